#!/bin/bash
# LDS / VALU / MFMA counters of the C1 kernel, one rocprofv3 --pmc pass each
# (product library, tools/wpr_phase.py as the driver: 2 seal + 2 open launches).
# Usage (GPU box): bash tools/pmc_lds.sh <tag>
set -euo pipefail
TAG=${1:-lds}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for C in "$@"; do
  [ $i -eq 0 ] && { i=1; continue; }
  NAME=$(echo "$C" | tr ' ' '_' | cut -c1-60)
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$NAME" -o run -- python3 "$REPO/tools/wpr_phase.py" --lib "$REPO/suruga_amd/libsuruga_gpu.so" > "$OUT/$NAME.log" 2>&1 || echo "pass $NAME failed rc=$?"
done
echo "pmc done: $OUT"
