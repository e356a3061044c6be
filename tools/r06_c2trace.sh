#!/bin/bash
# Round 6: kernel timeline of C2 batches (rocprofv3 kernel trace, start/end of
# every dispatch) -> gpurun_out/<tag>/c2_trace/
set -uo pipefail
TAG=${1:-r06o}
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c2_trace" -o run -- python3 "$REPO/bench.py" --workload c2 --steps 6 --warmup 2 --no-cpu-baseline --no-bitexact --energy-seconds 0 --record-path-bytes 0 > "$OUT/c2_trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/c2_trace.log"; exit 1; }
find "$OUT/c2_trace" -name "*kernel_trace.csv" | head -3
