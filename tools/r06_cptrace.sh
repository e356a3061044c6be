#!/bin/bash
# Kernel and memory-copy traces of the registered record path: standalone
# (tools/record_path_bench.py in-process) and inside the bench process.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/r06cp
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/standalone" -o run -- \
  python3 "$REPO/tools/record_path_bench.py" --child --registered 1 --bytes 268435456 > "$OUT/standalone.log" 2>&1 || { echo standalone failed; tail -5 "$OUT/standalone.log"; exit 1; }
tail -c 600 "$OUT/standalone.log"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/bench" -o run -- \
  python3 "$REPO/bench.py" --steps 2 --warmup 1 --c2-steps 0 --no-cpu-baseline --no-bitexact --energy-seconds 0 --record-path-bytes 268435456 > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench.log"; exit 1; }
echo done
