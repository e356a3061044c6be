#!/bin/bash
# Profile the bench on one MI355X: kernel-trace stats + separate PMC passes.
# Usage (GPU box): bash tools/profile_round.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
# (no energy window and no C2 sub-record in the profiled runs: the kernel
# trace then holds exactly the bench line's timed and event-timed steps)
BENCH=("$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --energy-seconds 0 --c2-steps 0 --record-path-bytes 0 "$@")
# the kernel trace runs the bench's default step count, so that the summary's
# per-dispatch durations include the steady state (tools/pmc_traffic.py also
# writes the average over the dispatches after the first few)
KT_BENCH=("$REPO/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --energy-seconds 0 --c2-steps 0 --record-path-bytes 0 "$@")
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "${KT_BENCH[@]}" > "$OUT/kt_bench.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_MFMA"; do
  NAME=$(echo "$C" | tr ' ' '_' | cut -c1-40)
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/pmc_$NAME" -o run -- python3 "${BENCH[@]}" > "$OUT/pmc_$NAME.log" 2>&1 || { echo "pmc pass $NAME failed"; exit 1; }
done
echo "profile done: $OUT"
