#!/bin/bash
# Sample the GPU clock, power and temperature while a long C1 bench runs
# (is the kernel power-capped?).  Usage (GPU box): bash tools/clock_watch.sh [steps]
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/clock
mkdir -p "$OUT"
rocm-smi --showclocks --showpower --showtemp --showmaxpower > "$OUT/idle.txt" 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-bitexact --steps ${1:-300} --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" &
BP=$!
sleep 15
for i in 1 2 3 4 5 6; do
  rocm-smi --showclocks --showpower --showtemp > "$OUT/load_$i.txt" 2>&1
  sleep 4
done
wait $BP
echo "bench rc=$?"
