#!/bin/bash
# Sample the GPU clock and power every second while a long bench runs (is the
# kernel power-capped?), then summarise the samples taken under load.
# Usage (GPU box): bash tools/clock_watch.sh [steps] [bench args...]
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/clock${CW_TAG:-}
mkdir -p "$OUT"
STEPS=${1:-2000}; shift || true
rocm-smi --showclocks --showpower --showtemp --showmaxpower > "$OUT/idle.txt" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-bitexact --steps "$STEPS" --warmup 3 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" &
BP=$!
: > "$OUT/samples.txt"
while kill -0 $BP 2>/dev/null; do
  { date +%s.%N; rocm-smi --showclocks --showpower --showtemp; } >> "$OUT/samples.txt" 2>&1
  sleep 1
done
wait $BP
echo "bench rc=$?"
python3 - "$OUT/samples.txt" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
pw = [float(x) for x in re.findall(r"Graphics Package Power \(W\): ([0-9.]+)", txt)]
sc = [int(x) for x in re.findall(r"sclk clock level: \S+ \((\d+)Mhz\)", txt)]
load = [(p, s) for p, s in zip(pw, sc) if p > 600]
if load:
    ps, ss = zip(*load)
    print(f"samples under load: {len(load)}; power W min/mean/max {min(ps):.0f}/{sum(ps)/len(ps):.0f}/{max(ps):.0f}; "
          f"sclk MHz min/mean/max {min(ss)}/{sum(ss)/len(ss):.0f}/{max(ss)}")
else:
    print("no sample under load")
PY
