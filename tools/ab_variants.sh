#!/bin/bash
# Time experiment builds of the library side by side on one box.
# Usage: bash tools/ab_variants.sh <tag>=<env assignments or lib path> ... (see below)
#   each argument is NAME:LIB:LOCKSTEP, LIB "-" = the product library
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/abv
mkdir -p "$OUT"
for spec in "$@"; do
  IFS=: read -r name lib ls <<< "$spec"
  if [ "$lib" = "-" ]; then
    SG_LOCKSTEP=$ls timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > "$OUT/$name.json" 2> "$OUT/$name.err"; rc=$?; [ $rc -eq 0 -o $rc -eq 3 ] || exit 1
  else
    SURUGA_GPU_LIB=$lib SG_LOCKSTEP=$ls timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > "$OUT/$name.json" 2> "$OUT/$name.err"; rc=$?; [ $rc -eq 0 -o $rc -eq 3 ] || exit 1
  fi
  python -c "import json,sys; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], 'seal', d['kernel_ms']['seal'], 'open', d['kernel_ms']['open'], 'correct', d['correct'])"
done
