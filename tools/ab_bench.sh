#!/bin/bash
# A/B a kernel variant on one GPU box: alternate bench runs of the product
# library (A) and an experiment build (B, via SURUGA_GPU_LIB) so that device
# and clock differences between boxes do not enter the comparison.
# Usage: bash tools/ab_bench.sh <variant.so> [rounds] [bench args...]
set -euo pipefail
B=$1; R=${2:-3}; shift 2 || shift $#
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/ab
mkdir -p "$OUT"
for i in $(seq 1 "$R"); do
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/a_$i.json"
  SURUGA_GPU_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/b_$i.json"
done
python - "$OUT" "$R" <<'PY'
import json, sys
out, r = sys.argv[1], int(sys.argv[2])
for tag in "ab":
    v = [json.loads(open(f"{out}/{tag}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, r + 1)]
    print(tag, [x["value"] for x in v], "seal", [x["kernel_ms"]["seal"] for x in v], "open", [x["kernel_ms"]["open"] for x in v])
PY
