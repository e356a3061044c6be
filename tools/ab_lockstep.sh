#!/bin/bash
# Same-box A/B of the two kernel forms for uniform 16 KiB-class batches
# (sg_set_lockstep / SG_LOCKSTEP): alternating bench runs of the size-class
# kernel (A, SG_LOCKSTEP=0) and the lock-step kernel (B, SG_LOCKSTEP=1).
# Usage: bash tools/ab_lockstep.sh [rounds] [bench args...]
set -euo pipefail
R=${1:-2}; shift || true
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/ab_ls
mkdir -p "$OUT"
for i in $(seq 1 "$R"); do
  SG_LOCKSTEP=0 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/a_$i.json"
  SG_LOCKSTEP=1 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/b_$i.json"
done
python - "$OUT" "$R" <<'PY'
import json, sys
out, r = sys.argv[1], int(sys.argv[2])
for tag in "ab":
    v = [json.loads(open(f"{out}/{tag}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, r + 1)]
    print(tag, [x["value"] for x in v], "seal", [x["kernel_ms"]["seal"] for x in v], "open",
          [x["kernel_ms"]["open"] for x in v], "correct", [x["correct"] for x in v])
PY
