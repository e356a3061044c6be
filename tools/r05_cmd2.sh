#!/bin/bash
# round 5 check: GPU suite, swizzle A/B, default bench line (C1 + C2 sub-record + energy)
set -uo pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; fi
R=3 AB_TAG=_r05b timeout -k 10 600 bash tools/ab_libs.sh base=- sw4=ablib/wpr_sw4.so || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C1", j["value"], j["roofline"]["frac"], j["kernel_ms"], j["correct"], "energy", j["energy"])
c = j["c2"]
print("C2", c["value"], c["roofline"]["frac"], c["kernel_ms"]["seal"], c["kernel_ms"]["open"], c["correct"], c.get("bitexact_fold"), "energy", c["energy"])
PY
