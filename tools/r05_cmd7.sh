#!/bin/bash
# round 5: record layer stream layouts (SG_COPY_STREAMS 0/1): tests, C++ loopback and record-path lines
set -uo pipefail
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_record_layer.py tests/test_gpu_loopback.py tests/test_cpp_host.py tests/test_gpu_concurrency.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; fi
for cs in 0 1; do
  export SG_COPY_STREAMS=$cs
  timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py tests/test_record_layer.py -k "overlap or zero_copy" -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests_cs$cs.log 2>&1; echo "cs=$cs tests rc=$?"; tail -1 $O/tests_cs$cs.log
  for m in "" "--registered"; do
    tag=loopback_cpp${m:+_reg}_cs$cs
    timeout -k 10 300 ./tools/loopback_cpp $m --json-out $O/$tag.json > /dev/null 2> $O/$tag.err || { echo "$tag failed"; tail $O/$tag.err; exit 1; }
  done
  timeout -k 10 600 python -u tools/record_path_bench.py --threads 8 --registered 0,1 --json-out $O/record_path_cs$cs.json > $O/record_path_cs$cs.log 2>&1 || { echo record path failed; tail $O/record_path_cs$cs.log; exit 1; }
done
python - <<'PY'
import json
O = "gpurun_out/r05g"
for cs in (0, 1):
    for f in ("loopback_cpp", "loopback_cpp_reg"):
        j = json.load(open(f"{O}/{f}_cs{cs}.json")); print(cs, f, j["gibs"], j["correct"], "W", j["writer"]["per_gib_ms"], "R", j["reader"]["per_gib_ms"])
    j = json.load(open(f"{O}/record_path_cs{cs}.json"))
    for k, r in j["by_copy_threads"].items(): print(cs, k, r["write_gibs"], r["read_gibs"], r["correct"], r["write_split"], r["read_split"])
PY
