#!/bin/bash
# round 5: three-slot record pipeline (default) against two (SG_RECORD_SLOTS=2):
# record-layer GPU tests, then the record path per direction, alternating, twice
set -uo pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_record_layer.py tests/test_gpu_loopback.py tests/test_cpp_host.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for ns in 2 3; do
    SG_RECORD_SLOTS=$ns timeout -k 10 300 python -u tools/record_path_bench.py --threads 8 --registered 0,1 --json-out $O/rp_s${ns}_$i.json > $O/rp_s${ns}_$i.log 2>&1 || { echo "rp $ns failed"; tail $O/rp_s${ns}_$i.log; exit 1; }
    python -c "
import json
j = json.load(open('$O/rp_s${ns}_$i.json'))
for k, r in j['by_copy_threads'].items(): print('slots $ns run $i', k, r['write_gibs'], r['read_gibs'], r['correct'])
"
  done
done
