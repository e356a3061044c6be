#!/bin/bash
# round 5: record layer (zero-copy path with device framing): tests, C++ loopback and record-path lines
set -uo pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_record_layer.py tests/test_gpu_loopback.py tests/test_cpp_host.py tests/test_gpu_concurrency.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; fi
for m in "" "--registered"; do
  tag=loopback_cpp${m:+_reg}
  timeout -k 10 300 ./tools/loopback_cpp $m --json-out $O/$tag.json > /dev/null 2> $O/$tag.err || { echo "$tag failed"; tail $O/$tag.err; exit 1; }
done
python -c "
import json
for f in ('loopback_cpp', 'loopback_cpp_reg'):
    j = json.load(open('$O/' + f + '.json')); print(f, j['gibs'], j['correct'], 'W', j['writer']['per_gib_ms'], 'R', j['reader']['per_gib_ms'])
"
timeout -k 10 600 python -u tools/record_path_bench.py --threads 8 --registered 0,1 --json-out $O/record_path.json > $O/record_path.log 2>&1 || { echo record path failed; tail $O/record_path.log; exit 1; }
python -c "
import json
j = json.load(open('$O/record_path.json'))
for k, r in j['by_copy_threads'].items(): print(k, r['write_gibs'], r['read_gibs'], r['correct'], r['write_split'], r['read_split'])
"
