#!/bin/bash
# round 5: GPU suite (zero-copy record path, C++ loopback), energy per record of
# the product and the C1 timing variants, C4 lines (record path, C++ loopback)
set -uo pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; fi
R=2 AB_TAG=_r05e AB_ALLOW_WRONG=1 timeout -k 10 900 bash tools/ab_libs.sh base=- nomac=ablib/wpr_nomac.so nomfma=ablib/wpr_nomfma.so noff=ablib/wpr_noff.so noepi=ablib/wpr_noepi.so nopro=ablib/wpr_nopro.so sw4=ablib/wpr_sw4.so || exit 1
timeout -k 10 300 ./tools/loopback_cpp --json-out $O/loopback_cpp.json > /dev/null 2> $O/loopback_cpp.err || { echo loopback staged failed; cat $O/loopback_cpp.err | tail; exit 1; }
timeout -k 10 300 ./tools/loopback_cpp --registered --json-out $O/loopback_cpp_reg.json > /dev/null 2> $O/loopback_cpp_reg.err || { echo loopback registered failed; tail $O/loopback_cpp_reg.err; exit 1; }
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
