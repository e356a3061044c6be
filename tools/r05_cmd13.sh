#!/bin/bash
# round 5: wave placement probe (three 512-thread workgroups per CU), then the
# packed kernel's setup-rotation variant: its packed/C2 parity tests and a
# same-box C2 A/B against the product
set -uo pipefail
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 60 ./tools/hwid_probe > $O/hwid_probe.txt 2>&1 || { echo probe failed; cat $O/hwid_probe.txt; exit 1; }
cat $O/hwid_probe.txt
SURUGA_ALLOW_VARIANT=1 SURUGA_GPU_LIB=ablib/pk_setrot.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "packed or c2" -x -q --timeout 240 --timeout-method thread > $O/setrot_tests.log 2>&1
rc=$?; tail -2 $O/setrot_tests.log; [ $rc -eq 0 ] || exit $rc
R=3 AB_TAG=_r05k BENCH_ARGS="--workload c2 --steps 60" timeout -k 10 900 bash tools/ab_libs.sh base=- setrot=ablib/pk_setrot.so
