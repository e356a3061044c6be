#!/bin/bash
# round 5 (after the toggle prune): GPU suite, then energy per record of the
# product and the C1 timing-only variants (same box)
set -uo pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; fi
R=2 AB_TAG=_r05d AB_ALLOW_WRONG=1 timeout -k 10 900 bash tools/ab_libs.sh base=- nomac=ablib/wpr_nomac.so nomfma=ablib/wpr_nomfma.so noff=ablib/wpr_noff.so noepi=ablib/wpr_noepi.so nopro=ablib/wpr_nopro.so sw4=ablib/wpr_sw4.so
