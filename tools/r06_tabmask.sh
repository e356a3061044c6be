set -uo pipefail
# parity of the masked-table variant first (C2 full-size fold + packed tests), then timing
SURUGA_ALLOW_VARIANT=1 SURUGA_GPU_LIB=ablib/pk_tabmask.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "packed or mixed" tests/test_gpu_full_size.py > gpurun_out/r06q_tabmask_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06q_tabmask_tests.log; [ $rc -eq 0 ] || exit $rc
R=3 AB_TAG=_r06q BENCH_ARGS="--workload c2 --steps 40" timeout -k 10 800 bash tools/ab_libs.sh base=- tabmask=ablib/pk_tabmask.so
