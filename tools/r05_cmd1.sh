set -uo pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 120 ./tools/valu_probe_nb2 > $O/probe_nb2.txt 2>&1 || { echo probe failed; cat $O/probe_nb2.txt; exit 1; }
cat $O/probe_nb2.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_full_size.py > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
R=3 AB_TAG=_r05a timeout -k 10 600 bash tools/ab_libs.sh base=- sw4=ablib/wpr_sw4.so || exit 1
