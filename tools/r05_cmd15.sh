#!/bin/bash
# round 5: C1 output stored straight from registers (wpr_dst, bit-exact) against
# the LDS staging + lane-contiguous read-out: C1 parity with the variant, then a
# same-box A/B with energy per record, then one WRITE_SIZE pass of each
set -uo pipefail
O=gpurun_out/r05m; mkdir -p $O
SURUGA_ALLOW_VARIANT=1 SURUGA_GPU_LIB=ablib/wpr_dst2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/dst_tests.log 2>&1
rc=$?; tail -2 $O/dst_tests.log; [ $rc -eq 0 ] || exit $rc
R=3 AB_TAG=_r05m timeout -k 10 900 bash tools/ab_libs.sh base=- dst2=ablib/wpr_dst2.so || exit 1
export TMPDIR=/tmp
for v in dst; do
  lib=suruga_amd/libsuruga_gpu.so; [ $v = dst ] && lib=ablib/wpr_dst2.so
  SURUGA_ALLOW_VARIANT=1 SURUGA_GPU_LIB=$lib timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_ws_$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bitexact --energy-seconds 0 --c2-steps 0 > $O/pmc_ws_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
