#!/bin/bash
# round 5: staggered start of the packed kernel's co-resident workgroups
# (tools/variants/pk_stagger.py): phase stamps, parity, same-box C2 A/B
set -uo pipefail
O=gpurun_out/r05q; mkdir -p $O
SURUGA_ALLOW_VARIANT=1 SURUGA_GPU_LIB=ablib/pk_stagger_prof.so timeout -k 10 300 python tools/pack_phase.py > $O/pk_stagger_prof.txt 2>&1 || { echo prof failed; tail $O/pk_stagger_prof.txt; exit 1; }
grep -v amdgpu.ids $O/pk_stagger_prof.txt
SURUGA_ALLOW_VARIANT=1 SURUGA_GPU_LIB=ablib/pk_stagger.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "packed or c2" -x -q --timeout 240 --timeout-method thread > $O/stagger_tests.log 2>&1
rc=$?; tail -1 $O/stagger_tests.log; [ $rc -eq 0 ] || exit $rc
R=3 AB_TAG=_r05q BENCH_ARGS="--workload c2 --steps 60" timeout -k 10 900 bash tools/ab_libs.sh base=- stagger=ablib/pk_stagger.so
