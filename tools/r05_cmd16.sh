#!/bin/bash
# round 5: the packed kernel's chunk rounds split into before / in / after the
# ChaCha20 asm (s_memtime sums of wave 0, tools/variants/pk_prof2.py), with
# three (the product), two and one workgroup(s) per CU
set -uo pipefail
O=gpurun_out/r05p; mkdir -p $O
for v in pk_prof2 pk_prof2_wg2 pk_prof2_wg1; do
  echo "== $v"
  SURUGA_ALLOW_VARIANT=1 SURUGA_GPU_LIB=ablib/$v.so timeout -k 10 300 python tools/pack_phase.py > $O/$v.txt 2>&1 || { echo "$v failed"; tail $O/$v.txt; exit 1; }
  grep -v amdgpu.ids $O/$v.txt
done
