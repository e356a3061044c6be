#!/bin/bash
# Same-box A/B of library builds: alternating bench runs (C1, 10 steps, no
# CPU baseline) of every NAME=LIB argument ("-" = the product library), R rounds.
# Variant libraries live in ablib/ (tools/exp/ does not travel to the GPU box).
# Usage (GPU box): R=2 bash tools/ab_libs.sh base=- v=ablib/lib_v.so ...
# BENCH_ARGS: extra bench.py arguments (e.g. --workload c2); AB_ALLOW_WRONG=1 times
# variants whose output is knowingly wrong (tools/archive/variants/, timing only)
set -uo pipefail
R=${R:-2}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/ab_libs${AB_TAG:-}
mkdir -p "$OUT"
for i in $(seq 1 "$R"); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "-" ]; then lib=suruga_amd/libsuruga_gpu.so; fi
    SURUGA_ALLOW_VARIANT=${SURUGA_ALLOW_VARIANT:-1} SURUGA_GPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-bitexact --steps 10 --c2-steps 0 --record-path-bytes 0 ${BENCH_ARGS:-} > "$OUT/${name}_$i.json"
    rc=$?
    # rc 3 = ran but not correct: accepted for timing-only variants (AB_ALLOW_WRONG=1)
    if [ $rc -ne 0 ] && ! { [ $rc -eq 3 ] && [ "${AB_ALLOW_WRONG:-0}" = 1 ]; }; then echo "$name rc=$rc"; exit $rc; fi
    python -c "import json; d=json.loads(open('$OUT/${name}_$i.json').read().strip().splitlines()[-1]); e=d.get('energy') or {}; print('$name', '$i', d['value'], 'seal', d['kernel_ms']['seal'], 'open', d['kernel_ms']['open'], 'keying', d['kernel_ms']['keying'], 'correct', d['correct'], 'W', e.get('board_power_w'), 'MHz', e.get('sclk_mhz'), 'uJ', e.get('seal_uj_per_record'), e.get('open_uj_per_record'))"
  done
done
