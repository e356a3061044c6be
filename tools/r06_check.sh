#!/bin/bash
# Round-6 GPU steps (one gpurun call each, chained with &&, every step under
# its own time limit).  Usage (GPU box): bash tools/r06_check.sh <step> <tag>
#   rp    record-path tests and tools/record_path_bench.py (registered and
#         pageable, duplex) for the product and, if present, ablib/rp_base.so
#   arx   C1 A/B of the ARX-share timing variants (tools/variants/wpr_*.py)
set -uo pipefail
STEP=$1; TAG=${2:-r06}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
case $STEP in
  rp)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_concurrency.py tests/test_record_layer.py tests/test_gpu_loopback.py > "$OUT/rp_tests.log" 2>&1
    rc=$?; tail -3 "$OUT/rp_tests.log"; [ $rc -eq 0 ] || exit $rc
    for m in ${RP_MODES:-1}; do
      SG_COPY_STREAMS=$m timeout -k 10 400 python -u tools/record_path_bench.py --threads 8 --registered 0,1 --json-out "$OUT/record_path_cs$m.json" > "$OUT/record_path_cs$m.log" 2>&1 || { echo "record_path cs$m failed"; tail -20 "$OUT/record_path_cs$m.log"; exit 1; }
    done
    if [ -f ablib/rp_base.so ]; then
      SURUGA_ALLOW_VARIANT=foreign SURUGA_GPU_LIB=ablib/rp_base.so timeout -k 10 400 python -u tools/record_path_bench.py --threads 8 --registered 0,1 --json-out "$OUT/record_path_base.json" > "$OUT/record_path_base.log" 2>&1 || { echo "record_path base failed"; tail -20 "$OUT/record_path_base.log"; exit 1; }
    fi
    python - "$OUT" <<'PY'
import json, sys, os
for f in sorted(os.listdir(sys.argv[1])):
    if not (f.startswith("record_path") and f.endswith(".json")): continue
    p = os.path.join(sys.argv[1], f)
    if not os.path.exists(p): continue
    j = json.load(open(p))
    for k, r in j["by_copy_threads"].items():
        print(f, k, "write", r["write_gibs"], "read", r["read_gibs"], "duplex", r["duplex"]["gibs"], "vs_slower", r["duplex"]["vs_slower_single"], "vs_serial", r["duplex"]["vs_serial"], "ok", r["correct"], r["duplex"]["correct"])
PY
    ;;
  arx)
    SURUGA_ALLOW_VARIANT=foreign R=${R:-2} AB_TAG=_$TAG AB_ALLOW_WRONG=1 timeout -k 10 900 bash tools/ab_libs.sh base=- noarx=ablib/wpr_noarx.so noarx_bar=ablib/wpr_noarx_bar.so arxonly=ablib/wpr_arxonly.so nomac=ablib/wpr_nomac.so
    ;;
esac
