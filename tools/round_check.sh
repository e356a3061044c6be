#!/bin/bash
# GPU-box check of one build: the GPU suite, smoke(), and the two bench lines
# (C1 = the metric's config, C2 = Zipf), into gpurun_out/<tag>/.
# Usage (GPU box): bash tools/round_check.sh <tag>
set -uo pipefail
TAG=${1:-check}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -1 "$OUT/gpu_tests.log"
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err" || { echo "bench c1 failed"; exit 1; }
timeout -k 10 400 python -u bench.py --workload c2 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { echo "bench c2 failed"; exit 1; }
python - "$OUT" <<'PY'
import json, sys
for w in ("c1", "c2"):
    j = json.loads(open(f"{sys.argv[1]}/bench_{w}.json").read().strip().splitlines()[-1])
    print(w, j["value"], "ms/step", j["ms_per_step"], "frac", j["roofline"]["frac"], "kernel_ms", j["kernel_ms"]["seal"],
          j["kernel_ms"]["open"], j["kernel_ms"]["keying"], "correct", j["correct"], "cpu", (j["cpu_baseline"] or {}).get("value"),
          "traffic", j["roofline"].get("traffic"), "valu", (j.get("valu_roofline") or {}).get("frac"),
          "uJ", j.get("energy_per_record_uj"))
    if "c2" in j:
        c = j["c2"]
        print("  c2 sub-record", c["value"], "frac", c["roofline"]["frac"], "traffic", c["roofline"].get("traffic"),
              "valu", (c.get("valu_roofline") or {}).get("frac"), "correct", c["correct"], "fold", c.get("bitexact_fold"))
PY
# C4 host side and the loopback stream with the same build (round 4)
timeout -k 10 600 python -u tools/record_path_bench.py --registered 0,1 --json-out "$OUT/record_path.json" > "$OUT/record_path.log" 2>&1 || echo "record_path failed"
tail -c 400 "$OUT/record_path.log"; echo
timeout -k 10 600 python -u tools/tls_loopback.py --json-out "$OUT/loopback.json" --watchdog 500 > "$OUT/loopback.log" 2>&1 || echo "loopback failed"
tail -c 400 "$OUT/loopback.log"; echo
# C4 from C++ (round 5): staged and registered (zero-copy) buffers
for m in "" "--registered"; do
  tag=loopback_cpp${m:+_reg}
  timeout -k 10 300 ./tools/loopback_cpp $m --json-out "$OUT/$tag.json" > /dev/null 2> "$OUT/$tag.err" || echo "$tag failed"
done
python -c "
import json
for f in ('loopback_cpp', 'loopback_cpp_reg'):
    try:
        j = json.load(open('$OUT/' + f + '.json')); print(f, j['gibs'], j['correct'])
    except OSError as e:
        print(f, 'missing', e)
"

