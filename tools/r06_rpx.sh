# round-6 record-path A/B of an environment switch (VAR, values VALS),
# standalone (tools/record_path_bench.py) and in bench.py; e.g.
# VAR=SG_RECORD_KD2H VALS="0 1", VAR=SG_STREAM_PRIO VALS="0 1 2"
VAR=${VAR:-SG_RECORD_KD2H}
set -uo pipefail
O=gpurun_out/${1:-r06z}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_record_layer.py tests/test_gpu_concurrency.py tests/test_gpu_loopback.py tests/test_abi.py > $O/rp_tests.log 2>&1; rc=$?; tail -2 $O/rp_tests.log; [ $rc -eq 0 ] || exit $rc
for kd in ${VALS:-0 1}; do
  t=$VAR$kd
  env $VAR=$kd timeout -k 10 200 python -u tools/record_path_bench.py --threads 8 --registered 0,1 --json-out $O/rp_$t.json > $O/rp_$t.log 2>&1 || { echo "$t failed"; tail -5 $O/rp_$t.log; exit 1; }
  env $VAR=$kd timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --c2-steps 3 --no-cpu-baseline --no-bitexact --energy-seconds 0 > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -5 $O/bench_$t.err; exit 1; }
  python - $O $t <<'PY'
import json, sys
o, t = sys.argv[1], sys.argv[2]
j = json.load(open(f"{o}/rp_{t}.json"))
for k, r in j["by_copy_threads"].items():
    print(t, "standalone", k, r["write_gibs"], r["read_gibs"], "duplex", r["duplex"]["gibs"], "vs_serial", r["duplex"]["vs_serial"], r["correct"] and r["duplex"]["correct"])
b = json.loads(open(f"{o}/bench_{t}.json").read().strip().splitlines()[-1])["record_path"]
for k in ("pageable", "registered"):
    r = b[k]
    print(t, "in-bench  ", k, r["write_gibs"], r["read_gibs"], "duplex", r["duplex"]["gibs"], "vs_serial", r["duplex"]["vs_serial"], r["correct"] and r["duplex"]["correct"] and r["wire_sample_ok"])
PY
done
