set -uo pipefail
O=gpurun_out/r06b; mkdir -p $O
for cfg in "dw0:SG_PIPE_DEVWAIT=0" "dw1:SG_PIPE_DEVWAIT=1" "dw2:SG_PIPE_DEVWAIT=2" "cs0:SG_COPY_STREAMS=0" "dw2cs0:SG_PIPE_DEVWAIT=2 SG_COPY_STREAMS=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python -u tools/record_path_bench.py --threads 8 --registered 1 --json-out $O/rp_$name.json > $O/rp_$name.log 2>&1 || { echo "$name failed"; tail -5 $O/rp_$name.log; exit 1; }
  python -c "
import json; j=json.load(open('$O/rp_$name.json'))
for k,r in j['by_copy_threads'].items(): print('$name', k, r['write_gibs'], r['read_gibs'], 'duplex', r['duplex']['gibs'], r['duplex']['vs_slower_single'], r['write_split'])"
done
