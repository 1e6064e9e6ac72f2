set -o pipefail
# GET /search during commits under: 1 background stream instead of 8; the search on
# a normal-priority stream; 2 hardware queues per process
O=gpurun_out/r05w; mkdir -p $O
for V in "FUGU_BG_STREAMS=1" "FUGU_BG_STREAMS=2" "FUGU_SEARCH_PRIO=0" "GPU_MAX_HW_QUEUES=2" "FUGU_BG_STREAMS=1 GPU_MAX_HW_QUEUES=2"; do
  N=$(echo $V | tr ' =' '__')
  env $V timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$N.json 2> $O/db_$N.err || { tail -30 $O/db_$N.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$N.json')); a=d['db_api_default_search']; c=d['commit']
print('$V idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
