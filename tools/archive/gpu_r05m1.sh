set -o pipefail
# final build: GET /search during commits, three more runs (the bar's robustness)
O=gpurun_out/r05m1; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$i.json 2> $O/db_$i.err || { tail -30 $O/db_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$i.json')); a=d['db_api_default_search']; c=d['commit']
print('run $i idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches','p99_over_idle_p99')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
