set -o pipefail
# with the K-th reuse: GET /search during commits under a background grid cap
# (2 / 4 per CU) and one background stream, against the default
O=gpurun_out/r05j1; mkdir -p $O
for V in "FUGU_BG_GRID=0" "FUGU_BG_GRID=2" "FUGU_BG_GRID=4" "FUGU_BG_STREAMS=1"; do
  N=$(echo $V | tr ' =' '__')
  env $V timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$N.json 2> $O/db_$N.err || { tail -30 $O/db_$N.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$N.json')); a=d['db_api_default_search']; c=d['commit']
print('$V idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches','p99_over_idle_p99')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
