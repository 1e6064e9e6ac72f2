set -o pipefail
# confirm: one background stream against eight (each twice), and one stream with a 2-per-CU cap
O=gpurun_out/r05j2; mkdir -p $O
for V in "FUGU_BG_STREAMS=1" "FUGU_BG_STREAMS=8" "FUGU_BG_STREAMS=1" "FUGU_BG_STREAMS=8" "FUGU_BG_STREAMS=1 FUGU_BG_GRID=2"; do
  N=$(echo $V | tr ' =' '__')_$RANDOM
  env $V timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$N.json 2> $O/db_$N.err || { tail -30 $O/db_$N.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$N.json')); a=d['db_api_default_search']; c=d['commit']
print('$V idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches','p99_over_idle_p99')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
