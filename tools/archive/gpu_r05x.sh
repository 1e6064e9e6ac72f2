set -o pipefail
# searches beside a rescore's device work alone (no commit around it); GET /search
# during commits with the HIP runtime's direct dispatch off / on
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 300 python -u tools/rescore_stall.py > $O/rescore_stall.json 2> $O/rescore_stall.err || { tail -30 $O/rescore_stall.err; exit 1; }
cat $O/rescore_stall.json
for V in "AMD_DIRECT_DISPATCH=0" "AMD_DIRECT_DISPATCH=1"; do
  N=$(echo $V | tr ' =' '__')
  env $V timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$N.json 2> $O/db_$N.err || { tail -30 $O/db_$N.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$N.json')); a=d['db_api_default_search']; c=d['commit']
print('$V idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
