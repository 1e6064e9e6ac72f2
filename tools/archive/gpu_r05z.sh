set -o pipefail
# background scorings capped at FUGU_BG_GRID workgroups per CU per launch, read-back
# by a copy kernel: correctness (ktop, segments, db), then searches beside rescores
# and GET /search during commits per cap
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ktop.py tests/test_gpu_segments.py tests/test_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for V in 2 1 4 0; do
  FUGU_BG_GRID=$V timeout -k 10 300 python -u tools/rescore_stall.py --rescores 12 > $O/rs_$V.json 2> $O/rs_$V.err || { tail -30 $O/rs_$V.err; exit 1; }
  echo "grid $V $(cat $O/rs_$V.json)"
done
for V in 2 1; do
  FUGU_BG_GRID=$V timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$V.json 2> $O/db_$V.err || { tail -30 $O/db_$V.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$V.json')); a=d['db_api_default_search']; c=d['commit']
print('grid $V idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches','p99_over_idle_p99')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
