set -o pipefail
# rescores without new deletions reuse the base's K-th scores as a scaled lower
# bound (no k_ktop): GPU tests, searches beside rescores, GET /search during commits
O=gpurun_out/r05h1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ktop.py tests/test_host.py tests/test_gpu_segments.py tests/test_gpu_floor.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/rescore_stall.py --rescores 12 > $O/rs.json 2> $O/rs.err || { tail -30 $O/rs.err; exit 1; }
echo "reuse $(cat $O/rs.json)"
for V in 1 0; do
  FUGU_KTOP_REUSE=$V timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$V.json 2> $O/db_$V.err || { tail -30 $O/db_$V.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$V.json')); a=d['db_api_default_search']; c=d['commit']
print('reuse $V idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches','p99_over_idle_p99')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
