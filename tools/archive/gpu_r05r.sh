set -o pipefail
# stream-ordered allocations keep their pool; background streams low priority (no
# CU mask); multi-snapshot k_conj items divided over the snapshots: GPU tests of
# the db / segment / multi paths, GET /search during commits, k_disj parts split
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_host.py tests/test_gpu_segments.py tests/test_gpu_multi.py tests/test_gpu_sharded.py tests/test_gpu_occur.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/db_api_bench.py --no-ref > $O/db_api.json 2> $O/db_api.err || { tail -30 $O/db_api.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/db_api.json')); a=d['db_api_default_search']; c=d['commit']
print('idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p99_ms','max_ms','searches','p99_over_idle_p99','slowest_1pct_phases_ms_mean')}, 'commit', c['p50_ms'], c['p99_ms'])"
timeout -k 10 400 python -u tools/c5_parts.py > $O/c5_parts.json 2> $O/c5_parts.err || { tail -30 $O/c5_parts.err; exit 1; }
grep "\[parts\]" $O/c5_parts.err
timeout -k 10 400 python -u tools/c4_ab.py --units 1 --rounds 7 base: gpq8:FUGU_CONJ_GPQ=8 gpq32:FUGU_CONJ_GPQ=32 maxg16:FUGU_CONJ_MAXGROUP=16 gpq8maxg16:FUGU_CONJ_GPQ=8,FUGU_CONJ_MAXGROUP=16 gpq4maxg32:FUGU_CONJ_GPQ=4,FUGU_CONJ_MAXGROUP=32 > $O/and3_ab.json 2> $O/and3_ab.err || { tail -30 $O/and3_ab.err; exit 1; }
grep "\[ab\]" $O/and3_ab.err
