set -o pipefail
# (1) GPU tests of the db / commit / segment paths with CU-masked background
# streams; (2) GET /search during commits: background work on 3/4 of the CUs
# (default), 1/2, and unmasked low-priority streams (FUGU_BG_CU_FRAC=1);
# (3) the XCD query groups balanced per launch set (single-list items apart)
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_host.py tests/test_gpu_segments.py tests/test_gpu_sharded.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for F in 0.75 1 0.5; do
  FUGU_BG_CU_FRAC=$F timeout -k 10 400 python -u tools/stall_trace.py run --out $O/stall_$F > $O/stall_$F.json 2> $O/stall_$F.err || { tail -30 $O/stall_$F.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/stall_$F/bench.json')); a=d['db_api_default_search']; c=d['commit']
print('bg_cu_frac=$F idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p99_ms','max_ms','searches')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
timeout -k 10 600 python -u tools/ab_env.py --rounds 5 --workloads and3,mixed sweep:FUGU_XCD_PART=0 second: lead:FUGU_XCD_KEY=0 \
  > $O/ab_xcd_key.json 2> $O/ab_xcd_key.err || { tail -30 $O/ab_xcd_key.err; exit 1; }
grep "\[ab\]" $O/ab_xcd_key.err | tail -2
