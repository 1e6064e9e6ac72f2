set -o pipefail
# per-device plan-workspace / pinned pools (a commit's rescored snapshots reuse
# them): GPU tests of the db / segment / multi paths, GET /search during
# commits; the k_conj XCD split by lead list with single-list items on the sweep
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_host.py tests/test_gpu_segments.py tests/test_gpu_sharded.py tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/stall_trace.py run --out $O/stall > $O/stall.json 2> $O/stall.err || { tail -30 $O/stall.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/stall/bench.json')); a=d['db_api_default_search']; c=d['commit']
print('idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p99_ms','max_ms','searches','slowest_1pct_phases_ms_mean')}, 'commit', c['p50_ms'], c['p99_ms'])"
head -c 1500 $O/stall.json
timeout -k 10 600 python -u tools/ab_env.py --rounds 5 --workloads and3,mixed sweep:FUGU_XCD_PART=0 lead: \
  > $O/ab_xcd.json 2> $O/ab_xcd.err || { tail -30 $O/ab_xcd.err; exit 1; }
grep "\[ab\]" $O/ab_xcd.err | tail -2
