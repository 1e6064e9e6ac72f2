set -o pipefail
# k_conj XCD split: the GPU suites it touches, C4 (multi-snapshot) with and
# without it; the high-priority search stream: GET /search during commits with
# and without it
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multi.py tests/test_gpu_sharded.py tests/test_host.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for X in 1 0; do
  FUGU_XCD_PART=$X timeout -k 10 200 python -u tools/c4_bench.py > $O/c4_part$X.json 2> $O/c4_part$X.err || { tail -20 $O/c4_part$X.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/c4_part$X.json')); print('xcd_part=$X', d['ms_per_step'], d['multi_plan_kernels_ms'], d['fg_search_sharded']['ms_per_batch'])"
done
for P in 1 0; do
  FUGU_SEARCH_PRIO=$P timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_api_prio$P.json 2> $O/db_api_prio$P.err || { tail -30 $O/db_api_prio$P.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_api_prio$P.json')); a=d['db_api_default_search']; c=d['commit']
print('prio=$P', {k: a[k] for k in ('p50_ms','p99_ms')}, {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','slowest_1pct_phases_ms_mean')}, {k: c[k] for k in ('p50_ms','p99_ms')})"
done
