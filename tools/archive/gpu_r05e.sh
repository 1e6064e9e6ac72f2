set -o pipefail
# GET /search during commits: do the latency path's small transfers queue behind
# a commit's bulk copies?  Copy engines for everything (FUGU_KCOPY=0), the
# compute-queue copy kernel for the small ones (default), every copy a blit
# kernel (HSA_ENABLE_SDMA=0)
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_host.py tests/test_gpu_boundary.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
FUGU_KCOPY=0 timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_api_sdma.json 2> $O/db_api_sdma.err || { tail -30 $O/db_api_sdma.err; exit 1; }
timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_api_kcopy.json 2> $O/db_api_kcopy.err || { tail -30 $O/db_api_kcopy.err; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_api_blit.json 2> $O/db_api_blit.err || { tail -30 $O/db_api_blit.err; exit 1; }
for f in sdma kcopy blit; do python3 -c "
import json; d=json.load(open('$O/db_api_$f.json')); a=d['db_api_default_search']; c=d['commit']
print('$f', {k: a[k] for k in ('p50_ms','p99_ms')}, a['during_commits'], {k: c[k] for k in ('p50_ms','p99_ms')})"; done
