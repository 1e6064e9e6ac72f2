set -o pipefail
# round 5: k_seed correctness (seeded == unseeded == oracle) and the OR suites it
# runs under; A/B of the seed and of the layouts; GET /search during commits
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_seed.py tests/test_gpu_floor.py tests/test_gpu_parity.py tests/test_gpu_occur.py tests/test_gpu_multi.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u tools/ab_env.py --rounds 4 --workloads or20,or1000,and3 \
  seed: noseed:FUGU_SEED=0 rf2:FUGU_RANK_FACTOR=2 f32top16:FUGU_RANK_SKIP_TOP=16,FUGU_DENSE_GIB=0.6 \
  > $O/ab_layout.json 2> $O/ab_layout.err || { tail -30 $O/ab_layout.err; exit 1; }
grep "\[ab\]" $O/ab_layout.err
timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_api.json 2> $O/db_api.err || { tail -30 $O/db_api.err; exit 1; }
tail -c 2500 $O/db_api.json
