set -o pipefail
# round 5, first GPU pass: the floor / ladder tests and the k_ktop kernels they
# touch, the driver's default bench (C5 with the independent shard lines), and a
# gloo N = 2 rehearsal of the headline's fan-out count
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 360 python -u -m pytest tests/test_gpu_floor.py tests/test_gpu_ktop.py tests/test_gpu_sharded.py tests/test_host.py tests/test_gpu_boundary.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 500 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -30 $O/bench_full.err; exit 1; }
tail -c 1500 $O/bench_full.json
FUGU_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { tail -30 $O/bench_n2_gloo.err; exit 1; }
tail -c 1500 $O/bench_n2_gloo.json
