set -o pipefail
# GPU suite + the driver's default bench command on the current build
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 520 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -30 $O/bench_default.err; exit 1; }
tail -c 400 $O/bench_default.json
