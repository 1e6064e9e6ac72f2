set -o pipefail
# the GPU suite and the driver's default bench command at the frozen sources
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 450 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -30 $O/bench_full.err; exit 1; }
tail -c 3000 $O/bench_full.json
