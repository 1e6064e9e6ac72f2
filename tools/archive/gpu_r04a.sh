set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 20 > $O/bench_and.json 2> $O/bench_and.err && tail -c 600 $O/bench_and.json
timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 10 --disj --k 1000 > $O/bench_or.json 2> $O/bench_or.err && tail -c 600 $O/bench_or.json
