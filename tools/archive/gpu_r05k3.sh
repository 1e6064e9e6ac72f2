set -o pipefail
# final build: the part-order guard's GPU test, then the driver's default bench.py
# against the complete registry (every line's traffic at this lib_id)
O=gpurun_out/r05k3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_floor.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
head -c 1500 $O/bench.json
