set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
L=fugu_amd/libfugu.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_parity.py tests/test_gpu_ktop.py tests/test_host.py tests/test_gpu_occur.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/rescore_bench.py > $O/rb.out 2> $O/rb.err && cat $O/rb.out
timeout -k 10 300 python -u tools/ab_variants.py --rounds 2 $L "$L@FUGU_SWEEP_TERM=1" > $O/ab_sweep_and.log 2>&1 && tail -1 $O/ab_sweep_and.log
timeout -k 10 300 python -u tools/ab_variants.py --rounds 2 --disj --k 1000 $L "$L@FUGU_SWEEP_TERM=1" > $O/ab_sweep_k1000.log 2>&1 && tail -1 $O/ab_sweep_k1000.log
