set -o pipefail
# A/B: k_disj segments trimmed to their first..last essential block (FG_TRIM=1) vs whole tiles (0);
# then the OR parity suites on the trimmed build
O=gpurun_out/r04tr; mkdir -p $O
V=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768
for k in 1000 20; do
  timeout -k 10 400 python -u tools/ab_variants.py --disj --k $k --rounds 3 $V"t0.so" $V"t1.so" > $O/ab_k$k.log 2> $O/ab_k$k.err || { tail -20 $O/ab_k$k.err; exit 1; }
  tail -1 $O/ab_k$k.log
done
FUGU_LIB=$GRAFT_REPO_ROOT/$V"t1.so" timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_occur.py tests/test_gpu_sharded.py tests/test_gpu_segments.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
