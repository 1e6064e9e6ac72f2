set -o pipefail
# A/B: k_disj bound 1 from sub-tile bounds (s1, LDS 31.9 KB) vs tile bounds (s0: u16 tile lengths, 29.8 KB) vs HEAD (30.4 KB);
# then the OR parity suites on s1
O=gpurun_out/r04sb; mkdir -p $O
V=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768
for k in 1000 20; do
  timeout -k 10 500 python -u tools/ab_variants.py --disj --k $k --rounds 3 fugu_amd/variants/libfugu_head.so $V"s0.so" $V"s1.so" > $O/ab_k$k.log 2> $O/ab_k$k.err || { tail -20 $O/ab_k$k.err; exit 1; }
  tail -1 $O/ab_k$k.log
done
FUGU_LIB=$GRAFT_REPO_ROOT/$V"s1.so" timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_occur.py tests/test_gpu_sharded.py tests/test_gpu_segments.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
