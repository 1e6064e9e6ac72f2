set -o pipefail
# A/B of k_disj's sub-tile split and bound 1 (FG_SUB=1) against tile-only (0): OR top-1000 / top-20
# (identical hashes = identical results), DRAM per launch of each, then the GPU suite on the default build
O=gpurun_out/r04s; mkdir -p $O
V=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768
timeout -k 10 400 python -u tools/ab_variants.py --disj --k 1000 --rounds 3 $V"b0.so" $V"b1.so" > $O/ab_k1000.log 2> $O/ab_k1000.err || { tail -20 $O/ab_k1000.err; exit 1; }
tail -1 $O/ab_k1000.log
timeout -k 10 400 python -u tools/ab_variants.py --disj --k 20 --rounds 3 $V"b0.so" $V"b1.so" > $O/ab_k20.log 2> $O/ab_k20.err || { tail -20 $O/ab_k20.err; exit 1; }
tail -1 $O/ab_k20.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for q in 0 1; do
  FUGU_LIB=$R/$V"b$q.so" timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B --output-format csv -d $R/$O/dram_b$q -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --p50-queries 0 --no-extra --disj --k 1000 > $R/$O/dram_b$q.log 2>&1 || exit 1
done
cd $R && python3 tools/pmc_summary.py $O/dram_b0 > $O/dram_b0.json && python3 tools/pmc_summary.py $O/dram_b1 > $O/dram_b1.json && grep -h -A2 '"k_disj"' $O/dram_b0.json $O/dram_b1.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_occur.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
