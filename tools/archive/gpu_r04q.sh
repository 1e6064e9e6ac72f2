set -o pipefail
# A/B of k_disj bound 2 from u8 tile-relative posting bounds (FG_QB2=1) against psc (0):
# OR top-1000 and top-20 (identical hashes = identical results), then DRAM bytes of each
O=gpurun_out/r04q; mkdir -p $O
V=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768
timeout -k 10 400 python -u tools/ab_variants.py --disj --k 1000 --rounds 3 $V"q0.so" $V"q1.so" > $O/ab_k1000.log 2> $O/ab_k1000.err || { tail -20 $O/ab_k1000.err; exit 1; }
cat $O/ab_k1000.log
timeout -k 10 400 python -u tools/ab_variants.py --disj --k 20 --rounds 3 $V"q0.so" $V"q1.so" > $O/ab_k20.log 2> $O/ab_k20.err || { tail -20 $O/ab_k20.err; exit 1; }
cat $O/ab_k20.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for q in 0 1; do
  FUGU_LIB=$R/$V"q$q.so" timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B --output-format csv -d $R/$O/dram_q$q -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --p50-queries 0 --no-extra --disj --k 1000 > $R/$O/dram_q$q.log 2>&1 || exit 1
done
cd $R && python3 tools/pmc_summary.py $O/dram_q0 > $O/dram_q0.json; python3 tools/pmc_summary.py $O/dram_q1 > $O/dram_q1.json; cat $O/dram_q0.json $O/dram_q1.json | head -60
