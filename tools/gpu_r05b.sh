set -o pipefail
# round 5 A/B batch:
#  1. snapshot layouts (rank-word budget for the HBM footprint; f32 score tables
#     in place of rank words for the densest terms), AND + OR, one process
#  2. k_disj item size (tiles per item, items per query: the concurrent doc
#     window each XCD's L2 has to hold), time at k = 20 / 1000 ...
#  3. ... and the DRAM bytes per k_disj launch at k = 20 (one --pmc pass each)
O=gpurun_out/r05b; mkdir -p $O
V=fugu_amd/variants
B=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768.so
G16=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o128_16z12y11u5r512h9g1s16k32768.so
G8=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o256_8z12y11u5r512h9g1s16k32768.so
timeout -k 10 600 python -u tools/ab_env.py --rounds 4 --workloads and3,or1000,or20 \
  base: rf2:FUGU_RANK_FACTOR=2 rf2.5:FUGU_RANK_FACTOR=2.5 f32top16:FUGU_RANK_SKIP_TOP=16,FUGU_DENSE_GIB=0.6 \
  > $O/ab_layout.json 2> $O/ab_layout.err || { tail -30 $O/ab_layout.err; exit 1; }
grep "\[ab\]" $O/ab_layout.err
for K in 20 1000; do
  timeout -k 10 400 python -u tools/ab_variants.py --disj --k $K --steps 6 --rounds 2 $B $G16 $G8 > $O/ab_items_k$K.log 2>&1 || { tail -20 $O/ab_items_k$K.log; exit 1; }
  tail -1 $O/ab_items_k$K.log
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in $B $G16 $G8; do
  n=$(basename $L .so)
  FUGU_LIB=$R/$L timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B --output-format csv -d $R/$O/pmc_$n -o run -- python3 $R/tools/ab_variants.py --child --disj --k 20 --steps 3 > $R/$O/pmc_$n.log 2>&1 || { tail -20 $R/$O/pmc_$n.log; exit 1; }
  python3 $R/tools/pmc_summary.py $R/$O/pmc_$n > $R/$O/pmc_$n.json
  echo $n; grep -A3 k_disj $R/$O/pmc_$n.json | head -4
done
