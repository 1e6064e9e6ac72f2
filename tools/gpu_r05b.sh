set -o pipefail
# round 5: A/B of snapshot layouts (rank-word budget for the HBM footprint; f32
# score tables in place of rank words for the densest terms) on the 10M corpus
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u tools/ab_env.py --rounds 5 --workloads and3,or1000,or20,mixed \
  base: rf2:FUGU_RANK_FACTOR=2 rf2.5:FUGU_RANK_FACTOR=2.5 f32top16:FUGU_RANK_SKIP_TOP=16,FUGU_DENSE_GIB=0.6 \
  > $O/ab_layout.json 2> $O/ab_layout.err || { tail -30 $O/ab_layout.err; exit 1; }
grep "\[ab\]" $O/ab_layout.err
