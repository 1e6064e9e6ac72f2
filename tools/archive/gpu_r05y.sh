set -o pipefail
# bisect the stall of searches beside a rescore (tools/rescore_stall.py): skip the
# k_ktop pass (1), the tables' read-back (2), k_score / k_bucket / k_tsub (4)
O=gpurun_out/r05y; mkdir -p $O
for V in 0 1 2 4 3 6; do
  FUGU_DIAG_SCORE_SKIP=$V timeout -k 10 300 python -u tools/rescore_stall.py --rescores 12 > $O/skip_$V.json 2> $O/skip_$V.err || { tail -30 $O/skip_$V.err; exit 1; }
  echo "skip $V $(cat $O/skip_$V.json)"
done
