set -o pipefail
# k_disj knobs after the block split: items per query (DGPQ), pass / flush size (DROUND), tiles per item (DGROUP)
O=gpurun_out/r04v; mkdir -p $O
L=$(ls fugu_amd/variants/*.so)
for k in 1000 20; do
  timeout -k 10 600 python -u tools/ab_variants.py --disj --k $k --rounds 2 $L > $O/ab_k$k.log 2> $O/ab_k$k.err || { tail -20 $O/ab_k$k.err; exit 1; }
  tail -1 $O/ab_k$k.log
done
