set -o pipefail
# A/B: k_disj's hits into the query histogram + its threshold re-read at every flush (FG_MIDHIST=1) vs at item end only (0)
O=gpurun_out/r04mh; mkdir -p $O
V=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768
for k in 1000 20; do
  timeout -k 10 400 python -u tools/ab_variants.py --disj --k $k --rounds 3 $V"h0.so" $V"h1.so" > $O/ab_k$k.log 2> $O/ab_k$k.err || { tail -20 $O/ab_k$k.err; exit 1; }
  tail -1 $O/ab_k$k.log
done
