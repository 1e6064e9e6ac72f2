set -o pipefail
# A/B builds, interleaved rounds on one box (tools/ab_variants.py), all from one source tree
# (every variant spill-free in k_conj / k_disj's single-snapshot instantiations):
#   e0 = k_disj tile ranges from the bucket directory (round-3 shape), e1 = the tile directory
#   l1 = packed (doc, score) postings for the streamed lead / essential lists
#   p1 = k_conj probes a rank term's presence bitmap before its rank word
#   w1 = 40-doc rank words (40 presence bits + 24-bit rank)
#   b1 = k_disj bound 2 prunes a posting once its partial bound falls below the threshold
O=gpurun_out/r04c; mkdir -p $O
V=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768
timeout -k 10 600 python -u tools/ab_variants.py --rounds 2 ${V}l0e1p0w0b0.so ${V}l0e1p1w0b0.so ${V}l1e1p0w0b0.so ${V}l0e1p0w1b0.so ${V}l1e1p0w1b0.so > $O/ab_and.log 2>&1 && tail -1 $O/ab_and.log &&
timeout -k 10 600 python -u tools/ab_variants.py --rounds 2 --disj --k 1000 ${V}l0e1p0w0b0.so ${V}l0e1p0w0b1.so ${V}l0e1p0w1b0.so ${V}l0e1p0w1b1.so ${V}l1e1p0w0b0.so > $O/ab_k1000.log 2>&1 && tail -1 $O/ab_k1000.log &&
timeout -k 10 300 python -u tools/ab_variants.py --rounds 2 --disj --k 20 ${V}l0e1p0w0b0.so ${V}l0e1p0w0b1.so ${V}l0e1p0w1b1.so > $O/ab_k20.log 2>&1 && tail -1 $O/ab_k20.log
