set -o pipefail
# A/B of the packed (doc, score) lead layout (FG_LEADPACK) against the product
# shape, AND headline batch and OR top-1000 batch, interleaved rounds
O=gpurun_out/r04b; mkdir -p $O
V=fugu_amd/variants
A=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768l0.so
B=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768l1.so
timeout -k 10 500 python -u tools/ab_variants.py --rounds 2 $A $B > $O/ab_leadpack_and.log 2>&1 && tail -1 $O/ab_leadpack_and.log &&
timeout -k 10 500 python -u tools/ab_variants.py --rounds 2 --disj --k 1000 $A $B > $O/ab_leadpack_k1000.log 2>&1 && tail -1 $O/ab_leadpack_k1000.log
