set -o pipefail
# k_conj items per query / chunks per item on the headline (3-term) and C3 (1-5 term) batches
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 400 python -u tools/c4_ab.py --units 1 --rounds 9 base: gpq8:FUGU_CONJ_GPQ=8 gpq8maxg16:FUGU_CONJ_GPQ=8,FUGU_CONJ_MAXGROUP=16 gpq12maxg12:FUGU_CONJ_GPQ=12,FUGU_CONJ_MAXGROUP=12 > $O/and3.json 2> $O/and3.err || { tail -30 $O/and3.err; exit 1; }
grep "\[ab\]" $O/and3.err
timeout -k 10 400 python -u tools/c4_ab.py --units 1 --rounds 9 --terms 1,5 base: gpq8:FUGU_CONJ_GPQ=8 gpq8maxg16:FUGU_CONJ_GPQ=8,FUGU_CONJ_MAXGROUP=16 gpq12maxg12:FUGU_CONJ_GPQ=12,FUGU_CONJ_MAXGROUP=12 > $O/c3.json 2> $O/c3.err || { tail -30 $O/c3.err; exit 1; }
grep "\[ab\]" $O/c3.err
