set -o pipefail
# k_disj item-size ramp (FUGU_DISJ_RAMP): the first items of every query short
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 400 python -u tools/c4_ab.py --units 1 --mode 1 --terms 2,5 --k 1000 --rounds 5 base: ramp2:FUGU_DISJ_RAMP=2 ramp3:FUGU_DISJ_RAMP=3 ramp5:FUGU_DISJ_RAMP=5 ramp8:FUGU_DISJ_RAMP=8 > $O/or1000_ramp.json 2> $O/or1000_ramp.err || { tail -30 $O/or1000_ramp.err; exit 1; }
grep "\[ab\]" $O/or1000_ramp.err
timeout -k 10 400 python -u tools/c4_ab.py --units 1 --mode 1 --terms 2,5 --k 20 --rounds 5 base: ramp2:FUGU_DISJ_RAMP=2 ramp3:FUGU_DISJ_RAMP=3 ramp5:FUGU_DISJ_RAMP=5 ramp8:FUGU_DISJ_RAMP=8 > $O/or20_ramp.json 2> $O/or20_ramp.err || { tail -30 $O/or20_ramp.err; exit 1; }
grep "\[ab\]" $O/or20_ramp.err
