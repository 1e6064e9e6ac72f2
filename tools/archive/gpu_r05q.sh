set -o pipefail
# stall probe: short workgroups vs long, priorities, stream-ordered allocation with
# the pool kept; C5 rehearsal (each shard's exchanged rounds back to back); C4 item
# counts per snapshot and the XCD key by snapshot
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 150 tools/stall_probe 1.5 idle short short_lowprio long_half long_half_lowprio spin_short_lowprio stream_lowprio malloc_async malloc_async_small malloc_async_keep idle > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; cat $O/probe.json; exit 1; }
cat $O/probe.json
timeout -k 10 400 python -u tools/c4_ab.py --rounds 7 base: div4:FUGU_CONJ_SEG_DIV=4 div8:FUGU_CONJ_SEG_DIV=8 div16:FUGU_CONJ_SEG_DIV=16 snapdiv8:FUGU_XCD_KEY=s,FUGU_CONJ_SEG_DIV=8 snapdiv16:FUGU_XCD_KEY=s,FUGU_CONJ_SEG_DIV=16 > $O/c4_ab.json 2> $O/c4_ab.err || { tail -30 $O/c4_ab.err; exit 1; }
grep "\[ab\]" $O/c4_ab.err
timeout -k 10 500 python -u tools/c5_bench.py --steps 5 > $O/c5.json 2> $O/c5.err || { tail -30 $O/c5.err; exit 1; }
grep "\[bench\] C5" $O/c5.err
