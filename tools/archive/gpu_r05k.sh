set -o pipefail
# (1) where the plain / sparse rank split goes (df >= N/32 default, N/16, N/8, N/4);
# (2) what the k_conj XCD split groups queries by; (3) the stall trace of GET
# /search during commits; (4) k_disj item sizes, time then DRAM bytes
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 700 python -u tools/ab_env.py --rounds 5 --workloads and3,mixed,or1000,or20 p32: p16:FUGU_RANK_PLAIN_DIV=16 p8:FUGU_RANK_PLAIN_DIV=8 p4:FUGU_RANK_PLAIN_DIV=4 \
  > $O/ab_rank_split.json 2> $O/ab_rank_split.err || { tail -30 $O/ab_rank_split.err; exit 1; }
grep "\[ab\]" $O/ab_rank_split.err
timeout -k 10 600 python -u tools/ab_env.py --rounds 5 --workloads and3,mixed sweep:FUGU_XCD_PART=0 second: lead:FUGU_XCD_KEY=0 last:FUGU_XCD_KEY=2 query:FUGU_XCD_KEY=q \
  > $O/ab_xcd_key.json 2> $O/ab_xcd_key.err || { tail -30 $O/ab_xcd_key.err; exit 1; }
grep "\[ab\]" $O/ab_xcd_key.err | tail -2
timeout -k 10 600 python -u tools/stall_trace.py run --out $O/stall > $O/stall.json 2> $O/stall.err || { tail -30 $O/stall.err; tail -30 $O/stall/trace.err; exit 1; }
head -c 3000 $O/stall.json
