set -o pipefail
# what the k_conj XCD split groups by: the second list (default), the lead, the
# last list, or nothing (queries balanced by items) vs the doc sweep
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 600 python -u tools/ab_env.py --rounds 5 --workloads and3,mixed sweep:FUGU_XCD_PART=0 second: lead:FUGU_XCD_KEY=0 last:FUGU_XCD_KEY=2 query:FUGU_XCD_KEY=q \
  > $O/ab_xcd_key.json 2> $O/ab_xcd_key.err || { tail -30 $O/ab_xcd_key.err; exit 1; }
grep "\[ab\]" $O/ab_xcd_key.err
