set -o pipefail
# sparse rank words: the rank layouts A/B (plain only = the round-4 layout; the
# plain/sparse split at df = N/32, N/128, N/512; budget factor 1), then the GPU suite
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 900 python -u tools/ab_env.py --rounds 5 --workloads and3,mixed,or1000,or20 old:FUGU_RANK_PLAIN_DIV=16384 p128: f1:FUGU_RANK_FACTOR=1 p32:FUGU_RANK_PLAIN_DIV=32 p512:FUGU_RANK_PLAIN_DIV=512 \
  > $O/ab_rank_layout.json 2> $O/ab_rank_layout.err || { tail -30 $O/ab_rank_layout.err; exit 1; }
grep "\[ab\]" $O/ab_rank_layout.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
