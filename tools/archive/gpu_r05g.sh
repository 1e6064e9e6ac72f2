set -o pipefail
# XCD query partition (FUGU_XCD_PART=1: queries probing one list on one XCD's L2)
# vs the doc sweep: time (k_conj headline, OR top-20 / top-1000), then L2 hit /
# miss and DRAM counters of each for the headline AND batch
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 500 python -u tools/ab_env.py --rounds 4 --workloads and3,or20,or1000 base: part:FUGU_XCD_PART=1 \
  > $O/ab_xcd.json 2> $O/ab_xcd.err || { tail -30 $O/ab_xcd.err; exit 1; }
grep "\[ab\]" $O/ab_xcd.err
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for V in base: part:FUGU_XCD_PART=1; do
  n=${V%%:*}
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_32B --output-format csv -d $R/$O/pmc_$n -o run -- python3 $R/tools/ab_env.py --rounds 1 --steps 2 --workloads and3,or20 $V > $R/$O/pmc_$n.log 2>&1 || { tail -20 $R/$O/pmc_$n.log; exit 1; }
  python3 $R/tools/pmc_summary.py $R/$O/pmc_$n > $R/$O/pmc_$n.json
  python3 -c "
import json; d=json.load(open('$R/$O/pmc_$n.json'))
for k in ('k_conj','k_disj'):
    c=d[k]; h,m=c['TCC_HIT_sum'],c['TCC_MISS_sum']; print('$n', k, 'L2 hit rate', round(h/(h+m),4), 'DRAM GB', round(32*c['TCC_EA0_RDREQ_DRAM_32B']/1e9,3))"
done
