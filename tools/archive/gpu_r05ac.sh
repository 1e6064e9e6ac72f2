set -o pipefail
# sparse-vs-plain rank-word split (FUGU_RANK_PLAIN_DIV: terms under N/div of the docs
# get sparse words; default 32): DRAM bytes per OR top-1000 / top-20 / AND launch
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05ac; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
DRAM="TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B"
BASE="--steps 5 --warmup 1 --no-cpu --p50-queries 0 --no-extra --no-model"
for DIV in 8 16 64; do
  for W in or1000 or20 and3; do
    case $W in or1000) A="--disj --k 1000";; or20) A="--disj --k 20";; and3) A="";; esac
    D=$O/d${DIV}_$W; mkdir -p $D
    FUGU_RANK_PLAIN_DIV=$DIV timeout -s KILL 300 rocprofv3 --pmc $DRAM --output-format csv -d $D/dram -o run -- python3 $R/bench.py $BASE $A > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
    cd $R; python3 tools/pmc_summary.py $D/dram > $D/dram.json; python3 -c "
import json; d=json.load(open('$D/dram.json')); b=json.loads(open('$D/bench.json').readline())
k='k_disj' if 'k_disj' in d else 'k_conj'
print('div $DIV $W', k, 'GB', round(32*(d[k]['TCC_EA0_RDREQ_DRAM_32B']+d[k]['TCC_EA0_WRREQ_WRITE_DRAM_32B'])/1e9,3), 'ms', b['roofline']['kernel_ms'])"; cd /tmp
  done
done
