set -o pipefail
# C4 with sparse rank words and the scratch-free multi-snapshot k_conj; then
# kernel traces + DRAM bytes of and3 / or20 / or1000 / c4 at this lib_id
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 200 python -u tools/c4_bench.py > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c4.json')); print('c4', d['ms_per_step'], d['multi_plan_kernels_ms'], d['fg_search_sharded']['ms_per_batch'])"
timeout -k 10 1000 bash tools/profile_workloads.sh r05l and3 or20 or1000 c4 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
cd $GRAFT_REPO_ROOT
for W in and3 or20 or1000 c4; do
  D=gpurun_out/prof_r05l/$W
  python3 tools/pmc_summary.py $D/dram > $D/dram.json 2>/dev/null && python3 -c "
import json; d=json.load(open('$D/dram.json'))
for k in ('k_conj','k_disj'):
    if k in d: print('$W', k, 'DRAM GB per launch', round(32*(d[k]['TCC_EA0_RDREQ_DRAM_32B']+d[k]['TCC_EA0_WRREQ_WRITE_DRAM_32B'])/1e9, 3))
"
  grep -h "k_conj\|k_disj" $D/kernel_stats.csv | cut -d, -f1-8
done
# GET /search during commits under runtime settings: more hardware queues per
# process (streams otherwise share HIP's default 4), copies without the SDMA engines
for V in "GPU_MAX_HW_QUEUES=16" "HSA_ENABLE_SDMA=0" "GPU_MAX_HW_QUEUES=16 HSA_ENABLE_SDMA=0"; do
  N=$(echo $V | tr ' =' '__')
  env $V timeout -k 10 400 python -u tools/stall_trace.py run --out $O/stall_$N > $O/stall_$N.json 2> $O/stall_$N.err || { tail -30 $O/stall_$N.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/stall_$N/bench.json')); a=d['db_api_default_search']; c=d['commit']
print('$V idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p99_ms','max_ms','searches')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
