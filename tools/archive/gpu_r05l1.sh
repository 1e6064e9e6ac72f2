set -o pipefail
# hardware counters (SQ / TCP / TCC / DRAM passes) of k_conj (headline) and k_disj
# (OR top-1000, OR top-20) at the final build
O=gpurun_out/r05l1; mkdir -p $O
timeout -k 10 400 bash tools/pmc_conj.sh final_and3 > $O/and3.log 2>&1 || { tail -20 $O/and3.log; exit 1; }
timeout -k 10 400 bash tools/pmc_conj.sh final_or1000 --disj --k 1000 > $O/or1000.log 2>&1 || { tail -20 $O/or1000.log; exit 1; }
timeout -k 10 400 bash tools/pmc_conj.sh final_or20 --disj --k 20 > $O/or20.log 2>&1 || { tail -20 $O/or20.log; exit 1; }
for W in and3 or1000 or20; do python3 -c "
import json; d=json.load(open('gpurun_out/pmc_final_$W/summary.json')); k='k_conj' if 'k_conj' in d else 'k_disj'; x=d[k]
w=x.get('SQ_WAIT_ANY',0)/max(x.get('SQ_WAVE_CYCLES',1),1); h=x.get('TCC_HIT_sum',0); m=x.get('TCC_MISS_sum',0)
print('$W', k, 'wait/wave', round(w,3), 'L2 hit', round(h/max(h+m,1),3), 'DRAM GB', round(32*(x.get('TCC_EA0_RDREQ_DRAM_32B',0)+x.get('TCC_EA0_WRREQ_WRITE_DRAM_32B',0))/1e9,3))"; done
