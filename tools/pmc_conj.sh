#!/bin/bash
# Hardware-counter passes of the bench's k_conj (or k_disj: pass --disj --k 1000) (run on the MI355X box through
# gpurun).  One rocprofv3 --pmc run per pass (slot limits: 8 SQ, 4 TCP, 2 TA,
# 2 TD, 4 TCC), each under its own hard time limit, then tools/pmc_summary.py.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-conj}
shift || true
ARGS="--steps 3 --warmup 1 --no-cpu --p50-queries 0 --no-extra $*"
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$R/bench.py" $ARGS \
    > "$OUT/$name.log" 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum
pass tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_GUI_ACTIVE GRBM_COUNT
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_REQ_sum
pass dram TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json"
echo "pmc done: $OUT"
