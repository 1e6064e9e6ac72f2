#!/bin/bash
# rocprofv3 evidence for every bench.py line that carries a roofline (run on the
# MI355X box through gpurun):
#   calibration (once): tools/calib_fetch under --pmc FETCH_SIZE and under the
#     size-aware DRAM request counters (known byte / line counts);
#   per workload W: python3 bench.py <W's flags> under
#     1. --kernel-trace --stats  -> per-kernel durations (kernel_stats.csv)
#     2. --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B -> DRAM bytes
#   (separate passes: no trace domains with --pmc; each under its own limit).
# Then tools/pmc_registry.py files them by the bench line's workload_key.
#   bash tools/profile_workloads.sh TAG [W ...]     W in: and3 c3 or1000 or20 c5 c4
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:?tag}
shift
WL=${*:-and3 c3 or1000 or20 c5}
OUT=$R/gpurun_out/prof_$TAG
DRAM="TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B"
BASE="--steps 5 --warmup 1 --no-cpu --p50-queries 0 --no-extra --no-model"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ ! -d "$OUT/calib_dram" ]; then
  echo "[prof] calib"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- "$R/tools/calib_fetch" > "$OUT/calib_fetch.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $DRAM --output-format csv -d "$OUT/calib_dram" -o run -- "$R/tools/calib_fetch" > "$OUT/calib_dram.log" 2>&1
fi
for W in $WL; do
  case $W in
    and3) A="" ;;
    c3) A="--mixed" ;;
    or1000) A="--disj --k 1000" ;;
    or20) A="--disj --k 20" ;;
    c5) A="--config c5" ;;
    c4) A="--config c4" ;;
    *) echo "unknown workload $W"; exit 2 ;;
  esac
  D=$OUT/$W
  mkdir -p "$D"
  echo "$A" > "$D/bench_args.txt"
  echo "[prof] $W trace"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 "$R/bench.py" $BASE $A > "$D/trace_bench.json" 2> "$D/trace_bench.err"
  echo "[prof] $W dram"
  timeout -s KILL 420 rocprofv3 --pmc $DRAM --output-format csv -d "$D/dram" -o run -- python3 "$R/bench.py" $BASE $A > "$D/dram_bench.json" 2> "$D/dram_bench.err"
  find "$D/trace" -name "*kernel_stats.csv" -exec cp {} "$D/kernel_stats.csv" \;
done
echo "profile done: $OUT"
