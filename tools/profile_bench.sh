#!/bin/bash
# rocprofv3 evidence for bench.py (run on the MI355X box through gpurun):
#   1. kernel trace + stats of the bench command  -> per-kernel durations
#   2-3. tools/calib_fetch (known byte / line counts) under --pmc FETCH_SIZE, then
#        under the size-aware DRAM request counters
#   4-6. the bench command under --pmc FETCH_SIZE, WRITE_SIZE, and the DRAM counters
#   (separate --pmc passes: a pass holds <= 4 TCC counters; no trace domains with --pmc)
# then tools/pmc_traffic.py -> per-launch HBM bytes.  Every step has its own limit.
#   bash tools/profile_bench.sh TAG [bench args...]   (default: the headline workload)
#   CALIB_FROM=<an earlier OUT dir> reuses its calib_fetch / calib_dram passes
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r02}
shift || true
# --p50-queries 0: only the batch dispatches, so the trace's average kernel
# duration is the batch kernel the bench's roofline line is computed on
ARGS="--steps 5 --warmup 1 --no-cpu --p50-queries 0 --no-extra $*"
OUT=$R/gpurun_out/prof_$TAG
DRAM="TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
echo "[prof] trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
if [ -n "${CALIB_FROM:-}" ]; then
  # the calibration of an earlier pass of the same call (same box, same counters)
  echo "[prof] calib from $CALIB_FROM"
  cp -r "$CALIB_FROM/calib_fetch" "$CALIB_FROM/calib_dram" "$OUT/"
else
  echo "[prof] calib"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- "$R/tools/calib_fetch" > "$OUT/calib_fetch.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $DRAM --output-format csv -d "$OUT/calib_dram" -o run -- "$R/tools/calib_fetch" > "$OUT/calib_dram.log" 2>&1
fi
echo "[prof] fetch"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
echo "[prof] write"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
echo "[prof] dram"
timeout -s KILL 300 rocprofv3 --pmc $DRAM --output-format csv -d "$OUT/dram" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/dram_bench.json" 2> "$OUT/dram_bench.err"
python3 "$R/tools/pmc_traffic.py" "$OUT" "$OUT/pmc.json"
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
echo "profile done: $OUT"
