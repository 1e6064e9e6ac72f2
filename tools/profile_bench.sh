#!/bin/bash
# rocprofv3 evidence for bench.py (run on the MI355X box through gpurun):
#   1. kernel trace + stats of the bench command  -> per-kernel durations
#   2. FETCH_SIZE calibration on a known 1 GiB stream (tools/calib_fetch)
#   3. FETCH_SIZE of the bench command, 4. WRITE_SIZE of the bench command
#   (separate --pmc passes: TCC slots cannot hold both; no trace domains with --pmc)
# then tools/pmc_traffic.py -> per-launch HBM bytes.  Every step has its own limit.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r01}
shift || true
# --p50-queries 0: only the batch dispatches, so the trace's average k_conj
# duration is the batch kernel the bench's roofline line is computed on
ARGS="--steps 5 --warmup 1 --no-cpu --p50-queries 0 --no-extra $*"
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib" -o run -- "$R/tools/calib_fetch" > "$OUT/calib.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
python3 "$R/tools/pmc_traffic.py" "$OUT/fetch" "$OUT/write" "$OUT/calib" "$OUT/pmc.json"
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
echo "profile done: $OUT"
