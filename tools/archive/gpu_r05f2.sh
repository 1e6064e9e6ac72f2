set -o pipefail
# final build: kernel traces + DRAM counters of the OR top-1000, OR top-20 and C4 lines
O=gpurun_out/r05f2; mkdir -p $O
timeout -k 10 1100 bash tools/profile_workloads.sh r05f or1000 or20 c4 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
