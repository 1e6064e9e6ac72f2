set -o pipefail
# final build: C4 and C5 traces + DRAM counters, every workload of prof_r05g filed
# into the registry on the box, then the driver's default bench.py against it
O=gpurun_out/r05k2; mkdir -p $O/reg
timeout -k 10 800 bash tools/profile_workloads.sh r05k c4 c5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
python3 tools/pmc_registry.py r05k r05 > $O/registry.log 2>&1 || { tail -20 $O/registry.log; exit 1; }
tail -6 $O/registry.log
cp profiles/latest.json $O/reg/ && cp -r profiles/r05/c4 profiles/r05/c5 $O/reg/
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
head -c 2500 $O/bench.json
