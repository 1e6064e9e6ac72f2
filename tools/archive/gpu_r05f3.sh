set -o pipefail
# final build: C5's kernel trace + DRAM counters, filed into the registry on the box,
# then the driver's default bench.py against that registry
O=gpurun_out/r05f3; mkdir -p $O/reg
timeout -k 10 800 bash tools/profile_workloads.sh r05f c5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
python3 tools/pmc_registry.py r05f r05 > $O/registry.log 2>&1 || { tail -20 $O/registry.log; exit 1; }
tail -6 $O/registry.log
cp profiles/latest.json $O/reg/ && cp -r profiles/r05/c5 $O/reg/
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
head -c 2500 $O/bench.json
