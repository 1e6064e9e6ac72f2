set -o pipefail
# final build: the whole GPU suite, then kernel traces + DRAM counters of the
# headline, C3, OR top-1000 and OR top-20 lines
O=gpurun_out/r05k1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/profile_workloads.sh r05k and3 c3 or1000 or20 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
