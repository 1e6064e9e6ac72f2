set -o pipefail
# final build (lib_id of HEAD): the whole GPU suite, then rocprofv3 kernel traces +
# DRAM counters of the headline and C3 bench lines
O=gpurun_out/r05f1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/profile_workloads.sh r05f and3 c3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
