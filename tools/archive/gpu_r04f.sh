set -o pipefail
# rocprofv3 evidence of every roofline workload at the frozen sources (lib_id in profiles/latest.json)
python3 tools/lib_id.py
timeout -k 10 1150 bash tools/profile_workloads.sh r04f and3 c3 or1000 or20 c4 c5
