set -o pipefail
bash tools/gpu_r05t.sh && bash tools/gpu_r05s.sh
