set -o pipefail
bash tools/gpu_r05e.sh && bash tools/gpu_r05b.sh
