set -o pipefail
bash tools/gpu_r05g.sh && bash tools/gpu_r05e.sh
