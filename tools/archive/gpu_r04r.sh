set -o pipefail
# C5 / C4 rocprofv3 passes, then the N = 2 rehearsal on one GPU (gloo)
timeout -k 10 700 bash tools/profile_workloads.sh r04b c5 c4 > gpurun_out/prof_r04b.log 2>&1 || { tail -20 gpurun_out/prof_r04b.log; exit 1; }
tail -2 gpurun_out/prof_r04b.log
mkdir -p gpurun_out/r04r
FUGU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --no-cpu --no-extra --steps 10 > gpurun_out/r04r/bench_n2_gloo.json 2> gpurun_out/r04r/bench_n2_gloo.err || { tail -30 gpurun_out/r04r/bench_n2_gloo.err; exit 1; }
tail -c 1500 gpurun_out/r04r/bench_n2_gloo.json
