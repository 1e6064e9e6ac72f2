set -o pipefail
# stall probe: short-workgroup background kernels on 1 / 2 / 4 / 8 streams at once,
# under HIP's default hardware queues and 16 of them
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 120 tools/stall_probe 1.5 idle short short8 short8_lowprio short4_lowprio short2_lowprio idle > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; cat $O/probe.json; exit 1; }
cat $O/probe.json
GPU_MAX_HW_QUEUES=16 timeout -k 10 120 tools/stall_probe 1.5 idle short short8 short8_lowprio short4_lowprio short2_lowprio idle > $O/probe_hwq16.json 2> $O/probe_hwq16.err || { tail -20 $O/probe_hwq16.err; cat $O/probe_hwq16.json; exit 1; }
cat $O/probe_hwq16.json
