set -o pipefail
# HEAD: smoke(), then the N = 2 headline path rehearsed over gloo on this one GPU
O=gpurun_out/r05g4; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
FUGU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 2 > $O/n2_gloo.json 2> $O/n2_gloo.err || { tail -30 $O/n2_gloo.err; exit 1; }
grep "^{" $O/n2_gloo.json | head -c 1200
