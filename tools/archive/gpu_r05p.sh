set -o pipefail
# the histogram exchange between parts of the k_disj sweep (fg_plan_execute_part):
# GPU tests, the one-GPU C5 rehearsal (shards alone, exchanged at 1/16, 1/8, 1/4),
# C5 over 2 gloo ranks on this GPU (same result_sha1 as N = 1); the stall probe
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_floor.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 150 tools/stall_probe 1.5 > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; cat $O/probe.json; exit 1; }
cat $O/probe.json
timeout -k 10 500 python -u tools/c5_bench.py --steps 5 > $O/c5.json 2> $O/c5.err || { tail -30 $O/c5.err; exit 1; }
grep "\[bench\] C5" $O/c5.err
FUGU_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --config c5 --steps 5 --warmup 2 > $O/c5_n2_gloo.json 2> $O/c5_n2_gloo.err || { tail -30 $O/c5_n2_gloo.err; exit 1; }
head -c 1500 $O/c5_n2_gloo.json
timeout -k 10 400 python -u tools/c4_ab.py --rounds 7 base: snap:FUGU_XCD_KEY=s div2:FUGU_CONJ_SEG_DIV=2 div8:FUGU_CONJ_SEG_DIV=8 snapdiv2:FUGU_XCD_KEY=s,FUGU_CONJ_SEG_DIV=2 nopart:FUGU_XCD_PART=0 > $O/c4_ab.json 2> $O/c4_ab.err || { tail -30 $O/c4_ab.err; exit 1; }
grep "\[ab\]" $O/c4_ab.err
