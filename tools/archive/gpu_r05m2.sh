set -o pipefail
# final build: C4 and C5 over 2 gloo ranks on this GPU (same result_sha1 as earlier rounds)
O=gpurun_out/r05m2; mkdir -p $O
FUGU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --config c5 --steps 3 --warmup 1 > $O/c5.json 2> $O/c5.err || { tail -30 $O/c5.err; exit 1; }
grep "^{" $O/c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c5', d['result_sha1'], d['value'])"
FUGU_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --config c4 --steps 5 --warmup 1 > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
grep "^{" $O/c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c4', d['result_sha1'], d['value'])"
