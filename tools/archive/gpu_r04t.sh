set -eo pipefail
# (1) the traffic model's line floor by array (OR top-1000, AND headline)
# (2) A/B of the multi-snapshot k_conj with / without deferred probes on C4 (bench.py --config c4)
O=gpurun_out/r04t; mkdir -p $O
FUGU_MODEL_TRACE=1 timeout -k 10 250 python -u bench.py --disj --k 1000 --no-cpu --no-extra --steps 3 --p50-queries 0 > $O/or.json 2> $O/or.err && grep "fg model" $O/or.err
FUGU_MODEL_TRACE=1 timeout -k 10 250 python -u bench.py --no-cpu --no-extra --steps 3 --p50-queries 0 > $O/and.json 2> $O/and.err && grep "fg model" $O/and.err
V=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768
for r in 0 1; do
  for m in 1 0; do
    FUGU_LIB=$V"e1m$m.so" timeout -k 10 200 python -u bench.py --config c4 --no-cpu --steps 10 > $O/c4_m${m}_r$r.json 2> $O/c4_m${m}_r$r.err || exit 1
    python -c "import json,sys; d=json.loads(open('$O/c4_m${m}_r$r.json').read().strip().splitlines()[-1]); print('m$m r$r', d['ms_per_step'], d['kernels_ms_per_step_max_rank'], d['result_sha1'])"
  done
done
# (3) the commit path after shared structure arrays / weights and pooled pinned read-backs
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_segments.py tests/test_host.py -m gpu > $O/segtests.log 2>&1 && tail -3 $O/segtests.log
timeout -k 10 300 python -u tools/rescore_bench.py > $O/rb.out 2> $O/rb.err && cat $O/rb.out
timeout -k 10 400 python -u tools/commit_trace.py --commits 24 > $O/commit.out 2> $O/commit.err && cat $O/commit.out
