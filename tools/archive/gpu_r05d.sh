set -o pipefail
# round 5: per-query floors across shards (k_seed ladders): correctness, then the
# C5 shards alone (unseeded / per-term floors / per-query floors) vs linked
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_floor.py tests/test_gpu_seed.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u tools/c5_bench.py > $O/c5.json 2> $O/c5.err || { tail -30 $O/c5.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c5.json'))
print(json.dumps({k: d[k] for k in ('ms_per_step','multi_plan_kernels_ms','k_disj_ms_per_shard_linked_mean','k_disj_ms_per_shard_independent','multi_plan_unseeded','same_hits_seeded_unseeded')}))"
