set -o pipefail
# the commit path after pinned staging of a build's uploads: segment / host GPU tests, commit trace
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_segments.py tests/test_host.py -m gpu > $O/segtests.log 2>&1 || { tail -30 $O/segtests.log; exit 1; }
tail -2 $O/segtests.log
timeout -k 10 400 python -u tools/commit_trace.py --commits 24 > $O/commit.out 2> $O/commit.err && cat $O/commit.out
