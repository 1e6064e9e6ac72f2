set -o pipefail
# timeline of GET /search during commits: rocprofv3 kernel + HIP API + copy traces
# of tools/db_api_bench.py, then what ran while each slow search kernel waited
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d $O/tl -o run -- python3 $R/tools/db_api_bench.py --no-ref > $O/db_api.json 2> $O/db_api.err || { tail -30 $O/db_api.err; exit 1; }
cd $R
timeout -k 10 300 python3 tools/stall_timeline.py $O/tl > $O/timeline.json 2> $O/timeline.err || { tail -20 $O/timeline.err; exit 1; }
head -c 6000 $O/timeline.json
find $O/tl -name "*hip_api_trace.csv" -delete
find $O/tl -name "*.csv" -exec gzip {} \;
du -sh $O
