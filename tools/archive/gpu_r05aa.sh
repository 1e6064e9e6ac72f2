set -o pipefail
# background read-back by a copy kernel (no cap); k_ktop chunk 32768 / 8192 / 4096
# (FUGU_LIB variants): searches beside rescores, GET /search during commits
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ktop.py tests/test_gpu_segments.py tests/test_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
V8=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k8192.so
V4=fugu_amd/variants/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k4096.so
for L in default $V8 $V4; do
  N=$(basename $L .so | tail -c 6)
  if [ $L = default ]; then E=""; else E="FUGU_LIB=$L"; fi
  env $E timeout -k 10 300 python -u tools/rescore_stall.py --rescores 12 > $O/rs_$N.json 2> $O/rs_$N.err || { tail -30 $O/rs_$N.err; exit 1; }
  echo "lib $N $(cat $O/rs_$N.json)"
  env $E timeout -k 10 300 python -u tools/db_api_bench.py --no-ref > $O/db_$N.json 2> $O/db_$N.err || { tail -30 $O/db_$N.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/db_$N.json')); a=d['db_api_default_search']; c=d['commit']
print('lib $N idle', a['p50_ms'], a['p99_ms'], 'during', {k: a['during_commits'][k] for k in ('p50_ms','p90_ms','p99_ms','max_ms','searches','p99_over_idle_p99')}, 'commit', c['p50_ms'], c['p99_ms'])"
done
