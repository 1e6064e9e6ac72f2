set -o pipefail
# ceiling of a better starting threshold: k_disj with every execute after the first starting at the
# threshold the previous one ended with (FUGU_DIAG_KEEP_THRESH, a diagnostic build) vs the product
O=gpurun_out/r04k; mkdir -p $O
for k in 1000 20; do
  timeout -k 10 200 python -u bench.py --disj --k $k --no-cpu --no-extra --steps 10 > $O/prod_k$k.json 2> $O/prod_k$k.err || exit 1
  FUGU_LIB=fugu_amd/variants/libfugu_keepthr.so FUGU_DIAG_KEEP_THRESH=1 timeout -k 10 200 python -u bench.py --disj --k $k --no-cpu --no-extra --steps 10 > $O/keep_k$k.json 2> $O/keep_k$k.err || exit 1
  python3 -c "
import json
for n in ('prod','keep'):
    d=json.loads(open('$O/'+n+'_k$k.json').read().strip().splitlines()[-1])
    print(n, $k, d['kernels_ms_per_step'], d.get('result_sha1'))
"
done
