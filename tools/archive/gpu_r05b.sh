set -o pipefail
# k_disj item size (tiles per item, items per query): the concurrent doc window
# each XCD's L2 has to hold.  Time at k = 20 / 1000, then DRAM bytes per launch
O=gpurun_out/r05k/items; mkdir -p $O
V=fugu_amd/variants
B=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o64_32z12y11u5r512h9g1s16k32768.so
G16=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o128_16z12y11u5r512h9g1s16k32768.so
G8=$V/libfugu_i8w4t1024b4d256m0g8f4096q896x448h10n16o256_8z12y11u5r512h9g1s16k32768.so
for K in 20 1000; do
  timeout -k 10 400 python -u tools/ab_variants.py --disj --k $K --steps 6 --rounds 2 $B $G16 $G8 > $O/ab_items_k$K.log 2>&1 || { tail -20 $O/ab_items_k$K.log; exit 1; }
  tail -1 $O/ab_items_k$K.log
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for K in 20 1000; do for L in $B $G16 $G8; do
  n=$(basename $L .so)_k$K
  FUGU_LIB=$R/$L timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B --output-format csv -d $R/$O/pmc_$n -o run -- python3 $R/tools/ab_variants.py --child --disj --k $K --steps 3 > $R/$O/pmc_$n.log 2>&1 || { tail -20 $R/$O/pmc_$n.log; exit 1; }
  python3 $R/tools/pmc_summary.py $R/$O/pmc_$n > $R/$O/pmc_$n.json
  python3 -c "
import json; d=json.load(open('$R/$O/pmc_$n.json'))['k_disj']; print('$n', 'DRAM GB per launch', round(32*(d['TCC_EA0_RDREQ_DRAM_32B']+d['TCC_EA0_WRREQ_WRITE_DRAM_32B'])/1e9, 3))"
done; done
