set -o pipefail
# end-to-end pipelined batches: workers 2 / 4 / 6 / 8 over 96 batches, twice
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 600 python -u tools/e2e_workers.py --workers 2,4,6,8 --steps 96 --repeat 2 > $O/e2e.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
cat $O/e2e.json
