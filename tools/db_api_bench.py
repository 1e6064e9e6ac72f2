"""bench.py's GET /search + commit lines alone (bench_db_api): a 10M-doc
namespace ingested as 8 bulk segments, batch-of-one GET /search latency idle
and while 16 commits of 1000 docs run, with fg_search_trace phase times.

  python tools/db_api_bench.py [--docs N]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--no-ref", action="store_true", help="skip the oracle parity sample")
    args = ap.parse_args()
    import bench
    from fugu_amd import native, synth
    threads = bench.host_threads(bench.host_cores())
    corp = synth.corpus(args.docs, synth.VOCAB, 1.0, threads=threads)
    ctx = native.Context((0,))
    ref = None
    if not args.no_ref:
        from oracle import oracle as orc
        ref = orc.OracleIndex(synth.VOCAB, corp.off, corp.tok, threads=threads)
    out, commits = bench.bench_db_api(ctx, corp, native, synth, ref, threads)
    print(json.dumps({"db_api_default_search": out, "commit": commits}))


if __name__ == "__main__":
    main()
