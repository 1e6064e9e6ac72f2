"""Rescore cost of a 10M-doc snapshot (the device work of every commit on a
10M namespace): wall time of fg_index_rescore with FUGU_BUILD_TRACE phases,
and of fg_index_rescore_many over the same snapshot cut into 8 segments.
Run under rocprofv3 --kernel-trace --stats for the scoring kernels' times.

  python tools/rescore_bench.py [--docs N] [--reps R]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    c = synth.corpus(args.docs, threads=16)
    V = synth.VOCAB
    g = native.docs_stats(c.off, c.tok, V, threads=16)
    ix = native.Index.from_docs(ctx, c.off, c.tok, V, threads=16)
    segs = []
    for i in range(8):
        a, b = args.docs * i // 8, args.docs * (i + 1) // 8
        segs.append(native.Index.from_docs(ctx, c.off[a:b + 1] - c.off[a], c.tok[c.off[a]:c.off[b]], V, threads=16,
                                           global_stats=g))
    os.environ["FUGU_BUILD_TRACE"] = "1"
    for r in range(args.reps):
        t = time.perf_counter()
        re = ix.rescore(g)
        print(f"rescore one 10M snapshot: {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
        re.close()
    for r in range(args.reps):
        t = time.perf_counter()
        res = native.Index.rescore_many(segs, g)
        print(f"rescore_many 8 x {args.docs // 8} docs: {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
        for x in res:
            x.close()


if __name__ == "__main__":
    main()
