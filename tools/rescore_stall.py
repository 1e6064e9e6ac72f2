"""Is a batch-of-one search held up by a rescore's DEVICE work alone?  A 10M-doc
namespace as 8 segments with global statistics; the main thread runs
batch-of-one OR top-20 searches over the 8 segments (fg_search_sharded, the
GET /search path) idle, then while a second thread rescores the segments
(fg_index_rescore_many, a commit's device work without the rest of the commit:
no upsert, analysis, segment build or snapshot swap) back to back.  Prints the
search latency percentiles of both phases and the rescore times.

  python tools/rescore_stall.py [--docs N] [--rescores R] [--mode background|plain]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(v):
    v = np.sort(np.asarray(v))
    q = lambda p: round(float(v[min(len(v) - 1, int(p * len(v)))]), 4)
    return {"n": len(v), "p50_ms": q(0.5), "p90_ms": q(0.9), "p99_ms": q(0.99), "max_ms": round(float(v[-1]), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--rescores", type=int, default=16)
    ap.add_argument("--mode", default="background", help="background: the rescoring thread on the background streams")
    args = ap.parse_args()
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    c = synth.corpus(args.docs, threads=16)
    V = synth.VOCAB
    g = native.docs_stats(c.off, c.tok, V, threads=16)
    segs = []
    for i in range(8):
        a, b = args.docs * i // 8, args.docs * (i + 1) // 8
        segs.append(native.Index.from_docs(ctx, c.off[a:b + 1] - c.off[a], c.tok[c.off[a]:c.off[b]], V, threads=16,
                                           global_stats=g))
    q_off, terms = synth.queries(4096, 1, 3, seed_q=5)

    def search(i):
        j = i % (len(q_off) - 1)
        qo = np.array([0, q_off[j + 1] - q_off[j]], np.uint32)
        t = time.perf_counter()
        native.search_sharded(segs, qo, terms[q_off[j]:q_off[j + 1]], 20, mode=native.MODE_OR, ctx=ctx)
        return (time.perf_counter() - t) * 1e3

    for i in range(200):
        search(i)
    idle = [search(i) for i in range(2000)]
    done = threading.Event()
    rs = []

    def rescorer():
        if args.mode == "background":
            native._lib.fg_thread_background(1)
        for _ in range(args.rescores):
            t = time.perf_counter()
            out = native.Index.rescore_many(segs, g)
            rs.append((time.perf_counter() - t) * 1e3)
            for x in out:
                x.close()
        done.set()

    th = threading.Thread(target=rescorer)
    th.start()
    during, i = [], 0
    while not done.is_set():
        during.append(search(i))
        i += 1
    th.join()
    print(json.dumps({"idle": pct(idle), "during_rescores": pct(during), "rescore_ms": pct(rs), "mode": args.mode}))


if __name__ == "__main__":
    main()
