"""Phase times of fg_search_sharded (FUGU_SHARD_TRACE=1 prints plan / link / launch /
kernels+merge per call): the C4 fan-out (8 namespaces x 1.25M on one GPU) as a
1024-query batch and as single queries.

  FUGU_SHARD_TRACE=1 python tools/shard_trace.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    from fugu_amd import native, synth
    from fugu_amd.shard import shard_ranges
    ctx = native.Context((0,))
    corp = synth.corpus(10_000_000, threads=16)
    ixs = []
    for b, e in shard_ranges(corp.n_docs, 8):
        ixs.append(native.Index.from_docs(ctx, corp.off[b:e + 1] - corp.off[b], corp.tok[corp.off[b]:corp.off[e]],
                                          synth.VOCAB, threads=16, keep_host=False))
    q_off, terms = synth.queries(1024, 3, 3)
    for mode, name in ((native.MODE_AND, "AND"), (native.MODE_OR, "OR")):
        for _ in range(3):
            t0 = time.perf_counter()
            native.search_sharded(ixs, q_off, terms, 100, mode=mode)
            print(f"[shard_trace] batch {name}: {(time.perf_counter() - t0) * 1e3:.3f} ms", file=sys.stderr, flush=True)
        lat = []
        for i in range(20):
            a, b = int(q_off[i]), int(q_off[i + 1])
            t0 = time.perf_counter()
            native.search_sharded(ixs, np.array([0, b - a], np.uint32), terms[a:b], 20, mode=mode)
            lat.append((time.perf_counter() - t0) * 1e3)
        print(f"[shard_trace] single {name}: p50 {np.median(lat):.3f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
