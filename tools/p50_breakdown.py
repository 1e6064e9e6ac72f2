"""Where a batch-of-one search spends its time (bench.py's p50 line): host
planning + plan upload (fg_plan_create), execute (memset + kernels, HIP events)
and the D2H of the hits (fg_plan_results), per query over the headline batch's
first queries.  python tools/p50_breakdown.py [--docs N] [--queries Q]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--queries", type=int, default=200)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    c = synth.corpus(args.docs, threads=16)
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, keep_host=False)
    q_off, terms = synth.queries(args.queries, 3, 3)
    rows = {"plan_ms": [], "exec_ms": [], "kernel_ms": [], "results_ms": [], "total_ms": [], "search_batch_ms": []}
    for rep in range(2):
        for i in range(args.queries):
            a, b = int(q_off[i]), int(q_off[i + 1])
            one = np.array([0, b - a], np.uint32)
            t0 = time.perf_counter()
            p = ix.plan(one, terms[a:b], 100)
            t1 = time.perf_counter()
            p.profile(True)
            p.execute()
            t2 = time.perf_counter()
            p.results()
            t3 = time.perf_counter()
            ms, n = p.kernel_ms()
            p.close()
            t4 = time.perf_counter()
            ix.search_batch(one, terms[a:b], 100)
            t5 = time.perf_counter()
            if rep:
                rows["plan_ms"].append((t1 - t0) * 1e3)
                rows["exec_ms"].append((t2 - t1) * 1e3)
                rows["results_ms"].append((t3 - t2) * 1e3)
                rows["kernel_ms"].append(float(ms.sum()))
                rows["total_ms"].append((t3 - t0) * 1e3)
                rows["search_batch_ms"].append((t5 - t4) * 1e3)
    print(json.dumps({k: {"p50": round(float(np.median(v)), 4), "p90": round(float(np.percentile(v, 90)), 4)}
                      for k, v in rows.items()}))


if __name__ == "__main__":
    main()
