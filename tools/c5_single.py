"""C5 (100M docs, Zipf s = 1.1, 2-5-term OR top-1000, 1024 queries) as ONE
snapshot on one GPU (5.6e9 postings, past 2^32) instead of 8 doc shards: one
threshold per query instead of eight.  Prints one JSON line.

  python tools/c5_single.py [--rank-gib G]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank-gib", default=None)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    if args.rank_gib:
        os.environ["FUGU_RANK_GIB"] = args.rank_gib
    from fugu_amd import native, synth
    t0 = time.time()
    c = synth.corpus(100_000_000, synth.VOCAB, 1.1, threads=16)
    ctx = native.Context((0,))
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, keep_host=False)
    build_s = time.time() - t0
    del c
    st = ix.stats()
    q_off, terms = synth.queries(1024, 2, 5)
    plan = ix.plan(q_off, terms, 1000, native.MODE_OR)
    for _ in range(2):
        plan.execute()
    plan.results()
    plan.profile(True)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute()
    s, d, n = plan.results()
    el = (time.perf_counter() - t1) / args.steps
    ms, cnt = plan.kernel_ms()
    h = hashlib.sha1()
    for i in range(len(n)):
        h.update(d[i, :n[i]].tobytes())
        h.update(s[i, :n[i]].tobytes())
    print(json.dumps({"workload": "C5 as one 100M-doc snapshot on one GPU", "n_postings": int(st.n_postings),
                      "device_gib": round(st.device_bytes / 2**30, 2), "build_s": round(build_s, 1),
                      "ms_per_batch": round(el * 1e3, 3), "queries_per_s": round(1024 / el, 1),
                      "k_disj_ms": round(ms[0] / cnt, 3), "k_final_ms": round(ms[1] / cnt, 3),
                      "hits": int(n.sum()), "result_sha1": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
