"""A/B of planner environment settings on one 10M-doc index in one process:
for each (k, setting) a fresh plan of the same OR batch, timed interleaved over
rounds with HIP events (median / min), results hashed to check they agree.

  python tools/ab_env.py VAR v1 v2 ... [--k 20 1000] [--rounds 5] [--mode or|and]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("var")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--k", type=int, nargs="+", default=[20, 1000])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--mode", choices=["or", "and"], default="or")
    args = ap.parse_args()
    import numpy as np
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, threads=16)
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16, keep_host=False)
    mode = native.MODE_OR if args.mode == "or" else native.MODE_AND
    q_off, terms = synth.queries(1024, 2, 5) if mode == native.MODE_OR else synth.queries(1024, 3, 3)
    out = {}
    for k in args.k:
        plans = {}
        for v in args.values:
            os.environ[args.var] = v
            plans[v] = ix.plan(q_off, terms, k, mode)
            plans[v].profile(True)
            for _ in range(2):
                plans[v].execute()
        t = {v: [] for v in args.values}
        for _ in range(args.rounds):
            for v in args.values:
                for _ in range(args.steps):
                    plans[v].execute()
                    ms, n = plans[v].kernel_ms()
                    t[v].append(float(ms[0]))
        res = {}
        for v in args.values:
            s, d, n = plans[v].results()
            h = hashlib.sha1()
            for i in range(len(n)):
                h.update(d[i, :n[i]].tobytes())
                h.update(s[i, :n[i]].tobytes())
            res[v] = {"ms_med": round(float(np.median(t[v])), 4), "ms_min": round(float(np.min(t[v])), 4),
                      "hash": h.hexdigest()[:16]}
        res["identical"] = len({r["hash"] for r in res.values()}) == 1
        out[f"k{k}"] = res
        print(f"[ab_env] {args.var} k={k}: {json.dumps(res)}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
