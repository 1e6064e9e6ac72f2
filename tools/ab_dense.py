"""A/B of the dense probe structures on one corpus, in one process: the same
batches run against snapshots built with different FUGU_DENSE_GIB /
FUGU_RANK_GIB budgets (f32 score tables vs rank words vs directory only),
interleaved round by round (cdna_hip_programming.md §5.4 rule 24: report
median and min), with the outputs of every variant checked identical.

  python tools/ab_dense.py [--docs N] [--rounds R] NAME=DENSE_GIB,RANK_GIB ...
  e.g. python tools/ab_dense.py rank=0,64 f32=64,0 dir=0,0
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
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--s", type=float, default=1.0)
    ap.add_argument("--workloads", default="and3,mixed,or")
    args = ap.parse_args()
    import numpy as np
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, synth.VOCAB, args.s, threads=16)
    ixs = {}
    for v in args.variants:
        name, spec = v.split("=")
        dg, rg = spec.split(",")
        os.environ["FUGU_DENSE_GIB"], os.environ["FUGU_RANK_GIB"] = dg, rg
        t0 = time.time()
        ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16, keep_host=False)
        st = ix.stats()
        print(f"[ab] {name}: f32 tables {st.n_dense_f32}, rank terms {st.n_rank_terms}, "
              f"{st.device_bytes / 2**30:.1f} GiB, built in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        ixs[name] = ix
    specs = {"and3": (3, 3, 100, native.MODE_AND), "mixed": (1, 5, 100, native.MODE_AND),
             "or": (2, 5, 1000, native.MODE_OR)}
    out = {"docs": args.docs, "s": args.s, "variants": args.variants, "workloads": {}}
    for wl in args.workloads.split(","):
        m0, m1, k, mode = specs[wl]
        q_off, terms = synth.queries(1024, m0, m1)
        plans = {n: ix.plan(q_off, terms, k, mode) for n, ix in ixs.items()}
        times = {n: [] for n in plans}
        hashes = {}
        for n, p in plans.items():
            p.execute()
            s, d, c = p.results()
            h = hashlib.sha1()
            for i in range(len(c)):
                h.update(d[i, :c[i]].tobytes())
                h.update(s[i, :c[i]].tobytes())
            hashes[n] = h.hexdigest()[:16]
        for _ in range(args.rounds):
            for n, p in plans.items():
                p.profile(True)
                for _ in range(args.steps):
                    p.execute()
                ms, cnt = p.kernel_ms()
                times[n].append(ms[0] / cnt)
        res = {n: {"kernel_ms_med": round(float(np.median(t)), 4), "kernel_ms_min": round(float(np.min(t)), 4),
                   "hash": hashes[n]} for n, t in times.items()}
        res["identical"] = len(set(hashes.values())) == 1
        out["workloads"][wl] = res
        print(f"[ab] {wl}: {json.dumps(res)}", file=sys.stderr, flush=True)
        del plans
    print(json.dumps(out))


if __name__ == "__main__":
    main()
