"""A/B of snapshot build settings (environment knobs read at fg_index build) on
one corpus in one process: the same batches run against snapshots built under
different environments, interleaved round by round (median and min reported),
with the outputs of every variant checked identical.

  python tools/ab_env.py [--docs N] [--rounds R] [--workloads and3,or1000,or20] NAME:ENV=V,ENV=V ...
  e.g. python tools/ab_env.py base: f32top15:FUGU_RANK_SKIP_TOP=15,FUGU_DENSE_GIB=2
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SPECS = {"and3": (3, 3, 100, 0), "mixed": (1, 5, 100, 0), "or1000": (2, 5, 1000, 1), "or20": (2, 5, 20, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--s", type=float, default=1.0)
    ap.add_argument("--workloads", default="and3,or1000,or20")
    args = ap.parse_args()
    import numpy as np
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, synth.VOCAB, args.s, threads=16)
    ixs = {}
    base_env = dict(os.environ)
    for v in args.variants:
        name, _, spec = v.partition(":")
        env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update(env)
        t0 = time.time()
        ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16, keep_host=False)
        st = ix.stats()
        print(f"[ab] {name} {env}: f32 tables {st.n_dense_f32}, rank terms {st.n_rank_terms} "
              f"({st.n_sparse_rank_terms} sparse, {st.rank_bytes / 2**30:.2f} GiB), "
              f"{st.device_bytes / 2**30:.2f} GiB, built in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        ixs[name] = (ix, st.device_bytes, env)
    os.environ.clear()
    os.environ.update(base_env)
    out = {"docs": args.docs, "s": args.s, "variants": args.variants,
           "device_gib": {n: round(b / 2**30, 3) for n, (_, b, _) in ixs.items()},
           "rank": {n: {"terms": ix.stats().n_rank_terms, "sparse": ix.stats().n_sparse_rank_terms,
                        "gib": round(ix.stats().rank_bytes / 2**30, 3)} for n, (ix, _, _) in ixs.items()},
           "workloads": {}}
    for wl in args.workloads.split(","):
        m0, m1, k, mode = SPECS[wl]
        q_off, terms = synth.queries(1024, m0, m1)
        plans = {}
        for n, (ix, _, env) in ixs.items():  # plan-time knobs (FUGU_SEED) under the variant's environment too
            os.environ.update(env)
            plans[n] = ix.plan(q_off, terms, k, mode)
            os.environ.clear()
            os.environ.update(base_env)
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
