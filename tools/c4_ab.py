"""A/B of PLAN-time knobs (environment read at fg_plan_create[_multi]) on bench.py's
C4 shape (--units 1: the headline's one 10M snapshot instead): the 10M corpus as 8 namespaces x 1.25M (own statistics each), one
multi-snapshot plan per variant over the same 1024 3-term AND top-100 batch,
run interleaved round by round with the merged select; per variant the median
k_conj and k_final ms and the merged-hit hash (every variant must match).

  python tools/c4_ab.py [--rounds 7] NAME:ENV=V,ENV=V ...
  e.g. python tools/c4_ab.py base: snap:FUGU_XCD_KEY=s div2:FUGU_CONJ_SEG_DIV=2
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--units", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--terms", default="3,3")
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--s", type=float, default=1.0, help="corpus Zipf exponent (C5: 1.1)")
    args = ap.parse_args()
    import torch

    from fugu_amd import native, synth
    from fugu_amd.shard import shard_ranges
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, synth.VOCAB, args.s, threads=16)
    ixs = []
    for b, e in shard_ranges(corp.n_docs, args.units):
        off = corp.off[b:e + 1] - corp.off[b]
        ixs.append(native.Index.from_docs(ctx, off, corp.tok[corp.off[b]:corp.off[e]], synth.VOCAB, threads=16,
                                          keep_host=False))
    m0, m1 = (int(x) for x in args.terms.split(","))
    q_off, terms = synth.queries(1024, m0, m1)
    nq, K = len(q_off) - 1, args.k
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    base_env = dict(os.environ)
    plans = {}
    for v in args.variants:
        name, _, spec = v.partition(":")
        env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update(env)
        plans[name] = native.Plan(ixs if len(ixs) > 1 else ixs[0], q_off, terms, K, args.mode)
    os.environ.clear()
    os.environ.update(base_env)
    outs = [torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32)]
    outs.append(torch.empty(nq, dtype=torch.int32, device=dev))
    multi = len(ixs) > 1

    def run(p):  # a multi-snapshot plan: its merged select; one snapshot: its own lists (shard column unused)
        if multi:
            p.execute_merged(st, *[x.data_ptr() for x in outs])
        else:
            p.execute(st, outs[0].data_ptr(), outs[1].data_ptr(), outs[3].data_ptr())
    times = {n: [] for n in plans}
    sha = {}
    for r in range(args.rounds):
        for n, p in plans.items():
            run(p)
            torch.cuda.synchronize()
            p.kernel_ms()
            p.profile(True)
            for _ in range(args.steps):
                run(p)
            torch.cuda.synchronize()
            m, c = p.kernel_ms()
            p.profile(False)
            times[n].append((m[0] / c, m[1] / c))
            if r == 0:
                h = hashlib.sha1()
                mn = outs[3].cpu().numpy()
                a = [x.cpu().numpy().reshape(nq, K) for x in (outs[:3] if multi else outs[:2])]
                for i in range(nq):
                    for x in a:
                        h.update(x[i, :mn[i]].tobytes())
                sha[n] = h.hexdigest()[:16]
    res = {}
    for n, t in times.items():
        t = np.array(t)
        res[n] = {"kernel_ms_median": round(float(np.median(t[:, 0])), 4), "kernel_ms_min": round(float(t[:, 0].min()), 4),
                  "final_ms_median": round(float(np.median(t[:, 1])), 4), "sha": sha[n], "env": args.variants}
        print(f"[ab] {n}: kernel {res[n]['kernel_ms_median']} ms (min {res[n]['kernel_ms_min']}), final "
              f"{res[n]['final_ms_median']} ms, sha {sha[n]}", file=sys.stderr, flush=True)
    same = len(set(sha.values())) == 1
    print(json.dumps({"docs": args.docs, "units": args.units, "k": K, "terms": args.terms, "mode": args.mode,
                      "same_hits": same, "variants": res}))
    if not same:
        sys.exit(3)


if __name__ == "__main__":
    main()
