"""Rank-word budget sweep and the creation-order check.

  python tools/ab_rank_budget.py sweep [--factors 0.5,1,2,4,8]
      the 10M-doc corpus built with FUGU_RANK_FACTOR = f (rank words within f x
      the snapshot's posting bytes), one child process per factor: device bytes,
      rank terms, k_conj ms (3-term AND top-100) and k_disj ms (2-5-term OR
      top-1000), output hashes (identical for every f)
  python tools/ab_rank_budget.py order
      the 8 C4 namespaces (10M docs as 8 x 1.25M) built on one GPU in forward,
      then in reverse order: each namespace's k_conj ms against its solo time
Prints one JSON line per measurement.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_ms(native, ix, q_off, terms, k, mode, steps=6):
    plan = ix.plan(q_off, terms, k, mode)
    for _ in range(2):
        plan.execute()
    plan.results()
    plan.profile(True)
    for _ in range(steps):
        plan.execute()
    ms, n = plan.kernel_ms()
    s, d, cnt = plan.results()
    h = hashlib.sha1()
    for i in range(len(cnt)):
        h.update(d[i, :cnt[i]].tobytes())
        h.update(s[i, :cnt[i]].tobytes())
    return round(ms[0] / n, 4), h.hexdigest()[:12]


def child_sweep(factor):
    sys.path.insert(0, ROOT)
    os.environ["FUGU_RANK_FACTOR"] = str(factor)
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(10_000_000, threads=16)
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16, keep_host=False)
    st = ix.stats()
    qa = synth.queries(1024, 3, 3)
    qo = synth.queries(1024, 2, 5)
    a_ms, a_h = kernel_ms(native, ix, *qa, 100, native.MODE_AND)
    o_ms, o_h = kernel_ms(native, ix, *qo, 1000, native.MODE_OR)
    print(json.dumps({"factor": factor, "device_gib": round(st.device_bytes / 2**30, 2), "rank_terms": st.n_rank_terms,
                      "k_conj_ms": a_ms, "k_disj_ms": o_ms, "hash_and": a_h, "hash_or": o_h}), flush=True)


def child_order():
    sys.path.insert(0, ROOT)
    from fugu_amd import native, synth
    from fugu_amd.shard import shard_ranges
    ctx = native.Context((0,))
    corp = synth.corpus(10_000_000, threads=16)
    ranges = shard_ranges(corp.n_docs, 8)
    qa = synth.queries(1024, 3, 3)

    def build(u):
        b, e = ranges[u]
        return native.Index.from_docs(ctx, corp.off[b:e + 1] - corp.off[b], corp.tok[corp.off[b]:corp.off[e]],
                                      synth.VOCAB, threads=16, keep_host=False)
    solo = []
    for u in range(8):
        ix = build(u)
        solo.append((kernel_ms(native, ix, *qa, 100, native.MODE_AND)[0], ix.stats().device_bytes))
        ix.close()
        del ix
    for order in ("forward", "reverse"):
        us = list(range(8)) if order == "forward" else list(range(7, -1, -1))
        ixs = {u: build(u) for u in us}
        for u in range(8):
            ms = kernel_ms(native, ixs[u], *qa, 100, native.MODE_AND)[0]
            print(json.dumps({"order": order, "namespace": u, "k_conj_ms": ms, "solo_ms": solo[u][0],
                              "ratio": round(ms / solo[u][0], 3), "device_gib": round(ixs[u].stats().device_bytes / 2**30, 2),
                              "rank_terms": ixs[u].stats().n_rank_terms}), flush=True)
        for ix in ixs.values():
            ix.close()
        del ixs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["sweep", "order"])
    ap.add_argument("--factors", default="0.5,1,2,4,8")
    ap.add_argument("--child", default=None)
    args = ap.parse_args()
    if args.child is not None:
        return child_order() if args.what == "order" else child_sweep(float(args.child))
    runs = [None] if args.what == "order" else args.factors.split(",")
    for f in runs:
        cmd = [sys.executable, __file__, args.what, "--child", f if f is not None else "0"]
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        sys.stdout.write(out.stdout)
        if out.returncode != 0:
            print(json.dumps({"factor": f, "error": out.stderr[-600:]}), flush=True)
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
