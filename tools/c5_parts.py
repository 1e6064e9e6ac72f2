"""Where the time of a k_disj sweep run in two parts goes (fg_plan_execute_part):
one doc shard of a C5-shaped corpus (Zipf s = 1.1, global statistics over S
shards) planned alone, OR top-1000; per split point f the kernel ms of
  whole   : fg_plan_execute
  parts   : part [0, f) then [f, 1), nothing exchanged
  own     : the same with the plan's own histogram copied out and back in between
  summed  : the histogram summed over the S shards' first parts in between
(part 1 and part 2 reported apart), and the hits' hash of each mode.

  python tools/c5_parts.py [--docs 25000000] [--shards 2] [--fracs 0.0625,0.25,0.5]
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
    ap.add_argument("--docs", type=int, default=25_000_000)
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--fracs", default="0.0625,0.25,0.5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--k", type=int, default=1000)
    args = ap.parse_args()
    import torch

    from fugu_amd import native, synth
    from fugu_amd.shard import agree_hist_span, seed_kth_floor, shard_ranges
    ctx = native.Context((0,))
    c = synth.corpus(args.docs, synth.VOCAB, 1.1, threads=16)
    ranges = shard_ranges(args.docs, args.shards)
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in ranges]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, synth.VOCAB, threads=16)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=16, keep_host=False, global_stats=g)
           for off, tok in parts]
    del parts, c
    seed_kth_floor(ixs)
    q_off, terms = synth.queries(1024, 2, 5)
    K = args.k
    nq = len(q_off) - 1
    st = torch.cuda.current_stream().cuda_stream
    hb = torch.zeros((len(ixs), nq * native.HIST_BINS), dtype=torch.int32, device="cuda")

    def digest(p):
        s, d, n = p.results()
        h = hashlib.sha1()
        for i in range(nq):
            h.update(s[i, :n[i]].tobytes() + d[i, :n[i]].tobytes())
        return h.hexdigest()[:16], int(n.sum())

    def timed(p, fn):
        torch.cuda.synchronize()
        p.kernel_ms()
        p.profile(True)
        fn()
        torch.cuda.synchronize()
        m, n = p.kernel_ms()
        p.profile(False)
        return m[0] + m[1]

    out = {"docs": args.docs, "shards": args.shards, "k": K, "modes": {}}
    plans = [ix.plan(q_off, terms, K, native.MODE_OR) for ix in ixs]
    agree_hist_span(plans)
    p = plans[0]
    for _ in range(2):
        p.execute(st)
    whole = [timed(p, lambda: p.execute(st)) for _ in range(args.reps)]
    out["modes"]["whole"] = {"ms": round(float(np.median(whole)), 4), "hits": digest(p)}
    print(f"[parts] whole {out['modes']['whole']}", file=sys.stderr, flush=True)
    for f in (float(x) for x in args.fracs.split(",")):
        # the summed histogram of every shard's first part
        for r, q in enumerate(plans):
            q.execute_part(st, 0.0, f)
            q.hist_copy(st, hb[r].data_ptr(), False)
        tot = hb.sum(0, dtype=torch.int32)
        own = torch.zeros_like(tot)
        for mode in ("parts", "own", "summed"):
            t1, t2 = [], []
            for rep in range(args.reps + 1):
                a = timed(p, lambda: p.execute_part(st, 0.0, f))
                if mode == "own":
                    p.hist_copy(st, own.data_ptr(), False)
                    p.hist_copy(st, own.data_ptr(), True)
                elif mode == "summed":
                    p.hist_copy(st, tot.data_ptr(), True)
                b = timed(p, lambda: p.execute_part(st, f, 1.0))
                if rep:
                    t1.append(a)
                    t2.append(b)
            e = {"part1_ms": round(float(np.median(t1)), 4), "part2_ms": round(float(np.median(t2)), 4),
                 "sum_ms": round(float(np.median(np.array(t1) + np.array(t2))), 4), "hits": digest(p)}
            out["modes"][f"{mode}@{f}"] = e
            print(f"[parts] {mode}@{f} {e}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
