"""C5 (100M docs, Zipf s = 1.1, 2-5-term OR top-1000, 1024 queries) as 8 doc
shards on ONE GPU, rehearsing the 8-GPU split's threshold sharing
(fg_plan_set_peers): every mode's merged hits are hashed, and timed
  alone    : each shard's plan by itself (seeded: shard.seed_kth_floor), one
             after another -- what one GPU of the split runs with no sharing
  linked   : the 8 plans linked (one shared threshold / histogram), back to back
             on one stream -- per-shard times (the round-5 reference mean)
  linked_c : the linked plans on 8 streams at once
  peers_c  : the plans with their own words, peers of each other, on 8 streams
             at once (each publishes into all 8: the cross-device mechanism)
On one GPU the concurrent modes share it; wall / 8 is the per-GPU time of the
split (each shard progresses at 1/8 of the speed, so the thresholds evolve
per posting as they would on 8 GPUs, bar the xGMI latency of the atomics).

  python tools/c5_peers.py [--docs N] [--reps R]
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
    ap.add_argument("--docs", type=int, default=100_000_000)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--k", type=int, default=1000)
    args = ap.parse_args()
    import numpy as np
    import torch

    from fugu_amd import native, synth
    from fugu_amd.shard import agree_hist_span, merge_on_device, seed_kth_floor, shard_ranges
    t0 = time.time()
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
    print(f"[c5_peers] built in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    K, S = args.k, args.shards
    q_off, terms = synth.queries(1024, 2, 5)
    nq = len(q_off) - 1
    dev = torch.device("cuda:0")
    gs = torch.empty((S, nq * K), dtype=torch.float32, device=dev)
    gd = torch.empty((S, nq * K), dtype=torch.int32, device=dev)
    gn = torch.empty((S, nq), dtype=torch.int32, device=dev)
    main_s = torch.cuda.current_stream().cuda_stream
    streams = [torch.cuda.Stream() for _ in range(S)]

    def digest():
        ms, md, msh, mn = merge_on_device(gs, gd, gn, nq, K, main_s)
        torch.cuda.synchronize()
        h = hashlib.sha1()
        s, d, sh, n = ms.cpu().numpy(), md.cpu().numpy(), msh.cpu().numpy(), mn.cpu().numpy()
        for i in range(nq):
            m = int(n[i])
            h.update(s[i * K:i * K + m].tobytes() + d[i * K:i * K + m].tobytes() + sh[i * K:i * K + m].tobytes())
        return h.hexdigest()[:16]

    def run(plans, concurrent, reset):
        if reset:
            for p in plans:
                p.reset(main_s)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for r, p in enumerate(plans):
            st = streams[r].cuda_stream if concurrent else main_s
            p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    out = {"docs": args.docs, "shards": S, "k": K, "modes": {}}
    # alone
    alone = []
    for r, ix in enumerate(ixs):
        p = ix.plan(q_off, terms, K, native.MODE_OR)
        p.execute(main_s, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        p.profile(True)
        for _ in range(args.reps):
            p.execute(main_s, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        torch.cuda.synchronize()
        m, n = p.kernel_ms()
        alone.append(round(float(m[0] + m[1]) / max(n, 1), 4))
        p.close()
    out["modes"]["alone"] = {"per_shard_ms": alone, "max_ms": max(alone), "hits": digest()}
    print(f"[c5_peers] alone {out['modes']['alone']}", file=sys.stderr, flush=True)
    # linked (one stream: per-shard times; 8 streams: wall)
    plans = [ix.plan(q_off, terms, K, native.MODE_OR) for ix in ixs]
    native.link_plans(plans)
    run(plans, False, False)
    for p in plans:
        p.profile(True)
    walls = [run(plans, False, False) for _ in range(args.reps)]
    per = []
    for p in plans:
        m, n = p.kernel_ms()
        per.append(round(float(m[0] + m[1]) / max(n, 1), 4))
        p.profile(False)
    out["modes"]["linked"] = {"per_shard_ms": per, "mean_ms": round(float(np.mean(per)), 4),
                              "wall_ms": round(float(np.median(walls)), 4), "hits": digest()}
    print(f"[c5_peers] linked {out['modes']['linked']}", file=sys.stderr, flush=True)
    # linked, concurrent: plans[0] zeroes the shared words, so it goes first (its
    # memset is queued ahead of the other streams' work by an event)
    ev = torch.cuda.Event()

    def run_linked_c():
        torch.cuda.synchronize()
        t = time.perf_counter()
        plans[0].execute(streams[0].cuda_stream, gs[0].data_ptr(), gd[0].data_ptr(), gn[0].data_ptr())
        for r in range(1, S):
            plans[r].execute(streams[r].cuda_stream, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3
    run_linked_c()
    walls = [run_linked_c() for _ in range(args.reps)]
    out["modes"]["linked_c"] = {"wall_ms": round(float(np.median(walls)), 4),
                                "wall_over_shards_ms": round(float(np.median(walls)) / S, 4), "hits": digest()}
    print(f"[c5_peers] linked_c {out['modes']['linked_c']}", file=sys.stderr, flush=True)
    for p in plans:
        p.close()
    # peers, concurrent
    plans = [ix.plan(q_off, terms, K, native.MODE_OR) for ix in ixs]
    agree_hist_span(plans)
    for i, p in enumerate(plans):
        p.set_peers([x for j, x in enumerate(plans) if j != i])
    run(plans, True, True)
    walls = [run(plans, True, True) for _ in range(args.reps)]
    out["modes"]["peers_c"] = {"wall_ms": round(float(np.median(walls)), 4),
                               "wall_over_shards_ms": round(float(np.median(walls)) / S, 4), "hits": digest()}
    print(f"[c5_peers] peers_c {out['modes']['peers_c']}", file=sys.stderr, flush=True)
    for p in plans:
        p.set_peers([])
        p.close()
    lm = out["modes"]["linked"]["mean_ms"]
    out["peers_per_gpu_over_linked_mean"] = round(out["modes"]["peers_c"]["wall_over_shards_ms"] / lm, 3)
    out["alone_max_over_linked_mean"] = round(max(alone) / lm, 3)
    out["identical_hits"] = len({m["hits"] for m in out["modes"].values()}) == 1
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
