"""A/B of several snapshots on one GPU: per-snapshot plans (linked, back to back
on one stream, or unlinked on 8 streams) against ONE multi-snapshot plan
(fg_plan_create_multi: one launch per kernel over all snapshots), same batch,
identical merged hits required.  Also the single-query latency of
fg_search_sharded (the GET /search path over a namespace's segments) in a child
process per mode: one plan with per-slot lists + k_merge_rank (the default for
a small batch), one plan with its merged select (FUGU_SHARDED_MERGED_MIN=1), one
linked plan per shard (FUGU_SHARDED_PER_SHARD=1: the round-2 path).

  python tools/multi_ab.py [--docs 10000000] [--units 8] [--kind seg|ns] [--steps 10]
  python tools/multi_ab.py --latency-only ...   (child: prints one JSON line)
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(native, synth, ctx, docs, units, kind, threads=16, whole=False):
    from fugu_amd.shard import shard_ranges
    corp = synth.corpus(docs, threads=threads)
    if whole:  # the same corpus as ONE snapshot (the segmentation's cost)
        return native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=threads, keep_host=False)
    ranges = shard_ranges(docs, units)
    parts = [(corp.off[b:e + 1] - corp.off[b], corp.tok[corp.off[b]:corp.off[e]]) for b, e in ranges]
    g = None
    if kind == "seg":
        for off, tok in parts:
            x = native.docs_stats(off, tok, synth.VOCAB, threads=threads)
            g = x if g is None else g + x
    return [native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=threads, keep_host=False, global_stats=g)
            for off, tok in parts]


def digest(ms, md, msh, mn, nq, K):
    mn = mn.cpu().numpy()
    ms = ms.cpu().numpy().reshape(nq, K)
    md = md.cpu().numpy().view(np.uint32).reshape(nq, K)
    msh = msh.cpu().numpy().reshape(nq, K)
    h = hashlib.sha1()
    for i in range(nq):
        m = int(mn[i])
        h.update(ms[i, :m].tobytes() + md[i, :m].tobytes() + msh[i, :m].astype(np.uint32).tobytes())
    return h.hexdigest()[:16]


def latency(native, synth, ixs, args):
    out = {}
    for mode, K, name in ((native.MODE_AND, 100, "AND_top100"), (native.MODE_OR, 20, "OR_top20")):
        q_off, terms = synth.queries(200, 2 if mode else 3, 4 if mode else 3, seed_q=5)
        lat = []
        for i in range(200):
            a, b = int(q_off[i]), int(q_off[i + 1])
            one = np.array([0, b - a], np.uint32)
            t0 = time.perf_counter()
            native.search_sharded(ixs, one, terms[a:b], K, mode=mode)
            lat.append((time.perf_counter() - t0) * 1e3)
        lat = np.array(lat[20:])
        out[name] = {"p50_ms": round(float(np.median(lat)), 4), "p90_ms": round(float(np.percentile(lat, 90)), 4),
                     "p99_ms": round(float(np.percentile(lat, 99)), 4)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--units", type=int, default=8)
    ap.add_argument("--kind", choices=["seg", "ns"], default="seg")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--latency-only", action="store_true")
    ap.add_argument("--no-whole", action="store_true", help="skip the one-snapshot comparison")
    args = ap.parse_args()
    import torch
    from fugu_amd import native, synth
    from fugu_amd.shard import merge_on_device
    ctx = native.Context((0,))
    ixs = build(native, synth, ctx, args.docs, args.units, args.kind)
    if args.latency_only:
        print(json.dumps(latency(native, synth, ixs, args)), flush=True)
        return
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    S, nq = len(ixs), 1024
    res = {"docs": args.docs, "units": S, "kind": args.kind}
    whole = None if args.no_whole else build(native, synth, ctx, args.docs, 1, args.kind, whole=True)
    for mode, K, m0, m1, name in ((native.MODE_AND, 100, 3, 3, "AND_top100"), (native.MODE_OR, 20, 2, 4, "OR_top20"),
                                  (native.MODE_OR, 1000, 2, 5, "OR_top1000")):
        q_off, terms = synth.queries(nq, m0, m1)
        gs = torch.empty((S, nq * K), dtype=torch.float32, device=dev)
        gd = torch.empty((S, nq * K), dtype=torch.int32, device=dev)
        gn = torch.empty((S, nq), dtype=torch.int32, device=dev)
        ent = {}
        # (a) per-snapshot plans, linked, back to back on one stream
        plans = [ix.plan(q_off, terms, K, mode) for ix in ixs]
        native.link_plans(plans)
        out = {}

        def step_linked():
            for r, p in enumerate(plans):
                p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
            out["m"] = merge_on_device(gs, gd, gn, nq, K, st)

        for _ in range(2):
            step_linked()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_linked()
        torch.cuda.synchronize()
        ent["linked_ms"] = round((time.perf_counter() - t0) * 1e3 / args.steps, 4)
        ent["linked_sha"] = digest(*out["m"], nq, K)
        del plans
        # (b) one multi-snapshot plan
        t0 = time.perf_counter()
        mp = native.Plan(ixs, q_off, terms, K, mode)
        ent["multi_plan_create_ms"] = round((time.perf_counter() - t0) * 1e3, 3)

        def step_multi():
            mp.execute(st, gs.data_ptr(), gd.data_ptr(), gn.data_ptr())
            out["m"] = merge_on_device(gs, gd, gn, nq, K, st)

        for _ in range(2):
            step_multi()
        mp.profile(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_multi()
        torch.cuda.synchronize()
        ent["multi_ms"] = round((time.perf_counter() - t0) * 1e3 / args.steps, 4)
        kms, kn = mp.kernel_ms()
        ent["multi_kernel_ms"] = [round(kms[0] / max(kn, 1), 4), round(kms[1] / max(kn, 1), 4)]
        ent["multi_sha"] = digest(*out["m"], nq, K)
        ent["same_hits"] = ent["multi_sha"] == ent["linked_sha"]
        # (b2) the same plan through its merged select (no per-slot lists, no k_merge_rank)
        mo = [torch.empty(nq * K, dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32)] + [
            torch.empty(nq, dtype=torch.int32, device=dev)]

        def step_merged():
            mp.execute_merged(st, *[x.data_ptr() for x in mo])
            out["m"] = tuple(mo)

        for _ in range(2):
            step_merged()
        mp.kernel_ms()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_merged()
        torch.cuda.synchronize()
        ent["merged_select_ms"] = round((time.perf_counter() - t0) * 1e3 / args.steps, 4)
        kms, kn = mp.kernel_ms()
        ent["merged_select_kernel_ms"] = [round(kms[0] / max(kn, 1), 4), round(kms[1] / max(kn, 1), 4)]
        ent["merged_select_same_hits"] = digest(*out["m"], nq, K) == ent["linked_sha"]
        del mp
        # (c) the corpus as one snapshot, same batch (what the segmentation costs)
        if whole is not None:
            wp = whole.plan(q_off, terms, K, mode)
            wp.profile(True)
            for _ in range(2):
                wp.execute(st)
            torch.cuda.synchronize()
            wp.kernel_ms()
            for _ in range(args.steps):
                wp.execute(st)
            torch.cuda.synchronize()
            kms, kn = wp.kernel_ms()
            ent["one_snapshot_kernel_ms"] = [round(kms[0] / max(kn, 1), 4), round(kms[1] / max(kn, 1), 4)]
            del wp
        # (d) the ABI call: fg_search_sharded (host batch in, merged host hits out)
        native.search_sharded(ixs, q_off, terms, K, mode=mode)
        t0 = time.perf_counter()
        for _ in range(3):
            native.search_sharded(ixs, q_off, terms, K, mode=mode)
        ent["fg_search_sharded_ms"] = round((time.perf_counter() - t0) * 1e3 / 3, 4)
        res[name] = ent
        print(f"[multi_ab] {name}: {ent}", file=sys.stderr, flush=True)
        del gs, gd, gn
    del ixs, whole
    # single-query latency of fg_search_sharded, one child per mode
    lat = {}
    for label, env in (("multi_slot_lists_merge", {}), ("multi_merged_select", {"FUGU_SHARDED_MERGED_MIN": "1"}),
                       ("per_shard", {"FUGU_SHARDED_PER_SHARD": "1"})):
        cmd = [sys.executable, os.path.abspath(__file__), "--latency-only", "--docs", str(args.docs), "--units",
               str(args.units), "--kind", args.kind]
        r = subprocess.run(cmd, env={**os.environ, **env}, capture_output=True, text=True, timeout=600)
        lat[label] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"rc": r.returncode,
                                                                                           "err": r.stderr[-400:]}
        print(f"[multi_ab] latency {label}: {lat[label]}", file=sys.stderr, flush=True)
    res["single_query_latency"] = lat
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
