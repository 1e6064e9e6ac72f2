"""k_disj work breakdown from the -DFG_DIAG build: tile modes, postings, candidates.

Run on the GPU box:  FUGU_LIB=fugu_amd/libfugu_diag.so python tools/diag_disj.py [--docs N] [--k K]
Prints a JSON summary (totals over the 1024-query batch + per-WG time percentiles).
"""
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
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--mmin", type=int, default=2)
    ap.add_argument("--mmax", type=int, default=5)
    args = ap.parse_args()
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, threads=16)
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16)
    q_off, terms = synth.queries(1024, args.mmin, args.mmax)
    plan = ix.plan(q_off, terms, args.k, mode=native.MODE_OR)
    for _ in range(2):
        plan.execute()
    plan.results()
    plan.profile(True)
    plan.execute()
    plan.results()
    ms, n = plan.kernel_ms()
    wg, _ = plan.diag()
    dt = (wg[:, 1].astype(np.int64) - wg[:, 0].astype(np.int64)) * 10e-3  # us
    dfs = np.array([ix.df(int(t)) for t in terms], np.float64)
    out = {
        "k_disj_ms": round(ms[0] / max(n, 1), 3), "k_final_ms": round(ms[1] / max(n, 1), 3),
        "work_items": int(len(wg)),
        "tiles_skip": int(wg[:, 2].sum()), "tiles_exact": int(wg[:, 3].sum()), "tiles_filter": int(wg[:, 4].sum()),
        "postings_scattered": int(wg[:, 5].sum()), "postings_total": int(dfs.sum()),
        "candidates_probed": int((wg[:, 6] & np.uint64(0xFFFFFFFF)).sum()),
        "postings_past_bound1": int((wg[:, 6] >> np.uint64(32)).sum()), "truncations": int((wg[:, 7] >> 32).sum()),
        "wg_us": {p: round(float(np.percentile(dt, p)), 1) for p in (50, 90, 99, 100)},
        "wg_us_sum_ms": round(float(dt.sum()) * 1e-3, 1),
        "phase_ms_sum_over_wgs": {nm: round(float(wg[:, 8 + i].sum()) * 1e-5, 1) for i, nm in enumerate(
            ["ranges+hist_read", "split", "exhaustive_tiles", "segment_list", "filter_bound1_bound2", "rescore", "truncate_publish", "hist_add_flush"])},
        "cand_per_query": [int(x) for x in np.percentile(plan.candidate_counts(), [50, 90, 100])],
    }
    # timeline: the kernel span and its tail (s_memrealtime: 100 MHz)
    t0 = wg[:, 0].astype(np.int64)
    t1 = wg[:, 1].astype(np.int64)
    base = t0.min()
    st, en = (t0 - base) * 10e-3, (t1 - base) * 10e-3  # us
    span = float(en.max())
    grid = np.linspace(0, span, 201)
    busy = np.array([int(((st <= x) & (en > x)).sum()) for x in grid])
    peak = max(int(busy.max()), 1)
    out["timeline"] = {
        "span_us": round(span, 1), "peak_busy_wgs": peak,
        "us_below_half_busy": round(float((busy < peak / 2).mean() * span), 1),
        "busy_at_pct": {str(p): int(busy[p * 2]) for p in (10, 50, 80, 90, 95, 99)},
        "last_start_us": round(float(st.max()), 1),
    }
    post = wg[:, 5].astype(np.int64)
    b1 = (wg[:, 6] >> np.uint64(32)).astype(np.int64)
    # the sweep (rows in plan order) in sixteenths: workgroup time, streamed
    # postings, postings past bound 1 and candidates rescored in each
    cuts = np.linspace(0, len(wg), 17).astype(int)
    cand = (wg[:, 6] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    out["by_sweep_16th"] = {
        "wg_ms": [round(float(dt[a:b].sum()) * 1e-3, 1) for a, b in zip(cuts[:-1], cuts[1:])],
        "postings_M": [round(float(post[a:b].sum()) * 1e-6, 2) for a, b in zip(cuts[:-1], cuts[1:])],
        "past_bound1_M": [round(float(b1[a:b].sum()) * 1e-6, 3) for a, b in zip(cuts[:-1], cuts[1:])],
        "candidates_M": [round(float(cand[a:b].sum()) * 1e-6, 3) for a, b in zip(cuts[:-1], cuts[1:])],
    }
    qid = (wg[:, 7] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    top = np.argsort(-dt)[:12]
    out["longest_items"] = [{"q": int(qid[i]), "us": round(float(dt[i]), 1), "start_us": round(float(st[i]), 1),
                             "postings": int(post[i]), "past_bound1": int(b1[i]),
                             "q_terms_df": [int(x) for x in dfs[q_off[qid[i]]:q_off[qid[i] + 1]]]} for i in top]
    if post.sum() > 0:
        out["us_per_posting_p50"] = round(float(np.median(dt[post > 0] / post[post > 0])), 5)
        out["corr_us_postings"] = round(float(np.corrcoef(dt, post)[0, 1]), 3)
        out["corr_us_past_bound1"] = round(float(np.corrcoef(dt, b1)[0, 1]), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"[diag_disj] {time.time() - t:.1f}s", file=sys.stderr)
