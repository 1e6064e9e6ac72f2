"""Per-workgroup phase timing of k_conj / k_final from the -DFG_DIAG build.

Run on the GPU box:  FUGU_LIB=fugu_amd/libfugu_diag.so python tools/diag_phases.py [--docs N]
Stamps are s_memrealtime (100 MHz, 10 ns).  Prints a JSON summary.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(a, ps=(50, 90, 99, 100)):
    a = np.asarray(a, np.float64)
    if a.size == 0:
        return {}
    return {f"p{p}": round(float(np.percentile(a, p)), 2) for p in ps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--terms", type=int, default=3)
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--k", type=int, default=100)
    args = ap.parse_args()
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, threads=16)
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16)
    q_off, terms = synth.queries(1024, 1 if args.mixed else args.terms, 5 if args.mixed else args.terms)
    plan = ix.plan(q_off, terms, args.k)
    for _ in range(3):
        plan.execute()
    plan.results()
    conj, fin = plan.diag()
    cc = plan.candidate_counts()
    us = 1e-2  # 10 ns ticks -> us
    c_start, c_probe, c_keys, c_sel, c_end = (conj[:, i].astype(np.int64) for i in range(5))
    dur = (c_end - c_start) * us
    t0 = c_start.min()
    nchk = (conj[:, 6] >> np.uint64(40)).astype(np.int64)
    # occupancy over time: the tail where fewer than half of the resident
    # workgroup slots (4 per CU x 256 CUs) are busy
    ev = np.concatenate([np.stack([c_start, np.ones_like(c_start)], 1), np.stack([c_end, -np.ones_like(c_end)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    act = np.cumsum(ev[:, 1])
    busy = np.nonzero(act >= 512)[0]
    tail_us = float((c_end.max() - ev[busy[-1], 0]) * 1e-2) if len(busy) else None
    out = {
        "k_conj": {
            "tail_us_below_half_slots": tail_us, "max_active_wgs": int(act.max()),
            "work_items": int(len(conj)),
            "chunks": int(nchk.sum()),
            "span_us": round(float((c_end.max() - t0) * us), 1),
            "wg_us": pct(dur),
            "wg_us_sum": round(float(dur.sum()), 1),
            "probe_us_sum": round(float(c_probe.sum() * us), 1),
            "keys_us_sum": round(float(c_keys.sum() * us), 1),
            "select_us_sum": round(float(c_sel.sum() * us), 1),
            "appended_per_chunk": pct(conj[:, 5].astype(np.float64) / np.maximum(nchk, 1)),
            "written_total": int(conj[:, 7].sum()),
            # candidates alive at: lead load, after the first MaxScore bound, after probe i
            "alive_lead_b1_p1_p2": [int(conj[:, 8 + i].sum()) for i in range(4)], "lead_unpruned": int(conj[:, 15].sum()),
            # tile-bound headroom: candidates past the first bound that tile maxima would drop
            "b1_extra_pruned_by_tile_maxima": int(conj[:, 14].sum()),
        },
    }
    f_start, f_read, f_sel, f_end = (fin[:, i].astype(np.int64) for i in range(4))
    fdur = (f_end - f_start) * us
    out["k_final"] = {
        "span_us": round(float((f_end.max() - f_start.min()) * us), 1),
        "wg_us": pct(fdur),
        "read_us": pct((f_read - f_start) * us),
        "select_us": pct((f_sel - f_read) * us),
        "sort_us": pct((f_end - f_sel) * us),
        "cand_cnt": pct(cc),
        "slowest": [{"q": int(i), "us": round(float(fdur[i]), 1), "cand": int(cc[i]), "nk": int(fin[i, 6])}
                    for i in np.argsort(-fdur)[:8]],
        "start_spread_us": round(float((f_start.max() - f_start.min()) * us), 1),
    }
    # per-query k_conj cost
    qid = (conj[:, 6] & 0xFFFFFFFF).astype(np.int64)
    per_q = np.bincount(qid, weights=dur, minlength=len(q_off) - 1)
    top = np.argsort(-per_q)[:8]
    out["heaviest_queries"] = [{"q": int(i), "wg_us_sum": round(float(per_q[i]), 1),
                                "items": int((qid == i).sum()), "cand": int(cc[i]),
                                "dfs": [ix.df(int(t)) for t in terms[q_off[i]:q_off[i + 1]]]} for i in top]
    # WG time by query class: lead density and how many probed lists are dense tables
    n_docs = args.docs
    cls = {}
    for i in range(len(q_off) - 1):
        ts = terms[q_off[i]:q_off[i + 1]].tolist()
        dfs = sorted(ix.df(int(t)) for t in ts)
        lead = dfs[0] / n_docs
        dense = sum(1 for d in dfs[1:] if d * 8 >= n_docs)
        key = f"lead>={2 ** int(np.floor(np.log2(max(lead, 1e-9))))}|dense_probes={dense}/{len(dfs) - 1}"
        c = cls.setdefault(key, [0.0, 0, 0])
        c[0] += float(per_q[i])
        c[1] += 1
        c[2] += dfs[0]
    tot = sum(v[0] for v in cls.values())
    out["time_by_class"] = {k: {"share": round(v[0] / tot, 4), "queries": v[1], "lead_postings": v[2]}
                            for k, v in sorted(cls.items(), key=lambda kv: -kv[1][0])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
