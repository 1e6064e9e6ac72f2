"""Commit latency on a 10M-doc namespace, phase by phase (run on the box):
the namespace ingested by 8 POST /batch/upsert calls (8 segments), then 16
upserts of 1000 new docs, each one commit (bench.py's commit_10M line), with
FUGU_COMMIT_TRACE / FUGU_BUILD_TRACE phase times on stderr.

  python tools/commit_trace.py [--docs N] [--commits C] [--per D]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--commits", type=int, default=16)
    ap.add_argument("--per", type=int, default=1000)
    ap.add_argument("--segments", type=int, default=8)
    args = ap.parse_args()
    import numpy as np
    from fugu_amd import db as fdb, native, synth
    ctx = native.Context((0,))
    corp = synth.corpus(args.docs, threads=16)
    d = fdb.Database(ctx)
    d.create_namespace("api")
    tb, to = synth.render_text(corp, 16)
    ib, io = synth.render_ids(corp.n_docs)
    bounds = [corp.n_docs * i // args.segments for i in range(args.segments + 1)]
    t0 = time.time()
    for a, b in zip(bounds[:-1], bounds[1:]):
        d.upsert_batch("api", id_buf=ib[int(io[a]):int(io[b])], id_off=io[a:b + 1] - io[a],
                       text_buf=tb[int(to[a]):int(to[b])], text_off=to[a:b + 1] - to[a])
    print(f"ingest {args.docs} docs as {args.segments} commits: {time.time() - t0:.1f}s", flush=True)
    new = synth.corpus(args.per * args.commits, doc_begin=corp.n_docs, threads=16)
    tb2, to2 = synth.render_text(new, 16)
    ib2, io2 = synth.render_ids(args.per * args.commits, doc_begin=corp.n_docs)
    os.environ["FUGU_COMMIT_TRACE"] = "1"
    os.environ["FUGU_BUILD_TRACE"] = "1"
    lat = []
    for c in range(args.commits):
        a, b = c * args.per, (c + 1) * args.per
        print(f"--- commit {c}", file=sys.stderr, flush=True)
        t1 = time.perf_counter()
        d.upsert_batch("api", id_buf=ib2[int(io2[a]):int(io2[b])], id_off=io2[a:b + 1] - io2[a],
                       text_buf=tb2[int(to2[a]):int(to2[b])], text_off=to2[a:b + 1] - to2[a])
        lat.append((time.perf_counter() - t1) * 1e3)
    d.merge_wait("api")
    mi = d.merge_info("api")
    print({"commit_ms": [round(x, 1) for x in lat], "p50": round(float(np.percentile(lat, 50)), 1),
           "p99": round(float(np.percentile(lat, 99)), 1), "merges": mi["merges"],
           "merge_ms_max": round(mi["merge_ms_max"], 1), "segments": mi["segments"]}, flush=True)
    d.close()


if __name__ == "__main__":
    main()
