"""Phase times of one small commit segment (FUGU_BUILD_TRACE): 1000 new docs
built with a 10M namespace's statistics, the way fg_db_commit builds a segment.

  FUGU_BUILD_TRACE=1 python tools/segment_trace.py [--new 1000]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--new", type=int, default=1000)
    args = ap.parse_args()
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    base = synth.corpus(1_000_000, threads=16)
    g = native.docs_stats(base.off, base.tok, synth.VOCAB, threads=16)
    new = synth.corpus(args.new, doc_begin=base.n_docs)
    g = g + native.docs_stats(new.off, new.tok, synth.VOCAB)
    for r in range(3):
        t0 = time.perf_counter()
        ix = native.Index.from_docs(ctx, new.off, new.tok, synth.VOCAB, global_stats=g, keep_host=False)
        print(f"[segment_trace] run {r}: {(time.perf_counter() - t0) * 1e3:.2f} ms", file=sys.stderr, flush=True)
        ix.close()


if __name__ == "__main__":
    main()
