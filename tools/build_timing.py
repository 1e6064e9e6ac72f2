"""Snapshot build cost on the box: per-phase host/device time of
fg_index_build_from_docs (FUGU_BUILD_TRACE) for a corpus, plus the corpus
generation and shard statistics times the C4/C5 tests pay.

  FUGU_BUILD_TRACE=1 python tools/build_timing.py [--docs N] [--s S]
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
    ap.add_argument("--s", type=float, default=1.0)
    args = ap.parse_args()
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    t = time.time()
    c = synth.corpus(args.docs, synth.VOCAB, args.s, threads=16)
    print(f"corpus {args.docs} s={args.s}: {len(c.tok)} tokens in {time.time() - t:.2f}s", flush=True)
    t = time.time()
    st = native.docs_stats(c.off, c.tok, synth.VOCAB, threads=16)
    print(f"docs_stats {time.time() - t:.2f}s", flush=True)
    t = time.time()
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, keep_host=False)
    s = ix.stats()
    print(f"index {time.time() - t:.2f}s: {s.n_postings} postings, {s.n_rank_terms} rank terms, "
          f"{s.device_bytes / 2**30:.1f} GiB", flush=True)
    del st


if __name__ == "__main__":
    main()
