"""Per-term K-th best alive scores (fg_index_term_kth) against the term's own
single-term top-1000 list, for terms of every length (diagnostic for k_ktop).

  [FUGU_LIB=...] python tools/ktop_check.py [--docs N]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KS = (1, 10, 20, 100, 1000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    args = ap.parse_args()
    from fugu_amd import native, synth
    ctx = native.Context((0,))
    c = synth.corpus(args.docs)
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16)
    terms = [t for t in range(0, 4000, 7) if ix.df(t) > 0]
    q_off = np.arange(len(terms) + 1, dtype=np.uint32)
    s, d, n = ix.search_batch(q_off, np.array(terms, np.uint32), 1000)
    bad = []
    for i, t in enumerate(terms):
        got = ix.term_kth(t)
        want = np.array([s[i, k - 1] if n[i] >= k else 0.0 for k in KS], np.float32)
        if not np.array_equal(got, want):
            bad.append({"t": t, "df": int(ix.df(t)), "got": got.tolist(), "want": want.tolist(),
                        "ties_at_k": [int((s[i, :n[i]] == s[i, k - 1]).sum()) if n[i] >= k else 0 for k in KS]})
    print(json.dumps({"lib": os.environ.get("FUGU_LIB", "libfugu.so"), "terms": len(terms), "mismatches": len(bad),
                      "long_terms": sum(1 for t in terms if ix.df(t) > 32768), "first": bad[:6]}))


if __name__ == "__main__":
    main()
