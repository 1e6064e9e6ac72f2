"""Debug helper (test infrastructure: the oracle is the checker): k_disj vs the oracle on the 1M Zipf
corpus (FUGU_LIB selects the build).  python tests/diag/debug_disj.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fugu_amd import native, synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    c = synth.corpus(1_000_000)
    ox = orc.OracleIndex(1 << 20, c.off, c.tok, threads=16)
    ctx = native.Context((0,))
    ix = native.Index.from_docs(ctx, c.off, c.tok, 1 << 20, threads=16)
    for (nq, mmin, mmax, k) in [(128, 2, 3, 100), (128, 2, 2, 10), (128, 2, 2, 1000)]:
        q_off, terms = synth.queries(nq, mmin, mmax)
        s, d, n = ix.search_batch(q_off, terms, k, mode=1)
        rs, rd, rn, _, _ = ox.search_batch(q_off, terms, k, mode=1, threads=16)
        bad = [i for i in range(nq) if n[i] != rn[i] or not np.array_equal(d[i, :n[i]], rd[i, :rn[i]])]
        print(f"nq={nq} m={mmin}..{mmax} k={k}: {len(bad)} mismatched queries", bad[:10])
        for i in bad[:2]:
            t = terms[q_off[i]:q_off[i + 1]]
            s1, d1, n1 = ix.search_batch(np.array([0, len(t)], np.uint32), t, k, mode=1)
            solo = np.array_equal(d1[0, :n1[0]], rd[i, :rn[i]])
            missing = sorted(set(rd[i, :rn[i]].tolist()) - set(d[i, :n[i]].tolist()))[:8]
            print(f"  q{i} terms={t.tolist()} df={[ox.df(int(x)) for x in t]} solo_ok={solo} missing={missing}")
            for doc in missing[:3]:
                j = rd[i].tolist().index(doc)
                print(f"    doc {doc} score {rs[i, j]} tile {doc >> 12} rank {j}")


if __name__ == "__main__":
    main()
