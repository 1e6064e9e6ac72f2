"""The C corpus/query generator against its numpy mirror."""
import numpy as np

import synth_ref as sr
from fugu_amd import synth


def test_hash_functions():
    for x in [0, 1, 2**63, 2**64 - 1, 12345678901234567]:
        assert synth.mix64(x) == int(sr.mix64(np.uint64(x)))
    assert synth.h2(0x5EED1, 17) == int(sr.h2(0x5EED1, 17))
    assert synth.h3(20250808, 3, 9) == int(sr.h3(20250808, 3, 9))


def test_corpus_bit_exact_vs_numpy():
    for (n, v, s) in [(3000, 1 << 20, 1.0), (500, 1 << 12, 1.1), (200, 7, 1.0)]:
        c = synth.corpus(n, v, s, 0x5EED1, 20250808, threads=3)
        off, tok = sr.corpus(n, v, s, 0x5EED1, 20250808)
        assert np.array_equal(c.off, off)
        assert np.array_equal(c.tok, tok)
        assert tok.max() < v
        lens = np.diff(off.astype(np.int64))
        assert lens.min() >= 8 and lens.max() <= 120


def test_corpus_offset_start_matches_full():
    full = synth.corpus(2000, 1 << 16, 1.0, 1, 2)
    part = synth.corpus(500, 1 << 16, 1.0, 1, 2, doc_begin=1500)
    assert np.array_equal(part.tok, full.tok[int(full.off[1500]):])


def test_queries_bit_exact_vs_numpy():
    for (nq, a, b, r, seed) in [(200, 3, 3, 1 << 14, 7), (300, 1, 5, 1 << 14, 13), (50, 2, 4, 1 << 9, 23)]:
        q_off, q_terms = synth.queries(nq, a, b, r, 1.0, seed)
        n_off, n_terms = sr.queries(nq, a, b, r, 1.0, seed)
        assert np.array_equal(q_off, n_off) and np.array_equal(q_terms, n_terms)
        for i in range(nq):
            t = q_terms[q_off[i]:q_off[i + 1]]
            assert a <= len(t) <= b and len(set(t.tolist())) == len(t) and t.max() < r


def test_zipf_head_mass():
    # rank 1 has mass 1/H(V); with V = 2^20, H ~ 14.44 -> ~6.9% of tokens
    c = synth.corpus(20000, 1 << 20, 1.0, 0x5EED1, 20250808)
    frac = np.mean(c.tok == 0)
    assert 0.065 < frac < 0.074
