"""Query-time BM25 (round 6): scores are formed inside k_conj / k_disj from each
posting's tf / fieldnorm payload (DevIndex::tfn) and the query's weights, as
tantivy's TermScorer does at search time (reference src/db/search.rs:162); a
rescore (a commit's new Searcher statistics) runs no device work and scales the
build-time bounds instead (fugu.cpp rescore_one, term_ratio).

Checked against the oracle and against fresh builds under the same statistics:
  * `name` postings (the second payload array, DevPlan::feat bit 0) and tf >= 255
    (escaped tf bytes, feat bit 1), alone and together;
  * a rescore to much larger statistics (every bound scaled, q_rup != 1) and one
    with new deletions (the K-th seeds then step up a level: n_dead);
  * the rescore's per-term K-th values stay lower bounds of the fresh build's.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from fugu_amd import native as nat
    if nat.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    return nat


@pytest.fixture(scope="module")
def ctx(native):
    return native.Context((0,))


def _same(a, b, what):
    assert np.array_equal(a[2], b[2]), what
    for i in range(len(a[2])):
        m = int(a[2][i])
        assert np.array_equal(a[1][i, :m], b[1][i, :m]), (what, i)
        assert np.array_equal(a[0][i, :m], b[0][i, :m]), (what, i)


def _vs_oracle(gi, oi, q_off, qt, k, mode, what):
    s, d, n = gi.search_batch(q_off, qt, k, mode=mode)
    rs, rd, rn, _, _ = oi.search_batch(q_off, qt, k, mode=mode, threads=16)
    assert np.array_equal(n, rn), what
    for i in range(len(n)):
        m = int(n[i])
        assert np.array_equal(d[i, :m], rd[i, :m]), (what, i)
        assert np.allclose(s[i, :m], rs[i, :m], rtol=1e-5, atol=0), (what, i)


def _corpus(names: bool, escapes: bool, n=120_000):
    """A synthetic corpus; with `escapes` a few hundred docs repeat frequent query
    terms 255..1500 times (tf past the payload's byte), with `names` every third
    doc has a short name field."""
    from fugu_amd import synth
    c = synth.corpus(n)
    off, tok = c.off.astype(np.uint64), c.tok.astype(np.uint32)
    if escapes:
        rng = np.random.default_rng(61)
        docs = [tok[off[i]:off[i + 1]] for i in range(n)]
        q_off, qt = synth.queries(64, 1, 3, seed_q=7)
        hot = np.unique(qt)[:40]
        for j, i in enumerate(rng.choice(n, 300, replace=False)):
            t = int(hot[j % len(hot)])
            reps = int(rng.integers(255, 1500))
            docs[i] = np.concatenate([docs[i], np.full(reps, t, np.uint32)])
        off = np.cumsum([0] + [len(x) for x in docs]).astype(np.uint64)
        tok = np.concatenate(docs).astype(np.uint32)
    no = nt = None
    if names:
        rng = np.random.default_rng(62)
        lens = np.where(np.arange(n) % 3 == 0, rng.integers(1, 4, n), 0)
        no = np.cumsum(np.concatenate([[0], lens])).astype(np.uint64)
        nt = (rng.zipf(1.3, int(no[-1])) % (1 << 14)).astype(np.uint32)
        if escapes:  # a name field with an escaped tf too
            d0 = int(np.flatnonzero(lens)[0])
            nt = np.concatenate([nt[:no[d0]], np.full(300, nt[no[d0]], np.uint32), nt[no[d0]:]])
            no = no.copy()
            no[d0 + 1:] += 300
    return n, off, tok, no, nt


@pytest.mark.parametrize("names,escapes", [(False, False), (True, False), (False, True), (True, True)],
                         ids=["plain", "names", "escapes", "names_escapes"])
def test_query_time_scores_vs_oracle(native, ctx, names, escapes):
    from fugu_amd import synth
    from oracle import oracle as orc
    n, off, tok, no, nt = _corpus(names, escapes)
    gi = native.Index.from_docs(ctx, off, tok, synth.VOCAB, name_off=no, name_tok=nt, threads=16)
    st = gi.stats()
    assert bool(st.has_name) == names
    oi = orc.OracleIndex(synth.VOCAB, off, tok, name_off=no, name_tok=nt, threads=16)
    for (m0, m1, k, mode) in [(2, 3, 100, native.MODE_AND), (1, 4, 1000, native.MODE_AND),
                              (2, 4, 20, native.MODE_OR), (2, 5, 1000, native.MODE_OR)]:
        q_off, qt = synth.queries(256, m0, m1, seed_q=7)
        _vs_oracle(gi, oi, q_off, qt, k, mode, (names, escapes, m0, m1, k, mode))
    gi.close()
    oi.close()


@pytest.mark.parametrize("names,escapes", [(False, False), (True, True)], ids=["plain", "names_escapes"])
def test_rescore_scales_bounds_like_a_fresh_build(native, ctx, names, escapes):
    """A rescore to the statistics of a namespace 3x as large (every clause's
    bounds scaled by q_rup), then one with 3% of the docs deleted (K-th seeds a
    level up): the hits of fresh builds under the same statistics, bit for bit,
    and K-th values that never exceed the fresh build's."""
    from fugu_amd import synth
    n, off, tok, no, nt = _corpus(names, escapes)
    big = synth.corpus(3 * n)
    g1 = native.docs_stats(off, tok, synth.VOCAB, name_off=no, name_tok=nt, threads=16)
    gb = native.docs_stats(big.off, big.tok, synth.VOCAB, threads=16)
    g2 = g1 + gb
    ix = native.Index.from_docs(ctx, off, tok, synth.VOCAB, name_off=no, name_tok=nt, threads=16, global_stats=g1)
    re = ix.rescore(g2)
    fresh = native.Index.from_docs(ctx, off, tok, synth.VOCAB, name_off=no, name_tok=nt, threads=16, global_stats=g2)
    rng = np.random.default_rng(63)
    deleted = (rng.random(n) < 0.03).astype(np.uint8)
    re_d = re.rescore(g2, deleted)
    fresh_d = native.Index.from_docs(ctx, off, tok, synth.VOCAB, name_off=no, name_tok=nt, threads=16,
                                     global_stats=g2, deleted=deleted)
    for (m0, m1, k, mode) in [(3, 3, 100, native.MODE_AND), (1, 1, 20, native.MODE_AND),
                              (2, 4, 20, native.MODE_OR), (2, 5, 1000, native.MODE_OR)]:
        q_off, qt = synth.queries(256, m0, m1, seed_q=19)
        _same(re.search_batch(q_off, qt, k, mode=mode), fresh.search_batch(q_off, qt, k, mode=mode),
              ("rescore", m0, m1, k, mode))
        _same(re_d.search_batch(q_off, qt, k, mode=mode), fresh_d.search_batch(q_off, qt, k, mode=mode),
              ("rescore + deletions", m0, m1, k, mode))
    terms = [t for t in range(0, 100_000, 97) if ix.df(t) > 0]
    assert len(terms) > 300
    for t in terms:
        a, b = re.term_kth(t), fresh.term_kth(t)
        assert (a <= b).all(), (t, a, b)
        if not names:  # (the name field's avgdl falls 4x here: its ratio bound is loose)
            assert (a[b > 0] >= 0.9 * b[b > 0]).all(), (t, a, b)
        assert (re_d.term_kth(t) <= fresh_d.term_kth(t)).all(), t
    for x in (re_d, fresh_d, re, fresh, ix):
        x.close()
