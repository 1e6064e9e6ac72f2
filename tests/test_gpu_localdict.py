"""A snapshot's own term dictionary (fg_index::tmap): a build whose docs hold
fewer than a quarter of the vocabulary's terms -- a commit's new docs, as a
tantivy segment keeps its own term dictionary (reference src/db/document.rs:65
adds one segment per commit) -- numbers its terms locally, and the C ABI still
takes vocabulary ids.

Checked here: such snapshots answer like the oracle over the whole vocabulary
(queries holding terms the snapshot lacks included); df / bm25 / term_kth /
term_ladder / set_kth_floor speak vocabulary ids; a rescore of one equals a fresh
build under the same statistics, alone and beside a vocabulary-indexed snapshot
in one fg_index_rescore_many; a multi-snapshot plan over both kinds answers like
the single index.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SPREAD = 16  # vocabulary ids t * SPREAD + 5: the docs hold at most 1/16 of the vocabulary


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
        assert np.array_equal(a[0][i, :m].view(np.uint32), b[0][i, :m].view(np.uint32)), (what, i)


def _spread(t):
    return (np.asarray(t, np.uint64) * SPREAD + 5).astype(np.uint32)


def test_local_dictionary_vs_oracle(native, ctx):
    from fugu_amd import synth
    from oracle import oracle as orc
    V = synth.VOCAB * SPREAD
    c = synth.corpus(20_000)
    off, tok = c.off.astype(np.uint64), _spread(c.tok)
    gi = native.Index.from_docs(ctx, off, tok, V, threads=16)
    oi = orc.OracleIndex(V, off, tok, threads=16)
    assert gi.stats().n_terms == V
    for (m0, m1, k, mode) in [(2, 3, 100, native.MODE_AND), (1, 4, 1000, native.MODE_AND),
                              (2, 4, 20, native.MODE_OR), (2, 5, 1000, native.MODE_OR)]:
        q_off, qt = synth.queries(256, m0, m1, seed_q=5)
        qt = _spread(qt)
        qt[::7] += 1  # ids the snapshot lacks (t * SPREAD + 6)
        s, d, n = gi.search_batch(q_off, qt, k, mode=mode)
        rs, rd, rn, _, _ = oi.search_batch(q_off, qt, k, mode=mode, threads=16)
        assert np.array_equal(n, rn), (m0, m1, k, mode)
        for i in range(len(n)):
            m = int(n[i])
            assert np.array_equal(d[i, :m], rd[i, :m]), (mode, k, i)
            assert np.allclose(s[i, :m], rs[i, :m], rtol=1e-5, atol=0), (mode, k, i)
    present = np.unique(tok)
    for t in list(present[:: max(1, len(present) // 50)]) + [6, 22, V - 1]:
        t = int(t)
        assert gi.df(t, native.FIELD_TEXT) == oi.df(t), t
        assert gi.bm25(t)[0] == orc.term_weight(oi.df(t), 20_000), t
    # the ladder on vocabulary ids: zeros at ids the snapshot lacks; as a floor it
    # gives back the same K-th values
    lad = gi.term_ladder()
    assert lad.shape[0] == V
    absent = np.setdiff1d(np.arange(0, 4096, dtype=np.uint32), present)
    assert not lad[absent].any()
    kk = [native.LADDER_KS.index(x) for x in native.KTH_KS]
    floor = np.ascontiguousarray(lad[:, kk])
    for t in present[:2000:37]:  # the snapshot's own K-th values, now on vocabulary ids
        assert np.array_equal(gi.term_kth(int(t)), floor[int(t)]), int(t)
    gi.set_kth_floor(floor)
    q_off, qt = synth.queries(256, 2, 4, seed_q=6)
    qt = _spread(qt)
    s, d, n = gi.search_batch(q_off, qt, 20, mode=native.MODE_OR)
    rs, rd, rn, _, _ = oi.search_batch(q_off, qt, 20, mode=native.MODE_OR, threads=16)
    assert np.array_equal(n, rn)
    for i in range(len(n)):
        assert np.array_equal(d[i, :int(n[i])], rd[i, :int(n[i])]), i
    with pytest.raises(Exception):
        gi.set_kth_floor(np.zeros((synth.VOCAB, len(native.KTH_KS)), np.float32))  # not the vocabulary's size
    gi.close()
    oi.close()


def test_local_dictionary_rescores(native, ctx):
    """A 5000-doc segment (its own dictionary) and a 300K-doc one (vocabulary ids)
    rescored together to the statistics of both: each equals a fresh build under
    them; merged in one plan they answer like the single index."""
    from fugu_amd import synth
    V = synth.VOCAB
    c = synth.corpus(305_000)
    cut = 300_000
    ao, at = c.off[:cut + 1].copy(), c.tok[:c.off[cut]]
    bo, bt = c.off[cut:] - c.off[cut], c.tok[c.off[cut]:]
    ga = native.docs_stats(ao, at, V, threads=16)
    gb = native.docs_stats(bo, bt, V, threads=16)
    g = ga + gb
    a = native.Index.from_docs(ctx, ao, at, V, threads=16, global_stats=ga)
    b = native.Index.from_docs(ctx, bo, bt, V, threads=16, global_stats=gb)
    assert len(np.unique(bt)) * 4 < V <= len(np.unique(at)) * 4  # b local, a vocabulary ids
    dl = (np.arange(5000) % 9 == 2).astype(np.uint8)
    many = native.Index.rescore_many([a, b], g, deleted=[None, dl])
    fa = native.Index.from_docs(ctx, ao, at, V, threads=16, global_stats=g)
    fb = native.Index.from_docs(ctx, bo, bt, V, threads=16, global_stats=g, deleted=dl)
    one_b = b.rescore(g, deleted=dl)
    single = native.Index.from_docs(ctx, c.off, c.tok, V, threads=16)
    for (m0, m1, k, mode) in [(3, 3, 100, native.MODE_AND), (1, 1, 20, native.MODE_AND),
                              (2, 4, 20, native.MODE_OR), (2, 5, 1000, native.MODE_OR)]:
        q_off, qt = synth.queries(256, m0, m1, seed_q=8)
        _same(many[0].search_batch(q_off, qt, k, mode=mode), fa.search_batch(q_off, qt, k, mode=mode), ("a", k, mode))
        _same(many[1].search_batch(q_off, qt, k, mode=mode), fb.search_batch(q_off, qt, k, mode=mode), ("b", k, mode))
        _same(one_b.search_batch(q_off, qt, k, mode=mode), fb.search_batch(q_off, qt, k, mode=mode), ("b1", k, mode))
    for t in range(0, 50_000, 331):
        assert (many[1].term_kth(t) <= fb.term_kth(t)).all(), t
        assert many[1].df(t) == fb.df(t), t
    # the two fresh segments under the namespace's statistics in one plan = the single index
    r = native.Index.rescore_many([a, b], g)
    for (m0, m1, k, mode) in [(2, 5, 1000, native.MODE_OR), (2, 2, 100, native.MODE_AND)]:
        q_off, qt = synth.queries(256, m0, m1, seed_q=9)
        s, d, sh, n = native.search_sharded(r, q_off, qt, k, mode=mode)
        s1, d1, n1 = single.search_batch(q_off, qt, k, mode=mode)
        assert np.array_equal(n, n1)
        for i in range(len(n)):
            m = int(n[i])
            gdoc = d[i, :m] + np.array([0, cut], np.uint32)[sh[i, :m]]
            assert np.array_equal(gdoc, d1[i, :m]), (mode, i)
            assert np.array_equal(s[i, :m], s1[i, :m]), (mode, i)
    for x in many + r + [a, b, fa, fb, one_b, single]:
        x.close()
