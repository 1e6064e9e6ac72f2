"""Per-term K-th best alive scores (k_ktop / k_ktop_part / k_ktop_big, runs on
the MI355X box): the starting thresholds of k_disj and of single-list k_conj
queries.  A term's K-th best alive posting score must equal the K-th score of
the term's own single-term top-1000 (a different kernel path: k_conj's
single-list items), for K = 1, 10, 20, 100, 1000, and 0 when the term has fewer
alive postings -- for terms of every length, including those past kKtopChunk
postings (chunked selection) and with deleted docs (the alive filter).
Bar: bit-identical scores.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
KS = (1, 10, 20, 100, 1000)


@pytest.fixture(scope="module")
def native():
    from fugu_amd import native as nat
    if nat.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    return nat


@pytest.mark.parametrize("with_deletes", [False, True])
def test_term_kth_equals_single_term_topk(native, with_deletes):
    from fugu_amd import synth
    ctx = native.Context((0,))
    c = synth.corpus(1_000_000)
    deleted = None
    if with_deletes:
        rng = np.random.default_rng(7)
        deleted = (rng.random(c.n_docs) < 0.1).astype(np.uint8)
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, deleted=deleted)
    # terms of every length: dense (> kKtopChunk = 32768 postings: chunked), mid, short, tiny
    picked = {"long": [], "mid": [], "short": [], "tiny": []}
    for t in range(0, 200_000):
        df = ix.df(t)
        key = "long" if df > 32768 else "mid" if df > 2000 else "short" if df > 30 else "tiny" if df > 0 else None
        if key and len(picked[key]) < 12:
            picked[key].append(t)
        if all(len(v) >= 12 for v in picked.values()):
            break
    assert all(len(v) >= 4 for v in picked.values()), {k: len(v) for k, v in picked.items()}
    terms = [t for v in picked.values() for t in v]
    q_off = np.arange(len(terms) + 1, dtype=np.uint32)
    s, d, n = ix.search_batch(q_off, np.array(terms, np.uint32), 1000)
    for i, t in enumerate(terms):
        got = ix.term_kth(t)
        want = np.array([s[i, k - 1] if n[i] >= k else 0.0 for k in KS], np.float32)
        assert np.array_equal(got, want), (t, ix.df(t), int(n[i]), got.tolist(), want.tolist())


def test_background_capped_scoring_identical(native):
    """A commit's scorings run in the background with at most FUGU_BG_GRID
    workgroups per CU per launch (fg::ScoreJob::grid_cap: every scoring kernel
    loops over its items in steps of the grid) and read the per-term tables back
    through a copy kernel.  The rescored snapshot must equal the foreground
    (uncapped) one: per-term K-th scores and maxima bit for bit, and every
    search's hits."""
    from fugu_amd import synth
    ctx = native.Context((0,))
    c = synth.corpus(600_000)
    g = native.docs_stats(c.off, c.tok, synth.VOCAB, threads=16)
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, global_stats=g)
    rng = np.random.default_rng(3)
    deleted = (rng.random(c.n_docs) < 0.05).astype(np.uint8)
    fg = ix.rescore(g, deleted)
    prev = native._lib.fg_thread_background(1)
    try:
        bg = ix.rescore(g, deleted)
    finally:
        native._lib.fg_thread_background(prev)
    terms = [t for t in range(0, 300_000, 97) if ix.df(t) > 0]
    assert len(terms) > 1000
    for t in terms:
        assert np.array_equal(fg.term_kth(t), bg.term_kth(t)), t
    q_off, qt = synth.queries(256, 1, 4, seed_q=21)
    for mode, k in ((native.MODE_OR, 20), (native.MODE_OR, 1000), (native.MODE_AND, 100)):
        a = fg.search_batch(q_off, qt, k, mode=mode)
        b = bg.search_batch(q_off, qt, k, mode=mode)
        assert np.array_equal(a[2], b[2])
        for i in range(len(a[2])):
            m = int(a[2][i])
            assert np.array_equal(a[0][i, :m], b[0][i, :m]) and np.array_equal(a[1][i, :m], b[1][i, :m])
    for x in (fg, bg, ix):
        x.close()


def test_rescore_kth_is_a_lower_bound(native):
    """A rescore runs no device work: its per-term K-th scores are the build's
    times the smallest current / build score ratio of the term's postings
    (fugu.cpp term_ratio), with new deletions taken from the level K + the docs
    deleted since (term_kth_now).  They must never exceed the exact K-th scores
    under the new statistics (a fresh build with them), stay within 1% of them
    without deletions (a 10% larger namespace), and the searches must return the
    fresh build's hits."""
    from fugu_amd import synth
    ctx = native.Context((0,))
    c = synth.corpus(400_000)
    big = synth.corpus(440_000)  # statistics of the namespace after a commit of 40K more docs
    g1 = native.docs_stats(c.off, c.tok, synth.VOCAB, threads=16)
    g2 = native.docs_stats(big.off, big.tok, synth.VOCAB, threads=16)
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, global_stats=g1)
    re = ix.rescore(g2)
    fresh = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, global_stats=g2)
    terms = [t for t in range(0, 200_000, 53) if ix.df(t) > 0]
    assert len(terms) > 1000
    below, n = 0, 0
    for t in terms:
        a, b = re.term_kth(t), fresh.term_kth(t)
        assert (a <= b).all(), (t, a, b)
        assert np.array_equal(a > 0, b > 0), (t, a, b)
        nz = b > 0
        assert (a[nz] >= b[nz] * 0.99).all(), (t, a, b)
        below += int((a[nz] < b[nz]).sum())
        n += int(nz.sum())
    assert n > 1000
    q_off, qt = synth.queries(256, 1, 4, seed_q=23)
    for mode, k in ((native.MODE_OR, 20), (native.MODE_OR, 1000), (native.MODE_AND, 100)):
        x = re.search_batch(q_off, qt, k, mode=mode)
        y = fresh.search_batch(q_off, qt, k, mode=mode)
        assert np.array_equal(x[2], y[2])
        for i in range(len(x[2])):
            m = int(x[2][i])
            assert np.array_equal(x[1][i, :m], y[1][i, :m]) and np.array_equal(x[0][i, :m], y[0][i, :m])
    # new deletions: lower bounds still, and the fresh build's hits
    rng = np.random.default_rng(5)
    deleted = (rng.random(c.n_docs) < 0.02).astype(np.uint8)
    re2 = ix.rescore(g2, deleted)
    fresh2 = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, global_stats=g2, deleted=deleted)
    for t in terms[::7]:
        assert (re2.term_kth(t) <= fresh2.term_kth(t)).all(), t
    for mode, k in ((native.MODE_OR, 20), (native.MODE_AND, 100)):
        x = re2.search_batch(q_off, qt, k, mode=mode)
        y = fresh2.search_batch(q_off, qt, k, mode=mode)
        assert np.array_equal(x[2], y[2])
        for i in range(len(x[2])):
            m = int(x[2][i])
            assert np.array_equal(x[1][i, :m], y[1][i, :m]) and np.array_equal(x[0][i, :m], y[0][i, :m])
    for x in (re, re2, fresh, fresh2, ix):
        x.close()
