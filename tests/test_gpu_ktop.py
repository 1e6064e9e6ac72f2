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
