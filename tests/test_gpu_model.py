"""fg_model_batch (the roofline numerators, fugu_amd/csrc/model.cpp) against the
oracle on a 200K-doc corpus: the replay of k_conj's exhaustive cascade keeps
exactly the intersection |I_q| of every query, the lead stream is 8 B per
posting of the cheapest list, and at the final k-th score the replays of both
kernels keep at least the k hits the kernels returned (MaxScore at that
threshold never drops a top-k doc).  Line floors: the launch's distinct lines
never exceed the per-query sum."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    from fugu_amd import native, synth
    from oracle import oracle as orc
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    ctx = native.Context((0,))
    corp = synth.corpus(200_000, synth.VOCAB)
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, keep_host=True)
    ref = orc.OracleIndex(synth.VOCAB, corp.off, corp.tok, threads=8)
    yield native, synth, orc, ix, ref
    ix.close()


def test_and_exhaustive_keeps_the_intersection(setup):
    native, synth, orc, ix, ref = setup
    q_off, terms = synth.queries(96, 2, 4)
    tot, per = ix.model(q_off, terms, 100)
    inter = 0.0
    for i in range(len(q_off) - 1):
        t = terms[q_off[i]:q_off[i + 1]]
        inter += ref.bytes_model(t, 100)[3]  # |I_q|
        dfs = [ix.df(int(x)) for x in t]
        if min(dfs) > 0:
            assert per[i, 0] >= 8.0 * min(dfs)  # the lead list's doc ids + scores (+ nothing else for m > 1)
            if len(t) > 1:
                assert per[i, 0] == 8.0 * min(dfs)
    assert tot["candidates"] == inter
    assert tot["alg_bytes"] == pytest.approx(per[:, 3].sum())
    assert 0 < tot["line_bytes"] <= tot["query_line_bytes"]


def test_and_at_threshold_keeps_the_topk(setup):
    native, synth, orc, ix, ref = setup
    q_off, terms = synth.queries(96, 1, 4)
    k = 20
    s, d, n = ix.search_batch(q_off, terms, k)
    thr = np.where(n >= k, s[:, k - 1], 0.0).astype(np.float32)
    full, _ = ix.model(q_off, terms, k)
    tot, per = ix.model(q_off, terms, k, thr=thr)
    assert tot["candidates"] >= n.sum()
    assert tot["alg_bytes"] <= full["alg_bytes"]
    assert 0 < tot["line_bytes"] <= tot["query_line_bytes"]


def test_or_at_threshold_keeps_the_topk(setup):
    native, synth, orc, ix, ref = setup
    q_off, terms = synth.queries(64, 2, 5, seed_q=11)
    for k in (10, 1000):
        s, d, n = ix.search_batch(q_off, terms, k, mode=native.MODE_OR)
        thr = np.where(n >= k, s[:, k - 1], 0.0).astype(np.float32)
        tot, per = ix.model(q_off, terms, k, thr=thr, mode=native.MODE_OR)
        assert tot["candidates"] >= n.sum(), k
        assert tot["stream_bytes"] > 0 and tot["probe_bytes"] > 0
        assert 0 < tot["line_bytes"] <= tot["query_line_bytes"]
        # the per-query split is the legacy fg_bytes_model_or output
        assert np.allclose(per, ix.bytes_model_or(q_off, terms, k, thr))
