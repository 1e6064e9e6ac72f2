"""Seeded disjunction thresholds (k_seed, fg_internal.h kSeedKS).

Before k_disj, one workgroup per Should-only query scores exactly the union of
its clauses' best docs (each clause's best min(k, 256) alive keys, kept by the
k_ktop kernels, or all postings of a clause of <= 1024) and publishes the k-th
best of those distinct docs as the query's starting threshold, score-only.
It only moves where pruning starts: hits must be identical with FUGU_SEED=0
(no seed) and equal the oracle, for every k, with deletions, on a multi-snapshot
plan, and for queries whose clauses' candidate lists overlap (the dedupe rule).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
RTOL = 1e-5


@pytest.fixture(scope="module")
def native():
    from fugu_amd import native as nat
    if nat.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    return nat


@pytest.fixture(scope="module")
def corpus(native):
    from fugu_amd import synth
    from oracle import oracle as orc
    ctx = native.Context((0,))
    c = synth.corpus(1_000_000)
    V = synth.VOCAB
    dele = (np.arange(c.n_docs) % 13 == 5).astype(np.uint8)
    ix = native.Index.from_docs(ctx, c.off, c.tok, V, threads=16, keep_host=False, deleted=dele)
    ref = orc.OracleIndex(V, c.off, c.tok, threads=16, deleted=dele)
    return ctx, c, ix, ref, dele


def _run(native, ix, q_off, terms, k, monkeypatch, seed):
    monkeypatch.setenv("FUGU_SEED", "1" if seed else "0")
    return ix.search_batch(q_off, terms, k, mode=native.MODE_OR)


@pytest.mark.parametrize("k", [1, 10, 20, 100, 256, 1000])
def test_seeded_equals_unseeded_and_oracle(native, corpus, monkeypatch, k):
    from fugu_amd import synth
    ctx, c, ix, ref, dele = corpus
    # terms from the dense head too (overlapping candidate lists): ranks 1..64 half the time
    q_off, terms = synth.queries(160, 2, 5, seed_q=41)
    q_off2, terms2 = synth.queries(96, 2, 4, seed_q=42, max_rank=64)
    q_off = np.concatenate([q_off, q_off2[1:] + q_off[-1]]).astype(np.uint32)
    terms = np.concatenate([terms, terms2]).astype(np.uint32)
    s1, d1, n1 = _run(native, ix, q_off, terms, k, monkeypatch, True)
    s0, d0, n0 = _run(native, ix, q_off, terms, k, monkeypatch, False)
    assert np.array_equal(n0, n1)
    for i in range(len(n0)):
        m = int(n0[i])
        assert np.array_equal(d0[i, :m], d1[i, :m]) and np.array_equal(s0[i, :m], s1[i, :m]), i
    check = range(0, len(n1), 3) if k >= 256 else range(len(n1))
    rs_all, rd_all, rn_all, _, _ = ref.search_batch(q_off, terms, k, mode=1, threads=16)
    for i in check:
        m = int(n1[i])
        assert m == int(rn_all[i])
        assert np.array_equal(d1[i, :m], rd_all[i, :m]), (i, k)
        rel = np.abs(s1[i, :m].astype(np.float64) - rs_all[i, :m]) / np.maximum(np.abs(rs_all[i, :m]), 1e-30)
        assert (rel <= RTOL).all()


def test_seeded_multi_snapshot_plan(native, monkeypatch):
    """Three segments with the namespace's statistics in one multi-snapshot
    plan: every slot seeds the batch query's shared threshold from its own
    segment's docs (score-only); merged hits as without seeds."""
    from fugu_amd import synth
    from fugu_amd.shard import shard_ranges
    ctx = native.Context((0,))
    c = synth.corpus(600_000)
    V = synth.VOCAB
    ranges = shard_ranges(c.n_docs, 3)
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in ranges]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, V, threads=16)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, V, threads=16, keep_host=False, global_stats=g) for off, tok in parts]
    q_off, terms = synth.queries(128, 2, 5, seed_q=43)
    out = {}
    for seed in (True, False):
        monkeypatch.setenv("FUGU_SEED", "1" if seed else "0")
        for k in (20, 100):
            out[(seed, k)] = native.search_sharded(ixs, q_off, terms, k, mode=native.MODE_OR, ctx=ctx)
    for k in (20, 100):
        a, b = out[(True, k)], out[(False, k)]
        assert np.array_equal(a[3], b[3])
        for i in range(len(a[3])):
            m = int(a[3][i])
            for j in range(3):
                assert np.array_equal(a[j][i, :m], b[j][i, :m]), (k, i, j)
