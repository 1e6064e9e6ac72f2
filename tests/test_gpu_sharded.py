"""fg_search_sharded: one batch over several shard indexes of one logical index,
merged on the device by (score desc, shard asc, doc asc) (SURVEY.md §8b
`fg_search_sharded`, §8e).

- doc shards scored with the namespace's global statistics (tantivy's segment
  model, reference src/db/core.rs:49-79, one segment per commit
  src/db/document.rs:65): the merged result is the oracle's multi-segment search
  (`or_search_seg`: every segment orders its intersection by its own cost) --
  doc ids exact, scores within 1e-5 relative;
- independent namespaces (own statistics, a fan-out query, config C4's shape):
  the per-namespace fg_search_batch results merged by numpy.
The shards share the one MI355X here; on a node each shard's device runs its
own part and the lists cross xGMI to shards[0]'s device.
"""
import numpy as np
import pytest

from shard_ref import merge_topk_numpy

pytestmark = pytest.mark.gpu
RTOL = 1e-5


@pytest.fixture(scope="module")
def native():
    from fugu_amd import native as nat
    if nat.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    return nat


@pytest.fixture(scope="module")
def ctx(native):
    return native.Context((0,))


@pytest.fixture(scope="module")
def doc_shards(native, ctx):
    from fugu_amd import synth
    from fugu_amd.shard import shard_ranges
    from oracle import oracle as orc
    c = synth.corpus(1_000_000)
    V = synth.VOCAB
    ranges = shard_ranges(c.n_docs, 3)
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in ranges]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, V, threads=16)
        g = x if g is None else g + x
    shards = [native.Index.from_docs(ctx, off, tok, V, threads=16, keep_host=False, global_stats=g)
              for off, tok in parts]
    ref = orc.OracleIndex(V, c.off, c.tok, threads=16)
    return c, ranges, shards, ref


@pytest.mark.parametrize("m0,m1,k,mode", [(3, 3, 100, 0), (1, 5, 100, 0), (2, 5, 1000, 1), (2, 3, 10, 1),
                                          (2, 2, 1, 0)])
def test_doc_shards_equal_segmented_oracle(native, ctx, doc_shards, m0, m1, k, mode):
    from fugu_amd import synth
    c, ranges, shards, ref = doc_shards
    q_off, terms = synth.queries(128, m0, m1, seed_q=5)
    s, d, sh, n = native.search_sharded(shards, q_off, terms, k, mode=mode, ctx=ctx)
    base = np.array([b for b, _ in ranges], np.uint64)
    bounds = np.array([b for b, _ in ranges] + [c.n_docs], np.uint32)
    for i in range(len(n)):
        t = terms[q_off[i]:q_off[i + 1]]
        rs, rd = ref.search_segments(t, k, bounds, mode=mode)
        m = int(n[i])
        assert m == len(rd), (i, m, len(rd))
        gdoc = d[i, :m].astype(np.uint64) + base[sh[i, :m]]
        assert np.array_equal(gdoc, rd.astype(np.uint64)), (i, t.tolist())
        rel = np.abs(s[i, :m].astype(np.float64) - rs) / np.maximum(np.abs(rs), 1e-30)
        assert (rel <= RTOL).all(), (i, rel.max())
    assert (n > 0).mean() > 0.5


def test_namespaces_fanout_equals_numpy_merge(native, ctx):
    """Four namespaces with their own statistics: fg_search_sharded == the
    per-namespace batches merged by (score desc, namespace asc, doc asc)."""
    from fugu_amd import synth
    V = synth.VOCAB
    nss = [synth.corpus(200_000, V, 1.0, synth.SEED_L + r, synth.SEED_T + r) for r in range(4)]
    ixs = [native.Index.from_docs(ctx, c.off, c.tok, V, threads=16, keep_host=False) for c in nss]
    for m0, m1, k, mode in [(3, 3, 100, 0), (2, 4, 1000, 1)]:
        q_off, terms = synth.queries(256, m0, m1, seed_q=9)
        s, d, sh, n = native.search_sharded(ixs, q_off, terms, k, mode=mode)
        per = [ix.search_batch(q_off, terms, k, mode=mode) for ix in ixs]
        es, ed, esh, en = merge_topk_numpy(np.stack([p[0] for p in per]), np.stack([p[1] for p in per]),
                                           np.stack([p[2] for p in per]), k)
        assert np.array_equal(n, en)
        for i in range(len(n)):
            m = int(n[i])
            assert np.array_equal(s[i, :m], es[i, :m]) and np.array_equal(d[i, :m], ed[i, :m]), (mode, i)
            assert np.array_equal(sh[i, :m], esh[i, :m]), (mode, i)


def test_sharded_concurrent_callers(native, ctx):
    """Four host threads issue fan-out batches over the same namespaces at once
    (the side streams are shared by every caller; each call orders its own work
    with events): every call returns the single-caller result."""
    import threading

    from fugu_amd import synth
    V = synth.VOCAB
    nss = [synth.corpus(100_000, V, 1.0, synth.SEED_L + 10 + r, synth.SEED_T + 10 + r) for r in range(3)]
    ixs = [native.Index.from_docs(ctx, c.off, c.tok, V, threads=16, keep_host=False) for c in nss]
    batches = [synth.queries(128, 1, 4, seed_q=40 + t) for t in range(4)]
    want = [native.search_sharded(ixs, qo, qt, 100) for qo, qt in batches]
    errors = []

    def worker(t):
        try:
            for _ in range(5):
                got = native.search_sharded(ixs, *batches[t], 100)
                n = want[t][3]
                assert np.array_equal(got[3], n)
                for i in range(len(n)):
                    m = int(n[i])
                    for a, b in zip(got[:3], want[t][:3]):
                        assert np.array_equal(a[i, :m], b[i, :m]), (t, i)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errors, errors[:3]


def test_sharded_terms_outside_a_shard_and_errors(native, ctx):
    """A shard built before a term was interned (smaller n_terms) matches nothing
    for it; bad arguments are rejected before any launch."""
    from fugu_amd import synth
    c = synth.corpus(50_000)
    small = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16)
    # the same docs with every term id shifted past a 2^20 dictionary: none of the
    # query terms exists there
    big = native.Index.from_docs(ctx, c.off, c.tok + (1 << 20), 1 << 21, threads=16)
    q_off, terms = synth.queries(64, 2, 3, seed_q=3)
    # low ids: in both dictionaries, postings only in `small`
    s, d, sh, n = native.search_sharded([big, small], q_off, terms, 100)
    s1, d1, n1 = small.search_batch(q_off, terms, 100)
    assert np.array_equal(n, n1) and (n1 > 0).any()
    for i in range(len(n)):
        m = int(n1[i])
        assert (sh[i, :m] == 1).all() and np.array_equal(d[i, :m], d1[i, :m])
        assert np.array_equal(s[i, :m], s1[i, :m])
    # high ids: >= small's n_terms (unknown there), postings in `big`
    hi = terms + np.uint32(1 << 20)
    s, d, sh, n = native.search_sharded([big, small], q_off, hi, 100)
    s2, d2, n2 = big.search_batch(q_off, hi, 100)
    assert np.array_equal(n, n2) and (n2 > 0).any()
    for i in range(len(n)):
        m = int(n2[i])
        assert (sh[i, :m] == 0).all() and np.array_equal(d[i, :m], d2[i, :m])
    with pytest.raises(native.FuguError) as e:
        native.search_sharded([], q_off, terms, 100)
    assert e.value.code == native.FG_EINVAL
    with pytest.raises(native.FuguError):
        native.search_sharded([small], q_off, terms, 0)
