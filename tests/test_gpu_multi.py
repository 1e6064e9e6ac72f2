"""Multi-snapshot plans (fg_plan_create_multi): the segments / doc shards /
namespaces of one device planned as ONE batch and run by one launch per kernel,
their query slots sharing each query's threshold score-only (runs on the MI355X
box).  fg_search_sharded uses them for every device's shards.

Reference semantics: tantivy searches every segment of a namespace with the
namespace's statistics and merges the per-segment TopDocs by (score desc,
segment asc, doc asc) (src/db/search.rs:162, src/db/document.rs:65); here each
shard's own single-snapshot plan (already checked against the oracle) merged in
numpy is the reference, plus the oracle's segmented search (`or_search_seg`
model) on a sample.  Covered: AND / OR / mixed occurs (k_conj, single-list
k_conj, k_disj and k_scan items of several snapshots in one launch), facet
filters (k_fmask over several snapshots' facet postings), terms a snapshot
lacks, one query (the GET /search latency path) and 1024-query batches; the
merged select (fg_plan_execute_merged: one final select over all slots of a
query) against the per-slot lists through fg_merge_shards.
Bar: doc ids exact, scores within 1e-5 relative (bit-identical in practice).
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
def segs(native, ctx):
    """1M docs with facets as 5 uneven segments scored with the global statistics."""
    import synth_ref as sr
    from fugu_amd import synth
    c = synth.corpus(1_000_000)
    fo, ft, nf = sr.facet_tokens(1_000_000, 4242)
    V = synth.VOCAB
    cuts = [0, 100_000, 370_000, 380_000, 700_000, 1_000_000]  # one tiny segment, like a small late commit
    parts = []
    for b, e in zip(cuts[:-1], cuts[1:]):
        parts.append((b, c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]], (fo[b:e + 1] - fo[b], ft[fo[b]:fo[e]], nf)))
    g = None
    for _, off, tok, fc in parts:
        x = native.docs_stats(off, tok, V, threads=16, facets=fc)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, V, threads=16, global_stats=g, facets=fc, keep_host=False)
           for _, off, tok, fc in parts]
    from oracle import oracle as orc
    ref = orc.OracleIndex(V, c.off, c.tok, threads=16, facet_off=fo, facet_tok=ft, n_fterms=nf)
    return np.array(cuts, np.uint32), ixs, nf, ref


def random_occurs(q_off, seed):
    rng = np.random.default_rng(seed)
    occ = []
    for i in range(len(q_off) - 1):
        m = int(q_off[i + 1] - q_off[i])
        shape = rng.integers(0, 4)
        o = [0] * m if shape == 0 else [1] * m if shape == 1 else [int(x) for x in rng.choice(3, m, p=[.4, .4, .2])]
        if m and all(x == 2 for x in o):
            o[0] = 1
        occ += o
    return np.array(occ, np.uint8)


def facet_clauses(nq, ncl, nf, seed):
    rng = np.random.default_rng(seed)
    fl = [[int(x) for x in rng.integers(0, nf, rng.integers(0, ncl + 1))] for _ in range(nq)]
    f_off = np.cumsum([0] + [len(f) for f in fl]).astype(np.uint32)
    return f_off, np.array([t for f in fl for t in f], np.uint32)


def per_segment_merged(ixs, q_off, terms, k, mode, occur=None, f_off=None, f_terms=None):
    res = [ix.search_batch(q_off, terms, k, mode=mode, occur=occur, f_off=f_off, f_terms=f_terms) for ix in ixs]
    sc, dc, nn = (np.stack([r[j] for r in res]) for j in range(3))
    return (sc, dc, nn), merge_topk_numpy(sc, dc, nn, k)


def assert_merged(got, want, what=""):
    s, d, sh, n = got
    ws, wd, wsh, wn = want
    assert np.array_equal(n.astype(np.int64), wn.astype(np.int64)), what
    for i in range(len(n)):
        m = int(n[i])
        assert np.array_equal(sh[i, :m].astype(np.int64), wsh[i, :m]), (what, i)
        assert np.array_equal(d[i, :m], wd[i, :m]), (what, i)
        rel = np.abs(s[i, :m].astype(np.float64) - ws[i, :m]) / np.maximum(np.abs(ws[i, :m]), 1e-30)
        assert (rel <= RTOL).all(), (what, i, rel.max())


@pytest.mark.parametrize("m_min,m_max,k,mode,occ,ncl,nq", [
    (3, 3, 100, 0, False, 0, 1024),   # the headline shape over 5 segments
    (1, 5, 100, 0, False, 0, 512),    # single-list k_conj items too
    (2, 5, 1000, 1, False, 0, 128),   # k_disj
    (2, 4, 20, 1, False, 2, 256),     # OR + facet filters
    (1, 5, 50, 0, True, 3, 256),      # mixed occurs + facets: k_conj, k_disj, k_scan in one launch
    (0, 0, 100, 0, False, 3, 64),     # facet-only / AllQuery: k_scan
    (2, 3, 20, 1, True, 0, 1),        # one query: the GET /search latency path
])
def test_sharded_multi_plan_equals_per_segment_merge(native, ctx, segs, m_min, m_max, k, mode, occ, ncl, nq):
    from fugu_amd import synth
    cuts, ixs, nf, _ = segs
    if m_max == 0:
        q_off, terms = np.zeros(nq + 1, np.uint32), np.zeros(0, np.uint32)
    else:
        q_off, terms = synth.queries(nq, m_min, m_max, seed_q=301 + k + ncl)
    occur = random_occurs(q_off, k + nq) if occ else None
    f_off, f_terms = facet_clauses(nq, ncl, nf, 77 + k) if ncl else (None, None)
    _, want = per_segment_merged(ixs, q_off, terms, k, mode, occur, f_off, f_terms)
    got = native.search_sharded(ixs, q_off, terms, k, mode=mode, ctx=ctx, occur=occur, f_off=f_off, f_terms=f_terms)
    assert_merged(got, want, (m_min, m_max, k, mode, occ, ncl))
    assert (got[3] > 0).mean() > 0.3


def test_multi_plan_slots_are_prefixes_of_segment_lists(native, segs):
    """A slot's list is a prefix of its segment's own top-k that holds every hit
    scoring at least the merged k-th score (the shared threshold prunes strictly
    below the k-th best score any slot of the query has found)."""
    from fugu_amd import synth
    cuts, ixs, _, _ = segs
    k, nq = 100, 256
    q_off, terms = synth.queries(nq, 2, 4, seed_q=911)
    for mode in (0, 1):
        (sc, dc, nn), (ms, md, msh, mn) = per_segment_merged(ixs, q_off, terms, k, mode)
        p = native.Plan(ixs, q_off, terms, k, mode=mode)
        assert p.n_queries == len(ixs) * nq and p.info().n_queries == len(ixs) * nq
        p.execute()
        s, d, n = p.results()
        S = len(ixs)
        s, d, n = s.reshape(S, nq, k), d.reshape(S, nq, k), n.reshape(S, nq)
        for q in range(nq):
            kth = ms[q, mn[q] - 1] if mn[q] == k else -1.0
            for j in range(S):
                m = int(n[j, q])
                assert m <= nn[j, q], (mode, q, j)
                assert np.array_equal(d[j, q, :m], dc[j, q, :m]), (mode, q, j)
                assert np.array_equal(s[j, q, :m], sc[j, q, :m]), (mode, q, j)
                assert (sc[j, q, m:nn[j, q]] < kth).all(), (mode, q, j)
        p.close()


def test_sharded_multi_plan_vs_segmented_oracle(native, ctx, segs):
    """A sample against the oracle's multi-segment search directly (every
    segment orders its intersection by its own cost, global statistics)."""
    from fugu_amd import synth
    cuts, ixs, _, ref = segs
    for mode, k in ((0, 100), (1, 20), (1, 1000)):
        q_off, terms = synth.queries(48, 2, 4, seed_q=17 + k)
        s, d, sh, n = native.search_sharded(ixs, q_off, terms, k, mode=mode, ctx=ctx)
        for i in range(len(n)):
            rs, rd = ref.search_segments(terms[q_off[i]:q_off[i + 1]], k, cuts, mode=mode)
            m = int(n[i])
            assert m == len(rd), (mode, k, i)
            assert np.array_equal(d[i, :m].astype(np.int64) + cuts[sh[i, :m]], rd.astype(np.int64)), (mode, k, i)
            rel = np.abs(s[i, :m].astype(np.float64) - rs) / np.maximum(np.abs(rs), 1e-30)
            assert (rel <= RTOL).all(), (mode, k, i)


def test_multi_plan_errors(native, ctx, segs):
    from fugu_amd import synth
    _, ixs, _, _ = segs
    q_off, terms = synth.queries(4, 2, 2, seed_q=3)
    with pytest.raises(native.FuguError):
        native.Plan([], q_off, terms, 10)
    p = native.Plan(ixs[:2], q_off, terms, 10)
    with pytest.raises(native.Unsupported):  # a multi-snapshot plan shares its thresholds already
        native.link_plans([p, native.Plan(ixs[2], q_off, terms, 10)])
    with pytest.raises(native.Unsupported):
        native.Plan(ixs[:2], q_off, terms, 2000)


@pytest.mark.parametrize("mode,k,m0,m1,nq", [(0, 100, 3, 3, 256), (1, 20, 2, 4, 256), (1, 1000, 2, 5, 64),
                                             (0, 10, 1, 5, 256), (1, 20, 2, 3, 1)])
def test_merged_select_equals_slot_lists_merged(native, segs, mode, k, m0, m1, nq):
    """fg_plan_execute_merged (one final select over all slots of a query, keys
    shifted by the snapshots' bases) == the per-slot lists through
    fg_merge_shards, entry for entry; slots past the count are zero."""
    import torch
    from fugu_amd import synth
    from fugu_amd.shard import merge_on_device
    _, ixs, _, _ = segs
    S = len(ixs)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev).cuda_stream
    q_off, terms = synth.queries(nq, m0, m1, seed_q=77 + k)
    p = native.Plan(ixs, q_off, terms, k, mode)
    gs = torch.zeros((S, nq * k), dtype=torch.float32, device=dev)
    gd = torch.zeros((S, nq * k), dtype=torch.int32, device=dev)
    gn = torch.zeros((S, nq), dtype=torch.int32, device=dev)
    p.execute(st, gs.data_ptr(), gd.data_ptr(), gn.data_ptr())
    ms, md, msh, mn = merge_on_device(gs, gd, gn, nq, k, st)
    os_ = torch.full((nq * k,), 7.0, dtype=torch.float32, device=dev)
    od, osh = (torch.full((nq * k,), 7, dtype=torch.int32, device=dev) for _ in range(2))
    on = torch.zeros(nq, dtype=torch.int32, device=dev)
    p.execute_merged(st, os_.data_ptr(), od.data_ptr(), osh.data_ptr(), on.data_ptr())
    torch.cuda.synchronize()
    mn, on_h = mn.cpu().numpy(), on.cpu().numpy()
    assert np.array_equal(mn, on_h)
    a = [x.cpu().numpy().reshape(nq, k) for x in (ms, md, msh)]
    b = [x.cpu().numpy().reshape(nq, k) for x in (os_, od, osh)]
    for q in range(nq):
        n = int(on_h[q])
        for x, y in zip(a, b):
            assert np.array_equal(x[q, :n], y[q, :n]), q
            assert not y[q, n:].any(), q  # slots past the count: 0
    assert (on_h > 0).mean() > 0.5
    p.close()
    with pytest.raises(native.Unsupported):  # one snapshot: nothing to merge
        native.Plan(ixs[0], q_off, terms, k, mode).execute_merged(st, os_.data_ptr(), od.data_ptr(), osh.data_ptr(),
                                                                  on.data_ptr())


def test_many_small_segments(native, ctx):
    """17 small segments (a namespace between host merges, FG_MAX_SEGMENTS = 64):
    one multi-snapshot plan through fg_search_sharded, batch (merged select) and
    single queries (per-slot lists + k_merge_rank), against the per-segment merge."""
    from fugu_amd import synth
    c = synth.corpus(170_000)
    V = synth.VOCAB
    cuts = [i * 10_000 for i in range(18)]
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in zip(cuts[:-1], cuts[1:])]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, V)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, V, global_stats=g, keep_host=False) for off, tok in parts]
    for mode, k, nq in ((0, 100, 512), (1, 20, 512), (1, 10, 1), (0, 1000, 256)):
        q_off, terms = synth.queries(nq, 1 if mode == 0 else 2, 4, seed_q=5 + k + nq)
        _, want = per_segment_merged(ixs, q_off, terms, k, mode)
        got = native.search_sharded(ixs, q_off, terms, k, mode=mode, ctx=ctx)
        assert_merged(got, want, (mode, k, nq))
    for ix in ixs:
        ix.close()
