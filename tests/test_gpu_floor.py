"""Namespace-wide starting thresholds of doc shards on the device
(fg_index_term_ladder, fg_kth_floor_combine, fg_index_set_kth_floor).

- a shard's ladder (one k_ktop pass into temporaries) equals the K-th scores of
  the term's own top-1000 list from a single-term search of that shard, and its
  main columns equal fg_index_term_kth;
- the combined floor never exceeds the namespace-wide K-th score of the term
  (the oracle's single-term search over the whole corpus with its statistics);
- shards searched with the floor return exactly the hits they return without it,
  and the oracle's segmented search (OR top-k for k in 10..1000, single-term
  queries, AND): the floor only moves where each shard starts pruning.
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
def shards(native):
    from fugu_amd import synth
    from fugu_amd.shard import shard_ranges
    from oracle import oracle as orc
    ctx = native.Context((0,))
    c = synth.corpus(400_000)
    V = synth.VOCAB
    ranges = shard_ranges(c.n_docs, 4)
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in ranges]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, V, threads=16)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, V, threads=16, keep_host=False, global_stats=g) for off, tok in parts]
    ref = orc.OracleIndex(V, c.off, c.tok, threads=16)
    return ctx, c, ranges, ixs, ref


def test_ladder_equals_single_term_lists(native, shards):
    ctx, c, ranges, ixs, ref = shards
    terms = np.array([1, 2, 3, 7, 40, 300, 2000, 9000, 60000, 500000], np.uint32)
    LK = np.array(native.LADDER_KS)
    main = [list(LK).index(k) for k in native.KTH_KS]
    for ix in ixs[:2]:
        lad = ix.term_ladder()
        q_off = np.arange(len(terms) + 1, dtype=np.uint32)
        s, d, n = ix.search_batch(q_off, terms, 1000)
        for i, t in enumerate(terms):
            exp = np.array([s[i, k - 1] if k <= n[i] else 0.0 for k in LK], np.float32)
            assert np.array_equal(lad[t], exp), (int(t), lad[t], exp)
            assert np.array_equal(lad[t, main], ix.term_kth(int(t)))


def test_floor_bounds_namespace_kth(native, shards):
    from fugu_amd.shard import seed_kth_floor
    ctx, c, ranges, ixs, ref = shards
    floor = seed_kth_floor(ixs)
    LKK = native.KTH_KS
    own = np.stack([[ix.term_kth(int(t)) for t in range(1, 4000, 37)] for ix in ixs]).max(axis=0)
    for row, t in enumerate(range(1, 4000, 37)):
        rs, rd = ref.search(np.array([t], np.uint32), 1000, mode=1)
        for j, K in enumerate(LKK):
            exact = rs[K - 1] if K <= len(rs) else 0.0
            assert floor[t, j] <= exact * (1 + 1e-7), (t, K, floor[t, j], exact)
            assert floor[t, j] >= own[row, j]
    # what pruning gains: at K = 1000 over 4 shards the floor sits above every shard's own 1000th
    sample = floor[1:4000:37, 4]
    has = own[:, 4] > 0
    assert has.sum() >= 8 and (sample[has] > own[has, 4]).mean() > 0.9
    for ix in ixs:
        ix.set_kth_floor(None)


@pytest.mark.parametrize("m0,m1,k,mode", [(2, 5, 1000, 1), (2, 4, 100, 1), (2, 3, 20, 1), (2, 5, 10, 1),
                                          (1, 1, 100, 0), (1, 1, 1000, 0), (3, 3, 100, 0)])
def test_seeded_shards_same_hits(native, shards, m0, m1, k, mode):
    from fugu_amd import synth
    from fugu_amd.shard import seed_kth_floor
    ctx, c, ranges, ixs, ref = shards
    q_off, terms = synth.queries(96, m0, m1, seed_q=11)
    for ix in ixs:
        ix.set_kth_floor(None)
    s0, d0, sh0, n0 = native.search_sharded(ixs, q_off, terms, k, mode=mode, ctx=ctx)
    # every shard alone (no shared threshold) with and without the floor, merged on the host
    per0 = [ix.search_batch(q_off, terms, k, mode=mode) for ix in ixs]
    seed_kth_floor(ixs)
    try:
        s1, d1, sh1, n1 = native.search_sharded(ixs, q_off, terms, k, mode=mode, ctx=ctx)
        per1 = [ix.search_batch(q_off, terms, k, mode=mode) for ix in ixs]
    finally:
        for ix in ixs:
            ix.set_kth_floor(None)
    assert np.array_equal(n0, n1)
    for i in range(len(n0)):
        m = int(n0[i])
        assert np.array_equal(d0[i, :m], d1[i, :m]) and np.array_equal(sh0[i, :m], sh1[i, :m])
        assert np.array_equal(s0[i, :m], s1[i, :m])
    from shard_ref import merge_topk_numpy
    merged = []
    for per in (per0, per1):
        sc = np.stack([p[0] for p in per])
        dc = np.stack([p[1] for p in per])
        nn = np.stack([p[2] for p in per]).astype(np.int64)
        merged.append(merge_topk_numpy(sc, dc, nn, k))
    ms0, md0, msh0, mn0 = merged[0]
    ms1, md1, msh1, mn1 = merged[1]
    assert np.array_equal(mn0, mn1) and np.array_equal(mn0, n0.astype(mn0.dtype))
    base = np.array([b for b, _ in ranges], np.uint64)
    bounds = np.array([b for b, _ in ranges] + [c.n_docs], np.uint32)
    for i in range(len(n0)):
        m = int(mn0[i])
        assert np.array_equal(md0[i, :m], md1[i, :m]) and np.array_equal(msh0[i, :m], msh1[i, :m])
        rs, rd = ref.search_segments(terms[q_off[i]:q_off[i + 1]], k, bounds, mode=mode)
        assert m == len(rd)
        gdoc = md1[i, :m].astype(np.uint64) + base[msh1[i, :m]]
        assert np.array_equal(gdoc, rd.astype(np.uint64))
        rel = np.abs(ms1[i, :m].astype(np.float64) - rs) / np.maximum(np.abs(rs), 1e-30)
        assert (rel <= RTOL).all()


@pytest.mark.parametrize("m0,m1,k,mode,frac", [(2, 5, 1000, 1, 0.125), (2, 4, 100, 1, 0.5), (2, 3, 20, 1, 0.0625),
                                               (1, 1, 100, 0, 0.25), (3, 3, 100, 0, 0.5)])
def test_hist_exchange_same_hits(native, shards, m0, m1, k, mode, frac):
    """Every shard alone, its k_disj sweep in two parts (fg_plan_execute_part) with
    the shards' score histograms summed between them (what shard.exchange_hist's
    all-reduce does across GPUs): the hits merged from the shards' lists equal
    the multi-snapshot search's and the oracle's segmented search.  A shard's own
    list may hold fewer than k hits (its tail is below the namespace's k-th)."""
    import torch
    from fugu_amd import synth
    from fugu_amd.shard import agree_hist_span
    from shard_ref import merge_topk_numpy
    ctx, c, ranges, ixs, ref = shards
    q_off, terms = synth.queries(96, m0, m1, seed_q=13)
    nq = len(q_off) - 1
    s0, d0, sh0, n0 = native.search_sharded(ixs, q_off, terms, k, mode=mode, ctx=ctx)
    plans = [ix.plan(q_off, terms, k, mode) for ix in ixs]
    lo, hi = agree_hist_span(plans)
    assert (lo <= hi).all()
    st = torch.cuda.current_stream().cuda_stream
    hb = torch.zeros((len(plans), nq * native.HIST_BINS), dtype=torch.int32, device="cuda")
    for rnd in range(2):  # a second round re-zeroes the plans' state
        for p in plans:
            p.execute_part(st, 0.0, frac)
        for r, p in enumerate(plans):
            p.hist_copy(st, hb[r].data_ptr(), False)
        tot = hb.sum(0, dtype=torch.int32)
        for p in plans:
            p.hist_copy(st, tot.data_ptr(), True)
        # every plan now holds the sum of every shard's first-part counts
        chk = torch.zeros_like(tot)
        for p in plans:
            p.hist_copy(st, chk.data_ptr(), False)
            torch.cuda.synchronize()
            assert torch.equal(chk, tot), rnd
        assert int(tot.sum().item()) == int(hb.sum().item()) and (frac <= 0.1 or int(tot.sum().item()) > 0)
        for p in plans:
            p.execute_part(st, frac, 1.0)
        per = [p.results() for p in plans]
        sc = np.stack([x[0] for x in per])
        dc = np.stack([x[1] for x in per])
        nn = np.stack([x[2] for x in per]).astype(np.int64)
        ms, md, msh, mn = merge_topk_numpy(sc, dc, nn, k)
        assert np.array_equal(mn, n0.astype(mn.dtype))
        for i in range(nq):
            m = int(n0[i])
            assert np.array_equal(md[i, :m], d0[i, :m]) and np.array_equal(msh[i, :m], sh0[i, :m]), (rnd, i)
            assert np.array_equal(ms[i, :m], s0[i, :m])
    base = np.array([b for b, _ in ranges], np.uint64)
    bounds = np.array([b for b, _ in ranges] + [c.n_docs], np.uint32)
    for i in range(nq):
        m = int(mn[i])
        rs, rd = ref.search_segments(terms[q_off[i]:q_off[i + 1]], k, bounds, mode=mode)
        assert m == len(rd)
        assert np.array_equal(md[i, :m].astype(np.uint64) + base[msh[i, :m]], rd.astype(np.uint64))
    for p in plans:
        p.close()


def test_multi_plan_parts_equal_merged(native, shards):
    """A multi-snapshot plan run in two parts (its slots already share one
    histogram: the exchange of one rank) gives execute_merged's hits."""
    import torch
    from fugu_amd import synth
    ctx, c, ranges, ixs, ref = shards
    q_off, terms = synth.queries(64, 2, 5, seed_q=17)
    nq, k = len(q_off) - 1, 200
    mp = native.Plan(ixs, q_off, terms, k, native.MODE_OR)
    st = torch.cuda.current_stream().cuda_stream
    a = [torch.zeros(nq * k, dtype=t, device="cuda") for t in (torch.float32, torch.int32, torch.int32)]
    a.append(torch.zeros(nq, dtype=torch.int32, device="cuda"))
    b = [torch.zeros_like(x) for x in a]
    mp.execute_merged(st, *[x.data_ptr() for x in a])
    mp.execute_part(st, 0.0, 0.3)
    hb = torch.zeros(nq * native.HIST_BINS, dtype=torch.int32, device="cuda")
    mp.hist_copy(st, hb.data_ptr(), False)
    mp.hist_copy(st, hb.data_ptr(), True)
    mp.execute_part(st, 0.3, 1.0, *[x.data_ptr() for x in b])
    torch.cuda.synchronize()
    n = a[3].cpu().numpy()
    assert np.array_equal(n, b[3].cpu().numpy()) and n.sum() > 0
    for x, y in zip(a[:3], b[:3]):
        xa, ya = x.cpu().numpy().reshape(nq, k), y.cpu().numpy().reshape(nq, k)
        for i in range(nq):
            assert np.array_equal(xa[i, :n[i]], ya[i, :n[i]])
    assert int(hb.sum().item()) > 0
    with pytest.raises(native.FuguError):
        mp.execute_part(st, 0.5, 0.5)
    with pytest.raises(native.FuguError):  # parts must continue the sweep
        mp.execute_part(st, 0.3, 1.0, *[x.data_ptr() for x in b])
    mp.execute_part(st, 0.0, 0.5)
    with pytest.raises(native.FuguError):
        mp.execute_part(st, 0.6, 1.0, *[x.data_ptr() for x in b])
    mp.execute_part(st, 0.5, 1.0, *[x.data_ptr() for x in b])
    torch.cuda.synchronize()
    assert np.array_equal(n, b[3].cpu().numpy())
    mp.close()
