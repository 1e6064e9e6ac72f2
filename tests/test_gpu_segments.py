"""Snapshots scored on the device and rescored with new statistics
(fg_index_rescore): tantivy's commit model, where a commit adds a segment
(reference src/db/document.rs:65) and every segment is then scored with the
namespace's new N / df / token totals (Bm25StatisticsProvider).  A rescored
snapshot must answer exactly like a snapshot built from scratch with the same
statistics; segments merged by (score desc, segment asc, doc asc) must answer
like the single index.
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


@pytest.fixture(scope="module")
def parts():
    from fugu_amd import synth
    c = synth.corpus(1_000_000)
    cut = 800_000
    a = (c.off[:cut + 1].copy(), c.tok[:c.off[cut]])
    b = (c.off[cut:] - c.off[cut], c.tok[c.off[cut]:])
    return c, cut, a, b


def same(x, y, what):
    sx, dx, nx = x
    sy, dy, ny = y
    assert np.array_equal(nx, ny), what
    for i in range(len(nx)):
        m = int(nx[i])
        assert np.array_equal(dx[i, :m], dy[i, :m]), (what, i)
        assert np.array_equal(sx[i, :m].view(np.uint32), sy[i, :m].view(np.uint32)), (what, i)


@pytest.mark.parametrize("with_deletes", [False, True])
def test_rescore_equals_build_with_global_stats(native, ctx, parts, with_deletes):
    from fugu_amd import synth
    c, cut, (ao, at), (bo, bt) = parts
    V = synth.VOCAB
    g = native.docs_stats(ao, at, V, threads=16) + native.docs_stats(bo, bt, V, threads=16)
    dl = None
    if with_deletes:
        dl = (np.arange(cut) % 7 == 3).astype(np.uint8)
    local = native.Index.from_docs(ctx, ao, at, V, threads=16, deleted=dl)
    fresh = native.Index.from_docs(ctx, ao, at, V, threads=16, deleted=dl, global_stats=g)
    re = local.rescore(g, deleted=dl)
    sl, sf, sr = local.stats(), fresh.stats(), re.stats()
    assert sr.avgdl == sf.avgdl and sr.avgdl != sl.avgdl
    for t in (0, 5, 99, 1000, 20000):
        assert re.bm25(t)[:2] == fresh.bm25(t)[:2]
    for (m0, m1, k, mode) in [(3, 3, 100, native.MODE_AND), (1, 5, 10, native.MODE_AND),
                              (2, 5, 1000, native.MODE_OR), (2, 3, 1, native.MODE_OR)]:
        q_off, terms = synth.queries(256, m0, m1, seed_q=77)
        same(re.search_batch(q_off, terms, k, mode=mode), fresh.search_batch(q_off, terms, k, mode=mode),
             (m0, m1, k, mode))


def test_rescore_twice_and_segment_merge_equals_single_index(native, ctx, parts):
    """Commit 1 builds segment A with A's statistics; commit 2 adds segment B and
    rescores A with the statistics of A + B; the two segments merged on the
    device give the single index's results (OR exactly, 2-term AND exactly)."""
    import torch

    from fugu_amd import synth
    from fugu_amd.shard import merge_on_device
    c, cut, (ao, at), (bo, bt) = parts
    V = synth.VOCAB
    seg_a = native.Index.from_docs(ctx, ao, at, V, threads=16)
    g = native.docs_stats(ao, at, V, threads=16) + native.docs_stats(bo, bt, V, threads=16)
    seg_a2 = seg_a.rescore(g)
    seg_a3 = seg_a2.rescore(g)  # a rescored snapshot rescored again keeps the shared structure
    seg_b = native.Index.from_docs(ctx, bo, bt, V, threads=16, global_stats=g)
    single = native.Index.from_docs(ctx, c.off, c.tok, V, threads=16)
    seg_a.close()
    seg_a2.close()
    dev = torch.device("cuda:0")
    for (m0, m1, k, mode) in [(2, 5, 1000, native.MODE_OR), (2, 2, 100, native.MODE_AND)]:
        q_off, terms = synth.queries(256, m0, m1, seed_q=91)
        nq = len(q_off) - 1
        res = [seg_a3.search_batch(q_off, terms, k, mode=mode), seg_b.search_batch(q_off, terms, k, mode=mode)]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32) if a.dtype == np.uint32  # noqa: E731
                                       else np.ascontiguousarray(a)).to(dev)
        ms, md, msh, mn = merge_on_device(t(np.stack([r[0] for r in res]).reshape(2, -1)),
                                          t(np.stack([r[1] for r in res]).reshape(2, -1)),
                                          t(np.stack([r[2] for r in res])), nq, k)
        torch.cuda.synchronize()
        md = md.cpu().numpy().view(np.uint32).reshape(nq, k)
        msh = msh.cpu().numpy().reshape(nq, k)
        s1, d1, n1 = single.search_batch(q_off, terms, k, mode=mode)
        assert np.array_equal(mn.cpu().numpy(), n1)
        ms = ms.cpu().numpy().reshape(nq, k)
        for i in range(nq):
            m = int(n1[i])  # entries past the hit count are not written
            gdoc = md[i, :m] + np.array([0, cut], np.uint32)[msh[i, :m]]
            assert np.array_equal(gdoc, d1[i, :m]), (mode, i)
            assert np.array_equal(ms[i, :m], s1[i, :m]), (mode, i)


def test_rescore_many_equals_one_by_one(native, ctx, parts):
    """fg_index_rescore_many (a commit's older segments rescored side by side,
    the weights once) gives every snapshot exactly what fg_index_rescore gives it,
    with and without deletes."""
    from fugu_amd import synth
    c, cut, (ao, at), (bo, bt) = parts
    V = synth.VOCAB
    g = native.docs_stats(ao, at, V, threads=16) + native.docs_stats(bo, bt, V, threads=16)
    seg_a = native.Index.from_docs(ctx, ao, at, V, threads=16)
    seg_b = native.Index.from_docs(ctx, bo, bt, V, threads=16)
    da = (np.arange(cut) % 5 == 1).astype(np.uint8)
    many = native.Index.rescore_many([seg_a, seg_b], g, deleted=[da, None])
    one = [seg_a.rescore(g, deleted=da), seg_b.rescore(g)]
    for (m0, m1, k, mode) in [(3, 3, 100, native.MODE_AND), (2, 5, 1000, native.MODE_OR)]:
        q_off, terms = synth.queries(256, m0, m1, seed_q=123)
        for x, y in zip(many, one):
            same(x.search_batch(q_off, terms, k, mode=mode), y.search_batch(q_off, terms, k, mode=mode), (m0, k, mode))


def test_rescore_shares_structure_and_leaves_base_intact(native, ctx, parts):
    """A rescore shares its base's device arrays (structure and build-time
    bounds: query-time scoring leaves nothing to recompute) and host structure:
    the base answers as before while and after rescores come and go, and every
    rescore answers like a fresh build under the same statistics."""
    import os

    from fugu_amd import synth
    c, cut, (ao, at), (bo, bt) = parts
    V = synth.VOCAB
    g = native.docs_stats(ao, at, V, threads=16) + native.docs_stats(bo, bt, V, threads=16)
    env = {"FUGU_RANK_GIB": "0.02"}  # the directory for the dense terms past the rank budget
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        base = native.Index.from_docs(ctx, ao, at, V, threads=16)
        fresh = native.Index.from_docs(ctx, ao, at, V, threads=16, global_stats=g)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    cases = [(3, 3, 100, native.MODE_AND), (2, 5, 1000, native.MODE_OR)]
    qs = [synth.queries(256, m0, m1, seed_q=31) for (m0, m1, _, _) in cases]
    before = [base.search_batch(q_off, terms, k, mode=mode) for (q_off, terms), (_, _, k, mode) in zip(qs, cases)]
    kth = np.stack([base.term_kth(t) for t in (0, 7, 300)])
    first = None
    for rnd in range(3):
        re = base.rescore(g)
        assert re.stats().device_bytes == base.stats().device_bytes  # the same arrays
        got = [re.search_batch(q_off, terms, k, mode=mode) for (q_off, terms), (_, _, k, mode) in zip(qs, cases)]
        for x, (q_off, terms), (_, _, k, mode) in zip(got, qs, cases):
            same(x, fresh.search_batch(q_off, terms, k, mode=mode), ("rescore vs fresh", rnd, k, mode))
        if first is None:
            first = got
        for x, y in zip(got, first):
            same(x, y, ("rescore again", rnd))
        re.close()
        for x, y, cs in zip(before, [base.search_batch(q_off, terms, k, mode=mode)
                                     for (q_off, terms), (_, _, k, mode) in zip(qs, cases)], cases):
            same(x, y, ("base after rescore", rnd, cs))
        assert np.array_equal(np.stack([base.term_kth(t) for t in (0, 7, 300)]), kth)
    base.close()
    fresh.close()


def test_sharded_batch_in_halves_equals_quarters(native, ctx, parts):
    """fg_search_sharded plans a batch of >= 512 queries over several snapshots as
    two halves, the second planned while the first one's kernels run: the merged
    hits equal those of the same queries searched 256 at a time (one plan each)."""
    from fugu_amd import synth
    c, cut, (ao, at), (bo, bt) = parts
    V = synth.VOCAB
    g = native.docs_stats(ao, at, V, threads=16) + native.docs_stats(bo, bt, V, threads=16)
    segs = [native.Index.from_docs(ctx, ao, at, V, threads=16, global_stats=g),
            native.Index.from_docs(ctx, bo, bt, V, threads=16, global_stats=g)]
    for (m0, m1, k, mode) in [(2, 5, 1000, native.MODE_OR), (3, 3, 100, native.MODE_AND), (1, 4, 20, native.MODE_OR)]:
        q_off, terms = synth.queries(1024, m0, m1, seed_q=51)
        whole = native.search_sharded(segs, q_off, terms, k, mode=mode, ctx=ctx)
        for b in range(0, 1024, 256):
            qo = (q_off[b:b + 257] - q_off[b]).astype(q_off.dtype)
            part = native.search_sharded(segs, qo, terms[q_off[b]:q_off[b + 256]], k, mode=mode, ctx=ctx)
            assert np.array_equal(part[3], whole[3][b:b + 256]), (k, mode, b)
            for i in range(256):
                m = int(part[3][i])
                for a in range(3):
                    assert np.array_equal(part[a][i, :m], whole[a][b + i, :m]), (k, mode, b + i, a)
    for x in segs:
        x.close()
