"""BASELINE.json configs C3 and C4 at full size on one MI355X, vs the oracle.

C3  10M-doc Zipf corpus, mixed 1-5-term AND, batch 1024, top-100 (the HBM-
    roofline run): every query of the batch against the oracle.
C4  the same 10M docs as 8 namespaces x 1.25M, each its own index with its own
    BM25 statistics (one fugu namespace = one tantivy index, reference
    src/db/core.rs:49-79); a fan-out 3-term AND top-100 runs on every namespace
    and the per-namespace top-100 lists are merged on the device
    (fg_merge_shards) by (score desc, namespace asc, doc asc) -- the 8-GPU
    RCCL gather's merge, with the namespaces resident on one GPU here.  Checked
    against the per-namespace oracle results merged in numpy.
Bar: doc ids and order identical, scores within 1e-5 relative.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-5
N_DOCS = 10_000_000


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
def corpus_10m():
    from fugu_amd import synth
    return synth.corpus(N_DOCS, threads=16)


def check(s, d, n, rs, rd, rn, what):
    assert np.array_equal(n, rn), what
    for i in range(len(n)):
        m = int(n[i])
        assert np.array_equal(d[i, :m], rd[i, :m]), (what, i)
        rel = np.abs(s[i, :m].astype(np.float64) - rs[i, :m]) / np.maximum(np.abs(rs[i, :m]), 1e-30)
        assert (rel <= RTOL).all(), (what, i, rel.max())


def test_c3_mixed_and_10m_batch1024(native, ctx, corpus_10m):
    from fugu_amd import synth
    from oracle import oracle as orc
    c = corpus_10m
    ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=16, keep_host=False)
    q_off, terms = synth.queries(1024, 1, 5)
    p = ix.plan(q_off, terms, 100)
    p.execute()
    s, d, n = p.results()
    del p
    ix.close()
    ref = orc.OracleIndex(synth.VOCAB, c.off, c.tok, threads=16)
    rs, rd, rn, _, _ = ref.search_batch(q_off, terms, 100, threads=16)
    check(s, d, n, rs, rd, rn, "C3")
    assert (n == 100).mean() > 0.3  # most queries fill their top-100


def test_c4_8_namespaces_fanout_merge(native, ctx, corpus_10m):
    import torch

    from fugu_amd import synth
    from fugu_amd.shard import shard_ranges
    from oracle import oracle as orc
    from shard_ref import merge_topk_numpy
    c = corpus_10m
    k, nq = 100, 1024
    q_off, terms = synth.queries(nq, 3, 3)
    ranges = shard_ranges(N_DOCS, 8)
    dev = torch.device("cuda:0")
    gs = torch.empty((8, nq * k), dtype=torch.float32, device=dev)
    gd = torch.empty((8, nq * k), dtype=torch.int32, device=dev)
    gn = torch.empty((8, nq), dtype=torch.int32, device=dev)
    ref_s = np.zeros((8, nq, k), np.float32)
    ref_d = np.zeros((8, nq, k), np.uint32)
    ref_n = np.zeros((8, nq), np.uint32)
    st = torch.cuda.current_stream(dev).cuda_stream
    for r, (b, e) in enumerate(ranges):
        off = c.off[b:e + 1] - c.off[b]
        tok = c.tok[c.off[b]:c.off[e]]
        # namespace r: its own index and its own statistics (doc ids local to the namespace)
        ix = native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=16, keep_host=False)
        p = ix.plan(q_off, terms, k)
        p.execute(st, gs[r].data_ptr(), gd[r].data_ptr(), gn[r].data_ptr())
        torch.cuda.synchronize()
        del p
        ix.close()
        ref = orc.OracleIndex(synth.VOCAB, off, tok, threads=16)
        rs, rd, rn, _, _ = ref.search_batch(q_off, terms, k, threads=16)
        ref_s[r], ref_d[r], ref_n[r] = rs, rd, rn
        del ref
    # the per-namespace device results equal the per-namespace oracle results ...
    hs = gs.cpu().numpy().reshape(8, nq, k)
    hd = gd.cpu().numpy().view(np.uint32).reshape(8, nq, k)
    hn = gn.cpu().numpy().view(np.uint32)
    for r in range(8):
        check(hs[r], hd[r], hn[r], ref_s[r], ref_d[r], ref_n[r], f"C4 namespace {r}")
    # ... and the device merge equals the numpy merge of the oracle lists
    from fugu_amd.shard import merge_on_device
    ms, md, msh, mn = merge_on_device(gs, gd, gn, nq, k, st)
    torch.cuda.synchronize()
    es, ed, esh, en = merge_topk_numpy(ref_s, ref_d, ref_n, k)
    assert np.array_equal(mn.cpu().numpy(), en)
    ms, md, msh = (x.cpu().numpy().reshape(nq, k) for x in (ms, md, msh))
    for q in range(nq):
        m = int(en[q])
        assert np.array_equal(md[q, :m].view(np.uint32), ed[q, :m]), q
        assert np.array_equal(msh[q, :m], esh[q, :m]), q
        assert np.array_equal(ms[q, :m], es[q, :m]), q
    assert (en == k).mean() > 0.5
