"""Peer plans (fg_plan_set_peers / fg_plan_set_ipc_peers): the doc shards of one
namespace, each with its own per-query threshold and histogram, publishing
their thresholds and hit counts into each other DURING the launch -- what the
shards of C5 on 8 GPUs do over xGMI (BASELINE configs[4]; tantivy's
Searcher-global statistics, reference src/db/search.rs:162).

Checked: shards run concurrently on their own streams with peers set give,
merged, the hits of the oracle's segmented search, round after round (reset
between rounds); and the same through HIP IPC with the shards' plans in two
processes on one device (what the ranks of a multi-GPU job do).
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_DOCS, SHARDS, NQ, K = 2_000_000, 4, 256, 100


@pytest.fixture(scope="module")
def native():
    from fugu_amd import native as nat
    if nat.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    return nat


@pytest.fixture(scope="module")
def setup(native):
    from fugu_amd import synth
    from fugu_amd.shard import shard_ranges
    from oracle import oracle as orc
    ctx = native.Context((0,))
    c = synth.corpus(N_DOCS, synth.VOCAB, 1.1, threads=16)
    ranges = shard_ranges(N_DOCS, SHARDS)
    parts = [(c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]]) for b, e in ranges]
    g = None
    for off, tok in parts:
        x = native.docs_stats(off, tok, synth.VOCAB, threads=16)
        g = x if g is None else g + x
    ixs = [native.Index.from_docs(ctx, off, tok, synth.VOCAB, threads=16, global_stats=g) for off, tok in parts]
    ref = orc.OracleIndex(synth.VOCAB, c.off, c.tok, threads=16)
    yield ctx, c, ranges, ixs, ref
    for ix in ixs:
        ix.close()
    ref.close()


def _check_vs_oracle(native, plans, ranges, c, ref, q_off, terms, k, mode, what):
    from shard_ref import merge_topk_numpy
    per = [p.results() for p in plans]
    ms, md, msh, mn = merge_topk_numpy(np.stack([x[0] for x in per]), np.stack([x[1] for x in per]),
                                       np.stack([x[2] for x in per]).astype(np.int64), k)
    base = np.array([b for b, _ in ranges], np.uint64)
    bounds = np.array([b for b, _ in ranges] + [c.n_docs], np.uint32)
    for i in range(len(q_off) - 1):
        rs, rd = ref.search_segments(terms[q_off[i]:q_off[i + 1]], k, bounds, mode=mode)
        m = int(mn[i])
        assert m == len(rd), (what, i)
        assert np.array_equal(md[i, :m].astype(np.uint64) + base[msh[i, :m]], rd.astype(np.uint64)), (what, i)
        assert np.allclose(ms[i, :m], rs, rtol=1e-5, atol=0), (what, i)


@pytest.mark.parametrize("m0,m1,k,mode", [(2, 5, 100, 1), (2, 3, 20, 1), (3, 3, 100, 0)])
def test_peers_concurrent_shards_equal_oracle(native, setup, m0, m1, k, mode):
    import torch

    from fugu_amd import synth
    from fugu_amd.shard import agree_hist_span
    ctx, c, ranges, ixs, ref = setup
    q_off, terms = synth.queries(NQ, m0, m1, seed_q=29)
    plans = [ix.plan(q_off, terms, k, mode) for ix in ixs]
    agree_hist_span(plans)
    for i, p in enumerate(plans):
        p.set_peers([x for j, x in enumerate(plans) if j != i])
    streams = [torch.cuda.Stream() for _ in plans]
    for rnd in range(2):
        for p in plans:
            p.reset(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()  # every reset before any peer's execute
        for p, s in zip(plans, streams):
            p.execute(s.cuda_stream)
        torch.cuda.synchronize()
        _check_vs_oracle(native, plans, ranges, c, ref, q_off, terms, k, mode, ("peers", rnd, k, mode))
    for p in plans:
        p.set_peers([])
    for p in plans:
        p.close()


def _ipc_child(conn, shard, m0, m1, k, mode):
    """A second process: its own context, its shard's index and plan, peers
    through the parent's exported words."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from fugu_amd import native, synth
    from fugu_amd.shard import shard_ranges
    ctx = native.Context((0,))
    c = synth.corpus(N_DOCS, synth.VOCAB, 1.1, threads=8)
    ranges = shard_ranges(N_DOCS, SHARDS)
    b, e = ranges[shard]
    g = None
    for bb, ee in ranges:
        x = native.docs_stats(c.off[bb:ee + 1] - c.off[bb], c.tok[c.off[bb]:c.off[ee]], synth.VOCAB, threads=8)
        g = x if g is None else g + x
    ix = native.Index.from_docs(ctx, c.off[b:e + 1] - c.off[b], c.tok[c.off[b]:c.off[e]], synth.VOCAB, threads=8,
                                global_stats=g)
    q_off, terms = synth.queries(NQ, m0, m1, seed_q=29)
    p = ix.plan(q_off, terms, k, mode)
    lo, hi = p.hist_span()
    conn.send((lo, hi))
    lo, hi = conn.recv()
    p.set_hist_span(lo, hi)
    conn.send(p.ipc_export())
    p.set_ipc_peers(conn.recv())
    p.reset()
    native_sync()
    conn.send("reset")
    assert conn.recv() == "go"
    p.execute()
    s, d, n = p.results()
    conn.send((s, d, n))
    assert conn.recv() == "done"  # the parent no longer publishes into us
    p.close()
    ix.close()


def native_sync():
    import torch
    torch.cuda.synchronize()


def test_ipc_peers_two_processes(native, setup):
    """Shard 0 in this process, shard 1 in a child process on the same device:
    peers through fg_plan_ipc_export / fg_plan_set_ipc_peers; the two shards'
    merged hits equal the oracle's over those two shards."""
    import torch

    from fugu_amd import synth
    from shard_ref import merge_topk_numpy
    ctx, c, ranges, ixs, ref = setup
    m0, m1, k, mode = 2, 5, 100, 1
    q_off, terms = synth.queries(NQ, m0, m1, seed_q=29)
    p = ixs[0].plan(q_off, terms, k, mode)
    ctxm = mp.get_context("spawn")
    a, b = ctxm.Pipe()
    child = ctxm.Process(target=_ipc_child, args=(b, 1, m0, m1, k, mode))
    child.start()
    try:
        lo0, hi0 = p.hist_span()
        lo1, hi1 = a.recv()
        lo, hi = np.maximum(lo0, lo1), np.maximum(hi0, hi1)
        a.send((lo, hi))
        p.set_hist_span(lo, hi)
        theirs = a.recv()
        a.send([p.ipc_export()])
        p.set_ipc_peers([theirs])
        p.reset()
        torch.cuda.synchronize()
        assert a.recv() == "reset"
        a.send("go")
        p.execute()
        s0, d0, n0 = p.results()
        s1, d1, n1 = a.recv()
        a.send("done")
        child.join(120)
        assert child.exitcode == 0
    finally:
        if child.is_alive():
            child.kill()
    p.set_ipc_peers([])
    p.close()
    ms, md, msh, mn = merge_topk_numpy(np.stack([s0, s1]), np.stack([d0, d1]), np.stack([n0, n1]).astype(np.int64), k)
    base = np.array([ranges[0][0], ranges[1][0]], np.uint64)
    for i in range(NQ):
        # the oracle over shards 0-1 with the namespace's statistics: the full
        # oracle's segmented search restricted to docs < ranges[1][1]
        rs, rd = ref.search_segments(terms[q_off[i]:q_off[i + 1]], 10 * k, np.array(
            [b for b, _ in ranges] + [c.n_docs], np.uint32), mode=mode)
        keep = rd < ranges[1][1]
        rs, rd = rs[keep][:k], rd[keep][:k]
        m = int(mn[i])
        assert m == len(rd), i
        assert np.array_equal(md[i, :m].astype(np.uint64) + base[msh[i, :m]], rd.astype(np.uint64)), i
