"""N > 1 path on CPU: world_size-2 (and 4) gloo groups, one namespace per rank.

Each rank searches its own namespace (the CPU oracle stands in for the
device, whose per-shard results are checked against the same oracle by the
gpu tests), the per-shard top-k lists go through fugu_amd.shard.gather_packed
(the exact collective bench.py uses), and the merged fan-out result must equal
searching every namespace and merging by (score desc, shard asc, doc asc).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_results(rank, n_docs, q_off, terms, k):
    import sys
    sys.path.insert(0, ROOT)
    from fugu_amd import synth
    from oracle import oracle as orc
    c = synth.corpus(n_docs, 1 << 16, 1.0, synth.SEED_L + rank, synth.SEED_T + rank)
    ix = orc.OracleIndex(1 << 16, c.off, c.tok)
    s, d, n, _, _ = ix.search_batch(q_off, terms, k)
    return s, d, n


def _worker(rank, world, port, n_docs, k, outq):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fugu_amd.shard import gather_packed
    from fugu_amd import synth
    q_off, terms = synth.queries(64, 1, 3, max_rank=1 << 9)
    s, d, n = _shard_results(rank, n_docs, q_off, terms, k)
    gs, gd, gn = gather_packed(torch.from_numpy(s.reshape(-1)), torch.from_numpy(d.reshape(-1).view(np.int32)),
                               torch.from_numpy(n.view(np.int32)))
    if rank == 0:
        outq.put((gs.numpy(), gd.numpy().view(np.uint32), gn.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_two_rank_fanout_matches_direct_merge(world):
    n_docs, k = 3000, 10
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_docs, k, outq)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = None
    for _ in range(240):
        try:
            got = outq.get(timeout=1)
            break
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, "a rank failed"
    assert got is not None, "rank 0 produced no result"
    gs, gd, gn = got
    from fugu_amd import synth
    from shard_ref import merge_topk_numpy
    q_off, terms = synth.queries(64, 1, 3, max_rank=1 << 9)
    nq = len(q_off) - 1
    per = [_shard_results(r, n_docs, q_off, terms, k) for r in range(world)]
    # the gathered buffers are exactly the per-shard results
    for r in range(world):
        assert np.array_equal(gn[r], per[r][2])
        assert np.array_equal(gd[r].reshape(nq, k), per[r][1])
        assert np.array_equal(gs[r].reshape(nq, k), per[r][0])
    sc = np.stack([gs[r].reshape(nq, k) for r in range(world)])
    dc = np.stack([gd[r].reshape(nq, k) for r in range(world)])
    ms, md, msh, mn = merge_topk_numpy(sc, dc, gn.astype(np.int64), k)
    for q in range(nq):
        rows = sorted([(float(per[r][0][q, i]), r, int(per[r][1][q, i]))
                       for r in range(world) for i in range(int(per[r][2][q]))], key=lambda x: (-x[0], x[1], x[2]))[:k]
        assert mn[q] == len(rows)
        assert [(int(msh[q, i]), int(md[q, i])) for i in range(mn[q])] == [(r[1], r[2]) for r in rows]


def _stats_worker(rank, world, port, outq):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fugu_amd import native, synth
    from fugu_amd.shard import allreduce_stats, shard_ranges
    c = synth.corpus(6000, 1 << 16)
    b, e = shard_ranges(6000, world)[rank]
    off = c.off[b:e + 1] - c.off[b]
    tok = c.tok[c.off[b]:c.off[e]]
    import synth_ref as sr
    fo, ft, nf = sr.facet_tokens(6000, 31)
    facets = (fo[b:e + 1] - fo[b], ft[fo[b]:fo[e]], nf)
    g = allreduce_stats(native.docs_stats(off, tok, 1 << 16, facets=facets))
    if rank == 0:
        outq.put((g.n_docs, g.tot_tokens, g.df_text, g.df_name, g.df_facet, g.tot_facet_tokens))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_two_rank_global_stats_allreduce(world):
    """Doc-sharded namespace: the summed shard statistics equal the whole corpus's."""
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, world, port, outq)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = None
    for _ in range(240):
        try:
            got = outq.get(timeout=1)
            break
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, "a rank failed"
    assert got is not None
    n, tot, dft, dfn, dff, totf = got
    from fugu_amd import native, synth
    import synth_ref as sr
    c = synth.corpus(6000, 1 << 16)
    full = native.docs_stats(c.off, c.tok, 1 << 16, facets=sr.facet_tokens(6000, 31))
    assert n == full.n_docs and tot == full.tot_tokens
    assert np.array_equal(dft, full.df_text) and np.array_equal(dfn, full.df_name)
    assert np.array_equal(dff, full.df_facet) and totf == full.tot_facet_tokens > 0


# ---- doc shards across ranks: histogram bins agreed, then summed mid-sweep ----
def _bin_shift(lo, hi, bins=512):
    sh = 0
    while sh < 31 and ((hi - lo) >> sh) >= bins - 1:
        sh += 1
    return sh


def _hist_threshold(h, K, lo, sh):
    """kernels.hip hist_threshold restated: the lower edge (f32 bits) of the highest
    bin with >= K counted docs at or above it, or 0."""
    c = 0
    for b in range(len(h) - 1, -1, -1):
        c += int(h[b])
        if c >= K:
            return lo + (b << sh)
    return 0


class _FakePlan:
    """The plan methods shard.agree_hist_span / exchange_hist call, over host
    memory (hist_copy's 'device' buffer is a CPU tensor here)."""

    def __init__(self, lo, hi, hist):
        self.n_batch = len(lo)
        self.lo, self.hi, self.hist = lo.astype(np.uint32), hi.astype(np.uint32), hist.astype(np.int32)

    def hist_span(self):
        return self.lo.copy(), self.hi.copy()

    def set_hist_span(self, lo, hi):
        self.lo, self.hi = np.asarray(lo, np.uint32), np.asarray(hi, np.uint32)

    def hist_copy(self, stream, ptr, into_plan):
        import ctypes
        src, dst = (ptr, self.hist.ctypes.data) if into_plan else (self.hist.ctypes.data, ptr)
        ctypes.memmove(dst, src, self.hist.nbytes)


def _scores(rank, nq):
    rng = np.random.default_rng(100 + rank)
    return [rng.gamma(2.0, 3.0, size=int(rng.integers(0, 400))).astype(np.float32) for _ in range(nq)]


def _hist_worker(rank, world, port, outq):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fugu_amd.shard import agree_hist_span, exchange_hist
    nq, K = 48, 50
    sc = _scores(rank, nq)
    # this rank's own spans (query 5: no work on rank 0)
    lo = np.array([max(1, int(np.float32(x.max() / 256 if len(x) else 0).view(np.uint32))) for x in sc], np.uint32)
    hi = np.array([int(np.float32(x.max() if len(x) else 0).view(np.uint32)) for x in sc], np.uint32)
    if rank == 0:
        lo[5] = hi[5] = 0
    p = _FakePlan(lo, hi, np.zeros(nq * 512, np.int32))
    alo, ahi = agree_hist_span([p])
    # count this rank's scores into the agreed bins (kernels.hip qbin)
    hist = np.zeros((nq, 512), np.int32)
    for q in range(nq):
        sh = _bin_shift(int(alo[q]), int(max(ahi[q], alo[q])))
        for v in sc[q].view(np.uint32):
            if v >= alo[q]:
                hist[q, min((int(v) - int(alo[q])) >> sh, 511)] += 1
    p.hist = hist.reshape(-1).copy()
    buf = torch.zeros(nq * 512, dtype=torch.int32)
    merged = exchange_hist(p, 0, buf)
    thr = [_hist_threshold(p.hist.reshape(nq, 512)[q], K, int(alo[q]), _bin_shift(int(alo[q]), int(max(ahi[q], alo[q]))))
           for q in range(nq)]
    after1 = p.hist.reshape(nq, 512).copy()
    # a third part of the sweep: this rank counts more docs into the merged
    # histogram, and the second exchange sums only what is new (prev)
    more = np.zeros((nq, 512), np.int32)
    rng = np.random.default_rng(200 + rank)
    for q in range(nq):
        more[q, rng.integers(0, 512, int(rng.integers(0, 30)))] += 1
    p.hist = (after1 + more).reshape(-1).copy()
    exchange_hist(p, 0, buf, prev=merged)
    outq.put((rank, alo, ahi, hist, after1, thr, more, p.hist.reshape(nq, 512).copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_hist_exchange():
    """C5 over N ranks (bench.py's step, shard.agree_hist_span / exchange_hist):
    every rank gets the elementwise max of the ranks' bin spans (a rank without
    work for a query does not count), the exchanged histogram is the bin-wise sum,
    and its threshold never exceeds the K-th best score of the union of the
    ranks' counted docs -- so pruning with it keeps the merged top-K."""
    world = 2
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hist_worker, args=(r, world, port, outq)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = {}
    for _ in range(240):
        try:
            r, *rest = outq.get(timeout=1)
            got[r] = rest
            if len(got) == world:
                break
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, "a rank failed"
    assert len(got) == world
    nq, K = 48, 50
    sc = [_scores(r, nq) for r in range(world)]
    for r in range(world):
        alo, ahi, own, summed, thr, _, summed2 = got[r]
        assert np.array_equal(alo, got[0][0]) and np.array_equal(ahi, got[0][1])
        assert np.array_equal(summed, got[0][2] + got[1][2])
        # the second exchange: every rank's counts exactly once
        assert np.array_equal(summed2, got[0][2] + got[1][2] + got[0][5] + got[1][5])
        for q in range(nq):
            los = [max(1, int(np.float32(s[q].max() / 256 if len(s[q]) else 0).view(np.uint32))) for s in sc]
            his = [int(np.float32(s[q].max() if len(s[q]) else 0).view(np.uint32)) for s in sc]
            if q == 5:  # rank 0 reported no work: rank 1's span alone
                los[0] = his[0] = 0
            assert alo[q] == max(los) and ahi[q] == max(his)
            union = np.sort(np.concatenate([s[q] for s in sc]))[::-1]
            if len(union) >= K:
                assert thr[q] <= int(union[K - 1].view(np.uint32))
            else:
                assert thr[q] == 0 or int(summed[q].sum()) >= K
    assert sum(1 for q in range(nq) if got[0][4][q] > 0) > nq // 2  # the exchange gives most queries a threshold


class _FakePeerPlan:
    """Stands in for a native.Plan in the peer-linking exchange: ipc_export()
    returns this rank's 112-byte fg_plan_ipc words, set_ipc_peers() / reset()
    record what the exchange hands it (the device side runs in the gpu tests)."""

    def __init__(self, rank):
        self.blob = bytes([rank + 1]) * 112
        self.peers = None
        self.resets = 0

    def ipc_export(self):
        return self.blob

    def set_ipc_peers(self, blobs):
        self.peers = list(blobs)

    def reset(self, stream=None):
        self.resets += 1


def _peer_worker(rank, world, port, outq):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fugu_amd.shard as shard
    p = _FakePeerPlan(rank)
    n = shard.link_peers(p)
    torch.cuda.synchronize = lambda *a, **k: None  # (no device here: the barrier is what is checked)
    shard.reset_peers(p)
    outq.put((rank, n, p.peers, p.resets))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_link_peers_exchange(world):
    """shard.link_peers over a gloo group: every rank's plan gets the IPC words of
    every OTHER rank's plan, in rank order, through one all-gather; reset_peers
    resets the rank's own plan before its barrier (bench.py's C5 step over N GPUs)."""
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer_worker, args=(r, world, port, outq)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    import queue
    for _ in range(240):
        try:
            r, *rest = outq.get(timeout=1)
            got[r] = rest
            if len(got) == world:
                break
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, "a rank failed"
    for r in range(world):
        n, peers, resets = got[r]
        assert n == world - 1 and resets == 1
        assert peers == [bytes([q + 1]) * 112 for q in range(world) if q != r]
