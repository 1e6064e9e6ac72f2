"""Namespace-wide starting thresholds of a doc-sharded namespace (CPU).

fg_kth_floor_combine turns the shards' score ladders (each shard's K-th best
alive score per term at the ranks FG_LADDER_KS) into lower bounds of the
namespace-wide K-th scores (K = 1, 10, 20, 100, 1000).  Checked here against a
brute-force restatement of its rule and against the exact K-th scores of the
concatenated score lists they summarise; the all-gather that carries the
ladders between ranks (fugu_amd.shard.exchange_ladders) with a world-2 gloo
group.  The device ladders themselves are checked in tests/test_gpu_floor.py.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

native = pytest.importorskip("fugu_amd.native")
LK = np.array(native.LADDER_KS)
KK = np.array(native.KTH_KS)


def ladder_of(scores):
    """A shard's ladder of one term from its alive posting scores (fg_index_term_ladder's definition)."""
    s = np.sort(np.asarray(scores, np.float32))[::-1]
    return np.array([s[k - 1] if k <= len(s) else 0.0 for k in LK], np.float32)


def brute_floor(lads):
    """Largest x with sum over shards of max{K_l : ladder_s(K_l) >= x} >= K (0 if none)."""
    cands = sorted({float(v) for lad in lads for v in lad if v > 0}, reverse=True)
    out = np.zeros(len(KK), np.float32)
    for j, K in enumerate(KK):
        for x in cands:
            tot = 0
            for lad in lads:
                ok = [int(k) for k, v in zip(LK, lad) if v >= x and v > 0]
                tot += max(ok) if ok else 0
            if tot >= K:
                out[j] = x
                break
    return out


def test_combine_matches_brute_force_and_bounds_the_exact_kth():
    rng = np.random.default_rng(5)
    S, V = 4, 40
    lists = [[rng.gamma(2.0, 1.0, size=int(rng.integers(0, 1500))).astype(np.float32) for _ in range(V)]
             for _ in range(S)]
    # a few terms with exact ties across shards
    for s in range(S):
        lists[s][0] = np.full(300, 2.5, np.float32)
    lads = [np.stack([ladder_of(lists[s][t]) for t in range(V)]) for s in range(S)]
    floor = native.kth_floor_combine(lads)
    assert floor.shape == (V, len(KK))
    for t in range(V):
        exp = brute_floor([lads[s][t] for s in range(S)])
        assert np.array_equal(floor[t], exp), (t, floor[t], exp)
        allv = np.sort(np.concatenate([lists[s][t] for s in range(S)]))[::-1]
        for j, K in enumerate(KK):
            exact = allv[K - 1] if K <= len(allv) else 0.0
            assert floor[t, j] <= exact  # a valid lower bound of the namespace-wide K-th score
            if K <= len(allv):
                assert floor[t, j] > 0 or K > 1  # K = 1: the largest shard maximum is exact
        assert floor[t, 0] == (allv[0] if len(allv) else 0.0)
    # tie term: 1200 docs at 2.5 -> every K <= 1000 is 2.5 exactly
    assert np.all(floor[0] == np.float32(2.5))


def test_combine_one_shard_is_its_own_ladder():
    rng = np.random.default_rng(1)
    lists = [rng.random(int(n)).astype(np.float32) + 0.1 for n in (0, 1, 9, 10, 999, 1000, 4000)]
    lad = np.stack([ladder_of(x) for x in lists])
    floor = native.kth_floor_combine([lad])
    main = [list(LK).index(k) for k in KK]
    assert np.array_equal(floor, lad[:, main])


def test_combine_tightens_large_k_over_shards():
    """K = 1000 over 8 equal shards: each shard's 125th (the ladder has it) instead of its 1000th."""
    rng = np.random.default_rng(2)
    allv = rng.random(80000).astype(np.float32)
    parts = np.array_split(rng.permutation(allv), 8)
    lads = [ladder_of(p)[None, :] for p in parts]
    floor = native.kth_floor_combine(lads)[0]
    exact = np.sort(allv)[::-1][999]
    own = max(lad[0, list(LK).index(1000)] for lad in lads)
    assert own < floor[4] <= exact
    assert floor[4] >= min(lad[0, list(LK).index(125)] for lad in lads)


def test_combine_rejects_bad_shapes():
    with pytest.raises(ValueError):
        native.kth_floor_combine([np.zeros((4, 5), np.float32)])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _exchange_worker(rank, world, port, outq):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fugu_amd import native as nat
    from fugu_amd.shard import exchange_ladders
    rng = np.random.default_rng(100 + rank)
    local = np.sort(rng.random((2, 64, len(nat.LADDER_KS))).astype(np.float32), axis=2)[:, :, ::-1]
    got = exchange_ladders(local)
    floor = nat.kth_floor_combine(list(got))
    outq.put((rank, got, floor))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_ladder_exchange():
    world = 2
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, outq)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    res = {}
    for _ in range(240):
        try:
            r, got, floor = outq.get(timeout=1)
            res[r] = (got, floor)
            if len(res) == world:
                break
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, "a rank failed"
    assert len(res) == world
    exp = np.concatenate([np.sort(np.random.default_rng(100 + r).random((2, 64, len(LK))).astype(np.float32),
                                  axis=2)[:, :, ::-1] for r in range(world)])
    for r in range(world):
        assert np.array_equal(res[r][0], exp)  # every rank holds every shard's ladder, in rank order
        assert np.array_equal(res[r][1], res[0][1])  # and computes the same floor
