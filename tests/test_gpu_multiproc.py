"""The N > 1 fan-out path with libfugu on the device: two
processes, one namespace each (own corpus, own statistics), every rank runs its
batch through libfugu into device buffers, the per-namespace top-k lists go
through fugu_amd.shard.gather_packed (the collective bench.py uses; a gloo group
here because both ranks share the box's one GPU -- the driver's 8-GPU runs use
RCCL) and rank 0 merges them on the device with fg_merge_shards.

Checked: every rank's own hits against the CPU oracle of its namespace, and the
merged fan-out result against the oracles of both namespaces merged by (score
desc, namespace asc, doc asc).
"""
import os
import queue
import socket

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N_DOCS, NQ, K = 200_000, 256, 100


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpus(rank):
    from fugu_amd import synth
    return synth.corpus(N_DOCS, synth.VOCAB, 1.0, synth.SEED_L + rank, synth.SEED_T + rank)


def _oracle_hits(c, q_off, terms):
    from fugu_amd import synth
    from oracle import oracle as orc
    ref = orc.OracleIndex(synth.VOCAB, c.off, c.tok, threads=8)
    s, d, n, _, _ = ref.search_batch(q_off, terms, K, threads=8)
    return s, d, n


def _worker(rank, world, port, outq):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from fugu_amd import native, synth
        from fugu_amd.shard import gather_packed, merge_on_device
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        c = _corpus(rank)
        ctx = native.Context((0,))
        ix = native.Index.from_docs(ctx, c.off, c.tok, synth.VOCAB, threads=8, keep_host=False)
        q_off, terms = synth.queries(NQ, 3, 3, seed_q=11)
        plan = ix.plan(q_off, terms, K)
        os_ = torch.empty(NQ * K, dtype=torch.float32, device=dev)
        od = torch.empty(NQ * K, dtype=torch.int32, device=dev)
        on = torch.empty(NQ, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev)
        plan.execute(st.cuda_stream, os_.data_ptr(), od.data_ptr(), on.data_ptr())
        gs, gd, gn = gather_packed(os_, od, on)
        ms, md, msh, mn = merge_on_device(gs, gd, gn, NQ, K, st.cuda_stream)
        torch.cuda.synchronize()
        # this rank's own hits vs its namespace's oracle
        rs, rd, rn = _oracle_hits(c, q_off, terms)
        n = on.cpu().numpy()
        s = os_.cpu().numpy().reshape(NQ, K)
        d = od.cpu().numpy().view(np.uint32).reshape(NQ, K)
        assert np.array_equal(n, rn.astype(n.dtype)), f"rank {rank}: hit counts"
        for i in range(NQ):
            m = int(n[i])
            assert np.array_equal(d[i, :m], rd[i, :m]), f"rank {rank} query {i}: doc ids"
            assert np.allclose(s[i, :m], rs[i, :m], rtol=1e-5, atol=0), f"rank {rank} query {i}: scores"
        if rank == 0:
            outq.put(("merged", ms.cpu().numpy(), md.cpu().numpy().view(np.uint32), msh.cpu().numpy(),
                      mn.cpu().numpy(), q_off, terms))
        dist.barrier()
        dist.destroy_process_group()
        del plan, ix
    except Exception as e:  # noqa: BLE001
        outq.put(("error", rank, repr(e)))
        raise


def test_two_process_fanout_through_libfugu():
    import torch.multiprocessing as mp
    world = 2
    mpc = mp.get_context("spawn")
    outq = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(r, world, port, outq)) for r in range(world)]
    for p in procs:
        p.start()
    got = None
    for _ in range(240):
        try:
            got = outq.get(timeout=1)
            break
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=120)
        if p.is_alive():
            p.kill()
            p.join(timeout=10)
    assert got is not None, "no result from the ranks"
    assert got[0] == "merged", got
    for p in procs:
        assert p.exitcode == 0, "a rank failed"
    _, ms, md, msh, mn, q_off, terms = got
    from shard_ref import merge_topk_numpy
    per = [_oracle_hits(_corpus(r), q_off, terms) for r in range(world)]
    es, ed, esh, en = merge_topk_numpy(np.stack([p[0] for p in per]), np.stack([p[1] for p in per]),
                                       np.stack([p[2] for p in per]), K)
    assert np.array_equal(mn, en)
    ms, md, msh = ms.reshape(NQ, K), md.reshape(NQ, K), msh.reshape(NQ, K)
    for i in range(NQ):
        m = int(mn[i])
        assert np.array_equal(md[i, :m], ed[i, :m]) and np.array_equal(msh[i, :m], esh[i, :m]), i
        assert np.allclose(ms[i, :m], es[i, :m], rtol=1e-5, atol=0), i
    assert (mn > 0).mean() > 0.5
