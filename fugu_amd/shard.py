"""Namespace sharding across GPUs.

One process per GPU; rank r holds namespace r's snapshot.  A fan-out query
runs on every shard, the per-shard top-k lists are exchanged with ONE
all-gather per batch (RCCL over xGMI when the group is "nccl"), and the global
top-k is merged on the device by (score desc, shard asc, doc asc)
(fg_merge_shards).  Scores are not renormalised across namespaces: each
namespace keeps its own BM25 statistics, exactly as each fugu namespace is its
own tantivy index (src/db/core.rs:49-79).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def pack_topk(score: torch.Tensor, doc: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
    """One int32 buffer [nq*k*2 + nq] so a batch needs a single all-gather."""
    return torch.cat([score.reshape(-1).view(torch.int32), doc.reshape(-1).view(torch.int32),
                      n.reshape(-1).view(torch.int32)])


def unpack_topk(out: torch.Tensor, nk: int):
    s = out[:, :nk].contiguous().view(torch.float32)
    d = out[:, nk:2 * nk].contiguous()
    c = out[:, 2 * nk:].contiguous()
    return s, d, c


def gather_packed(score: torch.Tensor, doc: torch.Tensor, n: torch.Tensor, group=None):
    """All-gather per-shard top-k buffers; returns ([world, nq*k] f32, [world, nq*k] i32, [world, nq] i32)
    on the input's device.  RCCL gathers device memory directly; a gloo group
    (CPU rehearsal of the N>1 path) goes through host memory."""
    world = dist.get_world_size(group)
    buf = pack_topk(score, doc, n)
    via_host = dist.get_backend(group) == "gloo" and buf.is_cuda
    src = buf.cpu() if via_host else buf
    out = torch.empty(world * src.numel(), dtype=torch.int32, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    if via_host:
        out = out.to(buf.device)
    return unpack_topk(out.view(world, src.numel()), score.numel())


def merge_on_device(s: torch.Tensor, d: torch.Tensor, c: torch.Tensor, nq: int, k: int, stream=None):
    """Device merge (fg_merge_shards) of gathered [world, nq*k] buffers."""
    from . import native
    world = s.shape[0]
    out_s = torch.empty(nq * k, dtype=torch.float32, device=s.device)
    out_d = torch.empty(nq * k, dtype=torch.int32, device=s.device)
    out_sh = torch.empty(nq * k, dtype=torch.int32, device=s.device)
    out_n = torch.empty(nq, dtype=torch.int32, device=s.device)
    st = stream if stream is not None else torch.cuda.current_stream(s.device).cuda_stream
    native.merge_shards(world, nq, k, s.data_ptr(), d.data_ptr(), c.data_ptr(), out_s.data_ptr(), out_d.data_ptr(),
                        out_sh.data_ptr(), out_n.data_ptr(), st)
    return out_s, out_d, out_sh, out_n


# ---- doc-sharded namespace ------------------------
def allreduce_stats(local, group=None, device=None):
    """Sum a shard's BM25 statistics over the group: ONE all-reduce of
    [n_docs, tot_text, tot_name, tot_facet, df_text[V], df_name[V], df_facet[VF]]
    as int64 (RCCL when the group is "nccl": pass the rank's cuda device).
    Every rank must pass the same vocabularies (one term / facet dictionary per
    namespace).  Returns native.ShardStats of the whole namespace, identical on
    every rank."""
    import numpy as np

    from .native import ShardStats
    V = len(local.df_text)
    VF = 0 if local.df_facet is None else len(local.df_facet)
    buf = np.empty(4 + 2 * V + VF, np.int64)
    buf[0] = local.n_docs
    buf[1:3] = local.tot_tokens
    buf[3] = local.tot_facet_tokens
    buf[4:4 + V] = local.df_text
    buf[4 + V:4 + 2 * V] = local.df_name
    if VF:
        buf[4 + 2 * V:] = local.df_facet
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    out = t.cpu().numpy()
    dff = out[4 + 2 * V:].astype(np.uint32) if local.df_facet is not None else None
    return ShardStats(int(out[0]), (int(out[1]), int(out[2])), out[4:4 + V].astype(np.uint32),
                      out[4 + V:4 + 2 * V].astype(np.uint32), dff, int(out[3]))


def exchange_ladders(local, group=None, device=None):
    """All-gather the score ladders of every rank's shards ([n_local, V, L] f32,
    fg_index_term_ladder each) -> [world * n_local, V, L] in rank order: ONE
    all-gather at build (RCCL when `device` is the rank's cuda device).  Every
    rank must hold the same number of shards of one vocabulary."""
    import numpy as np
    loc = np.ascontiguousarray(local, np.float32)
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return loc
    world = dist.get_world_size(group)
    t = torch.from_numpy(loc.reshape(-1))
    if device is not None:
        t = t.to(device)
    out = torch.empty(world * t.numel(), dtype=torch.float32, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu().numpy().reshape((world * loc.shape[0],) + loc.shape[1:])


def seed_kth_floor(indexes, group=None, device=None):
    """Doc-sharded namespace (C5): give every shard the namespace-wide floor of its
    per-term K-th scores, so each shard's disjunctions start from a threshold
    valid for the whole namespace instead of its own docs' (fg_index_term_ladder
    -> exchange_ladders -> fg_kth_floor_combine -> fg_index_set_kth_floor).  The
    floor is score-only and the merged results are unchanged.  Returns the floor
    [V, 5] (identical on every rank)."""
    import numpy as np

    from . import native
    lad = np.stack([ix.term_ladder() for ix in indexes])
    allv = exchange_ladders(lad, group, device)
    floor = native.kth_floor_combine(list(allv))
    for ix in indexes:
        ix.set_kth_floor(floor)
    return floor


def agree_hist_span(plans, group=None, device=None):
    """Doc shards on several ranks: give the plans of one batch the same
    histogram bins on every rank -- the elementwise max of their spans
    (fg_plan_hist_span) over this rank's plans, then over the ranks (one
    all-reduce MAX of 2 x n_batch u32 when a group is up) -- so the histograms
    can be summed bin by bin (exchange_hist).  Returns (lo, hi)."""
    import numpy as np
    lo = hi = None
    for p in plans:
        a, b = p.hist_span()
        lo = a if lo is None else np.maximum(lo, a)
        hi = b if hi is None else np.maximum(hi, b)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.from_numpy(np.concatenate([lo, hi]).astype(np.int64))
        if device is not None:
            t = t.to(device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        t = t.cpu().numpy().astype(np.uint32)
        lo, hi = t[:len(lo)], t[len(lo):]
    for p in plans:
        p.set_hist_span(lo, hi)
    return lo, hi


def exchange_hist(plan, stream: int, buf: torch.Tensor, group=None, prev: "torch.Tensor | None" = None):
    """Between two parts of a plan's k_disj sweep (fg_plan_execute_part): sum the
    per-query score histograms of every rank's shards into this plan's, ONE
    all-reduce of [n_batch * HIST_BINS] int32 (RCCL over xGMI with "nccl"; gloo
    through host memory).  `buf` is an int32 device tensor of that size, and
    `stream` torch's current stream of the plan's device (the copies and the
    collective are ordered on it).  The shards' counted docs are distinct, so
    the summed histogram's threshold is still a lower bound of the merged k-th
    score: merged results are unchanged.

    A second exchange in the same round (a sweep in three or more parts) passes
    `prev`, the tensor the previous exchange returned: the plan's histogram then
    already holds every rank's earlier counts, so only this rank's counts since
    (its histogram minus `prev`) are summed and added back -- summing the whole
    histogram again would count the earlier counts once per rank, and the
    threshold of an over-counted histogram can pass the merged k-th score
    (ADVICE r05).  Returns the merged histogram (a new tensor) for the next call."""
    plan.hist_copy(stream, buf.data_ptr(), False)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if prev is not None:
            buf.sub_(prev)  # this rank's counts since the last exchange
        if dist.get_backend(group) == "gloo" and buf.is_cuda:
            h = buf.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(h)
        else:
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        if prev is not None:
            buf.add_(prev)
    plan.hist_copy(stream, buf.data_ptr(), True)
    return buf.clone()


def link_peers(plan, group=None):
    """Doc shards on several ranks (C5 over N GPUs): make this rank's plan a PEER
    of every other rank's plan of the same batch -- its thresholds and hit counts
    published into theirs during the launch, over xGMI (fg_plan_set_ipc_peers)
    -- through ONE all-gather of the plans' IPC words (fg_plan_ipc_export, 96 B
    per rank).  Agree on the histogram span first (agree_hist_span).  Every
    round then runs reset_peers() before the executes.  Returns the peer count."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world <= 1:
        return 0
    me = dist.get_rank(group)
    blobs = [None] * world
    dist.all_gather_object(blobs, plan.ipc_export(), group=group)
    peers = [b for r, b in enumerate(blobs) if r != me]
    plan.set_ipc_peers(peers)
    return len(peers)


def reset_peers(plan, stream=None, group=None):
    """A round of peer plans: this rank's plan reset, then a barrier, so every
    rank's words are zero before any rank's kernels publish into them."""
    plan.reset(stream)
    torch.cuda.synchronize()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.barrier(group=group)


def shard_ranges(n_docs: int, world: int):
    """Contiguous doc-id ranges [b, e) of the shards (tantivy segments)."""
    step = (n_docs + world - 1) // world
    return [(min(r * step, n_docs), min((r + 1) * step, n_docs)) for r in range(world)]
