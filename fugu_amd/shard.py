"""Namespace sharding across GPUs.

One process per GPU; rank r holds namespace r's snapshot.  A fan-out query
runs on every shard, the per-shard top-k lists are exchanged with ONE
all-gather per batch (RCCL over xGMI when the group is "nccl"), and the global
top-k is merged on the device by (score desc, shard asc, doc asc).  Scores are
not renormalised across namespaces: each namespace keeps its own BM25
statistics, exactly as each fugu namespace is its own tantivy index
(src/db/core.rs:49-79).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def gather_topk(score: torch.Tensor, doc: torch.Tensor, n: torch.Tensor, group=None):
    """All-gather per-shard top-k buffers ([nq*k], [nq*k], [nq]) into
    ([world, nq*k], [world, nq*k], [world, nq]).  One collective per tensor."""
    world = dist.get_world_size(group)
    out_s = torch.empty((world,) + tuple(score.shape), dtype=score.dtype, device=score.device)
    out_d = torch.empty((world,) + tuple(doc.shape), dtype=doc.dtype, device=doc.device)
    out_n = torch.empty((world,) + tuple(n.shape), dtype=n.dtype, device=n.device)
    dist.all_gather_into_tensor(out_s, score.contiguous(), group=group)
    dist.all_gather_into_tensor(out_d, doc.contiguous(), group=group)
    dist.all_gather_into_tensor(out_n, n.contiguous(), group=group)
    return out_s, out_d, out_n


def pack_topk(score: torch.Tensor, doc: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
    """One int32 buffer [nq*k*2 + nq] so a batch needs a single all-gather."""
    return torch.cat([score.view(torch.int32), doc.view(torch.int32), n.view(torch.int32)])


def gather_packed(score: torch.Tensor, doc: torch.Tensor, n: torch.Tensor, group=None):
    world = dist.get_world_size(group)
    buf = pack_topk(score, doc, n)
    out = torch.empty((world, buf.numel()), dtype=torch.int32, device=buf.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    nk = score.numel()
    s = out[:, :nk].contiguous().view(torch.float32)
    d = out[:, nk:2 * nk].contiguous()
    c = out[:, 2 * nk:].contiguous()
    return s, d, c


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
