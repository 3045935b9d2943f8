"""Gallery sharding across the GPUs of one node (one process per GPU).

The reference has no parallelism.  Search shards naturally by
gallery rows: rank r of G holds rows [r*N/G, (r+1)*N/G) of the
gallery, W and the query batch are replicated, every rank computes its local
top-k (exact fp64 distances, global row indices via ``index_base``), and the
only data-path exchange is ONE all-gather of the B x k (distance, index)
lists (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X, "gloo"
on CPU for tests), followed by the ``ofr_topk_merge`` kernel.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(N, rank, world_size):
    """Contiguous, disjoint, covering row ranges."""
    return (N * rank) // world_size, (N * (rank + 1)) // world_size


def exchange_topk(d, i, group=None):
    """All-gather per-rank (B x k) lists -> (B x world*k) tensors, rank-major (list p = rank p)."""
    _, ws = world()
    if ws == 1:
        return d, i
    gd = [torch.empty_like(d) for _ in range(ws)]
    gi = [torch.empty_like(i) for _ in range(ws)]
    dist.all_gather(gd, d.contiguous(), group=group)
    dist.all_gather(gi, i.contiguous(), group=group)
    return torch.cat(gd, dim=1).contiguous(), torch.cat(gi, dim=1).contiguous()


def merge_topk(gd, gi, nlists, kin, k):
    """Device merge of the gathered lists (ofr_topk_merge)."""
    if nlists == 1 and kin == k:
        return gd, gi
    from ._device import topk_merge
    return topk_merge(gd, gi, nlists, kin, k)


def sharded_search(local_search, k, group=None):
    """local_search(k) -> (d, i) on this rank's shard with global indices; returns the global top-k."""
    d, i = local_search(k)
    _, ws = world()
    gd, gi = exchange_topk(d, i, group)
    return merge_topk(gd, gi, ws, k, k)
