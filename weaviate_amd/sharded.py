"""Corpus sharding over the GPUs of one node (one process per GPU).

The reference shards a class into independent indexes and merges their
results by distance (adapters/repos/db/index.go:967-1044, sorted by
sortby_distances.go).  Here rank r of W owns the contiguous id range
shard_bounds(N, r, W), searches it locally, and the per-shard [nq, k]
(dist, id) blocks are all-gathered over RCCL (torch.distributed "nccl") and
merged on every rank by the device kernel behind wv_merge_shards_device, in
(dist, id) order -- identical to a single-GPU search of the whole corpus.
"""
from __future__ import annotations

from typing import Callable, Optional


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """[lo, hi) of global ids owned by `rank` (contiguous, sizes differ by <= 1)."""
    return n * rank // world, n * (rank + 1) // world


def allgather_topk(ids, dists, counts, world: int, group=None):
    """All-gather per-shard results into [world, nq, k] / [world, nq] tensors."""
    import torch
    import torch.distributed as dist

    g_ids = torch.empty((world,) + tuple(ids.shape), dtype=ids.dtype, device=ids.device)
    g_d = torch.empty((world,) + tuple(dists.shape), dtype=dists.dtype, device=dists.device)
    g_n = torch.empty((world,) + tuple(counts.shape), dtype=counts.dtype, device=counts.device)
    if ids.is_cuda:
        dist.all_gather_into_tensor(g_ids, ids, group=group)
        dist.all_gather_into_tensor(g_d, dists, group=group)
        dist.all_gather_into_tensor(g_n, counts, group=group)
    else:  # gloo: list form
        dist.all_gather(list(g_ids.unbind(0)), ids, group=group)
        dist.all_gather(list(g_d.unbind(0)), dists, group=group)
        dist.all_gather(list(g_n.unbind(0)), counts, group=group)
    return g_ids, g_d, g_n


def merge_topk(g_ids, g_d, g_n, k: int, merge_fn: Optional[Callable] = None):
    """Merge gathered shard results.  On device tensors the HIP merge kernel
    runs; CPU tensors need an explicit merge_fn (tests only)."""
    import torch

    world, nq = g_n.shape
    if g_ids.is_cuda:
        from .index import merge_shards_device

        out_ids = torch.empty((nq, k), dtype=torch.int64, device=g_ids.device)
        out_d = torch.empty((nq, k), dtype=torch.float32, device=g_ids.device)
        out_n = torch.empty((nq,), dtype=torch.int32, device=g_ids.device)
        merge_shards_device(g_d.data_ptr(), g_ids.data_ptr(), g_n.data_ptr(), world, nq, k, out_d.data_ptr(),
                            out_ids.data_ptr(), out_n.data_ptr(),
                            stream=torch.cuda.current_stream(g_ids.device).cuda_stream)
        return out_ids, out_d, out_n
    if merge_fn is None:
        raise RuntimeError("merge_topk on CPU tensors needs merge_fn: the product merge runs on the GPU")
    return merge_fn(g_ids, g_d, g_n, k)
