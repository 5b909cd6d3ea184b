"""Multi-GPU plumbing for the hot path (one process per GPU, torch.distributed).

The reference is single-process; these are the
two collectives its data-parallel / sharded forms need:

* training: pure data parallelism -- rank 0's parameters are broadcast once, every
  rank differentiates its own batch of 64, the flat fp32 gradient buffer is
  averaged with one all-reduce (RCCL over xGMI: ReduceOp.AVG), then every rank runs
  the identical TF1-Adam update.  BN statistics stay per replica (no SyncBN), exactly
  the reference's 64-sample batch statistics.
* evaluation: frames shard by batch across ranks (``shard_range``); per-action fp64
  partial sums are combined with one all-reduce.

Everything here works on CPU tensors with the gloo backend too (tests/test_dist.py).
"""
from __future__ import annotations


def dist_state():
    """(initialized, rank, world) of the default process group."""
    import torch.distributed as dist
    on = dist.is_available() and dist.is_initialized()
    return on, (dist.get_rank() if on else 0), (dist.get_world_size() if on else 1)


def shard_range(n: int, rank: int, world: int):
    """Contiguous [lo, hi) slice of n items owned by ``rank`` (sizes differ by <= 1)."""
    return (n * rank) // world, (n * (rank + 1)) // world


def _host_staged(t):
    """gloo moves host memory: device tensors are staged through the host (tests only;
    the production multi-GPU path is RCCL, which reduces device memory directly)."""
    import torch.distributed as dist
    return dist.get_backend() != "nccl" and t.is_cuda


def allreduce_mean_(t):
    """In-place mean over ranks (the DP gradient average)."""
    import torch.distributed as dist
    on, _, world = dist_state()
    if not on or world == 1:
        return t
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
        return t
    h = t.cpu() if _host_staged(t) else t
    dist.all_reduce(h, op=dist.ReduceOp.SUM)
    h.div_(world)
    if h is not t:
        t.copy_(h)
    return t


def allreduce_sum_(t):
    import torch.distributed as dist
    on, _, world = dist_state()
    if on and world > 1:
        h = t.cpu() if _host_staged(t) else t
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        if h is not t:
            t.copy_(h)
    return t


def broadcast_(tensors, src: int = 0):
    import torch.distributed as dist
    on, _, world = dist_state()
    if on and world > 1:
        for t in tensors:
            if t is None:
                continue
            h = t.cpu() if _host_staged(t) else t
            dist.broadcast(h, src=src)
            if h is not t:
                t.copy_(h)
    return tensors
