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


def plan_buckets(ranges, min_elems):
    """Group per-layer gradient ranges into all-reduce buckets, in backward order.

    ``ranges[l] = (begin, end)`` is layer l's slice of the flat gradient buffer (layers
    are contiguous in TF creation order, layer 0 first).  The backward finishes the
    output layer first, so buckets are formed from the last layer down; a bucket closes
    once it holds ``min_elems`` floats and is ready when its lowest layer is.  A short
    remainder joins the previous bucket.  Returns [(begin, end, ready_layer)], covering
    every range exactly once.
    """
    out = []
    hi = None
    for l in range(len(ranges) - 1, -1, -1):
        lo, e = ranges[l]
        if hi is None:
            hi = e
        if hi - lo >= min_elems or l == 0:
            out.append([lo, hi, l])
            hi = None
    if len(out) > 1 and out[-1][1] - out[-1][0] < min_elems:
        lo, _, l = out.pop()
        out[-1][0], out[-1][2] = lo, l
    return [tuple(b) for b in out]


def allreduce_mean_buckets_(t, buckets, wait_ready, comm_stream, after=None):
    """Bucketed DP gradient average that overlaps the backward.

    For each bucket k (backward order), ``comm_stream`` waits for its gradient-ready event
    (``wait_ready(k, stream_handle)``, p3d_stream_wait_grad),
    then an async all-reduce(AVG) of that slice is issued from it (RCCL); the current
    stream finally waits for all of them.  Every byte of ``t`` is reduced exactly once, so
    the result equals ``allreduce_mean_`` (tests/test_gpu_dist.py).  Under gloo (tests:
    several ranks on one GPU) each bucket is copied to the host on ``comm_stream`` after
    its event -- the same event ordering, host-staged: a bucket read before its layer's
    gradients are final would differ from the single all-reduce.  ``after(k, stream_handle)``
    (optional) is issued on ``comm_stream`` behind bucket k's reduced slice -- the bucket's
    optimizer (p3d_adam_apply_bucket) -- and the current stream then waits for ``comm_stream``.
    """
    import torch
    import torch.distributed as dist
    if dist.get_backend() != "nccl":
        world = dist.get_world_size()
        with torch.cuda.stream(comm_stream):
            for k, (lo, hi, _) in enumerate(buckets):
                wait_ready(k, comm_stream.cuda_stream)
                h = t[lo:hi].to("cpu")          # synchronous on comm_stream, after the event
                dist.all_reduce(h, op=dist.ReduceOp.SUM)
                h.div_(world)
                t[lo:hi].copy_(h)
                if after is not None:
                    after(k, comm_stream.cuda_stream)
        torch.cuda.current_stream().wait_stream(comm_stream)
        return t
    works = []
    with torch.cuda.stream(comm_stream):
        for k, (lo, hi, _) in enumerate(buckets):
            wait_ready(k, comm_stream.cuda_stream)
            if after is None:
                works.append(dist.all_reduce(t[lo:hi], op=dist.ReduceOp.AVG, async_op=True))
            else:
                # a synchronous collective runs on the current stream (comm_stream) itself: the
                # bucket's optimizer queues right behind it.  (An async one plus work.wait() from
                # comm_stream crashed HIP graph capture at capture end.)
                dist.all_reduce(t[lo:hi], op=dist.ReduceOp.AVG)
                after(k, comm_stream.cuda_stream)
    if after is not None:
        torch.cuda.current_stream().wait_stream(comm_stream)
    for w in works:
        w.wait()
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
