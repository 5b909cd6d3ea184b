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

import os


def free_port(lo=20000, hi=29999):
    """A free 127.0.0.1 TCP port for a rendezvous, picked at random BELOW the kernel's ephemeral
    range (32768-60999): a port the OS handed out and we released can go to another socket (RCCL
    and gloo open many) before the rendezvous binds it -- the EADDRINUSE flake of r05_t20.  The one
    helper bench.py and the multi-process tests share."""
    import random
    import socket
    for _ in range(64):
        p = random.randint(lo, hi)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
        return p
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
    """Bucketed DP gradient average, host-staged (gloo: tests of several ranks on one GPU).

    For each bucket k (backward order), ``comm_stream`` waits for its gradient-ready event
    (``wait_ready(k, stream_handle)``, p3d_stream_wait_grad), the slice is copied to the host,
    all-reduced and copied back -- the event ordering of the device path (a bucket read before
    its layers' gradients are final would differ from the single all-reduce).
    ``after(k, stream_handle)`` (optional) is issued on ``comm_stream`` behind bucket k's reduced
    slice -- the bucket's optimizer (p3d_adam_apply_bucket) -- and the current stream then waits
    for ``comm_stream``.  Under RCCL the library reduces the buckets itself
    (p3d_train_step_dp, native_comm below)."""
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        raise RuntimeError("allreduce_mean_buckets_: RCCL data parallelism runs in libp3d (p3d_train_step_dp)")
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


def allreduce_sum_(t):
    import torch.distributed as dist
    on, _, world = dist_state()
    if on and world > 1:
        h = t.cpu() if _host_staged(t) else t
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        if h is not t:
            t.copy_(h)
    return t


_NATIVE = {}
_ATTACHED = None   # weakref.WeakSet of the models attached to a cached communicator


def attach_native(model):
    """Attach ``model`` to the process's library-owned communicator (p3d_dp_attach) and remember
    it, so that close_native_comms can detach it before the communicator is destroyed."""
    import weakref
    import _p3d
    global _ATTACHED
    if _ATTACHED is None:
        _ATTACHED = weakref.WeakSet()
    h = native_comm()
    _p3d.check(_p3d.lib().p3d_dp_attach(model._h, h), "p3d_dp_attach")
    _ATTACHED.add(model)
    return h


def librccl_path():
    """The librccl this process already uses (torch's bundled copy), for p3d_comm_load: one RCCL
    per process."""
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so.1"


def native_comm():
    """The library-owned RCCL communicator over the default process group's ranks (p3d_comm,
    include/p3d.h): rank 0 draws a unique id, it is broadcast over torch.distributed once, and
    every rank joins.  Cached per (world, rank); the data-parallel step reduces over it inside
    libp3d (p3d_train_step_dp), so a captured step holds no torch collective.
    RCCL process groups only (one GPU per rank); gloo tests use the host-staged path."""
    import ctypes
    import torch
    import torch.distributed as dist
    import _p3d
    on, rank, world = dist_state()
    if not on:
        raise RuntimeError("native_comm: no process group")
    key = (world, rank)
    c = _NATIVE.get(key)
    if c is not None:
        return c
    L = _p3d.lib()
    _p3d.check(L.p3d_comm_load(librccl_path().encode()), "p3d_comm_load")
    uid = (ctypes.c_uint8 * 128)()
    if rank == 0:
        _p3d.check(L.p3d_comm_unique_id(uid, 128), "p3d_comm_unique_id")
    t = torch.tensor(list(bytes(uid)), dtype=torch.uint8,
                     device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.broadcast(t, src=0)
    ctypes.memmove(uid, bytes(t.cpu().tolist()), 128)
    h = ctypes.c_void_p()
    _p3d.check(L.p3d_comm_create(uid, 128, world, rank, ctypes.byref(h)), "p3d_comm_create")
    _NATIVE[key] = h
    return h


def close_native_comms():
    """Destroy the cached communicators (before destroy_process_group; every rank calls it)."""
    import _p3d
    import torch
    if not _NATIVE:
        return
    torch.cuda.synchronize()
    # models first: a model still holding the communicator would reduce over a freed ncclComm
    for model in list(_ATTACHED or ()):
        h = getattr(model, "_h", None)
        if h is not None and h.value:
            _p3d.check(_p3d.lib().p3d_dp_attach(h, None), "p3d_dp_attach")
        model._native = None
        model._buckets = False      # the next DP step re-plans (and re-attaches)
    if _ATTACHED is not None:
        _ATTACHED.clear()
    for k in list(_NATIVE):
        _p3d.check(_p3d.lib().p3d_comm_destroy(_NATIVE.pop(k)), "p3d_comm_destroy")


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
