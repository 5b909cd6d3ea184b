"""Device-resident H3.6M data pipeline over libp3d's HIP kernels.

torch tensors in HBM in, torch tensors out, on the current stream; float64 like the
reference's numpy.  The reference-API wrappers (numpy in / numpy out) are
``cameras.project_point_radial / world_to_camera_frame / camera_to_world_frame`` and
``data_utils.transform_world_to_camera / project_to_cameras / postprocess_3d /
normalization_stats / normalize_data / unNormalizeData``.

There is no CPU path: without a GPU every function raises P3DError.
"""
from __future__ import annotations

import numpy as np

import _p3d
from _p3d import check, lib, ptr

CAM_DOUBLES = 21


def _torch():
    import torch
    return torch


def device():
    torch = _torch()
    if not torch.cuda.is_available():
        raise _p3d.P3DError("the H3.6M data pipeline runs on the GPU (libp3d); no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def as_device(a, dtype=None):
    """numpy / torch -> contiguous device tensor (float64 unless dtype is given)."""
    torch = _torch()
    dtype = dtype or torch.float64
    if isinstance(a, torch.Tensor):
        t = a
    else:
        t = torch.from_numpy(np.ascontiguousarray(a))
    return t.to(device=device(), dtype=dtype, non_blocking=True).contiguous()


def pack_camera(R, T, f, c, k, p):
    """The 21-double camera record of include/p3d.h from the reference's camera tuple
    (src/cameras.py:92-140): R row-major, T, f, c, k, p."""
    parts = [np.asarray(v, np.float64).reshape(-1) for v in (R, T, f, c, k, p)]
    sizes = [v.size for v in parts]
    if sizes != [9, 3, 2, 2, 3, 2]:
        raise ValueError("camera parameters must be R 3x3, T 3, f 2, c 2, k 3, p 2; got sizes %s" % sizes)
    return np.concatenate(parts)


def pack_cameras(cams):
    """[C, 21] from an iterable of (R, T, f, c, k, p[, name]) tuples."""
    return np.stack([pack_camera(*cam[:6]) for cam in cams])


def _stream():
    return _p3d.stream_handle()


def _points(P, what):
    t = as_device(P)
    if t.dim() != 2 or t.shape[1] != 3:
        raise ValueError("%s: expected points [N, 3], got %s" % (what, tuple(t.shape)))
    return t


def _out(out, shape, dev, what):
    torch = _torch()
    if out is None:
        return torch.empty(shape, dtype=torch.float64, device=dev)
    if tuple(out.shape) != tuple(shape) or out.dtype != torch.float64 or not out.is_contiguous() \
            or out.device != dev:
        raise ValueError("%s: out must be a contiguous float64 %s tensor on %s" % (what, tuple(shape), dev))
    return out


def world_to_camera(P, cams, out=None):
    """[n, 3] world points -> [C, n, 3] camera-frame points (one slab per camera)."""
    P = _points(P, "world_to_camera")
    cm = as_device(cams).reshape(-1, CAM_DOUBLES)
    out = _out(out, (cm.shape[0], P.shape[0], 3), P.device, "world_to_camera")
    check(lib().p3d_cam_transform(ptr(P), P.shape[0], 0, ptr(cm), cm.shape[0], 0, ptr(out), _stream()),
          "p3d_cam_transform")
    return out


def camera_to_world(X, cams):
    """Camera-frame points [n, 3] (one camera) or [C, n, 3] (camera c's own points) -> world [C, n, 3]."""
    torch = _torch()
    X = as_device(X)
    cm = as_device(cams).reshape(-1, CAM_DOUBLES)
    C = cm.shape[0]
    if X.dim() == 2 and X.shape[1] == 3:
        n, stride = X.shape[0], 0
    elif X.dim() == 3 and X.shape[0] == C and X.shape[2] == 3:
        n, stride = X.shape[1], 3 * X.shape[1]
    else:
        raise ValueError("camera_to_world: expected [N, 3] or [C, N, 3], got %s" % (tuple(X.shape),))
    out = torch.empty((C, n, 3), dtype=torch.float64, device=X.device)
    check(lib().p3d_cam_transform(ptr(X), n, stride, ptr(cm), C, 1, ptr(out), _stream()), "p3d_cam_transform")
    return out


def project(P, cams, aux=False, out=None):
    """[n, 3] world points -> projections [C, n, 2]; with aux also depth, radial, tan, r2 [C, n]."""
    torch = _torch()
    P = _points(P, "project")
    cm = as_device(cams).reshape(-1, CAM_DOUBLES)
    C, n = cm.shape[0], P.shape[0]
    proj = _out(out, (C, n, 2), P.device, "project")
    extra = [torch.empty((C, n), dtype=torch.float64, device=P.device) for _ in range(4)] if aux else [None] * 4
    check(lib().p3d_cam_project(ptr(P), n, ptr(cm), C, ptr(proj), *[ptr(e) for e in extra], _stream()),
          "p3d_cam_project")
    return (proj, *extra) if aux else proj


def root_center(poses):
    """poses [F, 3J] -> (poses - root tiled, root [F, 3])."""
    torch = _torch()
    x = as_device(poses)
    if x.dim() != 2 or x.shape[1] % 3 or x.shape[1] < 3:
        raise ValueError("root_center: expected poses [F, 3*joints], got %s" % (tuple(x.shape),))
    out = torch.empty_like(x)
    root = torch.empty((x.shape[0], 3), dtype=torch.float64, device=x.device)
    check(lib().p3d_root_center(ptr(x), x.shape[0], x.shape[1], ptr(out), ptr(root), _stream()), "p3d_root_center")
    return out, root


def _dims(dims, D, what):
    """Column indices as a device int32 tensor.  Host indices are range-checked here; a device
    int32 tensor is taken as already checked (no device -> host sync on the hot path)."""
    torch = _torch()
    if isinstance(dims, torch.Tensor) and dims.is_cuda and dims.dtype == torch.int32:
        return dims.reshape(-1).contiguous()
    d = np.asarray(dims.cpu() if isinstance(dims, torch.Tensor) else dims, np.int64).reshape(-1)
    if d.size and (d.min() < 0 or d.max() >= D):
        raise ValueError("%s: dimension indices out of range [0, %d)" % (what, D))
    return as_device(d.astype(np.int32), torch.int32)


def normalize(x, mean, std, dims_to_use, out_dtype=None, out=None):
    """(x[:, use] - mean[use]) / std[use]: [F, D] -> [F, U] (float64, or float32)."""
    torch = _torch()
    out_dtype = out_dtype or torch.float64
    x = as_device(x)
    if x.dim() != 2:
        raise ValueError("normalize: expected [F, D], got %s" % (tuple(x.shape),))
    D = x.shape[1]
    mean, std = as_device(mean).reshape(-1), as_device(std).reshape(-1)
    use = _dims(dims_to_use, D, "normalize")
    if mean.numel() != D or std.numel() != D:
        raise ValueError("normalize: mean/std must have %d entries" % D)
    if out is None:
        out = torch.empty((x.shape[0], use.numel()), dtype=out_dtype, device=x.device)
    elif tuple(out.shape) != (x.shape[0], use.numel()) or out.dtype != out_dtype or not out.is_contiguous():
        raise ValueError("normalize: out must be a contiguous %s [%d, %d] tensor"
                         % (out_dtype, x.shape[0], use.numel()))
    code = _p3d.P3D_DTYPE_F32 if out_dtype == torch.float32 else _p3d.P3D_DTYPE_F64
    check(lib().p3d_normalize(ptr(x), x.shape[0], D, ptr(mean), ptr(std), ptr(use), use.numel(), ptr(out), code,
                              _stream()), "p3d_normalize")
    return out


def unnormalize(xn, mean, std, dims_to_use, D=None, out=None):
    """Inverse of normalize as unNormalizeData computes it: [F, U] -> [F, D] float64."""
    torch = _torch()
    t = xn if isinstance(xn, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(xn))
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    t = t.to(device=device(), non_blocking=True).contiguous()
    if t.dim() != 2:
        raise ValueError("unnormalize: expected [F, U], got %s" % (tuple(t.shape),))
    mean, std = as_device(mean).reshape(-1), as_device(std).reshape(-1)
    D = D or mean.numel()
    use = _dims(dims_to_use, D, "unnormalize")
    if use.numel() != t.shape[1]:
        raise ValueError("unnormalize: %d columns for %d used dimensions" % (t.shape[1], use.numel()))
    out = _out(out, (t.shape[0], D), t.device, "unnormalize")
    code = _p3d.P3D_DTYPE_F32 if t.dtype == torch.float32 else _p3d.P3D_DTYPE_F64
    check(lib().p3d_unnormalize(ptr(t), code, t.shape[0], use.numel(), ptr(mean), ptr(std), ptr(use), D, ptr(out),
                                _stream()), "p3d_unnormalize")
    return out


def moments(x):
    """(mean, population std) over axis 0 of [F, D] float64."""
    torch = _torch()
    x = as_device(x)
    if x.dim() != 2 or x.shape[0] < 1:
        raise ValueError("moments: expected [F >= 1, D], got %s" % (tuple(x.shape),))
    F, D = x.shape
    nbytes = int(lib().p3d_moments_workspace(F, D))
    work = torch.empty(max(1, nbytes // 8), dtype=torch.float64, device=x.device)
    mean = torch.empty(D, dtype=torch.float64, device=x.device)
    std = torch.empty(D, dtype=torch.float64, device=x.device)
    check(lib().p3d_moments(ptr(x), F, D, ptr(mean), ptr(std), ptr(work), nbytes, _stream()), "p3d_moments")
    return mean, std
