"""ctypes binding of libp3d.so (include/p3d.h) -- the HIP hot path of the pose MLP.

There is deliberately NO fallback: if the shared library is missing or fails to
load, importing a module that needs it raises immediately.  Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (or ``make -C
3d-pose-baseline_amd``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_uint32, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("P3D_LIB", os.path.join(HERE, "libp3d.so"))  # P3D_LIB: dev builds (tools/)

P3D_CTR_GLOBAL_STEP = 0xFFFFFFFFFFFFFFFF
P3D_DTYPE_F32 = 0
P3D_DTYPE_BF16 = 1
P3D_DTYPE_F64 = 2
P3D_ERR_ARG = 1          # include/p3d.h status codes (check() maps 1 to ValueError)


class P3DCfg(ctypes.Structure):
    _fields_ = [("linear_size", c_int32), ("num_layers", c_int32), ("residual", c_int32),
                ("batch_norm", c_int32), ("max_norm", c_int32), ("input_size", c_int32),
                ("output_size", c_int32), ("dtype", c_int32), ("max_batch", c_int32),
                ("bn_eps", c_float), ("bn_momentum", c_float)]


class P3DError(RuntimeError):
    pass


# (name, restype, argtypes) -- exactly the entry points declared in include/p3d.h
SIGNATURES = [
    ("p3d_last_error", c_char_p, []),
    ("p3d_create", c_int32, [POINTER(P3DCfg), POINTER(c_void_p)]),
    ("p3d_destroy", c_int32, [c_void_p]),
    ("p3d_param_count", c_int32, [c_void_p, POINTER(c_int32)]),
    ("p3d_param_info", c_int32, [c_void_p, c_int32, POINTER(c_char_p), POINTER(c_int64),
                                 POINTER(c_int32), POINTER(c_int64)]),
    ("p3d_param_ptr", c_int32, [c_void_p, c_char_p, POINTER(c_void_p), POINTER(c_int64)]),
    ("p3d_flat_ptr", c_int32, [c_void_p, c_int32, POINTER(c_void_p), POINTER(c_int64)]),
    ("p3d_params_updated", c_int32, [c_void_p, c_void_p]),
    ("p3d_params_changed", c_int32, [c_void_p]),
    ("p3d_params_sync", c_int32, [c_void_p, c_void_p]),
    ("p3d_forward", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_float, c_uint64,
                              c_uint64, c_int64, c_void_p]),
    ("p3d_forward_ex", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_float, c_uint64,
                                 c_uint64, c_int64, c_int64, c_void_p]),
    ("p3d_serve", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    ("p3d_serve_mse", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("p3d_serve_mse_sync", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("p3d_serve_check", c_int32, [c_void_p]),
    ("p3d_sync_check", c_int32, [c_void_p]),
    ("p3d_error_flags", c_int32, [c_void_p, POINTER(c_int32), c_int32]),
    ("p3d_mse", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p]),
    ("p3d_backward", c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    ("p3d_adam_step", c_int32, [c_void_p, c_float, c_void_p]),
    ("p3d_adam_step_decay", c_int32, [c_void_p, c_float, c_float, c_float, c_void_p]),
    ("p3d_get_step", c_int32, [c_void_p, POINTER(c_int64), POINTER(c_float), POINTER(c_float)]),
    ("p3d_set_step", c_int32, [c_void_p, c_int64, c_float, c_float]),
    ("p3d_mpjpe_accum", c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                  c_void_p, c_void_p]),
    ("p3d_mpjpe_accum_ex", c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int64,
                                     c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    ("p3d_kernel_name", c_int32, [c_void_p, c_int32, c_char_p, c_int64]),
    ("p3d_dlpack_alias", c_void_p, [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int32]),
    ("p3d_train_step", c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_float, c_uint64, c_float,
                                 c_float, c_float, c_void_p, c_void_p]),
    ("p3d_train_fwd_bwd", c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_float, c_uint64, c_int64,
                                    c_void_p, c_void_p]),
    ("p3d_grad_events", c_int32, [c_void_p, c_int32]),
    ("p3d_grad_buckets", c_int32, [c_void_p, c_int32, c_void_p]),
    ("p3d_train_fwd_bwd_lr", c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_float, c_uint64, c_int64,
                                       c_float, c_float, c_float, c_void_p, c_void_p]),
    ("p3d_adam_apply", c_int32, [c_void_p, c_void_p]),
    ("p3d_adam_apply_bucket", c_int32, [c_void_p, c_int32, c_void_p]),
    ("p3d_layer_grad_range", c_int32, [c_void_p, c_int32, POINTER(c_int64), POINTER(c_int64)]),
    ("p3d_stream_wait_grad", c_int32, [c_void_p, c_int32, c_void_p]),
    ("p3d_profile_start", c_int32, [c_void_p, c_int32]),
    ("p3d_empty_launch", c_int32, [c_void_p, c_int32, c_void_p]),
    ("p3d_host_signal", c_int32, [c_void_p, c_void_p]),
    ("p3d_host_wait", c_int32, [c_void_p, c_uint32, c_void_p]),
    ("p3d_host_alloc", c_void_p, [c_int64]),
    ("p3d_host_free", c_int32, [c_void_p]),
    ("p3d_profile_stop", c_int32, [c_void_p, c_char_p, c_int64]),
    ("p3d_time_layer", c_int32, [c_void_p, c_int32, c_int64, c_int32, c_void_p]),
    ("p3d_cam_transform", c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    ("p3d_cam_project", c_int32, [c_void_p, c_int64, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p]),
    ("p3d_root_center", c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p]),
    ("p3d_normalize", c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                c_int32, c_void_p]),
    ("p3d_unnormalize", c_int32, [c_void_p, c_int32, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                                  c_void_p, c_void_p]),
    ("p3d_lift", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                           c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    ("p3d_lift_sync", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                                c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    ("p3d_moments_workspace", c_int64, [c_int64, c_int32]),
    ("p3d_moments", c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    ("p3d_crc32c", c_uint32, [c_void_p, c_int64, c_uint32]),
    ("p3d_comm_load", c_int32, [c_char_p]),
    ("p3d_comm_unique_id", c_int32, [c_void_p, c_int64]),
    ("p3d_comm_create", c_int32, [c_void_p, c_int64, c_int32, c_int32, POINTER(c_void_p)]),
    ("p3d_comm_destroy", c_int32, [c_void_p]),
    ("p3d_comm_allreduce", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p]),
    ("p3d_dp_attach", c_int32, [c_void_p, c_void_p]),
    ("p3d_train_step_dp", c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_float, c_uint64, c_int64,
                                    c_float, c_float, c_float, c_void_p, c_void_p]),
]


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise P3DError("libp3d.so not found at %s: the HIP extension is not built "
                       "(run __graft_entry__.build()); there is no CPU fallback" % path)
    # One HIP runtime per process: torch's libc10_hip pulls in its bundled libamdhip64 by the
    # unversioned name, libp3d.so by soname libamdhip64.so.7.  Loaded after torch, libp3d binds
    # to torch's copy (same soname); loaded first, it would bring /opt/rocm's and torch would
    # then add a second runtime, which sees no device (p3d_create: "no ROCm-capable device").
    import torch  # noqa: F401
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = load()
    return _LIB


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().p3d_last_error().decode()
        if rc == 1:
            raise ValueError("%s: %s" % (what, msg))
        raise P3DError("%s failed (%d): %s" % (what, rc, msg))


# --------------------------------------------------------------------------------------
# zero-copy torch views of library-owned device memory (DLPack, kDLROCM)
# --------------------------------------------------------------------------------------


def device_view(ptr: int, shape, device_index: int, dtype_code: int = 2, bits: int = 32):
    """torch tensor aliasing ``ptr`` (no copy).  The owner must outlive the view.  The
    DLPack record and its deleter are native (p3d_dlpack_alias): releasing the view never
    re-enters Python, also not during interpreter teardown."""
    from torch.utils.dlpack import from_dlpack

    shape = tuple(int(s) for s in shape)
    shp = (c_int64 * len(shape))(*shape)
    mt = lib().p3d_dlpack_alias(c_void_p(ptr), len(shape), shp, int(device_index), int(dtype_code), int(bits))
    if not mt:
        raise P3DError("p3d_dlpack_alias failed")
    PyCapsule_New = ctypes.pythonapi.PyCapsule_New
    PyCapsule_New.restype = ctypes.py_object
    PyCapsule_New.argtypes = [c_void_p, c_char_p, c_void_p]
    t = from_dlpack(PyCapsule_New(mt, b"dltensor", None))
    assert t.data_ptr() == ptr
    return t


def ptr(t) -> int:
    """Device pointer of a torch tensor (or 0 for None)."""
    return 0 if t is None else int(t.data_ptr())


def stream_handle(stream=None) -> int:
    import torch
    if stream is None:
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)   # no Stream object built
        if raw is not None:
            return int(raw(torch.cuda.current_device()))
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


__all__ = ["P3DCfg", "P3DError", "lib", "check", "device_view", "ptr", "stream_handle",
           "LIB_PATH", "SIGNATURES", "c_double"]
