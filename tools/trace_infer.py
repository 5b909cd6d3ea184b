"""Phase timestamps of the B=64 inference hidden-layer kernel (dev tool).

    hipcc ... -DP3D_TRACE -DP3D_TRACE_RS=1 -o 3d-pose-baseline_amd/libp3d_trace.so csrc/p3d.hip
    P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python tools/trace_infer.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import _p3d  # noqa: E402

model, _ = bench.make_model()
X = torch.randn(64, 32, device="cuda")
for _ in range(50):
    model.forward_device(X)
torch.cuda.synchronize()
lib = _p3d.lib()
lib.p3d_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(4096 * 8, np.uint64)
assert lib.p3d_debug_trace(buf.ctypes.data, buf.size) == 0
t = buf.reshape(4096, 8)[:256].astype(np.int64)   # 64 x 4 workgroups of the last hidden launch
t0 = t[:, 0].min()
probe = os.environ.get("P3D_TRACE_PROBE") == "1"   # library built with -DP3D_TRACE_PROBE
phases = [(0, "start")] + ([(7, "X landed")] if probe else []) + \
    [(1, "gemm w0"), (6, "gemm w7"), (2, "reduced"), (3, "epi"), (5, "stored")] + \
    ([(4, "drained")] if probe else [])
for k, n in phases:
    d = (t[:, k] - t0) * 10.0 / 1000.0
    print("%-9s min %6.2f  med %6.2f  max %6.2f us" % (n, d.min(), np.median(d), d.max()))
model.close()
