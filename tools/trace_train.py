"""Phase timestamps of the BN-train hidden forward kernel (dev tool).

Needs the tracing build (RS = 1: the default 256-workgroup exchange form):
    hipcc ... -DP3D_TRACE -DP3D_TRACE_RS=1 -o 3d-pose-baseline_amd/libp3d_trace.so
    P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python tools/trace_train.py [keep]
Prints, per phase, the min/median/max over workgroups of the wall_clock64 (100 MHz) delta
from the earliest workgroup start of the last traced launch.
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

keep = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
model, _ = bench.make_model()
X = torch.randn(64, 32, device="cuda")
T = torch.randn(64, 48, device="cuda")
for _ in range(20):
    model.train_step_device(X, T, keep)
torch.cuda.synchronize()
lib = _p3d.lib()
lib.p3d_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(4096 * 8, np.uint64)
assert lib.p3d_debug_trace(buf.ctypes.data, buf.size) == 0
nwg = int(os.environ.get("P3D_TRACE_NWG", "256"))   # workgroups of the traced launch
t = buf.reshape(4096, 8)[:nwg, :6].astype(np.int64)
t0 = t[:, 0].min()
t0f = t0
names = ["start", "gemm(w0)", "reduced", "bn+xchg", "philox", "stored"]
for k, n in enumerate(names):
    d = (t[:, k] - t0) * 10.0 / 1000.0
    print("%-9s min %6.2f  med %6.2f  max %6.2f us" % (n, d.min(), np.median(d), d.max()))
# per column tile: the latest sibling's GEMM end vs each sibling's exchange end (arrival skew)
gx = nwg // 4
g = (t[:, 2] - t0).reshape(4, gx) * 10.0 / 1000.0
b = (t[:, 3] - t0).reshape(4, gx) * 10.0 / 1000.0
print("sibling skew of 'reduced' (max-min over the 4 row tiles): med %.2f max %.2f us"
      % (np.median(g.max(0) - g.min(0)), (g.max(0) - g.min(0)).max()))
print("exchange done - latest sibling reduced: med %.2f max %.2f us"
      % (np.median(b - g.max(0)), (b - g.max(0)).max()))
x = buf.reshape(4096, 8)[:nwg, 7].astype(np.int64).reshape(4, gx)     # hardware XCD id per workgroup
same = (x == x[0:1]).all(0)
print("column tiles whose 4 row-tile siblings share an XCD: %d / %d" % (int(same.sum()), gx))
e = buf[16384:16384 + nwg * 8].astype(np.int64).reshape(nwg, 8)   # exchange detail (the last exchange launch)
t0 = e[:, 0].min() - 300   # (its own time base: the first get start, minus 3 us)
us = lambda v: (v - t0) * 10.0 / 1000.0   # noqa: E731
for k, n in ((0, "get start (w0)"), (1, "publish issue (w1)"), (2, "publish acked (w1)"), (3, "get done (w0)")):
    d = us(e[:, k])
    print("%-20s min %6.2f  med %6.2f  max %6.2f us" % (n, d.min(), np.median(d), d.max()))
print("sweeps per get: med %d max %d; memory-side sweeps med %d max %d"
      % (np.median(e[:, 4]), e[:, 4].max(), np.median(e[:, 5]), e[:, 5].max()))
pa = us(e[:, 2]).reshape(4, gx).max(0)         # the latest sibling's publish acked
print("get done - latest sibling acked: med %.2f max %.2f us"
      % (np.median(us(e[:, 3]).reshape(4, gx) - pa), (us(e[:, 3]).reshape(4, gx) - pa).max()))
for k, n in ((6, "fwd: moments done (w0)"),):   # (the forward's own time base)
    d = (e[:, k] - t0f) * 10.0 / 1000.0
    print("%-20s min %6.2f  med %6.2f  max %6.2f us" % (n, d.min(), np.median(d), d.max()))
