"""Dev tool: timeline of the training step's k_wgrad_multi (fused TF1 Adam) from a -DP3D_TRACE
build: per workgroup start, operands staged, contraction done, Adam tile done (stores drained),
in us from the earliest start; quantiles over the 1,056 workgroups and the dispatch rounds.

    P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python tools/trace_wgrad.py
"""
import ctypes
import json
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
T = torch.randn(64, 48, device="cuda")
for _ in range(20):
    model.train_step_device(X, T, 0.5)
torch.cuda.synchronize()
lib = _p3d.lib()
lib.p3d_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(4096 * 8, np.uint64)
assert lib.p3d_debug_trace(buf.ctypes.data, buf.size) == 0
n = int(os.environ.get("NWG", "1500"))
t = buf[4096:4096 + 8 * n].astype(np.int64).reshape(n, 8)[:, :5]
t = t[t[:, 4] > 0]                       # workgroups of the launch (slot 4: workgroup start)
t = t[t[:, 4] >= t[:, 4].max() - 10000]  # (the last launch: within 100 us of its latest start)
t[:, 0] = t[:, 4]                        # slot 0 = the workgroup's start (a pair's second tile re-stamps 0)
t0 = t[:, 0].min()
us = (t - t0) / 100.0
q = lambda a: [round(float(np.quantile(a, f)), 2) for f in (0, 0.1, 0.5, 0.9, 1.0)]  # noqa: E731
print(json.dumps({"start": q(us[:, 0]), "staged_last_tile": q(us[:, 1]), "contracted": q(us[:, 2]), "done": q(us[:, 3]),
                  "stage_dur": q(us[:, 1] - us[:, 0]), "mfma_dur": q(us[:, 2] - us[:, 1]),
                  "adam_dur": q(us[:, 3] - us[:, 2]), "wg_dur": q(us[:, 3] - us[:, 0])}))
# dispatch rounds: histogram of start times in 1-us bins
h = np.histogram(us[:, 0], bins=np.arange(0, us[:, 3].max() + 1, 1.0))[0]
print("starts per us:", h.tolist())
