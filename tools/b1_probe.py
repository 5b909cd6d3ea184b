"""Batch-1 latency probe (cfg2 model): graph-replayed device forward, eager device forward,
LinearModel.step() from numpy.  Dev tool for the OpenPose front-end path."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

model, _ = bench.make_model()
B = int(os.environ.get("B1", "1"))
X = torch.randn(64, B, 32, device="cuda")
Y = torch.empty(64, B, 48, device="cuda")
for i in range(20):
    model.forward_device(X[i], False, 1.0, out=Y[i], ctr=0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(20):
    for i in range(64):
        model.forward_device(X[i], False, 1.0, out=Y[i], ctr=0)
torch.cuda.synchronize()
print("eager forward_device B=%d: %.2f us/step" % (B, (time.perf_counter() - t0) / 1280 * 1e6))
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    for i in range(64):
        model.forward_device(X[i], False, 1.0, out=Y[i], ctr=0)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st):
    for i in range(64):
        model.forward_device(X[i], False, 1.0, out=Y[i], ctr=0)
g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(20):
    g.replay()
torch.cuda.synchronize()
print("graph forward B=%d: %.2f us/step" % (B, (time.perf_counter() - t0) / 1280 * 1e6))
xs = np.random.default_rng(0).standard_normal((B, 32))
ts = np.zeros((B, 48))
for i in range(20):
    model.step(None, xs, ts, 1.0, isTraining=False)
t0 = time.perf_counter()
for i in range(500):
    model.step(None, xs, ts, 1.0, isTraining=False)
print("step() API B=%d: %.2f us/call" % (B, (time.perf_counter() - t0) / 500 * 1e6))
prof = bench.profile_kernels(model, lambda: [model.forward_device(X[i], False, 1.0, out=Y[i], ctr=0) for i in range(64)])
for k, v in prof.items():
    print(k, v)
model.close()
