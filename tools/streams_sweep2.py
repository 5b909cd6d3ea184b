"""Independent batch-64 forward passes on S streams, each stream replaying its OWN graph
(one graph per stream -> one hardware queue per stream).  Dev tool."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

torch.cuda.set_device(0)


def run(S, G, reps=3, steps=2400):
    model, _ = bench.make_model(max_batch=64 * S)
    X = torch.randn(G, 64, 32, device="cuda")
    Y = torch.empty(G, 64, 48, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(S)]
    graphs = []
    per = G // S
    for j, st in enumerate(streams):
        with torch.cuda.stream(st):
            for i in range(per):
                model.forward_device(X[j * per + i], False, 1.0, out=Y[j * per + i], ctr=0, ws_row=64 * j)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for i in range(per):
                model.forward_device(X[j * per + i], False, 1.0, out=Y[j * per + i], ctr=0, ws_row=64 * j)
        graphs.append(g)
    torch.cuda.synchronize()

    def fn():
        for j, st in enumerate(streams):
            with torch.cuda.stream(st):
                graphs[j].replay()

    res = []
    for _ in range(reps):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps // G):
            fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.append((steps // G) * G * 64 / dt / 1e6)
    model.close()
    return res


if __name__ == "__main__":
  WK = os.environ.get("P3D_INFER_WK", "default")
  for S, G in [(1, 240), (2, 240), (3, 240), (4, 240), (6, 240), (8, 240)]:
      r = run(S, G)
      print("WK=%s S=%2d G=%3d per-stream graphs  Mposes/s %s" % (WK, S, G, " ".join("%.2f" % v for v in r)),
            flush=True)
