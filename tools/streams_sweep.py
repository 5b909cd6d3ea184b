"""Throughput of independent batch-64 forward passes vs stream count / graph size.
Dev tool: python tools/streams_sweep.py"""
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


def run(S, G, reps=3, steps=2400, graph=True):
    model, _ = bench.make_model(max_batch=64 * S)
    X = torch.randn(G, 64, 32, device="cuda")
    Y = torch.empty(G, 64, 48, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(S)]

    def multi():
        cur = torch.cuda.current_stream()
        for st in streams:
            st.wait_stream(cur)
        for j, st in enumerate(streams):
            with torch.cuda.stream(st):
                for i in range(j, G, S):
                    model.forward_device(X[i], False, 1.0, out=Y[i], ctr=0, ws_row=64 * j)
        for st in streams:
            cur.wait_stream(st)

    multi()
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            multi()
        fn = g.replay
    else:
        fn = multi
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


import sys as _s
WK = os.environ.get("P3D_INFER_WK", "16")
for S, G in [(1, 240), (2, 240), (3, 240), (4, 240), (8, 240)]:
    r = run(S, G)
    print("WK=%s S=%2d G=%3d graph  Mposes/s %s" % (WK, S, G, " ".join("%.2f" % v for v in r)), flush=True)
