"""Phase timestamps of the fused weight-gradient launch (k_wgrad_multi) of the cfg3 training step
(dev tool).  Needs the tracing build (-DP3D_TRACE):
    P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python tools/trace_wgrad.py
Per workgroup (P3D_WG_STAMP, p3d_layers.h): 4 entry, 0 tile start, 1 operands staged in LDS,
2 contraction done, 3 Adam + re-pack stores acknowledged.  Prints the quantiles of each stamp from
the launch's earliest entry, the per-phase durations, and how many tiles are in each phase over time
(the HBM-bound Adam phase's concurrency is what the launch's bandwidth follows).  One JSON line each.
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


def main():
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
    nwg = int(os.environ.get("P3D_TRACE_NWG", "1056"))
    t = buf[4096:4096 + nwg * 8].astype(np.int64).reshape(nwg, 8)
    t0 = t[:, 4].min()
    us = lambda v: (v - t0) / 100.0   # noqa: E731  (100 MHz wall clock)
    q = lambda a: [round(float(np.quantile(a, p)), 2) for p in (0.0, 0.1, 0.5, 0.9, 1.0)]   # noqa: E731
    out = {"workgroups": nwg}
    for k, n in ((4, "entry"), (0, "tile_start"), (1, "staged"), (2, "contracted"), (3, "adam_done")):
        out[n + "_q"] = q(us(t[:, k]))
    out["stage_us_q"] = q((t[:, 1] - t[:, 0]) / 100.0)
    out["contract_us_q"] = q((t[:, 2] - t[:, 1]) / 100.0)
    out["adam_us_q"] = q((t[:, 3] - t[:, 2]) / 100.0)
    end = us(t[:, 3]).max()
    grid = np.arange(0.0, end + 1.0, 1.0)
    in_adam = [int(((us(t[:, 2]) <= g) & (us(t[:, 3]) > g)).sum()) for g in grid]
    in_stage = [int(((us(t[:, 0]) <= g) & (us(t[:, 1]) > g)).sum()) for g in grid]
    out["launch_end_us"] = round(float(end), 2)
    out["tiles_in_adam_per_us"] = in_adam
    out["tiles_staging_per_us"] = in_stage
    print(json.dumps(out))
    model.close()


if __name__ == "__main__":
    main()
