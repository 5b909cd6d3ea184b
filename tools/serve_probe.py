"""Dev tool: throughput of p3d_serve (k_serve) vs steps per launch.

    python tools/serve_probe.py [steps_per_launch ...]
Prints, per launch size, the device time per launch (HIP events over 20 launches),
poses/s and the fp32 MFMA fraction of the whole launch (8,552,448 FLOP per pose).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import linear_model  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [8, 64, 240, 960]
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_probe", seed=3, max_batch=64)
    m.initialize(seed=3)
    flop = 8552448.0
    for nb in sizes:
        x = torch.randn((64 * nb, 32), device="cuda")
        y = torch.empty((64 * nb, 48), device="cuda")
        s = torch.cuda.current_stream()
        for _ in range(3):
            m.serve_device(x, out=y)
        torch.cuda.synchronize()
        m.serve_check()
        reps = max(3, min(50, 4000 // nb))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            m.serve_device(x, out=y)
        e1.record(s)
        torch.cuda.synchronize()
        m.serve_check()
        ms = e0.elapsed_time(e1) / reps
        pps = 64 * nb / (ms * 1e-3)
        print("steps/launch %5d: %8.3f ms/launch  %6.2f us/step  %.3f M poses/s  %.1f TF/s (%.3f of 157.3)" %
              (nb, ms, ms * 1e3 / nb, pps / 1e6, pps * flop / 1e12, pps * flop / 157.3e12), flush=True)
    m.close()


if __name__ == "__main__":
    main()
