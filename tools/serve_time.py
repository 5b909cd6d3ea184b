"""Dev tool: event-timed k_serve6 launches of 20 batch-64 steps at cfg2 (the headline's launch),
median over 200 launches, and a check against a second launch shape's bits."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import linear_model  # noqa: E402


def main():
    nb = int(os.environ.get("NB", "20"))
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_st", seed=3, max_batch=64 * nb)
    x = torch.randn((64 * nb, 32), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    y = torch.empty((64 * nb, 48), device="cuda")
    for _ in range(20):
        m.serve_device(x, out=y)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    for a, b in ev:
        a.record()
        m.serve_device(x, out=y)
        b.record()
    torch.cuda.synchronize()
    m.serve_check()
    ts = sorted(a.elapsed_time(b) * 1000 for a, b in ev)
    ref = m.forward_device(x)
    err = float((y - ref).abs().max())
    print(json.dumps({"median_us": round(ts[len(ts) // 2], 2), "p10": round(ts[20], 2), "p90": round(ts[180], 2),
                      "max_err_vs_fwd": err}))


if __name__ == "__main__":
    main()
