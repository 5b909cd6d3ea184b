"""Dev probe: k_serve6 launch time (20 steps) with random vs all-zero weights and inputs.

The MFMA cycle counts do not depend on the operands, the clock the chip holds under load does
(MI355X_MICROARCH.md, DVFS give-back): a large gap means the contraction is clock-bound.
    python tools/serve_clock_probe.py [steps] [launches]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def time_launches(model, x, y, n):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        model.serve_device(x, out=y)
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1000.0 for a, b in ev)
    return round(ts[len(ts) // 2], 2), round(ts[0], 2)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    out = {}
    for kind in ("random", "zero"):
        m, _ = bench.make_model()
        x = torch.randn((64 * nb, 32), device="cuda")
        if kind == "zero":
            m.set_weights({k: np.zeros(v.shape, np.float32) for k, v in m.get_weights(include_moving=False).items()})
            x.zero_()
        y = torch.empty((64 * nb, 48), device="cuda")
        time_launches(m, x, y, 20)
        out[kind] = time_launches(m, x, y, n)
        m.close()
    print(json.dumps({"steps": nb, "median_min_us": out}))


if __name__ == "__main__":
    main()
