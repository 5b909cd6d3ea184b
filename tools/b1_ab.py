"""Dev tool: device time of one batch-1 cfg2 forward under the library P3D_LIB names (tools/lib_ab.py
runs it alternately for two builds): a HIP graph of 50 forwards replayed back to back (bench.py's
forward_b1 measurement), plus the dispatch-attached average of the forward's kernels.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    model, _ = bench.make_model()
    x = torch.from_numpy(np.random.default_rng(7).standard_normal((1, bench.IN)).astype(np.float32)).cuda()
    y = torch.empty((1, bench.OUT), dtype=torch.float32, device="cuda")
    fwd = lambda: model.forward_device(x, False, 1.0, out=y, ctr=0)   # noqa: E731
    for _ in range(20):
        fwd()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(50):
            fwd()
    for _ in range(5):
        g.replay()
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res.append(round(1000.0 * e0.elapsed_time(e1) / 500, 3))
    prof = bench.profile_kernels(model, lambda: [fwd() for _ in range(100)])
    print(json.dumps({"us_per_forward": sorted(res)[len(res) // 2], "repeats_us": res,
                      "kernels_us": {k: round(v[1], 3) for k, v in prof.items()}}))
    model.close()


if __name__ == "__main__":
    main()
