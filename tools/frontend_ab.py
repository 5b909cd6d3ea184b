"""Dev tool: FrameLifter per-frame host round trip (pinned H2D, one graph, D2H, sync) with its
body as one p3d_lift call vs the three calls p3d_normalize + forward + p3d_unnormalize, on one
box, alternating; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import data_pipeline as dp  # noqa: E402
import data_utils  # noqa: E402
import linear_model  # noqa: E402
import openpose_frontend as of  # noqa: E402


def three_steps(self):
    self.din.copy_(self.hin, non_blocking=True)
    dp.normalize(self.din, self.m2, self.s2, self.u2, out_dtype=self.torch.float32, out=self.x)
    self.model.forward_device(self.x, False, 1.0, out=self.y, ctr=0)
    dp.unnormalize(self.y, self.m3, self.s3, self.u3, self.p3.shape[1], out=self.p3)
    self.hout.copy_(self.p3, non_blocking=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    rng = np.random.default_rng(600)
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_fab", seed=5)
    use2, _ = data_utils.dimension_sets(2)
    _, ign3 = data_utils.dimension_sets(3)
    stats = (rng.uniform(200, 600, 64), rng.uniform(50, 150, 64), use2, rng.uniform(-400, 400, 96),
             rng.uniform(30, 300, 96), ign3)
    e = of.map_frames(rng.uniform(100, 900, (1, 36)))
    fl_lift = of.FrameLifter(m, *stats, batch=1)
    orig = of.FrameLifter._body
    of.FrameLifter._body = three_steps
    fl_three = of.FrameLifter(m, *stats, batch=1)
    of.FrameLifter._body = orig
    out = {"lift_us": [], "three_us": []}
    a = fl_lift.lift_mapped(e)
    b = fl_three.lift_mapped(e)
    out["identical"] = bool(np.array_equal(a, b))
    for _ in range(3):
        for key, fl in (("lift_us", fl_lift), ("three_us", fl_three)):
            for _ in range(100):
                fl.lift_mapped(e)
            t0 = time.perf_counter()
            for _ in range(n):
                fl.lift_mapped(e)
            out[key].append(round(1e6 * (time.perf_counter() - t0) / n, 2))
    # device-only: the bodies without the copies, as a graph each and as eager calls
    dev = m.device
    fl = fl_lift
    fl.din.copy_(torch.from_numpy(e).to(dev))

    def body_lift():
        of.lift(m, fl.din, fl.m2, fl.s2, fl.u2, fl.m3, fl.s3, fl.u3, out=fl.p3)

    def body_three():
        dp.normalize(fl.din, fl.m2, fl.s2, fl.u2, out_dtype=torch.float32, out=fl.x)
        m.forward_device(fl.x, False, 1.0, out=fl.y, ctr=0)
        dp.unnormalize(fl.y, fl.m3, fl.s3, fl.u3, fl.p3.shape[1], out=fl.p3)

    side = torch.cuda.Stream(dev)
    graphs = {}
    for key, body in (("lift", body_lift), ("three", body_three)):
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            body()
        torch.cuda.current_stream(dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            body()
        graphs[key] = (g, body)
    for key in ("lift", "three"):
        out["graph_%s_us" % key] = []
        out["eager_%s_us" % key] = []
    for _ in range(3):
        for key, (g, body) in graphs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                g.replay()
            torch.cuda.synchronize()
            out["graph_%s_us" % key].append(round(1e6 * (time.perf_counter() - t0) / n, 2))
            with torch.cuda.stream(torch.cuda.Stream(dev)):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(n):
                    body()
                torch.cuda.synchronize()
            out["eager_%s_us" % key].append(round(1e6 * (time.perf_counter() - t0) / n, 2))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
