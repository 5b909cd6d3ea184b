"""Dev tool: a few eager cfg3 training steps (no HIP graph), for rocprofv3 --pmc passes
of the training kernels (graph replays under counter collection serialise badly).

    rocprofv3 --pmc FETCH_SIZE -d out -o run -- python3 tools/train_probe.py [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.cuda.set_device(0)
    m, _ = bench.make_model()
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.standard_normal((64, 32)).astype(np.float32)).cuda()
    t = torch.from_numpy(rng.standard_normal((64, 48)).astype(np.float32)).cuda()
    y = torch.empty((64, 48), device="cuda")
    for _ in range(steps):
        m.train_step_device(x, t, 0.5, out=y)
    torch.cuda.synchronize()
    print("loss", float(m._loss_dev.item()))
    m.close()


if __name__ == "__main__":
    main()
