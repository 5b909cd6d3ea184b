"""Per-kernel times of one large-M (cfg4 chunk) inference forward.  Dev probe."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

M = int(os.environ.get("BIG_M", "8192"))
model, _ = bench.make_model(max_batch=M)
X = torch.randn(M, 32, device="cuda")
Y = torch.empty(M, 48, device="cuda")
for _ in range(5):
    model.forward_device(X, False, 1.0, out=Y, ctr=0)
torch.cuda.synchronize()
prof = bench.profile_kernels(model, lambda: [model.forward_device(X, False, 1.0, out=Y, ctr=0) for _ in range(20)])
for k, v in prof.items():
    print("%-22s n=%4d avg %8.2f us  min %8.2f" % (k, v[0], v[1], v[2]))
model.close()
