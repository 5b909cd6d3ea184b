"""Probe: does touching N dummy streams before the S=4 run change its concurrency?"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
torch.cuda.set_device(0)
import streams_sweep2 as sw  # noqa: E402

pre = int(sys.argv[1])
dummy = [torch.cuda.Stream() for _ in range(pre)]
for st in dummy:
    with torch.cuda.stream(st):
        torch.zeros(16, device="cuda").add_(1)
torch.cuda.synchronize()
for k in range(2):
    print("pre=%d run %d S=4" % (pre, k), ["%.2f" % v for v in sw.run(4, 240)], flush=True)
