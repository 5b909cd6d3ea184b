"""Where the wall time of one 20-step serve launch goes on the host (dev probe).

    python tools/serve_host_probe.py [--spin]

--spin sets hipDeviceScheduleSpin before the HIP context exists (the host thread spins on the
completion signal instead of yielding).  Prints medians over 200 repetitions of: the bench's
timed region (serve_device + torch.cuda.synchronize), the same launch through a prebuilt ctypes
call, and with hipStreamSynchronize instead of torch's device synchronize."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-pose-baseline_amd")]

hip = ctypes.CDLL("libamdhip64.so")
if "--spin" in sys.argv:
    assert hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0          # hipDeviceScheduleSpin

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _p3d  # noqa: E402
import linear_model  # noqa: E402


def med(fn, n=200):
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return round(1e6 * ts[n // 2], 2)


m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_probe", seed=3, max_batch=64)
x = torch.randn((1280, 32), device="cuda")
y = torch.empty((1280, 48), device="cuda")
for _ in range(150):
    m.serve_device(x, out=y)
torch.cuda.synchronize()
lib = _p3d.lib()
h, xp, yp, st = m._h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(m.stream())
serve = lib.p3d_serve
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
out = {
    "spin": "--spin" in sys.argv,
    "bench_region": med(lambda: (m.serve_device(x, out=y), torch.cuda.synchronize())),
    "ctypes_launch_torch_sync": med(lambda: (serve(h, xp, 1280, yp, st), torch.cuda.synchronize())),
    "ctypes_launch_stream_sync": med(lambda: (serve(h, xp, 1280, yp, st), hip.hipStreamSynchronize(st))),
    "enqueue_only": med(lambda: serve(h, xp, 1280, yp, st)),
    "idle_sync": med(torch.cuda.synchronize),
}
print(out)
m.close()
