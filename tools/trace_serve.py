"""Dev tool: phase timeline of k_serve from a -DP3D_TRACE build.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -DP3D_TRACE \\
        -o 3d-pose-baseline_amd/libp3d_trace.so 3d-pose-baseline_amd/csrc/p3d.hip
    P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python tools/trace_serve.py [steps]
Prints, for XCD group 0's rank-0 workgroup, each phase of its first steps: compute time
and barrier wait (wall_clock64 at 100 MHz), averaged over steps 2..7.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _p3d  # noqa: E402
import linear_model  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 240
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_probe", seed=3, max_batch=64)
    m.initialize(seed=3)
    x = torch.randn((64 * nb, 32), device="cuda")
    for _ in range(3):
        m.serve_device(x)
    torch.cuda.synchronize()
    lib = _p3d.lib()
    lib.p3d_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.p3d_debug_trace(buf.ctypes.data, buf.size) == 0
    P = 5
    for rr in (0, 1):
        t = buf[8192 + rr * 8192: 8192 + rr * 8192 + 8192].astype(np.int64).reshape(8, 8, 16, 8)
        acc = np.zeros((P, 4)); cnt = 0
        for x_ in range(8):
            for jl in range(2, 8):
                if t[x_, jl, 0, 0] == 0 and t[x_, jl, 1, 0] == 0:
                    continue
                for ph in range(P):
                    if t[x_, jl, ph, 0] == 0:   # k_serve5 has no phase 0
                        continue
                    b, c, w, k3, k4 = (t[x_, jl, ph, k] for k in (0, 1, 2, 3, 4))
                    if ph == 0 or k3 == 0:
                        acc[ph] += (c - b, 0, 0, w - c)
                    else:
                        acc[ph] += (k3 - b, k4 - k3, c - k4, w - c)
                cnt += 1
        acc /= max(cnt, 1) * 100.0
        f0 = 0 if t[:, :, 0, 0].any() else 1
        step = [(t[x_, jl + 1, f0, 0] - t[x_, jl, f0, 0]) / 100.0 for x_ in range(8) for jl in range(2, 7)
                if t[x_, jl + 1, f0, 0] and t[x_, jl, f0, 0]]
        print("rank %d: step %.2f us; per phase [contraction, K-combine, epilogue, barrier] us:" %
              (rr, float(np.mean(step)) if step else 0.0))
        for ph in range(P):
            print("   phase %d: %s" % (ph, np.round(acc[ph], 2)))
        # k_serve4 stamps: 5 = prologue requested, 7 = first k-group's MFMAs issued (its
        # operands arrived), 3 = contraction done; 6 = shader cycles of the ring loop
        sub = [(t[x_, jl, ph, 5] - t[x_, jl, ph, 0], t[x_, jl, ph, 7] - t[x_, jl, ph, 5],
                t[x_, jl, ph, 3] - t[x_, jl, ph, 7], t[x_, jl, ph, 6])
               for x_ in range(8) for jl in range(2, 8) for ph in range(1, P)
               if t[x_, jl, ph, 7] > t[x_, jl, ph, 5] > 0]
        if sub:
            a = np.mean(np.array(sub, dtype=np.float64), axis=0)
            print("   hidden contraction: prologue %.2f us, first fragments %.2f us, loop %.2f us "
                  "(%.0f shader cycles -> %.2f GHz)" % (a[0] / 100, a[1] / 100, a[2] / 100, a[3],
                                                        a[3] / ((a[1] + a[2]) / 100) / 1e3))
    m.close()


if __name__ == "__main__":
    main()
