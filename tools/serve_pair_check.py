"""Dev tool: the k_serve6 pair form (P3D_SERVE6_PAIR=1) against the single-unit form on the same
weights and inputs -- every row bit for bit (the same per-tile association), over repeated launches
(both flag banks) and row counts that leave some groups a unit past the last row.
    P3D_LIB=... python tools/serve_pair_check.py
Prints one JSON line; exits 1 on a mismatch."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import _p3d  # noqa: E402
import linear_model  # noqa: E402


def make(pair):
    os.environ["P3D_SERVE6_PAIR"] = "1" if pair else "0"
    return linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_pair_check", seed=3, max_batch=64)


def kname(m):
    buf = ctypes.create_string_buffer(256)
    _p3d.lib().p3d_kernel_name(m._h, 3, buf, 256)
    return buf.value.decode()


def main():
    m0, m1 = make(False), make(True)
    torch.manual_seed(0)
    out = {"cases": []}
    ok = True
    for B in (1280, 1200, 1100, 1281 - 64, 64 * 20, 1024, 1000, 960):
        x = torch.randn((B, 32), device="cuda")
        y0 = m0.serve_device(x).clone()
        ys = [m1.serve_device(x).clone() for _ in range(3)]
        torch.cuda.synchronize()
        m0.serve_check()
        m1.serve_check()
        same = all(bool(torch.equal(y, y0)) for y in ys)
        d = max(float((y - y0).abs().max()) for y in ys)
        case = {"B": B, "k0": kname(m0), "k1": kname(m1), "bitwise": same, "max_abs": d,
                "finite": bool(torch.isfinite(ys[0]).all())}
        out["cases"].append(case)
        ok = ok and same and case["finite"]
    out["ok"] = ok
    print(json.dumps(out))
    m0.close()
    m1.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
