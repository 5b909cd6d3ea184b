"""Dev tool: timeline of one k_gemv_chain launch (the batch-1 forward) from a -DP3D_TRACE build.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -DP3D_TRACE \\
        -o 3d-pose-baseline_amd/libp3d_trace.so 3d-pose-baseline_amd/csrc/p3d.hip
    P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python tools/trace_chain.py [reps]

Per hidden layer: median / max over its workgroups of start, input ready (input layer computed
or the previous layer gathered), contracted, published; then workgroup 0's output-layer gather and
end (wave 0's gather, its contraction, the reduction barrier, the epilogue's end).  Times in us from the earliest workgroup start (wall_clock64, 100 MHz)."""
import ctypes
import json
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_probe", seed=3, max_batch=64)
    x = torch.randn((1, 32), device="cuda")
    lib = _p3d.lib()
    lib.p3d_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = []
    for rep in range(reps):
        m.forward_device(x, False, 1.0, ctr=0)
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 8, np.uint64)
        assert lib.p3d_debug_trace(buf.ctypes.data, buf.size) == 0
        t = buf[:256 * 8].astype(np.int64).reshape(256, 8)
        t0 = t[:, 0].min()
        us = (t - t0) / 100.0
        layers = {}
        for l in range(4):
            blk = us[64 * l:64 * (l + 1)]
            layers["layer%d" % (l + 1)] = {name: [round(float(np.median(blk[:, k])), 2), round(float(blk[:, k].max()), 2)]
                                           for k, name in enumerate(("start", "input", "contracted", "published"))}
        layers["layer2"]["in_published"] = [round(float(np.median(us[64:128, 4])), 2), round(float(us[64:128, 4].max()), 2)]
        layers["args_ready"] = [round(float(np.median(us[3:256, 5])), 2), round(float(us[3:256, 5].max()), 2)]
        layers["out"] = {"gathered": round(float(us[0, 4]), 2), "contracted": round(float(us[0, 6]), 2),
                         "barrier": round(float(us[0, 7]), 2), "end": round(float(us[0, 5]), 2)}
        out.append(layers)
        print(json.dumps({"rep": rep, **layers}), flush=True)


if __name__ == "__main__":
    main()
