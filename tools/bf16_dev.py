"""Development driver for tools/bf16_dev.hip (cfg5 hidden-layer bf16 GEMM variants).

Checks every variant against a float32 product of the same bf16-rounded operands, then times
them in interleaved rounds on one device (MI355X_MICROARCH / cdna guide §5.4 rule 24).
Usage: python tools/bf16_dev.py [--variants 0,1,2] [--rounds 5] [--iters 50] [--M 1024]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: "k_gemm_bf16p<64,4,8> 128x128", 1: "k_gemm_bf16s<3> 256x128 split2 8w",
         2: "k_gemm_bf16w<2,3> 256x128 split2 4w", 3: "k_gemm_bf16w<1,6>", 4: "k_gemm_bf16w<1,5>",
         5: "k_gemm_bf16p<64,4,4> 128x128 4w", 6: "bf16p<64,4,8> DIAG no-MFMA", 7: "bf16p DIAG no-DMA",
         8: "bf16p DIAG no-LDS-read", 9: "bf16p<64,4,8> asm reads", 10: "bf16p<64,4,4> asm reads",
         11: "bf16p<64,4,8> asm reads + prio", 12: "bf16p asm reads DIAG no-DMA",
         13: "k_gemm_bf16k<4> kg-split 64x64", 14: "k_gemm_bf16k<3>", 15: "k_gemm_bf16k<5>",
         16: "k_gemm_bf16k<3> K rotated per XCD group", 17: "k_gemm_bf16k<3> K rotated per WG%8"}


def unpack16(yp, M, N):
    r = np.arange(M)[:, None]
    c = np.arange(N)[None, :]
    ng = N // 32
    off = ((r >> 4) * ng + (c >> 5)) * 512 + ((r & 15) + ((c & 31) >> 3) * 16) * 8 + (c & 7)
    u = yp.reshape(-1)[off].astype(np.uint32) << 16
    return u.view(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4,5")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "bf16_dev.so"))
    vp = ctypes.c_void_p
    lib.dev_run.restype = ctypes.c_float
    lib.dev_run.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp,
                            ctypes.c_int]
    M, N, K = a.M, a.N, a.K
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.rand((M, K), generator=g) * 2 - 1).to(dev)
    w = ((torch.rand((K, N), generator=g) * 2 - 1) / 32).to(dev)
    bias = ((torch.rand((N,), generator=g) * 2 - 1) / 8).to(dev)
    A = torch.empty(M * K, dtype=torch.int16, device=dev)
    Bt = torch.empty(N * K, dtype=torch.int16, device=dev)
    assert lib.dev_pack_x(vp(x.data_ptr()), M, K, vp(A.data_ptr())) == 0
    assert lib.dev_pack_w(vp(w.data_ptr()), K, N, vp(Bt.data_ptr())) == 0
    ref = (x.to(torch.bfloat16).float() @ w.to(torch.bfloat16).float() + bias).cpu().numpy()
    T = (M // 256) * (N // 128)
    part = torch.zeros(T * 128 * 1024 // 4, dtype=torch.float32, device=dev)
    sync = torch.zeros(T * 64, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    Y = torch.empty(M * N, dtype=torch.int16, device=dev)
    variants = [int(v) for v in a.variants.split(",")]
    res = {"shape": [M, N, K], "flop": 2.0 * M * N * K, "variants": {}}
    for v in variants:
        Y.zero_()
        t = lib.dev_run(v, vp(A.data_ptr()), vp(Bt.data_ptr()), vp(Y.data_ptr()), vp(bias.data_ptr()), M, N, K,
                        vp(part.data_ptr()), vp(sync.data_ptr()), vp(err.data_ptr()), 1)
        torch.cuda.synchronize()
        y = unpack16(Y.cpu().numpy().view(np.uint16), M, N)
        d = np.abs(y - ref)
        rel = float(d.max() / np.abs(ref).max())
        ok = (v in (6, 7, 8, 12) or rel < 1e-2) and int(err.item()) == 0
        res["variants"][v] = {"name": NAMES.get(v, str(v)), "max_rel": rel, "err": int(err.item()), "ok": ok, "us": []}
        print("variant %d %-40s max|d|/max|ref| %.3e err %d %s" % (v, NAMES.get(v), rel, int(err.item()),
                                                                 "OK" if ok else "FAIL"), flush=True)
    for rd in range(a.rounds):
        for v in variants:
            t = lib.dev_run(v, vp(A.data_ptr()), vp(Bt.data_ptr()), vp(Y.data_ptr()), vp(bias.data_ptr()), M, N, K,
                            vp(part.data_ptr()), vp(sync.data_ptr()), vp(err.data_ptr()), a.iters)
            res["variants"][v]["us"].append(round(float(t), 3))
    for v in variants:
        us = sorted(res["variants"][v]["us"])
        med = us[len(us) // 2]
        res["variants"][v]["median_us"] = med
        res["variants"][v]["tflops"] = round(res["flop"] / med / 1e6, 1)
        res["variants"][v]["frac_bf16_2500"] = round(res["flop"] / med / 1e6 / 2500.0, 4)
        print("variant %d %-40s median %.2f us  min %.2f  %.0f TF/s  frac %.3f" % (
            v, NAMES.get(v), med, us[0], res["flop"] / med / 1e6, res["flop"] / med / 1e6 / 2500), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
