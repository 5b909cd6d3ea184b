"""Measured error distribution of the bf16 cfg5 path vs the oracle's bf16 emulation
(tests/test_gpu_parity.py::test_bf16_inference_matches_emulated_oracle sets its tolerances
from this).  Prints max / mean / p99.9 of |y - ref| relative to max|ref| per case."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-pose-baseline_amd")]
import linear_model  # noqa: E402
from oracle import ref_mlp  # noqa: E402

for L, N, B in [(256, 2, 128), (512, 1, 200), (4096, 4, 1024)]:
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=N, residual=True, batch_norm=True)
    for seed in (1, 5, 9):
        st = ref_mlp.init_state(cfg, seed=seed, bn_seed=seed + 1)
        m = linear_model.LinearModel(L, N, True, True, False, B, 1e-3, "/tmp/p3d_probe", dtype="bfloat16",
                                     seed=3, max_batch=B)
        m.set_weights({**st.params, **st.moving})
        x = np.random.default_rng(B + seed).standard_normal((B, 32)).astype(np.float32)
        y = m.forward_device(torch.from_numpy(x).cuda()).cpu().numpy()
        ref = ref_mlp.forward_bf16(st, x, acc=np.float32 if L >= 4096 else np.float64)
        scale = np.abs(ref).max()
        err = np.abs(y - ref) / scale
        ref32, _ = ref_mlp.forward(st, x, False)
        print("L=%d N=%d B=%d seed=%d  max %.3e  mean %.3e  p99.9 %.3e  exact %.3f  vs-fp32 mean rel %.3e"
              % (L, N, B, seed, err.max(), err.mean(), np.quantile(err, 0.999), np.mean(err == 0),
                 np.abs(y - ref32).mean() / np.abs(ref32).mean()), flush=True)
        m.close()
