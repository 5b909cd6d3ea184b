"""Reference point for the cfg5 GEMM: torch.matmul (hipBLASLt) bf16 [M, K] x [K, N]."""
import time
import torch

for M, N, K in [(1024, 4096, 4096), (4096, 4096, 4096), (8192, 1024, 1024)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        c = a @ b
    torch.cuda.synchronize()
    n = 200
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / n
    print("bf16 M=%d N=%d K=%d: %.1f us  %.0f TF/s" % (M, N, K, us, 2 * M * N * K / us / 1e6), flush=True)
    af, bf = a.float(), b.float()
    for _ in range(5):
        c = af @ bf
    torch.cuda.synchronize()
    e0.record()
    for _ in range(50):
        c = af @ bf
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 50
    print("fp32 M=%d N=%d K=%d: %.1f us  %.1f TF/s" % (M, N, K, us, 2 * M * N * K / us / 1e6), flush=True)
