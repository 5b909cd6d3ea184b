// Kernel-argument probe for k_gemv_chain's GemvChain block (1,880 B): every workgroup of a
// 256-workgroup launch decodes its layer / tile and the fields it reads, exactly as the chain does,
// and writes them (no other memory access) for the host to compare with what it passed -- through
// both launch paths the library uses (<<<>>> and hipExtLaunchKernelGGL with events).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/chain_kernarg_probe tools/chain_kernarg_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include "../3d-pose-baseline_amd/csrc/p3d_kernels.h"
#include "../3d-pose-baseline_amd/csrc/p3d_serve.h"
#include "../3d-pose-baseline_amd/csrc/p3d_gemv.h"

typedef unsigned long long u64;
__global__ __launch_bounds__(1024) void k_probe(GemvChain c, u64* out) {
  if (threadIdx.x) return;
  const int b = blockIdx.x, l = 1 + b / c.T, t = b - (l - 1) * c.T;
  GemvArgs p = c.ly[0];
#pragma unroll
  for (int k = 1; k < P3D_GEMV_CHAIN_MAXH; ++k)
    if (k == l - 1) p = c.ly[k];
  u64* o = out + b * 16;
  o[0] = c.T; o[1] = c.H; o[2] = l; o[3] = t; o[4] = p.K; o[5] = p.N; o[6] = p.M; o[7] = (u64)p.Wf;
  o[8] = (u64)c.hand; o[9] = (u64)c.epoch; o[10] = (u64)c.out.Y; o[11] = (u64)c.out.Wf; o[12] = (u64)c.in.X;
  o[13] = c.res; o[14] = (u64)c.err; o[15] = (u64)p.bias;
}

int main() {
  GemvChain c{};
  const int H = 4, T = 64;
  c.H = H; c.T = T; c.res = 1;
  c.hand = (float*)0x1111000ull; c.epoch = (unsigned*)0x2222000ull; c.err = (int*)0x3333000ull;
  c.in.X = (const float*)0x4444000ull; c.out.Y = (float*)0x5555000ull; c.out.Wf = (const float*)0x6666000ull;
  for (int l = 0; l < H; ++l) {
    c.ly[l].K = 1024; c.ly[l].N = 1024; c.ly[l].M = 1;
    c.ly[l].Wf = (const float*)(0x7000000ull + 0x100000ull * l);
    c.ly[l].bias = (const float*)(0x8000000ull + 0x100000ull * l);
  }
  u64* d = nullptr;
  if (hipMalloc(&d, 256 * 16 * 8) != hipSuccess) return 2;
  int bad = 0;
  for (int mode = 0; mode < 2; ++mode) {
    hipMemset(d, 0, 256 * 16 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    if (mode == 0) k_probe<<<dim3(256), dim3(1024)>>>(c, d);
    else hipExtLaunchKernelGGL(k_probe, dim3(256), dim3(1024), 0, 0, e0, e1, 0, c, d);
    if (hipDeviceSynchronize() != hipSuccess) { printf("sync failed\n"); return 3; }
    u64 h[256 * 16];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int b = 0; b < 256; ++b) {
      const u64* o = h + b * 16;
      const int l = 1 + b / T, t = b % T;
      const u64 want[16] = {(u64)T, (u64)H, (u64)l, (u64)t, 1024, 1024, 1, (u64)c.ly[l - 1].Wf, (u64)c.hand,
                            (u64)c.epoch, (u64)c.out.Y, (u64)c.out.Wf, (u64)c.in.X, 1, (u64)c.err, (u64)c.ly[l - 1].bias};
      for (int k = 0; k < 16; ++k)
        if (o[k] != want[k]) {
          if (bad < 20) printf("mode %d block %d field %d: got %llx want %llx\n", mode, b, k, o[k], want[k]);
          ++bad;
        }
    }
  }
  printf("sizeof(GemvChain)=%zu mismatches=%d\n", sizeof(GemvChain), bad);
  return bad ? 1 : 0;
}
