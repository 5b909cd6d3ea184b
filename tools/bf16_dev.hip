// Development harness for the cfg5 hidden-layer bf16 GEMM variants (not product code):
// packs operands with the library's own kernels and times each variant with HIP events
// over back-to-back launches.  Build: tools/bf16_dev.sh; driver: tools/bf16_dev.py.
#include "../3d-pose-baseline_amd/csrc/p3d_kernels.h"
#include "../3d-pose-baseline_amd/csrc/p3d_bf16.h"
#include "bf16_dev_kernels.h"

extern "C" int dev_pack_x(const float* x, int M, int K, unsigned short* out) {
  const int items = (M / 16) * (K / 32) * 64;
  k_x_to_bf16<<<(items + 255) / 256, 256>>>(x, M, K, out, M);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

extern "C" int dev_pack_w(const float* W, int K, int N, unsigned short* out) {
  const int64_t items = (int64_t)(N / 16) * (K / 32) * 64;
  k_pack_bf16<<<(unsigned)((items + 255) / 256), 256>>>(W, K, N, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

static void launch(int v, const GemmBf16Args& a, const GemmBf16SplitArgs& sa) {
  const unsigned g128 = (unsigned)((a.M / 128) * (a.N / 128));
  const unsigned t256 = (unsigned)((a.M / 256) * (a.N / 128));
  switch (v) {
    case 0: k_gemm_bf16p<64, 4, 8><<<g128, 512>>>(a); break;
    case 1: k_gemm_bf16s<3><<<2 * t256, 512>>>(sa); break;
    case 2: k_gemm_bf16w<2, 3><<<2 * t256, 256>>>(sa); break;
    case 3: k_gemm_bf16w<1, 6><<<2 * t256, 256>>>(sa); break;
    case 4: k_gemm_bf16w<1, 5><<<2 * t256, 256>>>(sa); break;
    case 5: k_gemm_bf16p<64, 4, 4><<<g128, 256>>>(a); break;
    case 6: k_gemm_bf16p<64, 4, 8, false, 1><<<g128, 512>>>(a); break;
    case 7: k_gemm_bf16p<64, 4, 8, false, 2><<<g128, 512>>>(a); break;
    case 8: k_gemm_bf16p<64, 4, 8, false, 3><<<g128, 512>>>(a); break;
    case 9: k_gemm_bf16p<64, 4, 8, false, 0, true><<<g128, 512>>>(a); break;
    case 10: k_gemm_bf16p<64, 4, 4, false, 0, true><<<g128, 256>>>(a); break;
    case 11: k_gemm_bf16p<64, 4, 8, true, 0, true><<<g128, 512>>>(a); break;
    case 12: k_gemm_bf16p<64, 4, 8, false, 2, true><<<g128, 512>>>(a); break;
    case 13: k_gemm_bf16k<4><<<g128, 512>>>(a); break;
    case 14: k_gemm_bf16k<3><<<g128, 512>>>(a); break;
    case 15: k_gemm_bf16k<5><<<g128, 512>>>(a); break;
    case 16: k_gemm_bf16k<3, 1><<<g128, 512>>>(a); break;
    case 17: k_gemm_bf16k<3, 2><<<g128, 512>>>(a); break;
    default: break;
  }
}

// avg microseconds per launch over iters back-to-back launches (after one untimed launch)
extern "C" float dev_run(int v, const unsigned short* A, const unsigned short* Bt, unsigned short* Y,
                         const float* bias, int M, int N, int K, float* part, unsigned* sync, int* err,
                         int iters) {
  GemmBf16Args a{};
  a.A = A; a.Bt = Bt; a.res = nullptr; a.Y = Y; a.M = M; a.N = N; a.K = K;
  a.epi.bias = bias; a.epi.inv = nullptr; a.epi.shift = nullptr; a.epi.relu = 0;
  GemmBf16SplitArgs sa{};
  sa.g = a; sa.part = part; sa.sync = sync; sa.err = err;
  launch(v, a, sa);
  if (hipDeviceSynchronize() != hipSuccess) return -1.f;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) launch(v, a, sa);
  (void)hipEventRecord(e1, 0);
  if (hipEventSynchronize(e1) != hipSuccess) return -2.f;
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 1000.f * ms / (float)iters;
}
