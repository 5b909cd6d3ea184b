// kbench.hip -- design-space microbenchmark for the hidden-layer forward kernel
// (M=64, K=N=1024, fp32, BN-eval + ReLU + residual epilogue).  Dev tool, not product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/kbench tools/kbench.hip && tools/kbench
//
// Every variant is validated against an fp64 host reference, then timed as
// (a) 400 back-to-back launches bracketed by one event pair (per-launch incl. boundary)
// (b) one event pair per launch (kernel-only estimate).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <string>
#include <functional>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(ck_), __FILE__, __LINE__); exit(1);} } while (0)

struct Args {
  const float* X; int ldx; const float* Wt; int ldw; const float* bias;
  const float* gamma; const float* beta; const float* mm; const float* mv; float eps;
  const float* res; float* Y; int M, K, N;
};

__device__ __forceinline__ float colsum16(float v) { v += __shfl_xor(v, 16, 64); v += __shfl_xor(v, 32, 64); return v; }

// Generic NT core with NACC independent accumulator chains (e-parity split)
template <int RS, int DEPTH, int NACC>
__device__ __forceinline__ void core(const float* __restrict__ A, int lda, int M, int m0, const float* __restrict__ Bt,
                                     int ldb, int N, int n0, int gb, int ge, f32x4 (&acc)[NACC][RS]) {
  const int lane = threadIdx.x & 63, i = lane & 15, q = lane >> 4;
  const float* pa[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) { int r = m0 + 16 * s + i; r = r < M ? r : M - 1; pa[s] = A + (size_t)r * lda + 4 * q; }
  int c = n0 + i; c = c < N ? c : N - 1;
  const float* pb = Bt + (size_t)c * ldb + 4 * q;
  const int ng = ge - gb;
  if (ng <= 0) return;
  f32x4 ra[DEPTH][RS], rb[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const int g = gb + (d < ng ? d : ng - 1);
#pragma unroll
    for (int s = 0; s < RS; ++s) ra[d][s] = *(const f32x4*)(pa[s] + 16 * g);
    rb[d] = *(const f32x4*)(pb + 16 * g);
  }
  for (int g0 = 0; g0 < ng; g0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int gi = g0 + d;
      if (gi < ng) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int s = 0; s < RS; ++s)
            acc[e % NACC][s] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][s][e], rb[d][e], acc[e % NACC][s], 0, 0, 0);
        if (gi + DEPTH < ng) {   // only issue real loads (DEPTH >= ng -> none)
          const int gn = gb + gi + DEPTH;
#pragma unroll
          for (int s = 0; s < RS; ++s) ra[d][s] = *(const f32x4*)(pa[s] + 16 * gn);
          rb[d] = *(const f32x4*)(pb + 16 * gn);
        }
      }
    }
  }
}

template <int RS, int WK, int DEPTH, int NACC, bool PRE>
__global__ __launch_bounds__(64 * WK) void kx(Args p) {
  __shared__ f32x4 red[(WK > 1) ? (WK - 1) * RS * 64 : 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 16 * RS;
  const int col = n0 + i;
  // optional epilogue prefetch (wave 0 only needs them)
  float b = 0, inv = 1, shift = 0, rv[RS][4];
  if (PRE && w == 0) {
    b = p.bias[col];
    const float g = p.gamma[col], be = p.beta[col], mu = p.mm[col], va = p.mv[col];
    inv = (1.0f / sqrtf(va + p.eps)) * g;
    shift = be - mu * inv;
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) rv[s][r] = p.res[(size_t)(m0 + 16 * s + 4 * q + r) * p.N + col];
  }
  const int ngt = p.K >> 4;
  const int gb = (ngt * w) / WK, ge = (ngt * (w + 1)) / WK;
  f32x4 acc[NACC][RS];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[a][s] = f32x4{0, 0, 0, 0};
  core<RS, DEPTH, NACC>(p.X, p.ldx, p.M, m0, p.Wt, p.ldw, p.N, n0, gb, ge, acc);
#pragma unroll
  for (int a = 1; a < NACC; ++a)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[0][s] += acc[a][s];
  if (WK > 1) {
    if (w > 0) {
#pragma unroll
      for (int s = 0; s < RS; ++s) red[((w - 1) * RS + s) * 64 + lane] = acc[0][s];
    }
    __syncthreads();
    if (w > 0) return;
#pragma unroll
    for (int u = 1; u < WK; ++u)
#pragma unroll
      for (int s = 0; s < RS; ++s) acc[0][s] += red[((u - 1) * RS + s) * 64 + lane];
  }
  if (!PRE) {
    b = p.bias[col];
    const float g = p.gamma[col], be = p.beta[col], mu = p.mm[col], va = p.mv[col];
    inv = (1.0f / sqrtf(va + p.eps)) * g;
    shift = be - mu * inv;
  }
#pragma unroll
  for (int s = 0; s < RS; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * s + 4 * q + r;
      float y = (acc[0][s][r] + b) * inv + shift;
      y = fmaxf(y, 0.f);
      y += PRE ? rv[s][r] : p.res[(size_t)row * p.N + col];
      p.Y[(size_t)row * p.N + col] = y;
    }
}

__global__ void knull(float* y) { if (threadIdx.x == 0 && blockIdx.x == 0 && y[0] == 12345.f) y[0] = 0; }

struct Variant { std::string name; std::function<void(const Args&, hipStream_t)> launch; };
const float* g_Wbase;

// ---- packed ("fragment-major") layouts: every operand load is 1 KB contiguous per wave
// Ap[rt][g][lane][4] = X[16rt+i][16g+4q+e], Bp[ct][g][lane][4] = Wt[16ct+i][16g+4q+e]
template <int WK, int DEPTH, int NACC, int MODE>   // MODE 0 full, 1 loads-only, 2 mfma-only
__global__ __launch_bounds__(64 * WK) void kp(Args p, const float* __restrict__ Ap, const float* __restrict__ Bp) {
  __shared__ f32x4 red[(WK > 1) ? (WK - 1) * 64 : 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, q = lane >> 4;
  const int ct = blockIdx.x, rt = blockIdx.y;
  const int n0 = ct * 16, m0 = rt * 16;
  const int col = n0 + i;
  float b, inv, shift, rv[4];
  if (w == 0) {
    b = p.bias[col];
    const float g = p.gamma[col], be = p.beta[col], mu = p.mm[col], va = p.mv[col];
    inv = (1.0f / sqrtf(va + p.eps)) * g;
    shift = be - mu * inv;
#pragma unroll
    for (int r = 0; r < 4; ++r) rv[r] = p.res[(size_t)(m0 + 4 * q + r) * p.N + col];
  }
  const int ngt = p.K >> 4;
  const int gb = (ngt * w) / WK, ng = (ngt * (w + 1)) / WK - gb;
  const f32x4* pa = (const f32x4*)Ap + ((size_t)rt * ngt + gb) * 64 + lane;
  const f32x4* pb = (const f32x4*)Bp + ((size_t)ct * ngt + gb) * 64 + lane;
  f32x4 acc[NACC];
#pragma unroll
  for (int a = 0; a < NACC; ++a) acc[a] = f32x4{0, 0, 0, 0};
  f32x4 ra[DEPTH], rb[DEPTH];
  if (MODE == 2) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) { ra[d] = f32x4{(float)lane, 1, 2, 3}; rb[d] = f32x4{1, (float)w, 1, 1}; }
  } else {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) { const int g = d < ng ? d : ng - 1; ra[d] = pa[g * 64]; rb[d] = pb[g * 64]; }
  }
  for (int g0 = 0; g0 < ng; g0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int gi = g0 + d;
      if (gi < ng) {
        if (MODE == 1) {
          acc[0] += ra[d] * rb[d];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[e % NACC] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][e], rb[d][e], acc[e % NACC], 0, 0, 0);
        }
        if (MODE != 2 && gi + DEPTH < ng) { ra[d] = pa[(gi + DEPTH) * 64]; rb[d] = pb[(gi + DEPTH) * 64]; }
      }
    }
  }
#pragma unroll
  for (int a = 1; a < NACC; ++a) acc[0] += acc[a];
  if (WK > 1) {
    if (w > 0) red[(w - 1) * 64 + lane] = acc[0];
    __syncthreads();
    if (w > 0) return;
#pragma unroll
    for (int u = 1; u < WK; ++u) acc[0] += red[(u - 1) * 64 + lane];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + 4 * q + r;
    float y = (acc[0][r] + b) * inv + shift;
    y = fmaxf(y, 0.f) + rv[r];
    p.Y[(size_t)row * p.N + col] = y;
  }
}

__global__ void knull0() {}
__global__ void knull1(const float* x, float* y) { float v = x[blockIdx.x * 256 + threadIdx.x]; if (v == 12345.f) y[0] = v; }

float* g_Ap; float* g_Bp;  // packed copies (layer 0); B rotated by layer index below
template <int WK, int DEPTH, int NACC, int MODE>
Variant mkp(const char* name) {
  return {name, [](const Args& a, hipStream_t st) {
            const size_t li = (a.Wt - g_Wbase) / ((size_t)a.N * a.K);
            kp<WK, DEPTH, NACC, MODE><<<dim3(a.N / 16, a.M / 16), 64 * WK, 0, st>>>(a, g_Ap, g_Bp + li * (size_t)a.N * a.K);
          }};
}


template <int RS, int WK, int DEPTH, int NACC, bool PRE>
Variant mk(const char* name) {
  return {name, [](const Args& a, hipStream_t st) {
            kx<RS, WK, DEPTH, NACC, PRE><<<dim3(a.N / 16, (a.M + 16 * RS - 1) / (16 * RS)), 64 * WK, 0, st>>>(a);
          }};
}

int main(int argc, char** argv) {
  const int M = 64, K = 1024, N = 1024;
  const int NL = 4;  // rotate over 4 distinct layers' weights so W comes from L2/MALL like the real chain
  std::vector<float> hX(M * K), hW(NL * (size_t)N * K), hb(N), hg(N), hbe(N), hm(N), hv(N), hr(M * N);
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& v : hX) v = rnd();
  for (auto& v : hW) v = rnd() * 0.05f;
  for (int j = 0; j < N; ++j) { hb[j] = rnd(); hg[j] = 1 + 0.5f * rnd(); hbe[j] = 0.1f * rnd(); hm[j] = 0.1f * rnd(); hv[j] = 1.2f + 0.7f * rnd(); }
  for (auto& v : hr) v = rnd();
  float *X, *W, *b, *g, *be, *mm, *mv, *r, *Y;
  CK(hipMalloc(&X, M * K * 4)); CK(hipMalloc(&W, hW.size() * 4)); CK(hipMalloc(&b, N * 4)); CK(hipMalloc(&g, N * 4));
  CK(hipMalloc(&be, N * 4)); CK(hipMalloc(&mm, N * 4)); CK(hipMalloc(&mv, N * 4)); CK(hipMalloc(&r, M * N * 4));
  CK(hipMalloc(&Y, M * N * 4));
  CK(hipMemcpy(X, hX.data(), M * K * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, hb.data(), N * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(g, hg.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(be, hbe.data(), N * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(mm, hm.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(mv, hv.data(), N * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(r, hr.data(), M * N * 4, hipMemcpyHostToDevice));
  g_Wbase = W;
  {
    std::vector<float> ap(M * K), bp(hW.size());
    const int NG = K / 16;
    for (int rt = 0; rt < M / 16; ++rt) for (int g = 0; g < NG; ++g) for (int l = 0; l < 64; ++l) for (int e = 0; e < 4; ++e)
      ap[(((size_t)rt * NG + g) * 64 + l) * 4 + e] = hX[(16 * rt + (l & 15)) * K + 16 * g + 4 * (l >> 4) + e];
    for (int li = 0; li < NL; ++li)
      for (int ct = 0; ct < N / 16; ++ct) for (int g = 0; g < NG; ++g) for (int l = 0; l < 64; ++l) for (int e = 0; e < 4; ++e)
        bp[(size_t)li * N * K + (((size_t)ct * NG + g) * 64 + l) * 4 + e] = hW[(size_t)li * N * K + (size_t)(16 * ct + (l & 15)) * K + 16 * g + 4 * (l >> 4) + e];
    CK(hipMalloc(&g_Ap, ap.size() * 4)); CK(hipMalloc(&g_Bp, bp.size() * 4));
    CK(hipMemcpy(g_Ap, ap.data(), ap.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(g_Bp, bp.data(), bp.size() * 4, hipMemcpyHostToDevice));
  }
  // reference for layer 0 (Wt layout [N][K])
  std::vector<double> ref(M * N);
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      double s = 0;
      for (int k = 0; k < K; ++k) s += (double)hX[m * K + k] * hW[(size_t)n * K + k];
      double inv = 1.0 / sqrt((double)hv[n] + 1e-3) * hg[n];
      double y = (s + hb[n]) * inv + (hbe[n] - hm[n] * inv);
      ref[m * N + n] = (y > 0 ? y : 0) + hr[m * N + n];
    }
  std::vector<Variant> vs = {
      mk<1, 4, 8, 1, false>("RS1 WK4 D8 acc1 (prod)"),
      mkp<4, 16, 2, 0>("PACK WK4 D16 acc2"),
      mkp<4, 8, 2, 0>("PACK WK4 D8 acc2"),
      mkp<8, 8, 2, 0>("PACK WK8 D8 acc2"),
      mkp<16, 4, 2, 0>("PACK WK16 D4 acc2"),
      mkp<4, 16, 2, 1>("PACK WK4 loads-only (bad err ok)"),
      mkp<4, 16, 2, 2>("PACK WK4 mfma-only (bad err ok)"),
      mkp<16, 4, 2, 1>("PACK WK16 loads-only (bad err)"),
      mk<1, 4, 16, 1, false>("RS1 WK4 D16 acc1"),
      mk<1, 4, 16, 2, true>("RS1 WK4 D16 acc2 pre"),
      mk<1, 4, 8, 2, true>("RS1 WK4 D8 acc2 pre"),
      mk<1, 8, 8, 2, true>("RS1 WK8 D8 acc2 pre"),
      mk<1, 16, 4, 2, true>("RS1 WK16 D4 acc2 pre"),
      mk<2, 4, 16, 1, true>("RS2 WK4 D16 pre"),
      mk<2, 8, 8, 1, true>("RS2 WK8 D8 pre"),
      mk<4, 4, 8, 1, true>("RS4 WK4 D8 pre"),
      mk<4, 8, 8, 1, true>("RS4 WK8 D8 pre"),
      mk<4, 16, 4, 1, true>("RS4 WK16 D4 pre"),
  };
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int ITERS = 400;
  std::vector<hipEvent_t> evs(2 * ITERS);
  for (auto& e : evs) CK(hipEventCreate(&e));
  // null kernel reference
  {
    for (int it = 0; it < 50; ++it) knull<<<256, 256, 0, st>>>(Y);
    CK(hipEventRecord(e0, st));
    for (int it = 0; it < ITERS; ++it) knull<<<256, 256, 0, st>>>(Y);
    CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s back-to-back %8.3f us/launch\n", "null kernel 256x256", 1000 * ms / ITERS);
    for (int grid : {1, 64, 256, 1024}) {
      for (int pass = 0; pass < 2; ++pass) {
        CK(hipEventRecord(e0, st));
        for (int it = 0; it < ITERS; ++it) { if (pass == 0) knull0<<<grid, 256, 0, st>>>(); else knull1<<<grid, 256, 0, st>>>(X, Y); }
        CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("null%d grid %5d              back-to-back %8.3f us/launch\n", pass, grid, 1000 * ms / ITERS);
      }
    }
  }
  for (auto& v : vs) {
    Args a{X, K, W, K, b, g, be, mm, mv, 1e-3f, r, Y, M, K, N};
    CK(hipMemset(Y, 0, M * N * 4));
    v.launch(a, st);
    CK(hipStreamSynchronize(st));
    CK(hipGetLastError());
    std::vector<float> hy(M * N);
    CK(hipMemcpy(hy.data(), Y, M * N * 4, hipMemcpyDeviceToHost));
    double err = 0;
    for (int k = 0; k < M * N; ++k) err = fmax(err, fabs(hy[k] - ref[k]));
    // back-to-back over 4 layer weight sets
    for (int it = 0; it < 50; ++it) { a.Wt = W + (size_t)(it % NL) * N * K; v.launch(a, st); }
    CK(hipEventRecord(e0, st));
    for (int it = 0; it < ITERS; ++it) { a.Wt = W + (size_t)(it % NL) * N * K; v.launch(a, st); }
    CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    // per-launch event pairs
    for (int it = 0; it < ITERS; ++it) {
      a.Wt = W + (size_t)(it % NL) * N * K;
      CK(hipEventRecord(evs[2 * it], st)); v.launch(a, st); CK(hipEventRecord(evs[2 * it + 1], st));
    }
    CK(hipStreamSynchronize(st));
    std::vector<float> t(ITERS);
    for (int it = 0; it < ITERS; ++it) CK(hipEventElapsedTime(&t[it], evs[2 * it], evs[2 * it + 1]));
    std::sort(t.begin(), t.end());
    printf("%-28s err %.2e  back-to-back %8.3f us/launch   pair median %8.3f us  min %8.3f\n", v.name.c_str(), err,
           1000 * ms / ITERS, 1000 * t[ITERS / 2], 1000 * t[0]);
  }
  return 0;
}
