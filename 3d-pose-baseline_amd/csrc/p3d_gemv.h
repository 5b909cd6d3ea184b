// p3d_gemv.h -- inference layers at batch <= 4 as weight-streaming GEMV kernels (gfx950).
//
// The OpenPose front end lifts one frame per model.step (src/openpose_3dpose_sandbox.py:353-356,
// SURVEY.md 8f rank 4).  At B = 1 a layer is a matrix-vector product: 4 MB of weights for 2 K
// FLOP per weight row, so the bound is the weight stream (HBM, or the XCD's L2 / MALL when the
// same model lifts frame after frame), never MFMA.  The 16-row MFMA tiles of k_fwd waste 15/16
// of every product at B = 1 and run K-slices of only 8 waves per column tile.
//
// k_gemv: one workgroup per 16 output features (the Wf fragment row tile, N/16 workgroups),
// WV waves split the K groups.  Every weight fragment (1 KB, lane i + 16q holding
// W[16ct + i][16g + 4q .. +3]) is requested before the first FMA -- a wave holds all of its
// fragments in registers (4 at K = 1024, WV = 16), so each CU has its whole 64 KB slice in flight
// at once (default cache policy: the same slice is read every frame, so it stays in the L2 of
// the XCD the workgroup lands on, or in MALL).  Lane (i, q) multiplies its fragment with x[r][16g + 4q .. +3] (one float4 load, the
// same address across the 16 lanes of a quarter) for every row r < M; the four quarters are
// summed with two cross-lane adds, the waves in fixed order through LDS (deterministic), and 16
// lanes per row apply the layer epilogue of k_fwd (max-norm divisor, bias, eval BN, ReLU,
// dropout, residual).  The epilogue operands are requested at kernel start by the lanes that
// use them.
//
// Why one launch per layer (not a persistent chain): the hand-off of a layer's 1024 features
// from the 64 producing workgroups to every consumer costs ~3-4 us inside a launch (price list
// rows allgather / barrier-xcd of MI355X_MICROARCH.md) against ~1.2 us for the dependent kernel
// boundary between short GEMV kernels (row boundary).
#pragma once
#include "p3d_kernels.h"

struct GemvArgs {
  const float* X; int64_t ldx; int xpk;   // X packed (hidden input) or row-major, leading dim ldx
  const float* Wf;                        // fragment-major [ceil(N/16)][K/16] 1 KB fragments
  const float* bias;
  const float* wsq;                       // max-norm: ||W||^2 or null
  int M, K, N;
  int bn;                                 // 0 none, 1 eval BN (moving statistics)
  const float* gamma; const float* beta; const float* mmean; const float* mvar; float eps;
  int relu;
  float keep; uint64_t seed; uint64_t ctr; int site; int64_t row_off;
  const int64_t* ctr_dev;
  const float* res;                       // residual, packed [M, N]
  float* Y; int64_t ldy; int ypk;         // packed (hidden) or row-major (output layer)
};

// MR: most rows per launch (B <= MR); WV: waves per workgroup; GC: K groups requested per
// chunk and wave (registers: 4 * GC).
template <int MR, int WV, int GC>
__global__ __launch_bounds__(64 * WV) void k_gemv(GemvArgs p) {
  __shared__ float red[WV][MR][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int ct = blockIdx.x;
  const int ngK = p.K >> 4;
  const int gb = (ngK * w) / WV, ge = (ngK * (w + 1)) / WV;
  const int M = p.M;
  // ---- epilogue operands, requested first (wave 0, lane (i, q) = row q, column 16ct + i) -----
  const int col = 16 * ct + i;
  const bool cok = col < p.N;
  const int cc = cok ? col : p.N - 1;
  float b = 0.f, gam = 1.f, bet = 0.f, mmu = 0.f, mva = 1.f, rv = 0.f, mxv = 1.f;
  uint64_t ctr = p.ctr;
  if (w == 0 && q < M) {
    b = p.bias[cc];
    if (p.bn) { gam = p.gamma[cc]; bet = p.beta[cc]; mmu = p.mmean[cc]; mva = p.mvar[cc]; }
    if (p.res) rv = p.res[p3d_pk(q, cc, (p.N + 15) >> 4)];
    if (p.wsq) mxv = *p.wsq;
    if (p.ctr_dev) ctr = (uint64_t)*p.ctr_dev;
  }
  // ---- contraction: this wave's K groups, GC fragments in flight per chunk -----------------
  float acc[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) acc[r] = 0.f;
  const f32x4* pw = (const f32x4*)p.Wf + (int64_t)ct * ngK * 64 + lane;
  for (int g0 = gb; g0 < ge; g0 += GC) {
    f32x4 wf[GC];
#pragma unroll
    for (int j = 0; j < GC; ++j) {
      const int g = g0 + j < ge ? g0 + j : ge - 1;
      wf[j] = pw[(int64_t)g * 64];   // default policy: frame after frame hits the XCD's L2 / MALL
    }
#pragma unroll
    for (int j = 0; j < GC; ++j) {
      if (g0 + j >= ge) break;
      const int k = 16 * (g0 + j) + 4 * q;
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        if (r >= M) break;
        const f32x4 xv = p.xpk ? *(const f32x4*)(p.X + ((int64_t)(g0 + j) << 8) + ((r + 16 * q) << 2))
                               : *(const f32x4*)(p.X + (int64_t)r * p.ldx + k);
        float a = acc[r];
        a = fmaf(wf[j].x, xv.x, a);
        a = fmaf(wf[j].y, xv.y, a);
        a = fmaf(wf[j].z, xv.z, a);
        a = fmaf(wf[j].w, xv.w, a);
        acc[r] = a;
      }
    }
  }
  // ---- quarters, then waves in fixed order ------------------------------------------------
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    acc[r] += __shfl_xor(acc[r], 16, 64);
    acc[r] += __shfl_xor(acc[r], 32, 64);
  }
  if (q == 0) {
#pragma unroll
    for (int r = 0; r < MR; ++r) red[w][r][i] = acc[r];
  }
  __syncthreads();
  if (w != 0 || q >= M || q >= MR) return;
  float zs = 0.f;
#pragma unroll
  for (int u = 0; u < WV; ++u) zs += red[u][q][i];
  // ---- epilogue of k_fwd for row q, column col ---------------------------------------------
  const float mx = p.wsq ? fmaxf(sqrtf(mxv), 1.0f) : 1.0f;
  const float z = (p.wsq ? zs / mx : zs) + b;
  float y = z;
  if (p.bn) {
    const float inv = (1.0f / sqrtf(mva + p.eps)) * gam;
    const float shift = bet - mmu * inv;
    y = z * inv + shift;
  }
  if (p.relu) y = fmaxf(y, 0.0f);
  if (p.keep < 1.0f) y = (y / p.keep) * p3d_dropout_mask(p.keep, p3d_uniform(p.seed, ctr, p.site, p.row_off + q, cc));
  if (p.res) y += rv;
  if (!cok) return;
  if (p.ypk) p.Y[p3d_pk(q, col, (p.N + 15) >> 4)] = y;
  else p.Y[(int64_t)q * p.ldy + col] = y;
}
