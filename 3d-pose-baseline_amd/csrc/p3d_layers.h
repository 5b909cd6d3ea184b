// p3d_layers.h -- the layer kernels of the fused training / batch-64 inference paths (gfx950):
// TF1 Adam primitives, k_fwd / k_out_part, the BN-train exchange and split forms, k_dgrad,
// k_bn_bwd, the weight-gradient kernels (k_wgrad, k_wgrad_multi, k_wgrad_grad), k_adam_pack,
// the weight (un)packing, k_mse and the max-norm helpers.  Device code only; included by p3d.hip (the
// host side) and by tools/kdev.hip (single-kernel resource builds: a kernel's registers and spills in
// seconds instead of the whole library's minutes).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include "p3d_kernels.h"
#include "p3d_xchg.h"
#include <math.h>
#include <stdint.h>

// =====================================================================================
// TF1 ApplyAdam primitives (linear_model.py:137,145) shared by k_adam_pack and the fused
// single-GPU train step (k_wgrad / k_bn_bwd apply the update where the gradient is formed)
// =====================================================================================
#define P3D_MAX_W 40
#define P3D_MAX_V 64
struct StepState {
  int64_t global_step;
  float beta1_power, beta2_power;
  unsigned int arrivals;
  unsigned int pad[3];
};

// Every operation rounded on its own (no FMA contraction), as the TF1 kernel's expression
// reads and as the oracle computes it -- and identically in every kernel that inlines it
// (the compiler contracted it in one context and not in another before).
__device__ __forceinline__ void p3d_adam1(float& w, float& m, float& v, float g, float alpha, float omb1,
                                          float omb2, float eps) {
#pragma clang fp contract(off)
  m = m + (g - m) * omb1;
  v = v + (g * g - v) * omb2;
  w = w - (m * alpha) / (sqrtf(v) + eps);
}

// Adam hyper-parameters + the device step state a fused kernel reads its alpha from.
struct AdamFuse {
  const StepState* st;
  float lr_host;        // >= 0: use as lr; < 0: device exponential decay of lr0
  float lr0, decay_steps, decay_rate;
  float b1, b2, eps;
  int wsrc;             // 1: weights read from their Wd copy, the TF-layout master not written (p3d_adam_tile64)
};

__device__ __forceinline__ float p3d_adam_alpha(const StepState* st, float lr_host, float lr0, float decay_steps,
                                                float decay_rate) {
  const float b1p = st->beta1_power, b2p = st->beta2_power;
  float lr = lr_host;
  if (lr < 0.f) lr = lr0 * powf(decay_rate, (float)st->global_step / decay_steps);
  return lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
}

// Adam on one 64x64 tile (rows k0.., cols n0..) of a weight W [K, N] (TF layout, flat
// offset `off` in w/m/v/g) + re-pack of the updated tile into Wf / Wd.  256 threads.
// g comes from `g` (global) or, when g == nullptr, from tile[k - k0][n - n0] (the fused
// weight-gradient kernel); tile ends holding the updated weights.  Bit-identical updates
// either way (same gradient values, same p3d_adam1).
//
// wsrc = 1 (every optimizer of a model without --max_norm): the weights are read from their Wd copy
// -- the TF layout tiled: Wd element (k, n) is lane (k & 15) + 16 ((n & 15) >> 2), component n & 3
// of 16x16 tile (k >> 4, n >> 4), a permutation, so the values are the master's bit for bit -- and
// the TF-layout master is NOT written: 4 of the 32 / 36 bytes per weight element the optimizer moves.
// The master is re-derived from Wd when something reads it (p3d_params_sync).
__device__ __forceinline__ int64_t p3d_wd_at(int k, int n, int ngd) {
  return ((int64_t)((k >> 4) * ngd + (n >> 4)) * 64 + (k & 15) + 16 * ((n & 15) >> 2)) * 4 + (n & 3);
}
// RB: rows of the thread's four requested together (4: one round trip; 2: two, 24 fewer registers
// live -- the fused weight-gradient kernel at five workgroups per CU).
template <int RB = 4>
__device__ __forceinline__ void p3d_adam_tile64(float (*tile)[65], const float* g, int64_t off, int K, int N,
                                                int k0, int n0, float* w, float* m, float* v, float* wd,
                                                float* wf, float alpha, float omb1, float omb2, float eps,
                                                int wsrc = 0) {
  const int tid = threadIdx.x;
  const bool vec = (N & 3) == 0;
  const int ngd_ = ((N + 15) & ~15) >> 4;
  if (vec) {
#pragma unroll
   for (int h = 0; h < 4; h += RB) {
    // all four rows' w / m / v (and g) requested before the first update, from clamped (always
    // valid) addresses, stores after: a load inside the per-row range branch made every row a
    // dependent memory round trip (with the previous row's stores in the same wait)
    f32x4 ww[RB], mm[RB], vv[RB], gg[RB];
    bool ok[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int it = h + j, r = it * 16 + (tid >> 4), c = 4 * (tid & 15);
      const int k = k0 + r, n = n0 + c;
      ok[j] = k < K && n < N;
      const int64_t base = ok[j] ? off + (int64_t)k * N + n : off;
      ww[j] = wsrc ? *(const f32x4*)(wd + (ok[j] ? p3d_wd_at(k, n, ngd_) : 0)) : *(const f32x4*)(w + base);
      mm[j] = *(const f32x4*)(m + base);
      vv[j] = *(const f32x4*)(v + base);
      if (g) gg[j] = *(const f32x4*)(g + base);
      else gg[j] = f32x4{tile[r][c], tile[r][c + 1], tile[r][c + 2], tile[r][c + 3]};
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int it = h + j, r = it * 16 + (tid >> 4), c = 4 * (tid & 15);
      const int64_t base = off + (int64_t)(k0 + r) * N + n0 + c;
      float wn[4] = {0.f, 0.f, 0.f, 0.f};
      if (ok[j]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float w1 = ww[j][e], m1 = mm[j][e], v1 = vv[j][e];
          p3d_adam1(w1, m1, v1, gg[j][e], alpha, omb1, omb2, eps);
          ww[j][e] = w1; mm[j][e] = m1; vv[j][e] = v1; wn[e] = w1;
        }
        if (!wsrc) *(f32x4*)(w + base) = ww[j];
        *(f32x4*)(m + base) = mm[j]; *(f32x4*)(v + base) = vv[j];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[r][c + e] = wn[e];   // each thread rewrites only what it read
    }
   }
  } else {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int r = it * 16 + (tid >> 4), c = 4 * (tid & 15);
      const int k = k0 + r, n = n0 + c;
      float wn[4] = {0.f, 0.f, 0.f, 0.f};
      if (k < K) {
        const int64_t base = off + (int64_t)k * N + n;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < N) {
            float ww = wsrc ? wd[p3d_wd_at(k, n + e, ngd_)] : w[base + e], mm = m[base + e], vv = v[base + e];
            p3d_adam1(ww, mm, vv, g ? g[base + e] : tile[r][c + e], alpha, omb1, omb2, eps);
            if (!wsrc) w[base + e] = ww;
            m[base + e] = mm; v[base + e] = vv;
            wn[e] = ww;
          }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[r][c + e] = wn[e];
    }
  }
  __syncthreads();
  const int NP = (N + 15) & ~15;
  const int ngf = K >> 4, ngd = NP >> 4;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int sub = it * 4 + (tid >> 6), l = tid & 63;
    const int sk = sub >> 2, sn = sub & 3;             // 16x16 sub-tile within the 64x64 tile
    const int kt = (k0 >> 4) + sk, nt = (n0 >> 4) + sn;
    if (16 * kt >= K || 16 * nt >= NP) continue;
    const int i = l & 15, q = l >> 4;
    // Wd (rows k, cols n): element (16kt+i, 16nt+4q+e)
    const f32x4 od = f32x4{tile[16 * sk + i][16 * sn + 4 * q], tile[16 * sk + i][16 * sn + 4 * q + 1],
                           tile[16 * sk + i][16 * sn + 4 * q + 2], tile[16 * sk + i][16 * sn + 4 * q + 3]};
    *(f32x4*)(wd + ((int64_t)(kt * ngd + nt) * 64 + l) * 4) = od;
    // Wf (rows n, cols k): element (16nt+i, 16kt+4q+e)
    const f32x4 of = f32x4{tile[16 * sk + 4 * q][16 * sn + i], tile[16 * sk + 4 * q + 1][16 * sn + i],
                           tile[16 * sk + 4 * q + 2][16 * sn + i], tile[16 * sk + 4 * q + 3][16 * sn + i]};
    *(f32x4*)(wf + ((int64_t)(nt * ngf + kt) * 64 + l) * 4) = of;
  }
}

// =====================================================================================
// forward
// =====================================================================================
struct FwdArgs {
  const float* X; int64_t ldx;    // [M, K]: packed (ldx unused) or row-major (input layer)
  const float* Wf;                // packed forward weight, ngB = K/16 groups per column tile
  const float* bias;              // [N]
  const float* wsq;               // max-norm: ||W||^2 (device scalar) or null
  int M, K, N;
  int bn;                         // 0 none, 1 eval (moving stats), 2 train (batch stats)
  const float* gamma; const float* beta;
  float* mmean; float* mvar;      // moving stats (read in eval, updated in train)
  float eps; float decay;         // decay = 1 - momentum (fp32, as TF computes it)
  float* z_save;                  // train: z = X*W + b, packed [M, N]
  float* mean_save; float* var_save;
  int relu;
  float keep; uint64_t seed; uint64_t ctr; int site; int64_t row_off;
  const int64_t* ctr_dev;         // if set, dropout counter = *ctr_dev (device global_step)
  const float* res;               // residual added after dropout, packed [M, N]
  float* Y; int64_t ldy;          // packed (hidden) or row-major (output layer)
  float* bnpart;                  // bn == 3: per (row tile, column) {sum z, sum (z - tile mean)^2}
  const float* tgt;               // fused MSE (training output layer, row-major like Y): targets,
  float* dy; float dscale;        //   dy = dscale * (y - t) stored row-major (leading dim lddy),
  int64_t lddy;
  float* lossp;                   //   per-workgroup sum of (y - t)^2
  XchgSite xs;                    // bn == 4 (BN-train exchange form, p3d_xchg.h)
  int remap_gy;                   // > 0: 1-D grid of gx * remap_gy blocks, tiles by p3d_sibling_remap
};

// Tile of block b in a 1-D grid of gx * gy blocks (gx % 8 == 0): the gy row-tile siblings of a
// column tile are blocks xcd + 8 j for gy consecutive j -- one XCD under the observed round-robin
// placement, dispatched together (the 2-D grid put them 64 blocks apart).  Speed only: the
// exchange is correct for any placement.
__device__ __forceinline__ void p3d_sibling_remap(int b, int gx, int gy, int& ct, int& rt) {
  const int xcd = b & 7, j = b >> 3;
  rt = j % gy;
  ct = (j / gy) * 8 + xcd;
  (void)gx;
}

// Phase timestamps for kernel development (build with -DP3D_TRACE; tools/trace_train.py).
#ifdef P3D_TRACE
#define P3D_STAMP(k)                                                                             \
  do {                                                                                           \
    if ((threadIdx.x & 63) == 0 && p3d_trace_idx < 4096)                                          \
      g_p3d_trace[p3d_trace_idx * 8 + (k)] = wall_clock64();                                     \
  } while (0)
extern "C" int p3d_debug_trace(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_p3d_trace), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : 2;
}
#else
#define P3D_STAMP(k) do { } while (0)
#endif

// RS row tiles of 16 per wave; WK waves split the contraction; KIND only separates the
// symbols of the input / hidden / output layers for rocprof.
template <int RS, int WK, int DEPTH, int NACC, bool APK, bool YPK, int KIND>
__global__ __launch_bounds__(64 * WK) void k_fwd(FwdArgs p) {
  __shared__ f32x4 red[(WK > 1) ? (WK - 1) * RS * 64 : 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  int tbx = blockIdx.x, tby = blockIdx.y, tgx = gridDim.x, tgy = gridDim.y;
  if (p.remap_gy > 0) {
    tgx = (p.N + 15) >> 4;
    tgy = p.remap_gy;
    p3d_sibling_remap(blockIdx.x, tgx, tgy, tbx, tby);
  }
  const int ct = tbx, n0 = ct * 16, m0 = tby * 16 * RS;
  const int col = n0 + i;
  const bool cok = col < p.N;
  const int cc = cok ? col : p.N - 1;
  const int ngN = (p.N + 15) >> 4;
  const int p3d_trace_idx = tbx + tgx * tby;
  (void)p3d_trace_idx;
#ifndef P3D_TRACE_RS
#define P3D_TRACE_RS 4
#endif
  const bool trace = (RS == P3D_TRACE_RS && KIND == 1 && w == 0);
  const bool trace_last = (RS == P3D_TRACE_RS && KIND == 1 && w == WK - 1);
  if (trace) P3D_STAMP(0);
#ifdef P3D_TRACE_PROBE  // first-touch latency of the activations (wave 1 only)
  if (RS == P3D_TRACE_RS && KIND == 1 && w == 1) {
    const float v = __builtin_nontemporal_load(p.X + lane * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (v == 12345.678f) p.Y[0] = v;
    P3D_STAMP(7);
  }
#endif
  // ---- epilogue operands issued before the GEMM so their latency overlaps it -------
  float b = 0.f, gam = 1.f, bet = 0.f, mmu = 0.f, mva = 1.f, rv[RS][4], tv[RS][4];
  uint64_t ctr = p.ctr;
  unsigned xtag = 0;
  if (w == 0) {
    if (p.bn == 4) xtag = p3d_xchg_tag(p.xs, ct, tby, tgy);
    if (p.ctr_dev) ctr = (uint64_t)*p.ctr_dev;
    b = p.bias[cc];
    if (p.bn) { gam = p.gamma[cc]; bet = p.beta[cc]; mmu = p.mmean[cc]; mva = p.mvar[cc]; }
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 16 * s + 4 * q + r;
        rv[s][r] = p.res ? p.res[p3d_pk(row, cc, ngN)] : 0.f;
        // fused MSE targets (training output layer): requested with the other epilogue
        // operands, not after the contraction (one dependent round trip less)
        tv[s][r] = (KIND == 2 && p.tgt && row < p.M) ? p.tgt[(int64_t)row * p.ldy + cc] : 0.f;
      }
  }
  const int ngt = p.K >> 4;
  const int gb = (ngt * w) / WK, ge = (ngt * (w + 1)) / WK;
  f32x4 acc[NACC][RS];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[a][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  p3d_core<RS, DEPTH, NACC, APK>(p.X, p.ldx, ngt, p.M, m0, p.Wf, ngt, ct, gb, ge, acc);
  if (trace) P3D_STAMP(1);
  if (trace_last) P3D_STAMP(6);
  __shared__ XchgPub xpub;                  // bn == 4: wave 0 posts its column pairs, wave 1 publishes
  if (WK > 1 && p.bn == 4 && w == 1) p3d_xchg_pub_reset(&xpub);
  if (!p3d_reduce_waves<RS, NACC, WK>(acc, red)) {
    if (WK > 1 && p.bn == 4 && w == 1) p3d_xchg_publish(p.xs, &xpub, p.N, tby, n0);
    return;
  }
  if (trace) P3D_STAMP(2);
  // ---- epilogue (wave 0): lane holds rows m0+16s+4q+r of column n0+i ---------------
  const float mx = p.wsq ? fmaxf(sqrtf(*p.wsq), 1.0f) : 1.0f;
  float z[RS][4];
#pragma unroll
  for (int s = 0; s < RS; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) z[s][r] = (p.wsq ? acc[0][s][r] / mx : acc[0][s][r]) + b;

  float xmean = 0.f, xvar = 1.f, sum = 0.f, sq = 0.f, uu_x[RS][4];
  if (p.bn == 3 || p.bn == 4) {
    // BN-train: this row tile's per-column count-weighted moments {sum, M2 about the tile
    // mean} for Chan's combination.  Split form (bn = 3): z and the moments out, k_bn_fwd
    // finishes the layer.  Exchange form (bn = 4): the row-tile siblings swap their moments
    // here (p3d_xchg.h) and every workgroup finishes its own tile below.
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (m0 + 16 * s + 4 * q + r < p.M) sum += z[s][r];
    sum = p3d_colsum16(sum);
    const int nt = min(16 * RS, p.M - m0);
    const float mt = sum / (float)nt;
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (m0 + 16 * s + 4 * q + r < p.M) { const float d = z[s][r] - mt; sq = __builtin_fmaf(d, d, sq); }
    sq = p3d_colsum16(sq);
    if (p.bn == 4) {
      const int R = tgy;
      if (WK > 1) p3d_xchg_post(&xpub, q == 0, i, sum, sq, xtag);
      else p3d_xchg_put(p.xs, p.N, tby, col, q == 0 && cok, sum, sq, xtag);
      // the dropout uniforms do not depend on the statistics: formed while the siblings arrive
      if (p.keep < 1.0f) {
#pragma unroll
        for (int s = 0; s < RS; ++s) p3d_uniform_rows4(p.seed, ctr, p.site, p.row_off + m0 + 16 * s + 4 * q, cc, uu_x[s]);
      }
      if (R <= 4) p3d_xchg_moments<4>(p.xs, p.N, R, cc, xtag, tby, p.M, xmean, xvar);   // (wave-uniform)
      else p3d_xchg_moments<P3D_XCHG_MAXR, (WK >= 16 ? 8 : P3D_XCHG_MAXR)>(p.xs, p.N, R, cc, xtag, tby, p.M, xmean, xvar);
      p3d_xchg_done(p.xs, ct, tby);
#ifdef P3D_TRACE
      if (trace && lane == 0 && ct + tgx * tby < 2048) g_p3d_trace[16384 + (ct + tgx * tby) * 8 + 6] = wall_clock64();
#endif
#ifdef P3D_TRACE
      if (trace && lane == 0 && p3d_trace_idx < 4096) {   // slot 7: the hardware XCD of this workgroup
        unsigned xr;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xr));
        g_p3d_trace[p3d_trace_idx * 8 + 7] = xr & 7u;
      }
#endif
    }
  }
  if (p.bn == 3) {
    if (!cok) return;
    if (q == 0) {
      p.bnpart[((int64_t)tby * p.N + col) * 2] = sum;
      p.bnpart[((int64_t)tby * p.N + col) * 2 + 1] = sq;
    }
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 16 * s + 4 * q + r;
        if (row < p.M) p.z_save[p3d_pk(row, col, ngN)] = z[s][r];
      }
    return;
  }
  float inv = 1.0f, shift = 0.0f;
  if (p.bn == 4) {
    p3d_bn_affine(xmean, xvar, p.eps, gam, bet, inv, shift);
    if (tby == 0 && q == 0 && cok) {
      p.mean_save[col] = xmean;
      p.var_save[col] = xvar;
      p.mmean[col] = p3d_bn_moving(mmu, xmean, p.decay);
      p.mvar[col] = p3d_bn_moving(mva, xvar, p.decay);
    }
  } else if (p.bn) {
    float mean = mmu, var = mva;
    if (p.bn == 2) {  // batch statistics over all M rows (host guarantees M <= 16*RS)
      float sum = 0.f;
#pragma unroll
      for (int s = 0; s < RS; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (m0 + 16 * s + 4 * q + r < p.M) sum += z[s][r];
      sum = p3d_colsum16(sum);
      mean = sum / (float)p.M;
      float sq = 0.f;
#pragma unroll
      for (int s = 0; s < RS; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (m0 + 16 * s + 4 * q + r < p.M) { const float d = z[s][r] - mean; sq += d * d; }
      sq = p3d_colsum16(sq);
      var = sq / (float)p.M;
      if (q == 0 && cok) {
        p.mean_save[col] = mean;
        p.var_save[col] = var;
        p.mmean[col] = mmu - (mmu - mean) * p.decay;
        p.mvar[col] = mva - (mva - var) * p.decay;
      }
    }
    inv = (1.0f / sqrtf(var + p.eps)) * gam;
    shift = bet - mean * inv;
  }
  if (trace) P3D_STAMP(3);
  float uu[RS][4];
  if (p.keep < 1.0f) {
#pragma unroll
    for (int s = 0; s < RS; ++s) {
      if (p.bn == 4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) uu[s][r] = uu_x[s][r];
      } else {
        p3d_uniform_rows4(p.seed, ctr, p.site, p.row_off + m0 + 16 * s + 4 * q, cc, uu[s]);
      }
    }
  }
  if (trace) P3D_STAMP(4);
  if (p.tgt) {
    // fused MSE of linear_model.py:129 (output layer: no BN / ReLU / dropout / residual)
    float ls = 0.f;
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 16 * s + 4 * q + r;
        if (cok && row < p.M) {
          const float d = z[s][r] - (KIND == 2 ? tv[s][r] : p.tgt[(int64_t)row * p.ldy + col]);
          p.dy[(int64_t)row * p.lddy + col] = d * p.dscale;
          ls += d * d;
        }
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
    if (lane == 0) p.lossp[tbx + tgx * tby] = ls;
  }
  if (!cok) return;
#pragma unroll
  for (int s = 0; s < RS; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * s + 4 * q + r;
      if (row >= p.M) continue;
      if (p.z_save) p.z_save[p3d_pk(row, col, ngN)] = z[s][r];
      float y = p.bn == 4 ? p3d_bn_y(z[s][r], inv, shift) : p.bn ? z[s][r] * inv + shift : z[s][r];
      if (p.relu) y = fmaxf(y, 0.0f);
      if (p.keep < 1.0f) y = (y / p.keep) * p3d_dropout_mask(p.keep, uu[s][r]);
      if (p.res) y += rv[s][r];
      if (YPK) p.Y[p3d_pk(row, col, ngN)] = y;
      else p.Y[(int64_t)row * p.ldy + col] = y;
    }
  if (trace) P3D_STAMP(5);
#ifdef P3D_TRACE_PROBE  // stores complete (slot 4: the dropout stamp, unused in inference)
  if (trace) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); P3D_STAMP(4); }
#endif
}

// =====================================================================================
// Training output layer as split-K partials (round 4).  The fused-MSE output layer (N = 48, 12
// tiles at B = 64) ran as 12 workgroups of 8 waves: 12 CUs each taking in 128 KB while 244 idled
// (6.3 us).  Here every (tile, K eighth) is its own one-wave workgroup (96 at B = 64): wave w of
// the 8-wave k_fwd becomes workgroup (ct, rt, w), same k-groups, same MFMA chains, in the
// transposed-accumulator form (p3d_core SWAP: the same products in the same order, lane (i, q)
// holding row 16 rt + i, columns 4q .. 4q+3 -- the A-fragment layout of the data gradient).  The
// output layer's data-gradient launch sums the 8 partials in wave order (k_fwd's association, so
// y and dy are bit-identical), adds the bias, forms y, dy = 2(y - t)/(B D) and the loss partials,
// and contracts dy with W^T straight from registers (p3d_dgrad_body, BwdArgs::opart).
// =====================================================================================
struct OutPartArgs {
  const float* X;     // packed [M, K] (the last hidden layer's output)
  const float* Wf;    // the output layer's forward operand
  int M, K;
  float* part;        // [R][NT][8] 1 KB tiles
};
template <int DEPTH>
__global__ __launch_bounds__(64) void k_out_part(OutPartArgs p) {
  const int lane = threadIdx.x;
  const int ct = blockIdx.x, rt = blockIdx.y, sl = blockIdx.z;
  const int ngt = p.K >> 4;
  const int gb = (ngt * sl) / 8, ge = (ngt * (sl + 1)) / 8;
  f32x4 acc[2][1];
  acc[0][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  p3d_core<1, DEPTH, 2, true, true>(p.X, 0, ngt, p.M, 16 * rt, p.Wf, ngt, ct, gb, ge, acc);
  acc[0][0] += acc[1][0];
  ((f32x4*)p.part)[(((int64_t)rt * gridDim.x + ct) * 8 + sl) * 64 + lane] = acc[0][0];
}

// =====================================================================================
// BN-train forward, second half (split form): batch statistics from the row-tile moments,
// then y = dropout(relu(BN(z))) (+ residual) on the packed layout: one 16x16 tile per
// 64-lane workgroup, lane l holding row 16rt + (l&15), columns 16ct + 4(l>>4) .. +3, so
// one float4 per operand and one Philox block per lane (its four dropout words).
// TF1 semantics as k_fwd bn == 2 (biased variance, moving m -= (m - stat) * (1 - momentum)).
// =====================================================================================
struct BnFwdArgs {
  const float* z; const float* part;   // packed [M, N]; [R][N][2]
  int M, N;
  const float* gamma; const float* beta;
  float* mmean; float* mvar; float eps; float decay;
  float* mean_save; float* var_save;
  int relu;
  float keep; uint64_t seed; uint64_t ctr; int site; int64_t row_off;
  const int64_t* ctr_dev;
  const float* res;                    // packed residual or null
  float* Y;                            // packed [M, N]
};

// The first <= 4 row-tile partial pairs of columns n0..n0+3 ([t][col][2] layout: 8
// consecutive floats per tile), all issued up front (tiles 4.. of B > 64 are read in the fold).
__device__ __forceinline__ void p3d_load_parts(const float* part, int M, int N, int n0, f32x4 (&pp)[4][2]) {
  const int R = (M + 15) >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int tt = t < R ? t : 0;
    const f32x4* src = (const f32x4*)(part + ((int64_t)tt * N + n0) * 2);
    pp[t][0] = src[0];
    pp[t][1] = src[1];
  }
}

__global__ __launch_bounds__(64) void k_bn_fwd(BnFwdArgs p) {
  const int lane = threadIdx.x, ct = blockIdx.x, rt = blockIdx.y;
  const int j = lane & 15, q = lane >> 4;
  const int n0 = 16 * ct + 4 * q, row = 16 * rt + j;
  const int ngN = p.N >> 4;
  const int R = (p.M + 15) >> 4;
  const int64_t off = ((int64_t)rt * ngN + ct) * 256 + lane * 4;
  // every operand load issued before any arithmetic
  f32x4 pp[4][2];
  p3d_load_parts(p.part, p.M, p.N, n0, pp);
  const f32x4 z4 = *(const f32x4*)(p.z + off);
  const f32x4 g4 = *(const f32x4*)(p.gamma + n0), b4 = *(const f32x4*)(p.beta + n0);
  f32x4 r4 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (p.res) r4 = *(const f32x4*)(p.res + off);
  f32x4 mm4 = f32x4{0.f, 0.f, 0.f, 0.f}, mv4 = mm4;
  const bool owner = (rt == 0 && j == 0);
  if (owner) { mm4 = *(const f32x4*)(p.mmean + n0); mv4 = *(const f32x4*)(p.mvar + n0); }
  const uint64_t ctr = p.ctr_dev ? (uint64_t)*p.ctr_dev : p.ctr;
  float u[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.keep < 1.0f) {
    const uint4 wq = p3d_philox(make_uint4((uint32_t)(p.row_off + row), (uint32_t)(n0 >> 2), (uint32_t)p.site,
                                           (uint32_t)ctr), (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
    const uint32_t xs[4] = {wq.x, wq.y, wq.z, wq.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) u[e] = __uint_as_float((xs[e] & 0x7FFFFFu) | 0x3F800000u) - 1.0f;
  }
  const float fm = (float)p.M;
  f32x4 o, mean4, var4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    // element e of column n0+e sits at float 2e (sum) / 2e+1 (M2) of the tile's 8 floats
    float S = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t < R) S += pp[t][e >> 1][(e & 1) * 2];
    for (int t = 4; t < R; ++t) S += p.part[((int64_t)t * p.N + n0 + e) * 2];   // B > 64
    const float mean = S / fm;
    float M2 = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t < R) M2 += p3d_chan_term(pp[t][e >> 1][(e & 1) * 2], pp[t][e >> 1][(e & 1) * 2 + 1], min(16, p.M - 16 * t), mean);
    for (int t = 4; t < R; ++t) {
      const float* pt = p.part + ((int64_t)t * p.N + n0 + e) * 2;
      M2 += p3d_chan_term(pt[0], pt[1], min(16, p.M - 16 * t), mean);
    }
    const float var = M2 / fm;
    mean4[e] = mean;
    var4[e] = var;
    float inv, shift;
    p3d_bn_affine(mean, var, p.eps, g4[e], b4[e], inv, shift);
    float y = p3d_bn_y(z4[e], inv, shift);
    if (p.relu) y = fmaxf(y, 0.0f);
    if (p.keep < 1.0f) y = (y / p.keep) * p3d_dropout_mask(p.keep, u[e]);
    if (p.res) y += r4[e];
    o[e] = row < p.M ? y : 0.0f;
  }
  *(f32x4*)(p.Y + off) = o;
  if (owner) {
    *(f32x4*)(p.mean_save + n0) = mean4;
    *(f32x4*)(p.var_save + n0) = var4;
    f32x4 nm, nv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      nm[e] = p3d_bn_moving(mm4[e], mean4[e], p.decay);
      nv[e] = p3d_bn_moving(mv4[e], var4[e], p.decay);
    }
    *(f32x4*)(p.mmean + n0) = nm;
    *(f32x4*)(p.mvar + n0) = nv;
  }
}

// =====================================================================================
// data gradient + previous layer's epilogue backward (whole batch per workgroup)
// =====================================================================================
struct BwdArgs {
  const float* dZ; int64_t ldz;   // A = dZ [M, N]: packed, or row-major (dy of the output layer)
  const float* Wd;                // packed dgrad weight: rows = K (in), cols = N padded (ngB groups)
  int ngB;
  const float* wsq;
  int M, K, N;                    // output [M, K]
  const float* dres;              // residual gradient added to dX (block output grad), packed [M,K]
  float* draw;                    // store dX (+dres) packed if non-null
  int prev;                       // 1: run prev layer's dropout/relu/BN backward
  int bn; const float* z; const float* mean; const float* var;   // prev layer: z packed [M,K]
  const float* gamma; const float* beta; float eps;
  int relu; float keep; uint64_t seed; uint64_t ctr; int site; int64_t row_off;
  const int64_t* ctr_dev;
  float* dz;                      // packed [M, K]: gradient wrt prev layer's z
  float* dgamma; float* dbeta;    // [K]
  float* bnpart;                  // split BN backward: per (row tile, column) {sum g, sum g*xhat};
                                  // dz then holds g (k_bn_bwd finishes it)
  const float* lossp; int nlossp; // fused MSE: workgroup 0 folds the forward's loss partials
  float* loss; float loss_scale;  //   (fixed order) into loss[0] = scale * sum
  XchgSite xs; int xchg;          // with bnpart: exchange form (p3d_xchg.h) -- dz, dgamma, dbeta here
  int remap_gy;                   // > 0: 1-D grid of (K/16) * remap_gy blocks (p3d_sibling_remap)
  float* alpha_out; AdamFuse af;  // fused Adam: tile (0, 0) stores the step's alpha for later launches
  // output layer from split-K partials (k_out_part): A = dy formed here, not loaded (dZ unused)
  const float* opart; int ont;    //   partials [R][ont][8] and the output layer's column tiles
  const float* obias; const float* otgt; int64_t oldt;   // bias [N], targets row-major
  float* oy; int64_t oldy;        //   y out (row-major, the caller's), written by column tile 0
  float* ody; int64_t oldd;       //   dy out (row-major, for the output layer's weight gradient)
  float odscale; float* olossp;   //   2 / (B N); per-(row tile, column tile) sum of (y - t)^2
};

// RS = 4: one workgroup owns all (<= 64) rows of its 16 columns (BN sums workgroup-local);
// RS = 1: 16x16 tiles over a (K/16, M/16) grid, BN sums left as row-tile partials (bnpart).
// The body on tile (bx, by) of a (K/16, gy) grid (k_dgrad).
template <int RS, int WK, int DEPTH, int NACC, bool APK, int KIND>
__device__ __forceinline__ void p3d_dgrad_body(const BwdArgs& p, int bx, int by, int gy) {
  __shared__ f32x4 red[(WK > 1) ? (WK - 1) * RS * 64 : 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int ct = bx, n0 = ct * 16, m0 = by * 16 * RS;
  const int col = n0 + i;
  const bool cok = col < p.K;
  const int cc = cok ? col : p.K - 1;
  const int ngK = p.K >> 4;
  // the step's Adam alpha and the folded loss (tile (0, 0)): side outputs nothing in this launch
  // reads, so with several waves the last one forms them after its share of the contraction
  // (done first by wave 0 they delayed the tile's operand requests by their load round trip,
  // and the whole launch by it, through the tile's exchange siblings)
  auto side_outputs = [&]() {
    if (p.alpha_out) *p.alpha_out = p3d_adam_alpha(p.af.st, p.af.lr_host, p.af.lr0, p.af.decay_steps, p.af.decay_rate);
    if (p.lossp) {
      float l = 0.f;
      for (int k = 0; k < p.nlossp; ++k) l += p.lossp[k];
      p.loss[0] = l * p.loss_scale;
    }
  };
  constexpr bool side_late = WK >= 3;
  if (!side_late && bx == 0 && by == 0 && threadIdx.x == 0) side_outputs();
  // prefetch the epilogue's per-column and per-element operands
  float mean = 0.f, var = 1.f, gam = 1.f, bet = 0.f, zz[RS][4], dr[RS][4];
  uint64_t ctr = p.ctr;
  unsigned xtag = 0;
  if (w == 0) {
    if (p.xchg) xtag = p3d_xchg_tag(p.xs, bx, by, gy);
    if (p.ctr_dev) ctr = (uint64_t)*p.ctr_dev;
    if (p.prev && p.bn) { mean = p.mean[cc]; var = p.var[cc]; gam = p.gamma[cc]; bet = p.beta[cc]; }
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 16 * s + 4 * q + r;
        zz[s][r] = p.prev ? p.z[p3d_pk(row, cc, ngK)] : 0.f;
        dr[s][r] = p.dres ? p.dres[p3d_pk(row, cc, ngK)] : 0.f;
      }
  }
  const int ngt = p.ngB;
  const int gb = (ngt * w) / WK, ge = (ngt * (w + 1)) / WK;
  f32x4 acc[NACC][RS];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[a][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (KIND == 2 && RS == 1 && p.opart) {
    // the output layer's dy from its split-K partials (k_out_part), one k-group = one output column
    // tile per wave: partials summed in wave order, bias, y, dy, loss partial; then dy x W^T
    const float mxo = p.wsq ? fmaxf(sqrtf(*p.wsq), 1.0f) : 1.0f;
    const int row = m0 + i;
    const int rt = m0 >> 4;
    for (int g = gb; g < ge; ++g) {
      // every operand requested before anything is stored (a store ahead of a load of another
      // array keeps the compiler from hoisting the load: one more round trip)
      const f32x4 rb = ((const f32x4*)p.Wd)[((int64_t)ct * ngt + g) * 64 + lane];
      const f32x4* pp = (const f32x4*)p.opart + (((int64_t)rt * p.ont + g) * 8) * 64 + lane;
      f32x4 pv[8];
#pragma unroll
      for (int sl = 0; sl < 8; ++sl) pv[sl] = pp[sl * 64];
      const int c0 = 16 * g + 4 * q;
      f32x4 t4, b4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool okc = c0 + e < p.N;
        t4[e] = (row < p.M && okc) ? p.otgt[(int64_t)(row < p.M ? row : 0) * p.oldt + c0 + e] : 0.f;
        b4[e] = okc ? p.obias[c0 + e] : 0.f;
      }
      f32x4 zs = pv[0];
#pragma unroll
      for (int sl = 1; sl < 8; ++sl) zs += pv[sl];
      f32x4 a4, z4;
      float ls = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = row < p.M && c0 + e < p.N;
        z4[e] = (p.wsq ? zs[e] / mxo : zs[e]) + b4[e];
        const float d = z4[e] - t4[e];
        a4[e] = ok ? d * p.odscale : 0.f;
        if (ok) ls += d * d;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[e % NACC][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[e], rb[e], acc[e % NACC][0], 0, 0, 0);
      if (bx == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (row < p.M && c0 + e < p.N) {
            p.oy[(int64_t)row * p.oldy + c0 + e] = z4[e];
            p.ody[(int64_t)row * p.oldd + c0 + e] = a4[e];
          }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ls += __shfl_xor(ls, o, 64);
        if (lane == 0) p.olossp[g + p.ont * rt] = ls;
      }
    }
  } else {
    p3d_core<RS, DEPTH, NACC, APK>(p.dZ, p.ldz, ngt, p.M, m0, p.Wd, ngt, ct, gb, ge, acc);
  }
  __shared__ XchgPub xpub;                  // exchange form: wave 0 posts its column sums, wave 1 publishes
  const bool pubw = WK > 1 && p.xchg && p.prev && p.bn && w == 1;
  if (pubw) p3d_xchg_pub_reset(&xpub);
  if (!p3d_reduce_waves<RS, NACC, WK>(acc, red)) {
    if (pubw) p3d_xchg_publish(p.xs, &xpub, p.K, by, n0);
    if (side_late && w == WK - 1 && lane == 0 && bx == 0 && by == 0) side_outputs();
    return;
  }
  const float mx = p.wsq ? fmaxf(sqrtf(*p.wsq), 1.0f) : 1.0f;
  // exchange form: the residual-gradient stores wait until after the swap (the sweeps' vmcnt
  // waits would otherwise wait for them too)
  const bool defer_draw = WK > 1 && p.xchg && p.prev && p.bn;
  float g[RS][4], dv[RS][4];
#pragma unroll
  for (int s = 0; s < RS; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * s + 4 * q + r;
      const float d = (p.wsq ? acc[0][s][r] / mx : acc[0][s][r]) + dr[s][r];
      if (p.draw && cok && row < p.M && !defer_draw) p.draw[p3d_pk(row, col, ngK)] = d;
      g[s][r] = d;
      dv[s][r] = d;
    }
  if (!p.prev) return;
  // previous layer: y = dropout(relu(BN(z))) ; recompute a = BN(z) for the relu mask
  float rstd = 1.f, inv = 1.f, shift = 0.f;
  if (p.bn) {
    rstd = 1.0f / sqrtf(var + p.eps);
    p3d_bn_affine(mean, var, p.eps, gam, bet, inv, shift);   // (1 / sqrt(var + eps)) * gamma, as rstd * gamma
  }
  float xh[RS][4];
  float sg = 0.f, sgx = 0.f;
  float uu[RS][4];
  if (p.keep < 1.0f) {
#pragma unroll
    for (int s = 0; s < RS; ++s) p3d_uniform_rows4(p.seed, ctr, p.site, p.row_off + m0 + 16 * s + 4 * q, cc, uu[s]);
  }
#pragma unroll
  for (int s = 0; s < RS; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * s + 4 * q + r;
      const bool ok = row < p.M;
      float gg = g[s][r];
      if (p.keep < 1.0f) gg = (gg * p3d_dropout_mask(p.keep, uu[s][r])) / p.keep;
      const float a = p.bn ? p3d_bn_y(zz[s][r], inv, shift) : zz[s][r];   // the forward's own rounding
      if (p.relu && !(a > 0.0f)) gg = 0.0f;
      if (!ok) gg = 0.0f;
      g[s][r] = gg;
      const float x = (zz[s][r] - mean) * rstd;
      xh[s][r] = x;
      sg += gg;
      sgx = __builtin_fmaf(gg, x, sgx);
    }
  if (p.bn) {
    sg = p3d_colsum16(sg);
    sgx = p3d_colsum16(sgx);
    if (p.xchg) {   // exchange form: the row-tile siblings swap {sum g, sum g xhat}
      const int R = gy;
      if (WK > 1) p3d_xchg_post(&xpub, q == 0, i, sg, sgx, xtag);
      else p3d_xchg_put(p.xs, p.K, by, col, q == 0 && cok, sg, sgx, xtag);
      float xsg, xsgx;
      if (R <= 4) p3d_xchg_sums<4>(p.xs, p.K, R, cc, xtag, by, xsg, xsgx);   // (wave-uniform)
      else p3d_xchg_sums<P3D_XCHG_MAXR, (WK >= 16 ? 8 : P3D_XCHG_MAXR)>(p.xs, p.K, R, cc, xtag, by, xsg, xsgx);
      p3d_xchg_done(p.xs, bx, by);
      if (defer_draw && p.draw && cok)
#pragma unroll
        for (int s = 0; s < RS; ++s)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + 16 * s + 4 * q + r;
            if (row < p.M) p.draw[p3d_pk(row, col, ngK)] = dv[s][r];
          }
      sg = xsg;
      sgx = xsgx;
      if (!cok) return;
      if (by == 0 && q == 0) { p.dgamma[col] = sgx; p.dbeta[col] = sg; }
      const float fmx = (float)p.M;
#pragma unroll
      for (int s = 0; s < RS; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + 16 * s + 4 * q + r;
          if (row < p.M) p.dz[p3d_pk(row, col, ngK)] = p3d_bn_dz(inv, fmx, g[s][r], sg, xh[s][r], sgx);
        }
      return;
    }
    if (p.bnpart) {   // split form: partials + g; k_bn_bwd forms dz, dgamma, dbeta
      if (!cok) return;
      if (q == 0) {
        p.bnpart[((int64_t)by * p.K + col) * 2] = sg;
        p.bnpart[((int64_t)by * p.K + col) * 2 + 1] = sgx;
      }
#pragma unroll
      for (int s = 0; s < RS; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + 16 * s + 4 * q + r;
          if (row < p.M) p.dz[p3d_pk(row, col, ngK)] = g[s][r];
        }
      return;
    }
    if (q == 0 && cok) { p.dgamma[col] = sgx; p.dbeta[col] = sg; }
  }
  if (!cok) return;
  const float fm = (float)p.M;
#pragma unroll
  for (int s = 0; s < RS; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * s + 4 * q + r;
      if (row >= p.M) continue;
      const float dz = p.bn ? p3d_bn_dz(inv, fm, g[s][r], sg, xh[s][r], sgx) : g[s][r];
      p.dz[p3d_pk(row, col, ngK)] = dz;
    }
}

template <int RS, int WK, int DEPTH, int NACC, bool APK, int KIND>
__global__ __launch_bounds__(64 * WK) void k_dgrad(BwdArgs p) {
  if (p.remap_gy > 0) {
    int bx, by;
    p3d_sibling_remap(blockIdx.x, (p.K + 15) >> 4, p.remap_gy, bx, by);
    p3d_dgrad_body<RS, WK, DEPTH, NACC, APK, KIND>(p, bx, by, p.remap_gy);
    return;
  }
  p3d_dgrad_body<RS, WK, DEPTH, NACC, APK, KIND>(p, blockIdx.x, blockIdx.y, gridDim.y);
}


// =====================================================================================
// BN-train backward, second half (split form): dz = inv/M * (M g - sum g - xhat sum g*xhat)
// from the row-tile partials, in place over g (packed), dgamma = sum g*xhat, dbeta = sum g.
// =====================================================================================
struct BnBwdArgs {
  float* dz; const float* z; const float* part;   // dz holds g on entry; [R][K][2]
  int M, K;
  const float* mean; const float* var; const float* gamma; float eps;
  float* dgamma; float* dbeta;
};

__global__ __launch_bounds__(64) void k_bn_bwd(BnBwdArgs p) {
  const int lane = threadIdx.x, ct = blockIdx.x, rt = blockIdx.y;
  const int j = lane & 15, q = lane >> 4;
  const int n0 = 16 * ct + 4 * q, row = 16 * rt + j;
  const int ngK = p.K >> 4;
  const int R = (p.M + 15) >> 4;
  const int64_t off = ((int64_t)rt * ngK + ct) * 256 + lane * 4;
  f32x4 pp[4][2];
  p3d_load_parts(p.part, p.M, p.K, n0, pp);
  const f32x4 g4 = *(const f32x4*)(p.dz + off);
  const f32x4 z4 = *(const f32x4*)(p.z + off);
  const f32x4 mu4 = *(const f32x4*)(p.mean + n0), va4 = *(const f32x4*)(p.var + n0);
  const f32x4 ga4 = *(const f32x4*)(p.gamma + n0);
  const float fm = (float)p.M;
  f32x4 o, sg4, sgx4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t < R) {
        sg += pp[t][e >> 1][(e & 1) * 2];
        sgx += pp[t][e >> 1][(e & 1) * 2 + 1];
      }
    for (int t = 4; t < R; ++t) {   // B > 64
      const float* pt = p.part + ((int64_t)t * p.K + n0 + e) * 2;
      sg += pt[0];
      sgx += pt[1];
    }
    sg4[e] = sg;
    sgx4[e] = sgx;
    const float rstd = 1.0f / sqrtf(va4[e] + p.eps);
    const float inv = rstd * ga4[e];
    const float xh = (z4[e] - mu4[e]) * rstd;
    o[e] = row < p.M ? p3d_bn_dz(inv, fm, g4[e], sg, xh, sgx) : 0.0f;
  }
  *(f32x4*)(p.dz + off) = o;
  if (rt == 0 && j == 0) {
    *(f32x4*)(p.dgamma + n0) = sgx4;
    *(f32x4*)(p.dbeta + n0) = sg4;
  }
}

// =====================================================================================
// weight gradient: dW[K,N] = X^T[K,M] * dZ[M,N];  db[N] = colsum(dZ)
// 64x64 output tile per 256-thread workgroup; wave w owns k-rows [16w,16w+16) and the
// four 16-column subtiles.  The batch (contraction) is staged through LDS in chunks of 64.
// =====================================================================================
struct WgradArgs {
  const float* X; int64_t ldx; int xpk;   // [M, K] packed (xpk) or row-major
  const float* dZ; int64_t ldz; int zpk;  // [M, N] packed (zpk) or row-major
  int M, K, N;
  float* dW;                      // [K, N] (TF layout, into the flat grads buffer)
  float* db;                      // [N] or null
  // fused Adam (single-GPU train step): instead of storing dW / db, apply the update to
  // W (flat offset woff) / b (boff) in w/m/v and re-pack the tile into Wf / Wd
  int adam; AdamFuse af;
  float* w; float* m; float* v; int64_t woff, boff;
  float* wd; float* wf;
  // ... and to the previous layer's BN gamma / beta ([K]; flat offsets goff / btoff), whose
  // gradients k_bn_bwd wrote to gflat just before (all readers of gamma/beta are done)
  int bn_adam; const float* gflat; int64_t goff, btoff;
  const float* alpha_dev;         // if set: the step's Adam alpha, formed by an earlier launch
};

#ifndef P3D_WG_PER_CU
// k_wgrad_multi / k_wgrad_grad workgroups per CU.  5 fits (32 KB LDS, <= 96 registers: cfg3's 1,056
// tiles in one round instead of 1,024 + a 32-tile tail) but measured SLOWER on the box: 28.6-28.9 vs
// 25.6-26.0 us per launch (r05_t8, three alternating pairs) -- five tiles' requests per CU contend
// more than the tail costs; 4 stays the default, 5 is a build option
#define P3D_WG_PER_CU 4
#endif
#define WG_LDS_STRIDE 80   // 64 + 16 pad: lanes q and q+1 (adjacent rows) hit disjoint banks

// Stage rows [mc, mc+64) x cols [c0, c0+64) of a packed or row-major [R, C] source, in two
// halves so that both operands' loads are in flight before the first LDS write: every load from
// a clamped (always valid) address, out-of-range elements zeroed after it.  (A load behind a
// per-element range branch made the compiler wait for each load on its own: 8 dependent memory
// round trips per staged chunk.)
struct Stage64 { float f[16]; unsigned ok; };
__device__ __forceinline__ void p3d_stage64_load(Stage64& st, const float* __restrict__ src, int pk, int64_t ld,
                                                 int R, int C, int mc, int c0, int tid = threadIdx.x) {
  st.ok = 0u;
  if (pk) {  // 16 packed 1 KB tiles (4 row tiles x 4 column groups); C is a multiple of 16
    const int ng = C >> 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + 256 * e, chunk = idx >> 6, ln = idx & 63;
      const int rt = chunk >> 2, gg = chunk & 3;
      const int row = 16 * rt + (ln & 15);
      const bool ok = mc + row < R && c0 + 16 * gg < C;
      st.ok |= ok ? (1u << e) : 0u;
      const int64_t off = ok ? ((int64_t)((mc >> 4) + rt) * ng + (c0 >> 4) + gg) * 64 + ln : 0;
      const f32x4 v = ((const f32x4*)src)[off];
#pragma unroll
      for (int j = 0; j < 4; ++j) st.f[4 * e + j] = v[j];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + 256 * k, m = e >> 6, c = e & 63;
      const bool ok = mc + m < R && c0 + c < C;
      st.ok |= ok ? (1u << k) : 0u;
      st.f[k] = src[ok ? (int64_t)(mc + m) * ld + c0 + c : 0];
    }
  }
}
// LDS image of a staged 64 x 64 chunk.  SW = false: rows WG_LDS_STRIDE floats apart; SW = true:
// rows 64 floats apart (16 KB per operand), column c of row r at c ^ (16 (r & 3)) -- the four
// row phases of a wave's MFMA operand reads land in four different 16-bank quarters.
template <bool SW>
__device__ __forceinline__ int p3d_wg_lidx(int r, int c) {
  return SW ? r * 64 + (c ^ ((r & 3) << 4)) : r * WG_LDS_STRIDE + c;
}
template <bool SW = false>
__device__ __forceinline__ void p3d_stage64_store(float* __restrict__ dst, const Stage64& st, int pk,
                                                  int tid = threadIdx.x) {
  if (pk) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + 256 * e, chunk = idx >> 6, ln = idx & 63;
      const int rt = chunk >> 2, gg = chunk & 3;
      const int row = 16 * rt + (ln & 15), col = 16 * gg + 4 * (ln >> 4);
      const bool ok = (st.ok >> e) & 1u;
      *(f32x4*)&dst[p3d_wg_lidx<SW>(row, col)] =
          ok ? f32x4{st.f[4 * e], st.f[4 * e + 1], st.f[4 * e + 2], st.f[4 * e + 3]} : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + 256 * k, m = e >> 6, c = e & 63;
      dst[p3d_wg_lidx<SW>(m, c)] = ((st.ok >> k) & 1u) ? st.f[k] : 0.f;
    }
  }
}

// dW tile (bx, by) = 64 columns x 64 rows of X^T dZ (and db from the by == 0 row of tiles)
#ifdef P3D_TRACE   // k_wgrad_multi timeline (tools/trace_wgrad.py): per workgroup at 4096 + 8 b
#define P3D_WG_STAMP(k)                                                                                 \
  do {                                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < 1500) g_p3d_trace[4096 + blockIdx.x * 8 + (k)] = wall_clock64(); \
  } while (0)
#else
#define P3D_WG_STAMP(k) do { } while (0)
#endif
// NOADAM: the gradient-only form (data-parallel steps, whose optimizer runs behind the
// all-reduce): no optimizer code.  Both forms: swizzled 16 KB operand images, db's partials in LDS
// the operands no longer need -- 32 KB of LDS -- and the staging addresses formed inside the chunk
// loop: 4 workgroups per CU (1,024 of cfg3's 1,056 tiles in the first round; round 4's 41 KB form
// held 3: 768 + 288).  With P3D_WG_PER_CU = 5 the fused Adam runs two rows of its four at a time and
// the layer is picked with constant indices: <= 96 registers, five per CU, one round -- measured
// slower (P3D_WG_PER_CU above).  The same arithmetic: the same bits.
template <bool NOADAM = false>
__device__ __forceinline__ void p3d_wgrad_tile(const WgradArgs& p, int bx, int by) {
  P3D_WG_STAMP(0);
  // both forms use the swizzled 16 KB operand images in one array, so the fused Adam's 64 x 65
  // transpose tile (16.6 KB) can run over into the dead dZ image
  constexpr int XS = 64 * 64;
  __shared__ __attribute__((aligned(16))) float xz[2 * XS];
  float* xs = xz;
  float* zs = xz + XS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int n0 = bx * 64, k0 = by * 64;
  f32x4 acc[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  // db's per-wave partials: in the X image once it is consumed (NOADAM), or past the part of the dZ
  // image the Adam transpose tile runs over (fused form: 64 x 65 floats from xs) -- no LDS of
  // their own, so the fused form fits five workgroups per CU (5 x 32 KB)
  float (*dbp)[64] = NOADAM ? reinterpret_cast<float (*)[64]>(xs) : reinterpret_cast<float (*)[64]>(zs + 1024);
  const bool do_db = p.db && by == 0;
  float dbs = 0.f;   // wave w: rows 16w .. 16w+15 of column `lane` (summed in row order)
  // the step's alpha, requested before the contraction (its latency hides there)
  const float alpha_pre = (!NOADAM && p.adam && p.alpha_dev) ? *p.alpha_dev : 0.f;
  for (int mc = 0; mc < p.M; mc += 64) {
    Stage64 sx, sz;
    // the staging addresses formed inside the chunk loop: hoisted out of it (a one-pass loop at
    // B = 64) they stayed live across the whole tile and, at five workgroups per CU, in scratch
    int tl = tid;
    asm volatile("" : "+v"(tl));
    p3d_stage64_load(sx, p.X, p.xpk, p.ldx, p.M, p.K, mc, k0, tl);
    p3d_stage64_load(sz, p.dZ, p.zpk, p.ldz, p.M, p.N, mc, n0, tl);
    p3d_stage64_store<true>(xs, sx, p.xpk, tl);
    p3d_stage64_store<true>(zs, sz, p.zpk, tl);
    __syncthreads();
    P3D_WG_STAMP(1);
#pragma unroll NOADAM ? 2 : 4
    for (int t = 0; t < 16; ++t) {
      const int m = 4 * t + q;
      const float a = xs[p3d_wg_lidx<true>(m, 16 * w + i)];
#pragma unroll
      for (int s = 0; s < 4; ++s)
        acc[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, zs[p3d_wg_lidx<true>(m, 16 * s + i)], acc[s], 0, 0, 0);
    }
    if (do_db) {
      if (NOADAM) {   // (the same sums, fewer registers live)
#pragma unroll
        for (int r = 0; r < 16; ++r) dbs += zs[p3d_wg_lidx<true>(16 * w + r, lane)];
      } else {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = zs[p3d_wg_lidx<true>(16 * w + r, lane)];
#pragma unroll
        for (int r = 0; r < 16; ++r) dbs += v[r];
      }
    }
    __syncthreads();
  }
  P3D_WG_STAMP(2);
  float alpha = 0.f;
  if (!NOADAM && p.adam)
    alpha = p.alpha_dev ? alpha_pre : p3d_adam_alpha(p.af.st, p.af.lr_host, p.af.lr0, p.af.decay_steps, p.af.decay_rate);
  if (do_db) {
    dbp[w][lane] = dbs;
    __syncthreads();
    if (w == 0 && n0 + lane < p.N) {
      const float gb = ((dbp[0][lane] + dbp[1][lane]) + dbp[2][lane]) + dbp[3][lane];
      if (!NOADAM && p.adam) {
        p.db[n0 + lane] = gb;   // the bias gradient stays visible in the grads buffer
        const int64_t o = p.boff + n0 + lane;
        float ww = p.w[o], mm = p.m[o], vv = p.v[o];
        p3d_adam1(ww, mm, vv, gb, alpha, 1.0f - p.af.b1, 1.0f - p.af.b2, p.af.eps);
        p.w[o] = ww; p.m[o] = mm; p.v[o] = vv;
      } else {
        p.db[n0 + lane] = gb;
      }
    }
  }
  if (!NOADAM && p.adam && p.bn_adam && bx == 0 && tid < 64 && k0 + tid < p.K) {
    const float omb1 = 1.0f - p.af.b1, omb2 = 1.0f - p.af.b2;
    const int64_t og = p.goff + k0 + tid, ob = p.btoff + k0 + tid;
    float w1 = p.w[og], m1 = p.m[og], v1 = p.v[og];
    p3d_adam1(w1, m1, v1, p.gflat[og], alpha, omb1, omb2, p.af.eps);
    p.w[og] = w1; p.m[og] = m1; p.v[og] = v1;
    float w2 = p.w[ob], m2 = p.m[ob], v2 = p.v[ob];
    p3d_adam1(w2, m2, v2, p.gflat[ob], alpha, omb1, omb2, p.af.eps);
    p.w[ob] = w2; p.m[ob] = m2; p.v[ob] = v2;
  }
  if (!NOADAM && p.adam) {
    // gradient tile -> LDS (reusing the staging buffer), then Adam + re-pack of W's tile
    float (*tile)[65] = reinterpret_cast<float (*)[65]>(xs);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[16 * w + 4 * q + r][16 * s + i] = acc[s][r];
    __syncthreads();
    p3d_adam_tile64<P3D_WG_PER_CU >= 5 ? 2 : 4>(tile, nullptr, p.woff, p.K, p.N, k0, n0, p.w, p.m, p.v, p.wd, p.wf, alpha,
                    1.0f - p.af.b1, 1.0f - p.af.b2, p.af.eps, p.af.wsrc);
#ifdef P3D_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    P3D_WG_STAMP(3);
    return;
  }
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 16 * w + 4 * q + r;
      const int n = n0 + 16 * s + i;
      if (k < p.K && n < p.N) p.dW[(int64_t)k * p.N + n] = acc[s][r];
    }
}

__global__ __launch_bounds__(256) void k_wgrad(WgradArgs p) { p3d_wgrad_tile(p, blockIdx.x, blockIdx.y); }

// Every layer's weight gradient in ONE launch (backward without fused Adam or gradient-ready
// events): a layer's dW / db depend only on its dZ and its input activations, which nothing
// later in the backward overwrites, so they can all wait for its end.  One grid over the
// tiles of all layers (1,056 workgroups at cfg2) replaces 2N + 2 launches of <= 256
// workgroups; every tile's arithmetic is k_wgrad's, so the gradients are bit-identical.
#define P3D_WG_MULTI 16
struct WgradLayer {
  const float* X; const float* dZ; float* dW; float* db;
  int64_t ldx, ldz; int xpk, zpk, M, K, N;
  // fused Adam (WgradArgs): flat offsets of W / b and of the previous layer's gamma / beta,
  // the layer's packed copies
  int bn_adam; int64_t woff, boff, goff, btoff; float* wd; float* wf;
};
struct WgradMulti {
  int n;
  int begin[P3D_WG_MULTI + 1];   // workgroup prefix over layers
  int gx[P3D_WG_MULTI];          // column tiles of each layer
  int adam; AdamFuse af; float* w; float* m; float* v; const float* gflat;
  const float* alpha_dev;        // fused Adam: alpha formed by an earlier launch of the step (or null)
  StepState* advance;            // if set: this launch's workgroup 0 advances the step state at its end
  WgradLayer ly[P3D_WG_MULTI];
};
template <bool NOADAM = false>
__device__ __forceinline__ void p3d_wgrad_multi_tile(const WgradMulti& mw, int b) {
  P3D_WG_STAMP(4);
  int j = 0;
  WgradArgs p{};
  int beg = 0, gx = 1;
  if (NOADAM) {
    // constant indices only (a runtime index into the argument block made the compiler copy it
    // to scratch at the 96-register budget)
#pragma unroll
    for (int k = 1; k < P3D_WG_MULTI; ++k)
      if (k < mw.n && b >= mw.begin[k]) j = k;
#pragma unroll
    for (int k = 0; k < P3D_WG_MULTI; ++k)
      if (k == j) {
        const WgradLayer& l = mw.ly[k];
        p.X = l.X; p.ldx = l.ldx; p.xpk = l.xpk; p.dZ = l.dZ; p.ldz = l.ldz; p.zpk = l.zpk;
        p.M = l.M; p.K = l.K; p.N = l.N; p.dW = l.dW; p.db = l.db;
        beg = mw.begin[k]; gx = mw.gx[k];
      }
    const int loc = b - beg;
    p3d_wgrad_tile<NOADAM>(p, loc % gx, loc / gx);
    return;
  }
#if P3D_WG_PER_CU >= 5
  // (the fused form at five per CU: the layer's fields picked with constant indices, as the
  // gradient-only form does -- mw.ly[j] at a runtime j kept 29 registers' worth in scratch)
#pragma unroll
  for (int k = 1; k < P3D_WG_MULTI; ++k)
    if (k < mw.n && b >= mw.begin[k]) j = k;
#pragma unroll
  for (int k = 0; k < P3D_WG_MULTI; ++k)
    if (k == j) {
      const WgradLayer& l = mw.ly[k];
      p.X = l.X; p.ldx = l.ldx; p.xpk = l.xpk; p.dZ = l.dZ; p.ldz = l.ldz; p.zpk = l.zpk;
      p.M = l.M; p.K = l.K; p.N = l.N; p.dW = l.dW; p.db = l.db;
      p.woff = l.woff; p.boff = l.boff; p.wd = l.wd; p.wf = l.wf;
      p.bn_adam = l.bn_adam; p.goff = l.goff; p.btoff = l.btoff;
      beg = mw.begin[k]; gx = mw.gx[k];
    }
  if (mw.adam) {
    p.adam = 1; p.af = mw.af; p.w = mw.w; p.m = mw.m; p.v = mw.v;
    p.gflat = mw.gflat; p.alpha_dev = mw.alpha_dev;
  }
  const int loc = b - beg;
  p3d_wgrad_tile<NOADAM>(p, loc % gx, loc / gx);
#else
  while (j + 1 < mw.n && b >= mw.begin[j + 1]) ++j;
  const WgradLayer& l = mw.ly[j];
  p.X = l.X; p.ldx = l.ldx; p.xpk = l.xpk; p.dZ = l.dZ; p.ldz = l.ldz; p.zpk = l.zpk;
  p.M = l.M; p.K = l.K; p.N = l.N; p.dW = l.dW; p.db = l.db;
  if (!NOADAM && mw.adam) {
    p.adam = 1; p.af = mw.af; p.w = mw.w; p.m = mw.m; p.v = mw.v; p.woff = l.woff; p.boff = l.boff;
    p.wd = l.wd; p.wf = l.wf;
    p.bn_adam = l.bn_adam; p.gflat = mw.gflat; p.goff = l.goff; p.btoff = l.btoff;
    p.alpha_dev = mw.alpha_dev;
  }
  const int loc = b - mw.begin[j];
  p3d_wgrad_tile<NOADAM>(p, loc % mw.gx[j], loc / mw.gx[j]);
#endif
}
template <bool NOADAM>
__device__ __forceinline__ void p3d_wgrad_multi_body(const WgradMulti& mw) {
  p3d_wgrad_multi_tile<NOADAM>(mw, blockIdx.x);
  // the step's last launch: nothing in it reads the step state (alpha came from alpha_dev),
  // so one thread may advance it here instead of a k_step_advance launch
  if (mw.advance && blockIdx.x == 0 && threadIdx.x == 0) {
    StepState* st = mw.advance;
    st->beta1_power = st->beta1_power * mw.af.b1;
    st->beta2_power = st->beta2_power * mw.af.b2;
    st->global_step = st->global_step + 1;
  }
}
__global__ __launch_bounds__(256, P3D_WG_PER_CU) void k_wgrad_multi(WgradMulti mw) { p3d_wgrad_multi_body<false>(mw); }
// the gradient-only form, P3D_WG_PER_CU workgroups per CU (see p3d_wgrad_tile)
__global__ __launch_bounds__(256, P3D_WG_PER_CU) void k_wgrad_grad(WgradMulti mw) { p3d_wgrad_multi_body<true>(mw); }

// =====================================================================================
// TF1 ApplyAdam fused with the weight re-pack (one launch per optimizer step)
//   alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
//   w -= (m*alpha)/(sqrt(v)+eps)                          (linear_model.py:137,145)
// Step state (global_step, beta powers) lives on the device so that whole training
// steps can be graph-captured: every block reads it first; the last block to finish
// (arrival counter) advances it.  lr is either given (lr_host >= 0) or the TF
// exponential decay lr0 * rate^(global_step / steps) computed on the device.
// Weight matrices are processed in 16x16 tiles (64 threads each) so that the updated
// tile is also written in both fragment-major layouts (Wd directly, Wf via an LDS
// transpose); 1-D tensors (biases, gamma, beta) are updated float-wise.
// =====================================================================================
struct AdamTable {
  int nw, nv;
  int K[P3D_MAX_W], N[P3D_MAX_W];
  int64_t off[P3D_MAX_W], wf[P3D_MAX_W], wd[P3D_MAX_W];
  int tile_begin[P3D_MAX_W + 1];   // 64x64 tiles, prefix over weights
  int64_t voff[P3D_MAX_V];
  int vlen[P3D_MAX_V];
  int vbegin[P3D_MAX_V + 1];       // 1024-element chunks, prefix over vectors
};

struct AdamArgs {
  float* w; float* m; float* v; const float* g;
  float* wpk;
  StepState* st;
  const float* alpha_dev;   // if set: the step's alpha, formed by the backward's first launch; block 0
  StepState* advance;       //   then advances the step state (nothing in the launch reads it) -- no
                            //   k_step_advance launch behind the optimizer
  float lr_host;        // >= 0: use as lr; < 0: device exponential decay of lr0
  float lr0, decay_steps, decay_rate;
  float b1, b2, eps;
  int wblocks;          // blocks spent on weight tiles (one 64x64 tile each)
  int wsrc;             // weights from Wd, TF-layout master not written (p3d_adam_tile64)
};

// One 64x64 weight tile per 256-thread block: 16 threads x float4 per 256-B row segment;
// the updated tile is staged in LDS and written as 16 Wd and 16 Wf fragment-major 1 KB
// chunks (64 lanes x float4 each, fully contiguous).
__global__ __launch_bounds__(256) void k_adam_pack(AdamArgs a, AdamTable tb) {
  __shared__ float tile[64][65];
  __shared__ float s_alpha;
  if (threadIdx.x == 0) {
    if (a.alpha_dev) {
      s_alpha = *a.alpha_dev;
      if (a.advance && blockIdx.x == 0) {
        StepState* st = a.advance;
        st->beta1_power = st->beta1_power * a.b1;
        st->beta2_power = st->beta2_power * a.b2;
        st->global_step = st->global_step + 1;
      }
    } else {
      const float b1p = a.st->beta1_power, b2p = a.st->beta2_power;
      float lr = a.lr_host;
      if (lr < 0.f) lr = a.lr0 * powf(a.decay_rate, (float)a.st->global_step / a.decay_steps);
      s_alpha = lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
    }
  }
  __syncthreads();
  const float alpha = s_alpha, omb1 = 1.0f - a.b1, omb2 = 1.0f - a.b2;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x < a.wblocks) {
    const int tile_id = blockIdx.x;
    int wi = 0;
    while (wi + 1 < tb.nw && tile_id >= tb.tile_begin[wi + 1]) ++wi;
    const int K = tb.K[wi], N = tb.N[wi];
    const int tnc = (N + 63) >> 6;
    const int local = tile_id - tb.tile_begin[wi];
    const int k0 = (local / tnc) * 64, n0 = (local % tnc) * 64;
    p3d_adam_tile64(tile, a.g, tb.off[wi], K, N, k0, n0, a.w, a.m, a.v, a.wpk + tb.wd[wi], a.wpk + tb.wf[wi],
                    alpha, omb1, omb2, a.eps, a.wsrc);
  } else {
    const int chunk = blockIdx.x - a.wblocks;
    if (chunk < tb.vbegin[tb.nv]) {
      int vi = 0;
      while (vi + 1 < tb.nv && chunk >= tb.vbegin[vi + 1]) ++vi;
      const int e0 = (chunk - tb.vbegin[vi]) * 1024 + 4 * tid;
      const int64_t i = tb.voff[vi] + e0;
      if (e0 + 3 < tb.vlen[vi]) {   // vectors start 256-B aligned in the flat buffer
        f32x4 ww = *(f32x4*)(a.w + i), mm = *(f32x4*)(a.m + i), vv = *(f32x4*)(a.v + i);
        const f32x4 gg = *(const f32x4*)(a.g + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float w1 = ww[e], m1 = mm[e], v1 = vv[e];
          p3d_adam1(w1, m1, v1, gg[e], alpha, omb1, omb2, a.eps);
          ww[e] = w1; mm[e] = m1; vv[e] = v1;
        }
        *(f32x4*)(a.w + i) = ww; *(f32x4*)(a.m + i) = mm; *(f32x4*)(a.v + i) = vv;
      } else {
        for (int e = 0; e < 4 && e0 + e < tb.vlen[vi]; ++e) {
          float ww = a.w[i + e], mm = a.m[i + e], vv = a.v[i + e];
          p3d_adam1(ww, mm, vv, a.g[i + e], alpha, omb1, omb2, a.eps);
          a.w[i + e] = ww; a.m[i + e] = mm; a.v[i + e] = vv;
        }
      }
    }
  }
}

// Advance the device step state after the optimizer (one thread; stream-ordered after
// every block of k_adam_pack has read the old state).
__global__ void k_step_advance(StepState* st, float b1, float b2) {
  st->beta1_power = st->beta1_power * b1;
  st->beta2_power = st->beta2_power * b2;
  st->global_step = st->global_step + 1;
}

// =====================================================================================
// pack every weight W [K, N] into Wf (rows n, cols k) and Wd (rows k, cols n padded)
// (after the host writes parameters; the optimizer re-packs inside k_adam_pack)
// =====================================================================================
struct PackTable {
  int n;
  int K[P3D_MAX_W], N[P3D_MAX_W];
  int64_t src[P3D_MAX_W], dstf[P3D_MAX_W], dstd[P3D_MAX_W];  // element offsets
  int64_t begin[P3D_MAX_W + 1];  // float4 prefix over (Wf + Wd) outputs
};

// The TF-layout master of every weight re-derived from its Wd copy (p3d_params_sync): a pure
// permutation, so the master equals what an optimizer writing it would have written, bit for bit.
struct UnpackTable {
  int n;
  int N[P3D_MAX_W];
  int64_t src[P3D_MAX_W], dstd[P3D_MAX_W];
  int64_t begin[P3D_MAX_W + 1];   // element prefix over the weights' K x N masters
};
__global__ __launch_bounds__(256) void k_unpack_w(const float* __restrict__ wpk, float* __restrict__ params,
                                                  UnpackTable ut) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= ut.begin[ut.n]) return;
  int t = 0;
  while (t + 1 < ut.n && o >= ut.begin[t + 1]) ++t;
  const int N = ut.N[t], ngd = ((N + 15) & ~15) >> 4;
  const int64_t e = o - ut.begin[t];
  const int k = (int)(e / N), n = (int)(e % N);
  params[ut.src[t] + e] = wpk[ut.dstd[t] + p3d_wd_at(k, n, ngd)];
}

__global__ __launch_bounds__(256) void k_pack(const float* __restrict__ params, float* __restrict__ wpk, PackTable pt) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= pt.begin[pt.n]) return;
  int t = 0;
  while (t + 1 < pt.n && o >= pt.begin[t + 1]) ++t;
  const int K = pt.K[t], N = pt.N[t], NP = (N + 15) & ~15;
  const float* W = params + pt.src[t];
  const int64_t local = o - pt.begin[t];
  const int64_t nf = (int64_t)NP * K / 4;   // float4s in Wf
  const bool isf = local < nf;
  const int64_t li = isf ? local : local - nf;
  const int64_t chunk = li >> 6;
  const int ln = (int)(li & 63);
  f32x4 v;
  if (isf) {  // rows n (NP), cols k (K): chunk = ct * (K/16) + g
    const int ngc = K >> 4;
    const int ctile = (int)(chunk / ngc), g = (int)(chunk % ngc);
    const int n = 16 * ctile + (ln & 15), k = 16 * g + 4 * (ln >> 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = n < N ? W[(int64_t)(k + e) * N + n] : 0.f;
    ((f32x4*)(wpk + pt.dstf[t]))[li] = v;
  } else {    // rows k (K), cols n (NP): chunk = kt * (NP/16) + g
    const int ngc = NP >> 4;
    const int kt = (int)(chunk / ngc), g = (int)(chunk % ngc);
    const int k = 16 * kt + (ln & 15), n = 16 * g + 4 * (ln >> 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (n + e) < N ? W[(int64_t)k * N + n + e] : 0.f;
    ((f32x4*)(wpk + pt.dstd[t]))[li] = v;
  }
}

// =====================================================================================
// MSE loss + gradient (single workgroup; deterministic)
// =====================================================================================
__global__ __launch_bounds__(256) void k_mse(const float* __restrict__ y, const float* __restrict__ t,
                                             int64_t n, float* loss, float* dy) {
  __shared__ float part[256];
  const float invn = 1.0f / (float)n;
  float s = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += 256) {
    const float d = y[e] - t[e];
    s += d * d;
    if (dy) dy[e] = invn * (d * 2.0f);
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) part[threadIdx.x] += part[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0 && loss) *loss = part[0] / (float)n;
}

// =====================================================================================
// per-tensor dot products (max-norm): out[t] = sum a_t * b_t   (two deterministic passes)
// =====================================================================================
struct DotTable {
  int n;
  int64_t off[P3D_MAX_W];
  int64_t len[P3D_MAX_W];
};

#define DOT_CHUNKS 64
__global__ __launch_bounds__(256) void k_dot_partial(const float* __restrict__ a, const float* __restrict__ b,
                                                     DotTable tb, float* __restrict__ part) {
  __shared__ float s[256];
  const int t = blockIdx.y;
  const float* pa = a + tb.off[t];
  const float* pb = b + tb.off[t];
  float acc = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tb.len[t]; e += (int64_t)DOT_CHUNKS * 256)
    acc += pa[e] * pb[e];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) s[threadIdx.x] += s[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[t * DOT_CHUNKS + blockIdx.x] = s[0];
}

__global__ void k_dot_final(const float* __restrict__ part, int n, float* __restrict__ out) {
  const int t = threadIdx.x;
  if (t >= n) return;
  float acc = 0.f;
  for (int c = 0; c < DOT_CHUNKS; ++c) acc += part[t * DOT_CHUNKS + c];
  out[t] = acc;
}

// max-norm gradient: g = G/m - [n>=1] <G,W> W / (m^2 n), n = ||W||, m = max(n,1)
__global__ __launch_bounds__(256) void k_maxnorm_grad(float* __restrict__ g, const float* __restrict__ w,
                                                      DotTable tb, const float* __restrict__ wsq,
                                                      const float* __restrict__ gw) {
  const int t = blockIdx.y;
  const float n = sqrtf(wsq[t]);
  const float m = fmaxf(n, 1.0f);
  const float c = n >= 1.0f ? gw[t] / (m * m * n) : 0.0f;
  float* pg = g + tb.off[t];
  const float* pw = w + tb.off[t];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tb.len[t]; e += (int64_t)gridDim.x * 256)
    pg[e] = pg[e] / m - c * pw[e];
}
