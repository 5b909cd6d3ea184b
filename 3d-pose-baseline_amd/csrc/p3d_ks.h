// p3d_ks.h -- batch-norm training layers with the contraction split over K across workgroups
// (round 4; included by p3d.hip after k_fwd / k_dgrad).
//
// The exchange form (p3d_xchg.h) runs a BN-train hidden layer as 16 x 16 tiles: each workgroup
// contracts 16 rows x 16 columns over the whole K = 1024, i.e. takes in 64 KB of activations and
// 64 KB of weights (128 KB per CU, the GEMM phase's 2.7 us), and the 4 row-tile siblings of a
// column tile swap their column moments.  Here a workgroup owns a 64-row x 32-column block (every
// row of the batch) for one EIGHTH of K: 32 KB of activations + 16 KB of weights.  Its 8 waves are
// exactly the 8 waves of the exchange form's tiles -- wave (rt, c) contracts row tile rt of column
// tile 2 cp + c over k-groups [K/16 s/8, K/16 (s+1)/8) with the same MFMA chains -- so the 8
// sibling workgroups (s = 0..7) of a column pair hold what the 8 waves of a tile workgroup held,
// and the swap carries those partial products instead of moments: sibling s finalises columns
// 32 cp + 4 s .. +3 for all rows, summing the 8 partials in s order (k_fwd's wave order), so z,
// and everything after it, is bit-identical to the split and exchange forms; the batch statistics
// are then workgroup-local (no second swap).  The partials travel as data-tagged 16-B granules
// {a, tag, b, tag} (p3d_xchg.h's transport: a plain copy that stays in the producer XCD's L2 and
// an sc1 copy for a sibling placed elsewhere; the tag is the column pair's epoch word + 1, advanced
// by slice 0 once it has read every sibling's granules).
#pragma once
#include "p3d_xchg.h"

struct KsSite {
  unsigned* epoch;   // per column pair one word, P3D_XCHG_EPOCH_STRIDE words apart
  float* slots;      // [cp][src][dst][rt 4][16 lanes][2] 16-B granules, sc1 copy
  float* near;       // the same, plain-stored
  int* err;
};

__device__ __forceinline__ int64_t p3d_ks_granule(int cp, int src, int dst, int rt, int ll, int g) {
  return ((((int64_t)(cp * 8 + src) * 8 + dst) * 4 + rt) * 16 + ll) * 2 + g;
}

// Tile-moment sums of one row tile in k_fwd's order, in the finaliser layout (lane = 4 r16 + j:
// row r16 of the tile, column j): per group of 4 rows ((v0 + v1) + v2) + v3, then
// (S0 + S1) + (S2 + S3) -- what k_fwd's per-lane row loop and p3d_colsum16 compute.  Every lane
// with the same j ends holding the column's sum.
__device__ __forceinline__ float p3d_ks_tile_sum(float v) {
  const int lane = threadIdx.x & 63;
  const float v1 = __shfl(v, lane + 4, 64), v2 = __shfl(v, lane + 8, 64), v3 = __shfl(v, lane + 12, 64);
  float a = v + v1;
  a = a + v2;
  a = a + v3;
  a += __shfl_xor(a, 16, 64);
  a += __shfl_xor(a, 32, 64);
  return a;
}
// the same for the squares, as k_fwd's explicit fmaf chain per lane
__device__ __forceinline__ float p3d_ks_tile_sq(float d) {
  const int lane = threadIdx.x & 63;
  const float d1 = __shfl(d, lane + 4, 64), d2 = __shfl(d, lane + 8, 64), d3 = __shfl(d, lane + 12, 64);
  float a = __builtin_fmaf(d, d, 0.0f);
  a = __builtin_fmaf(d1, d1, a);
  a = __builtin_fmaf(d2, d2, a);
  a = __builtin_fmaf(d3, d3, a);
  a += __shfl_xor(a, 16, 64);
  a += __shfl_xor(a, 32, 64);
  return a;
}

// Block b of a 1-D grid of 8 * ncp blocks (ncp % 8 == 0): slice s and column pair cp, the 8 slices
// of a pair on one XCD under the round-robin placement (equal b % 8), dispatched together.
__device__ __forceinline__ void p3d_ks_place(int b, int& s, int& cp) {
  const int xcd = b & 7, jj = b >> 3;
  s = jj & 7;
  cp = (jj >> 3) * 8 + xcd;
}

// The swap, finaliser side: wave fw (row tile), lane (r16, j) collects the 8 partials of element
// (row 16 fw + r16, column 32 cp + 4 s + j); its own slice's comes from LDS (mine).
__device__ __forceinline__ void p3d_ks_gather(const KsSite& ks, int cp, int s, int fw, int r16, int j, unsigned tag,
                                              float mine, float (&pv)[8]) {
  const __amdgpu_buffer_rsrc_t rn = p3d_rsrc(ks.near), rs = p3d_rsrc(ks.slots);
  const int ll = j + 4 * (r16 >> 2), g = (r16 & 3) >> 1;
  const bool hi = (r16 & 1) != 0;
  bool got[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) { got[t] = t == s; pv[t] = mine; }
  for (int spin = 0;; ++spin) {
    const bool far_sweep = (spin & 7) == 7;
    const __amdgpu_buffer_rsrc_t rr = far_sweep ? rs : rn;
    u32x4_t v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
      v[t] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                 rr, (int)(p3d_ks_granule(cp, t, s, fw, ll, g) * 16), 0, 16));
    bool ok = true;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const bool hit = !got[t] & (v[t].y == tag) & (v[t].w == tag);
      pv[t] = hit ? __uint_as_float(hi ? v[t].z : v[t].x) : pv[t];
      got[t] = got[t] | hit;
      ok &= got[t];
    }
    if (__all(ok)) break;
    if (spin > P3D_XCHG_SPIN) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(ks.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Publisher side: tile-wave sw's partial (C layout: lane (i, q) holds column i, rows 4q .. 4q+3)
// to the sibling that finalises column i: dst = 4 c + (i >> 2), two granules per lane.
__device__ __forceinline__ void p3d_ks_publish(const KsSite& ks, int cp, int s, int sw, f32x4 v, unsigned tag) {
  const int lane = threadIdx.x & 63, i = lane & 15, q = lane >> 4;
  const int srt = sw & 3, sc = sw >> 2, dst = 4 * sc + (i >> 2);
  if (dst == s) return;
  const int ll = (i & 3) + 4 * q;
  const u32x4_t g0 = {__float_as_uint(v[0]), tag, __float_as_uint(v[1]), tag};
  const u32x4_t g1 = {__float_as_uint(v[2]), tag, __float_as_uint(v[3]), tag};
  const int o0 = (int)(p3d_ks_granule(cp, s, dst, srt, ll, 0) * 16);
  const __amdgpu_buffer_rsrc_t rn = p3d_rsrc(ks.near), rs = p3d_rsrc(ks.slots);
  __builtin_amdgcn_raw_buffer_store_b128(g0, rn, o0, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(g1, rn, o0 + 16, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(g0, rs, o0, 0, 16);   // aux 16 = sc1
  __builtin_amdgcn_raw_buffer_store_b128(g1, rs, o0 + 16, 0, 16);
}

// ---- forward: GEMM + bias + batch-stat BN (+ moving averages) + ReLU + dropout + residual --------
// Grid: 8 * (N / 32) blocks of 512 threads (N % 256 == 0, K % 128 == 0, M <= 64).
template <int DEPTH>
__global__ __launch_bounds__(512) void k_fwd_ks(FwdArgs p, KsSite ks) {
  __shared__ f32x4 own[8][64];      // each tile-wave's partial, C layout
  __shared__ float chs[4][4][2];    // per row tile and finalised column: {sum, M2 about the tile mean}
  __shared__ unsigned stag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int s, cp;
  p3d_ks_place(blockIdx.x, s, cp);
  const int R = (p.M + 15) >> 4;
  const int ngN = p.N >> 4;
  const int rt = w & 3, c = w >> 2, ct = 2 * cp + c;
  const int ngt = p.K >> 4;
  const int gb = (ngt * s) / 8, ge = (ngt * (s + 1)) / 8;
  if (threadIdx.x == 0)
    stag = __hip_atomic_load(ks.epoch + cp * P3D_XCHG_EPOCH_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  // finaliser element of waves 0..3: row 16 w + r16, column 32 cp + 4 s + j
  const int r16 = lane >> 2, j = lane & 3;
  const int frow = 16 * w + r16, fcol = 32 * cp + 4 * s + j;
  const bool fin = w < 4 && w < R;
  const bool valid = fin && frow < p.M;
  float fb = 0.f, fg = 1.f, fbt = 0.f, fmm = 0.f, fmv = 1.f, frs = 0.f;
  uint64_t ctr = p.ctr;
  if (fin) {
    fb = p.bias[fcol];
    fg = p.gamma[fcol]; fbt = p.beta[fcol];
    if (w == 0 && r16 == 0) { fmm = p.mmean[fcol]; fmv = p.mvar[fcol]; }
    if (p.res) frs = p.res[p3d_pk(valid ? frow : 0, fcol, ngN)];
    if (p.ctr_dev) ctr = (uint64_t)*p.ctr_dev;
  }
  // ---- contraction: the exchange form's wave s of tile (rt, ct) ----------------------------
  f32x4 acc[2][1];
  acc[0][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1][0] = acc[0][0];
  if (rt < R) p3d_core<1, DEPTH, 2, true>(p.X, p.ldx, ngt, p.M, 16 * rt, p.Wf, ngt, ct, gb, ge, acc);
  acc[0][0] += acc[1][0];
  own[w][lane] = acc[0][0];
  __syncthreads();
  const unsigned tag = stag;
  if (w >= 4) {
    // waves 4..7 publish every tile-wave's partial (the finalisers' sweeps then wait on loads only)
    const int pw = w - 4;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int sw = pw + 4 * t2;
      if ((sw & 3) < R) p3d_ks_publish(ks, cp, s, sw, own[sw][lane], tag);
    }
  }
  float u = 0.f, z = 0.f;
  if (fin) {
    if (p.keep < 1.0f) u = p3d_uniform(p.seed, ctr, p.site, p.row_off + frow, fcol);   // while siblings arrive
    const float mine = own[w + 4 * (s >> 2)][(4 * (s & 3) + j) + 16 * (r16 >> 2)][r16 & 3];
    float pv[8];
    p3d_ks_gather(ks, cp, s, w, r16, j, tag, mine, pv);
    if (s == 0 && w == 0 && lane == 0)   // every sibling has published, i.e. read the epoch
      __hip_atomic_fetch_add(ks.epoch + cp * P3D_XCHG_EPOCH_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float zs = pv[0];
#pragma unroll
    for (int t = 1; t < 8; ++t) zs += pv[t];
    const float mx = p.wsq ? fmaxf(sqrtf(*p.wsq), 1.0f) : 1.0f;
    z = (p.wsq ? zs / mx : zs) + fb;
    // this row tile's moments about its own mean (k_fwd's order)
    const int nt = min(16, p.M - 16 * w);
    const float sum = p3d_ks_tile_sum(valid ? z : 0.0f);
    const float mt = sum / (float)nt;
    const float sq = p3d_ks_tile_sq(valid ? z - mt : 0.0f);
    if (r16 == 0) { chs[w][j][0] = sum; chs[w][j][1] = sq; }
  }
  __syncthreads();
  if (!valid) return;
  // Chan's combination over the row tiles (p3d_xchg_moments' order)
  float S = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (t < R) S += chs[t][j][0];
  const float fm = (float)p.M;
  const float mean = S / fm;
  float M2 = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (t < R) M2 += p3d_chan_term(chs[t][j][0], chs[t][j][1], min(16, p.M - 16 * t), mean);
  const float var = M2 / fm;
  float inv, shift;
  p3d_bn_affine(mean, var, p.eps, fg, fbt, inv, shift);
  if (w == 0 && r16 == 0) {
    p.mean_save[fcol] = mean;
    p.var_save[fcol] = var;
    p.mmean[fcol] = p3d_bn_moving(fmm, mean, p.decay);
    p.mvar[fcol] = p3d_bn_moving(fmv, var, p.decay);
  }
  const int64_t o = p3d_pk(frow, fcol, ngN);
  if (p.z_save) p.z_save[o] = z;
  float y = p3d_bn_y(z, inv, shift);
  if (p.relu) y = fmaxf(y, 0.0f);
  if (p.keep < 1.0f) y = (y / p.keep) * p3d_dropout_mask(p.keep, u);
  if (p.res) y += frs;
  p.Y[o] = y;
}

// sum over a row tile of g * xhat in the data gradient's order (per lane fmaf chain over its 4
// rows, then p3d_colsum16), finaliser layout
__device__ __forceinline__ float p3d_ks_tile_dot(float g, float x) {
  const int lane = threadIdx.x & 63;
  const float g1 = __shfl(g, lane + 4, 64), g2 = __shfl(g, lane + 8, 64), g3 = __shfl(g, lane + 12, 64);
  const float x1 = __shfl(x, lane + 4, 64), x2 = __shfl(x, lane + 8, 64), x3 = __shfl(x, lane + 12, 64);
  float a = __builtin_fmaf(g, x, 0.0f);
  a = __builtin_fmaf(g1, x1, a);
  a = __builtin_fmaf(g2, x2, a);
  a = __builtin_fmaf(g3, x3, a);
  a += __shfl_xor(a, 16, 64);
  a += __shfl_xor(a, 32, 64);
  return a;
}

// ---- data gradient: dX = dZ W^T (+ residual gradient) with the previous layer's dropout / ReLU /
// batch-norm backward (dz, dgamma, dbeta) -- the 8-wave k_dgrad's association (p3d_dgrad_body).
template <int DEPTH>
__global__ __launch_bounds__(512) void k_dgrad_ks(BwdArgs p, KsSite ks) {
  __shared__ f32x4 own[8][64];
  __shared__ float chs[4][4][2];    // per row tile and finalised column: {sum g, sum g xhat}
  __shared__ unsigned stag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int s, cp;
  p3d_ks_place(blockIdx.x, s, cp);
  const int R = (p.M + 15) >> 4;
  const int ngK = p.K >> 4;
  const int rt = w & 3, c = w >> 2, ct = 2 * cp + c;
  const int ngt = p.ngB;
  const int gb = (ngt * s) / 8, ge = (ngt * (s + 1)) / 8;
  if (threadIdx.x == 0)
    stag = __hip_atomic_load(ks.epoch + cp * P3D_XCHG_EPOCH_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int r16 = lane >> 2, j = lane & 3;
  const int frow = 16 * w + r16, fcol = 32 * cp + 4 * s + j;
  const bool fin = w < 4 && w < R;
  const bool valid = fin && frow < p.M;
  float mean = 0.f, var = 1.f, gam = 1.f, bet = 0.f, zz = 0.f, dr = 0.f;
  uint64_t ctr = p.ctr;
  if (fin) {
    if (p.ctr_dev) ctr = (uint64_t)*p.ctr_dev;
    mean = p.mean[fcol]; var = p.var[fcol]; gam = p.gamma[fcol]; bet = p.beta[fcol];
    const int64_t o = p3d_pk(valid ? frow : 0, fcol, ngK);
    zz = p.z[o];
    if (p.dres) dr = p.dres[o];
  }
  f32x4 acc[2][1];
  acc[0][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1][0] = acc[0][0];
  if (rt < R) p3d_core<1, DEPTH, 2, true>(p.dZ, p.ldz, ngt, p.M, 16 * rt, p.Wd, ngt, ct, gb, ge, acc);
  acc[0][0] += acc[1][0];
  own[w][lane] = acc[0][0];
  __syncthreads();
  const unsigned tag = stag;
  if (w >= 4) {
    const int pw = w - 4;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int sw = pw + 4 * t2;
      if ((sw & 3) < R) p3d_ks_publish(ks, cp, s, sw, own[sw][lane], tag);
    }
    // the step's Adam alpha / the folded loss (side outputs nothing in this launch reads)
    if (w == 7 && lane == 0 && s == 0 && cp == 0) {
      if (p.alpha_out) *p.alpha_out = p3d_adam_alpha(p.af.st, p.af.lr_host, p.af.lr0, p.af.decay_steps, p.af.decay_rate);
      if (p.lossp) {
        float l = 0.f;
        for (int k = 0; k < p.nlossp; ++k) l += p.lossp[k];
        p.loss[0] = l * p.loss_scale;
      }
    }
  }
  float g = 0.f, xh = 0.f, inv = 1.f, rstd = 1.f;
  if (fin) {
    float u = 0.f;
    if (p.keep < 1.0f) u = p3d_uniform(p.seed, ctr, p.site, p.row_off + frow, fcol);
    const float mine = own[w + 4 * (s >> 2)][(4 * (s & 3) + j) + 16 * (r16 >> 2)][r16 & 3];
    float pv[8];
    p3d_ks_gather(ks, cp, s, w, r16, j, tag, mine, pv);
    if (s == 0 && w == 0 && lane == 0)
      __hip_atomic_fetch_add(ks.epoch + cp * P3D_XCHG_EPOCH_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float zs = pv[0];
#pragma unroll
    for (int t = 1; t < 8; ++t) zs += pv[t];
    const float mx = p.wsq ? fmaxf(sqrtf(*p.wsq), 1.0f) : 1.0f;
    const float d = (p.wsq ? zs / mx : zs) + dr;
    if (p.draw && valid) p.draw[p3d_pk(frow, fcol, ngK)] = d;
    float shift = 0.f;
    rstd = 1.0f / sqrtf(var + p.eps);
    p3d_bn_affine(mean, var, p.eps, gam, bet, inv, shift);
    float gg = d;
    if (p.keep < 1.0f) gg = (gg * p3d_dropout_mask(p.keep, u)) / p.keep;
    const float a = p3d_bn_y(zz, inv, shift);
    if (p.relu && !(a > 0.0f)) gg = 0.0f;
    if (!valid) gg = 0.0f;
    g = gg;
    xh = (zz - mean) * rstd;
    const float sg = p3d_ks_tile_sum(g);
    const float sgx = p3d_ks_tile_dot(g, xh);
    if (r16 == 0) { chs[w][j][0] = sg; chs[w][j][1] = sgx; }
  }
  __syncthreads();
  if (!valid) return;
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (t < R) { sg += chs[t][j][0]; sgx += chs[t][j][1]; }
  if (w == 0 && r16 == 0) { p.dgamma[fcol] = sgx; p.dbeta[fcol] = sg; }
  p.dz[p3d_pk(frow, fcol, ngK)] = p3d_bn_dz(inv, (float)p.M, g, sg, xh, sgx);
}
