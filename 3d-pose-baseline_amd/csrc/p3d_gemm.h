// Large-batch fp32 layer: 128x128 output tile per workgroup on v_mfma_f32_16x16x4_f32.
//
// Used by the inference forward for the hidden layers of src/linear_model.py:154-201 when
// many independent batches are submitted in one launch (evaluateActionWise sweep,
// src/predict_3dpose.py:274-298, cfg4): M rows >= the large-M threshold.  The batch-64
// kernels (k_fwd) split K across eight waves of one 16x16 tile and are latency-bound;
// at M = 4096 that tiling re-reads every operand panel 64-256x from L2.  Here each wave
// owns a 64x64 sub-tile (4x4 MFMA tiles, 16 independent accumulator chains).  Operand
// tiles (fragment-major, 1 KB each, see p3d_kernels.h) stream into an NST-stage LDS ring
// by LDS-DMA (global_load_lds_dwordx4: one instruction moves one tile), KG k-groups per
// stage, each tile fetched once per workgroup and read by the two waves that share it
// (ds_read_b128).  Waits are explicit (s_waitcnt vmcnt on the DMA count): with plain
// register prefetch the compiler sinks the loads next to their use and waits vmcnt(0).
//
// The product is computed transposed (W fragment as MFMA A, X fragment as MFMA B), so a
// lane's four accumulator registers are four consecutive COLUMNS of one row -- exactly
// the packed activation layout: the epilogue (bias, max-norm scale, eval BN, ReLU,
// dropout, residual) works on float4s and stores each 16x16 tile as one 1 KB wave store.
#pragma once
#include "p3d_kernels.h"
#include "p3d_bf16.h"   // p3d_wait_stages

struct GemmF32Args {
  const float* A;            // packed [M, K] activations (ngA = K/16), or row-major [M, lda] (APK = false)
  int64_t lda;
  const float* Wf;           // packed [N, K] forward weight
  const float* bias;         // [N]
  const float* wsq;          // max-norm ||W||^2 or null
  int M, K, N;               // N % 128 == 0, K % 16 == 0
  int bn;                    // 0 / 1 (eval: moving statistics)
  const float* gamma; const float* beta; const float* mmean; const float* mvar; float eps;
  int relu;
  float keep; uint64_t seed; uint64_t ctr; int site; int64_t row_off;
  const int64_t* ctr_dev;
  const float* res;          // packed [M, N] residual (added after dropout) or null
  float* Y;                  // packed [M, N]
};

// APK = false: A is the row-major network input (the input layer, K = 32): lane (i, q) of
// A tile (rt, g) DMAs the 16 B at row 16rt+i (clamped to M-1), columns 16g+4q..+3 -- the same
// fragment the packed layout holds, so the rest of the kernel is unchanged.
template <int KG, int NST, bool APK = true>
__global__ __launch_bounds__(256) void k_gemm_f32(GemmF32Args p) {
  constexpr int STAGE = 16 * KG * 1024;   // 8 A + 8 B tiles per k-group
  constexpr int PER = 4 * KG;             // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) unsigned char smem[NST * STAGE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  // XCD-aware remap + grouped order (as k_gemm_bf16): an XCD's consecutive tile ids
  // cover GM row panels x (its share of) the column panels
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tiles_n = p.N / 128, tiles_m = (p.M + 127) / 128;
  const int GM = (tiles_m % 4 == 0) ? 4 : ((tiles_m % 2 == 0) ? 2 : 1);
  const int grp = tile_id / (GM * tiles_n), in_grp = tile_id % (GM * tiles_n);
  const int mt = grp * GM + (in_grp % GM), nt = in_grp / GM;
  const int ngA = p.K >> 4;
  const int nks = ngA / KG;
  const int rt_last = (p.M - 1) >> 4;   // last row tile holding valid rows

  // the PER tiles this wave DMAs per stage: source base (k-group 0) and LDS slot
  const unsigned char* src[PER];
  int slot[PER];
  int64_t sstep[PER];                     // source bytes per stage (KG k-groups)
#pragma unroll
  for (int c = 0; c < PER; ++c) {
    const int t = w * PER + c;            // 0 .. 16*KG-1
    const bool isB = t >= 8 * KG;
    const int tt = isB ? t - 8 * KG : t;
    const int jt = tt / KG, g = tt % KG;  // row tile jt (0..7) of the panel, k-group g
    int rt = isB ? 8 * nt + jt : 8 * mt + jt;
    if (!isB) rt = rt < rt_last ? rt : rt_last;   // tiles past M re-read the last one
    if (isB || APK) {
      src[c] = (const unsigned char*)(isB ? p.Wf : p.A) + ((int64_t)rt * ngA + g) * 1024 + lane * 16;
      sstep[c] = (int64_t)KG * 1024;
    } else {
      int row = 16 * rt + (lane & 15);
      row = row < p.M ? row : p.M - 1;
      src[c] = (const unsigned char*)(p.A + (int64_t)row * p.lda + 16 * g + 4 * (lane >> 4));
      sstep[c] = (int64_t)KG * 64;
    }
    slot[c] = t * 1024;
  }
  auto issue = [&](int ks, int buf) {
    unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int c = 0; c < PER; ++c)
      __builtin_amdgcn_global_load_lds((const void*)(src[c] + (int64_t)ks * sstep[c]), (void*)(base + slot[c]),
                                       16, 0, 0);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < NST - 1; ++s0)
    if (s0 < nks) issue(s0, s0);
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks % NST;
    if (ks + NST - 1 < nks) issue(ks + NST - 1, (ks + NST - 1) % NST);
    const int later = (nks - 1 - ks) < (NST - 1) ? (nks - 1 - ks) : (NST - 1);
    p3d_wait_stages<PER, NST>(later);
    __builtin_amdgcn_s_barrier();
    const unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      f32x4 af[4], bfr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) af[r] = *(const f32x4*)(base + ((4 * wm + r) * KG + g) * 1024 + lane * 16);
#pragma unroll
      for (int c = 0; c < 4; ++c) bfr[c] = *(const f32x4*)(base + (8 * KG + (4 * wn + c) * KG + g) * 1024 + lane * 16);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[c][e], af[r][e], acc[r][c], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // ---- epilogue: lane (j, q) of tile (r, c) holds row 16rt+j, columns 16ct+4q..+3 ----
  const int j = lane & 15, q = lane >> 4;
  const float mx = p.wsq ? fmaxf(sqrtf(*p.wsq), 1.0f) : 1.0f;
  const uint64_t ctr = p.ctr_dev ? (uint64_t)*p.ctr_dev : p.ctr;
  const int ngN = p.N >> 4;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ct = 8 * nt + 4 * wn + c;
    const int n0 = 16 * ct + 4 * q;
    const f32x4 b4 = *(const f32x4*)(p.bias + n0);
    f32x4 inv = f32x4{1.f, 1.f, 1.f, 1.f}, shift = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bn) {
      const f32x4 g4 = *(const f32x4*)(p.gamma + n0), be4 = *(const f32x4*)(p.beta + n0);
      const f32x4 mu4 = *(const f32x4*)(p.mmean + n0), va4 = *(const f32x4*)(p.mvar + n0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        inv[e] = (1.0f / sqrtf(va4[e] + p.eps)) * g4[e];
        shift[e] = be4[e] - mu4[e] * inv[e];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rt = 8 * mt + 4 * wm + r;
      if (rt > rt_last) continue;
      const int row = 16 * rt + j;
      const int64_t off = ((int64_t)rt * ngN + ct) * 256 + lane * 4;
      f32x4 rv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p.res) rv = *(const f32x4*)(p.res + off);
      float u[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.keep < 1.0f) {
        const uint4 wq = p3d_philox(make_uint4((uint32_t)(p.row_off + row), (uint32_t)(n0 >> 2), (uint32_t)p.site,
                                               (uint32_t)ctr), (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        const uint32_t xs[4] = {wq.x, wq.y, wq.z, wq.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = __uint_as_float((xs[e] & 0x7FFFFFu) | 0x3F800000u) - 1.0f;
      }
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z = (p.wsq ? acc[r][c][e] / mx : acc[r][c][e]) + b4[e];
        float y = p.bn ? z * inv[e] + shift[e] : z;
        if (p.relu) y = fmaxf(y, 0.0f);
        if (p.keep < 1.0f) y = (y / p.keep) * p3d_dropout_mask(p.keep, u[e]);
        if (p.res) y += rv[e];
        o[e] = y;
      }
      *(f32x4*)(p.Y + off) = o;
    }
  }
}
