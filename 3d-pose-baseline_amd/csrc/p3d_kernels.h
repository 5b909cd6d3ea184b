// p3d_kernels.h -- device-side building blocks shared by the p3d kernels (gfx950 only).
//
// Layout conventions (HBM):
//   activations  [B, features] row-major fp32, rows padded to a multiple of 4 floats
//   weights      TF layout [in, out] row-major (what p3d_param_ptr exposes), plus a
//                library-maintained transposed copy Wt [out, in] so that both the
//                forward (X * W) and the data-gradient (dZ * W^T) run as "NT" GEMMs whose
//                two operands are K-contiguous rows -> every operand load is a 16-byte
//                vector load straight into the MFMA fragment registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define P3D_WAVE 64

// ------------------------------------------------------------------------------------
// Philox4x32-10 (bit-identical with oracle/ref_mlp.py:philox4x32_10)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 p3d_philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
  }
  return c;
}

// U[0,1) for dropout element (global row g, col c) of site `site` at counter `ctr`.
__device__ __forceinline__ float p3d_uniform(uint64_t seed, uint64_t ctr, int site, int64_t g, int c) {
  const uint4 w = p3d_philox(make_uint4((uint32_t)g, (uint32_t)(c >> 2), (uint32_t)site, (uint32_t)ctr),
                             (uint32_t)seed, (uint32_t)(seed >> 32));
  const int s = c & 3;
  const uint32_t x = s == 0 ? w.x : s == 1 ? w.y : s == 2 ? w.z : w.w;
  return __uint_as_float((x & 0x7FFFFFu) | 0x3F800000u) - 1.0f;
}

// tf.nn.dropout (TF1): binary = floor(keep + U); y = x / keep * binary
__device__ __forceinline__ float p3d_dropout_mask(float keep, float u) { return floorf(keep + u); }

// ------------------------------------------------------------------------------------
// NT GEMM core on v_mfma_f32_16x16x4_f32.
//
// Computes, for one wave, RS accumulator tiles of 16x16:
//   acc[s][i][j] += sum_{k in [16*g_begin, 16*g_end)} A[m0+16s+i][k] * Bt[n0+j][k]
// Lane l = (i = l&15, q = l>>4).  For k-group g (16 k's) lane (i,q) loads the float4
// A[row][16g+4q .. +3] and Bt[col][16g+4q .. +3]; MFMA step e (0..3) feeds element e, so
// one step contracts k = {16g+4q+e : q=0..3} -- a permutation of k that makes every
// operand load a contiguous 16-byte vector (no LDS round trip needed).
// Loads run DEPTH groups ahead of the MFMAs (register ring, static indices).
// Out-of-range rows/cols are clamped (their results are never stored); K must be a
// multiple of 16 and rows 16-byte aligned (checked on the host).
// ------------------------------------------------------------------------------------
template <int RS, int DEPTH>
__device__ __forceinline__ void p3d_nt_core(const float* __restrict__ A, int64_t lda, int M, int m0,
                                            const float* __restrict__ Bt, int64_t ldb, int N, int n0,
                                            int g_begin, int g_end, f32x4 (&acc)[RS]) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, q = lane >> 4;
  const float* pa[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    int r = m0 + 16 * s + i;
    r = r < M ? r : M - 1;
    pa[s] = A + (int64_t)r * lda + 4 * q;
  }
  int c = n0 + i;
  c = c < N ? c : N - 1;
  const float* pb = Bt + (int64_t)c * ldb + 4 * q;

  const int ng = g_end - g_begin;
  if (ng <= 0) return;
  f32x4 ra[DEPTH][RS], rb[DEPTH];
  // prologue: issue DEPTH groups (indices clamped so every load is unconditional)
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const int g = g_begin + (d < ng ? d : ng - 1);
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
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int s = 0; s < RS; ++s)
            acc[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][s][e], rb[d][e], acc[s], 0, 0, 0);
        }
        int gn = gi + DEPTH;
        gn = g_begin + (gn < ng ? gn : ng - 1);
#pragma unroll
        for (int s = 0; s < RS; ++s) ra[d][s] = *(const f32x4*)(pa[s] + 16 * gn);
        rb[d] = *(const f32x4*)(pb + 16 * gn);
      }
    }
  }
}

// Sum across the 4 lane groups (lanes j, j+16, j+32, j+48) -> every lane gets the column total.
__device__ __forceinline__ float p3d_colsum16(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
