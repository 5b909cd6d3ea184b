// p3d_kernels.h -- device-side building blocks shared by the p3d kernels (gfx950 only).
//
// HBM layouts
//   * user I/O (x [B,32], y [B,48], dy, targets): row-major fp32.
//   * weights: TF layout W [in, out] row-major is the master copy (p3d_param_ptr, Adam).
//     The library derives two "fragment-major" packed copies after every update:
//       Wf  -- forward operand  Bt[n][k] = W[k][n]   (rows = out features, cols = in)
//       Wd  -- dgrad operand    Bt[k][n] = W[k][n]   (rows = in features,  cols = out)
//   * activations / z / dz between layers: fragment-major packed.
//
// Fragment-major packing of an [R, C] matrix (R padded to 16, C a multiple of 16):
// 16x16 tiles, tile (rt, g) is 1 KB = 64 lanes x float4, lane l = i + 16q holding
// element (16rt + i, 16g + 4q + e) in component e.  That is exactly the operand a
// v_mfma_f32_16x16x4_f32 wave needs for four k-steps, so every operand load of the
// GEMM core is one perfectly contiguous 1 KB wave load (16 B per lane) straight into
// registers -- no LDS round trip, no partial cache lines.  Measured on MI355X
// (tools/kbench.hip): hidden layer 6.9 -> 3.9 us per launch vs row-major operands.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifdef P3D_TRACE   // development builds only: in-kernel phase timestamps (tools/trace_*.py)
__device__ unsigned long long g_p3d_trace[4096 * 8];
#endif

// buffer resource over a whole allocation (raw buffer loads / stores with scalar offsets)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t p3d_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// 16-B load with sc1 (bypasses this CU's L1; served by the XCD's L2): every read of data
// another CU of the group produced goes through this
__device__ __forceinline__ f32x4 p3d_ld_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}

// float offset of element (r, c) in a packed matrix with ng = C/16 column groups
__device__ __host__ __forceinline__ int64_t p3d_pk(int r, int c, int ng) {
  return (((int64_t)(r >> 4) * ng + (c >> 4)) << 8) + (((r & 15) + ((c & 15) >> 2) * 16) << 2) + (c & 3);
}

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

// The uniforms of rows row0 .. row0+3 of this lane's column `col` (u[r] = p3d_uniform(..,
// row0 + r, col)) in the MFMA C layout, where lane i + 16q holds column n0 + i and rows
// 4q + r: one Philox block per lane instead of four.  Lane 4a + j computes the block of
// (row0 + j, col >> 2), whose four words are the four columns of its lane quad; four
// rotations through ds_bpermute hand every lane its own column's word of all four rows.
// Requires the 4 lanes of a quad to share col >> 2 (n0 a multiple of 4) and row0 to be
// uniform over each 16-lane group.  All 64 lanes must execute it.
__device__ __forceinline__ void p3d_uniform_rows4(uint64_t seed, uint64_t ctr, int site, int64_t row0, int col,
                                                  float u[4]) {
  const int lane = threadIdx.x & 63;
  const uint4 w = p3d_philox(make_uint4((uint32_t)(row0 + (lane & 3)), (uint32_t)(col >> 2), (uint32_t)site,
                                        (uint32_t)ctr), (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int c = (lane - t) & 3;                       // the word my quad-mate wants from me
    const uint32_t give = c == 0 ? w.x : c == 1 ? w.y : c == 2 ? w.z : w.w;
    const int src = (lane & ~3) + ((lane + t) & 3);
    const uint32_t got = (uint32_t)__shfl((int)give, src, 64);
    u[(lane + t) & 3] = __uint_as_float((got & 0x7FFFFFu) | 0x3F800000u) - 1.0f;
  }
}

// tf.nn.dropout (TF1): binary = floor(keep + U); y = x / keep * binary
__device__ __forceinline__ float p3d_dropout_mask(float keep, float u) { return floorf(keep + u); }

// ------------------------------------------------------------------------------------
// GEMM core on v_mfma_f32_16x16x4_f32 (exact fp32: one fmaf rounding per product).
//
// One wave accumulates RS 16x16 tiles (rows m0+16s.., the 16 B-rows of column tile ct):
//   acc[s][i][j] += sum_{g in [gb, ge)} sum_{k in group g} A[m0+16s+i][k] * Bt[16ct+j][k]
// For k-group g (16 k's), lane (i, q) holds the float4 A[row][16g+4q..+3] and the float4
// Bt[col][16g+4q..+3]; MFMA step e (0..3) feeds component e, contracting
// k = {16g+4q+e : q = 0..3}.  NACC independent accumulator chains (component parity)
// hide the 40-cycle dependent-MFMA latency.  Loads run DEPTH groups ahead.
//   APK = true : A packed (ngA groups per row tile)
//   APK = false: A row-major with leading dimension lda (rows clamped to M-1)
//   B always packed (ngB groups per column tile)
// ------------------------------------------------------------------------------------
// SWAP = true computes the transposed product (B fragment as the MFMA A operand): the
// accumulator of lane (i, q) then holds row 16s + i, columns 4q .. 4q+3 of the tile (the
// fragment-major layout itself) instead of column i, rows 4q .. 4q+3.
template <int RS, int DEPTH, int NACC, bool APK, bool SWAP = false>
__device__ __forceinline__ void p3d_core(const float* __restrict__ A, int64_t lda, int ngA, int M, int m0,
                                         const float* __restrict__ Bp, int ngB, int ct, int gb, int ge,
                                         f32x4 (&acc)[NACC][RS]) {
  const int lane = threadIdx.x & 63;
  const int ng = ge - gb;
  if (ng <= 0) return;
  const f32x4* pa[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) {
    if (APK) {
      pa[s] = (const f32x4*)A + ((int64_t)((m0 >> 4) + s) * ngA + gb) * 64 + lane;
    } else {
      int r = m0 + 16 * s + (lane & 15);
      r = r < M ? r : M - 1;
      pa[s] = (const f32x4*)(A + (int64_t)r * lda + 16 * gb + 4 * (lane >> 4));
    }
  }
  const f32x4* pb = (const f32x4*)Bp + ((int64_t)ct * ngB + gb) * 64 + lane;
  constexpr int ASTR = APK ? 64 : 4;  // f32x4 stride between consecutive k-groups
  f32x4 ra[DEPTH][RS], rb[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const int g = d < ng ? d : ng - 1;
#pragma unroll
    for (int s = 0; s < RS; ++s) ra[d][s] = pa[s][g * ASTR];
    rb[d] = pb[g * 64];
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
            acc[e % NACC][s] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x4f32(rb[d][e], ra[d][s][e], acc[e % NACC][s], 0, 0, 0)
                                    : __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][s][e], rb[d][e], acc[e % NACC][s], 0, 0, 0);
        if (gi + DEPTH < ng) {
#ifndef P3D_DIAG_GA  // diagnostic builds only (tools/): re-read group d instead of streaming
#define P3D_DIAG_GA(g) (g)
#endif
#ifndef P3D_DIAG_GB
#define P3D_DIAG_GB(g) (g)
#endif
#pragma unroll
          for (int s = 0; s < RS; ++s) ra[d][s] = pa[s][P3D_DIAG_GA(gi + DEPTH) * ASTR];
          rb[d] = pb[P3D_DIAG_GB(gi + DEPTH) * 64];
        }
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

// Fold NACC chains and the WK k-split waves into wave 0 (deterministic order).
// Returns false for waves other than 0 (which then exit).
template <int RS, int NACC, int WK>
__device__ __forceinline__ bool p3d_reduce_waves(f32x4 (&acc)[NACC][RS], f32x4* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 1; a < NACC; ++a)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[0][s] += acc[a][s];
  if (WK == 1) return true;
  if (w > 0) {
#pragma unroll
    for (int s = 0; s < RS; ++s) red[((w - 1) * RS + s) * 64 + lane] = acc[0][s];
  }
  __syncthreads();
  if (w > 0) return false;
#pragma unroll
  for (int u = 1; u < WK; ++u)
#pragma unroll
    for (int s = 0; s < RS; ++s) acc[0][s] += red[((u - 1) * RS + s) * 64 + lane];
  return true;
}
