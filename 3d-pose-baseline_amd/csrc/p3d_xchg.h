// p3d_xchg.h -- batch-norm training layers as ONE launch (gfx950).
//
// tf.layers.batch_normalization in training mode (src/linear_model.py:112,181,193) needs each
// column's mean / variance over the whole batch before any output element of that column can
// be formed; the backward needs the column sums of g and g * xhat the same way.  The GEMM of a
// layer runs as 16 x 16 tiles, so a column's B = 64 rows sit in R = 4 row-tile workgroups.
//
// Split form (k_fwd bn = 3 + k_bn_fwd, k_dgrad + k_bn_bwd): the GEMM stores z and per-tile
// moments, a second launch combines them -- one extra dependent launch per BN layer and
// direction (~4.4 us each at cfg3, 10 per step).
//
// Exchange form (this file): the R row-tile workgroups of a column tile swap their per-column
// partials inside the GEMM launch and each finishes its own tile.  The partials travel as
// data-tagged granules (the R2 form of cdna_hip_programming.md Guideline 16: the data IS the
// flag, no flag word, no fence, no drain before a signal):
//   1. at kernel start lane 0 of wave 0 reads its COLUMN TILE's epoch word (agent-scope load);
//      the launch's tag is epoch + 1;
//   2. after the GEMM, wave 0 stores its 16 columns' pairs as {a, tag, b, tag} granules, twice:
//      a plain 16-B store into the `near` array (the line stays in this XCD's L2) and a
//      write-through (sc1) 16-B store into the `slots` array (the line leaves L2 for the
//      memory side: visible from every XCD), one 256-B run per workgroup each;
//   3. wave 0 re-reads the R siblings' `near` entries of its column with sc1 loads (L1
//      bypassed, served by its XCD's L2) until every tag equals this launch's, every 8th sweep
//      the `slots` entries too (bounded spin, s_sleep between sweeps), and combines them in
//      row-tile order -- the association of the split form's second kernel, so both forms give
//      the same bits (the helpers below are shared and compiled without FMA contraction).
//      A sibling on this XCD (the observed placement: siblings share blockIdx % 8) is read
//      from L2 in ~0.2 us per sweep; the sc1 copy is what keeps a sibling on another XCD
//      correct (its `near` line never reaches this L2), at the memory-side round trip
//      (~1 us per sweep, the cost of every sweep when only the sc1 copy existed: 2.9 us from
//      the last sibling's arrival to the end of the swap, tools/trace_train.py);
//   4. the row-tile-0 workgroup of the column tile, once it has read every sibling's entry, adds
//      1 to the tile's epoch word (agent atomic, no return).  Every sibling read that word before
//      publishing, and row tile 0 adds only after it has seen all of them, so the word changes
//      only after every sibling of this launch holds its tag: each launch's tag is unique
//      without a memset in front (graph replays included), stale entries of earlier launches
//      never match.  The word is the column tile's own (one 128-B line per tile): a shared word
//      per site would move once per column tile, and a workgroup dispatched after another
//      column tile had finished its swap would read a tag its siblings do not hold.
// Each site (layer and direction) has its own epoch words and slot array.  The siblings of a
// column tile have equal blockIdx % 8, i.e. one XCD under the observed round-robin placement
// (speed only, never correctness).  Every sibling must be resident at once: the host uses this
// form only when the grid fits on the device's CUs at one workgroup each.  Every spin is
// bounded (~0.5 s) and sets *err (p3d_sync_check) instead of hanging the GPU.
#pragma once
#include "p3d_kernels.h"

#ifndef P3D_XCHG_MAXR
#define P3D_XCHG_MAXR 16          // row tiles per exchange (B <= 256)
#endif
#define P3D_XCHG_SPIN (1 << 19)

// ---- arithmetic shared by the split and exchange forms (no FMA contraction) -------------
// BN affine of TF1's non-fused batch norm: inv = rsqrt(var + eps) * gamma, shift = beta - mean * inv
__device__ __forceinline__ void p3d_bn_affine(float mean, float var, float eps, float gam, float bet, float& inv,
                                              float& shift) {
#pragma clang fp contract(off)
  inv = (1.0f / sqrtf(var + eps)) * gam;
  shift = bet - mean * inv;
}
__device__ __forceinline__ float p3d_bn_y(float z, float inv, float shift) {
#pragma clang fp contract(off)
  return z * inv + shift;
}
// UPDATE_OPS moving average (momentum 0.99): m - (m - stat) * (1 - momentum)
__device__ __forceinline__ float p3d_bn_moving(float m, float stat, float decay) {
#pragma clang fp contract(off)
  return m - (m - stat) * decay;
}
// Chan's combination, one row tile's term: M2_t + n_t * (mean_t - mean)^2
__device__ __forceinline__ float p3d_chan_term(float s_t, float q_t, int nt, float mean) {
#pragma clang fp contract(off)
  const float d = s_t / (float)nt - mean;
  return q_t + (float)nt * d * d;
}
// BN-train data gradient: dz = inv / M * (M g - sum g - xhat * sum g xhat)
__device__ __forceinline__ float p3d_bn_dz(float inv, float fm, float g, float sg, float xh, float sgx) {
#pragma clang fp contract(off)
  return (inv / fm) * (fm * g - sg - xh * sgx);
}

// ---- the exchange ------------------------------------------------------------------------
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

#define P3D_XCHG_EPOCH_STRIDE 32   // words between two column tiles' epoch words (one 128-B line each)

struct XchgSite {
  unsigned* epoch;   // per column tile one word, P3D_XCHG_EPOCH_STRIDE words apart
  float* slots;      // [P3D_XCHG_MAXR row tiles][N columns] 16-B entries {a, tag, b, tag}, sc1-stored
  float* near;       // the same entries, plain-stored (L2-resident on the producer's XCD)
  int* err;          // host-visible error word (pinned): 1 = a spin ran out
  int delay;         // test hook (env P3D_XCHG_TEST_DELAY): odd column tiles' last row tile sleeps
                     // ~delay x 3.4 us before reading its tag (a late-dispatched sibling)
};

// This launch's tag for column tile ct (wave-uniform; read at kernel start so its latency
// hides under the GEMM).
__device__ __forceinline__ unsigned p3d_xchg_tag(const XchgSite& x, int ct, int rt, int R) {
  if (x.delay && (ct & 1) && rt == R - 1)
    for (int i = 0; i < x.delay; ++i) __builtin_amdgcn_s_sleep(127);
  return __hip_atomic_load(x.epoch + ct * P3D_XCHG_EPOCH_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

// The publishing is done by ANOTHER wave than the polling one.  A wave's s_waitcnt vmcnt
// covers its stores and loads together, in issue order: had the poller stored its own pair, each
// of its sweeps would also wait for that write-through store to be acknowledged by the memory
// side (~1 us), whatever the siblings' readiness.  So wave 0 posts its 16 pairs and the tag in
// LDS (p3d_xchg_post), and wave 1 -- whose K slice is already combined and which would exit
// otherwise -- stores them (p3d_xchg_publish) while wave 0 goes straight to its sweeps.
struct XchgPub {
  float a[16], b[16];
  unsigned tag;      // 0 until wave 0 posts (wave 1 zeroes it before the K-combine barrier)
};

__device__ __forceinline__ void p3d_xchg_pub_reset(XchgPub* pub) {   // wave 1, before the barrier
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(&pub->tag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// wave 0: lanes with q0 (one per column, lane i = column n0 + i) post their pair, then the tag
__device__ __forceinline__ void p3d_xchg_post(XchgPub* pub, bool q0, int i, float a0, float b0, unsigned tag) {
  if (q0) { pub->a[i] = a0; pub->b[i] = b0; }
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(&pub->tag, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// wave 1: wait for the post, store the 16 granules twice (plain: L2-resident near copy; sc1:
// memory-side copy) for columns n0 .. n0 + 15 < N of row tile rt
__device__ __forceinline__ void p3d_xchg_publish(const XchgSite& x, XchgPub* pub, int N, int rt, int n0) {
  unsigned tag;
  for (int spin = 0; (tag = __hip_atomic_load(&pub->tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0; ++spin) {
    if (spin > P3D_XCHG_SPIN) return;        // (wave 0 always posts)
    __builtin_amdgcn_s_sleep(1);
  }
  const int i = threadIdx.x & 63;
#ifdef P3D_TRACE
  const int tix = (n0 >> 4) + (N >> 4) * rt;
  if (i == 0 && tix < 2048) g_p3d_trace[16384 + tix * 8 + 1] = wall_clock64();
#endif
  if (i < 16 && n0 + i < N) {
    const u32x4_t v = {__float_as_uint(pub->a[i]), tag, __float_as_uint(pub->b[i]), tag};
    __builtin_amdgcn_raw_buffer_store_b128(v, p3d_rsrc(x.near), (rt * N + n0 + i) * 16, 0, 0);     // plain
    __builtin_amdgcn_raw_buffer_store_b128(v, p3d_rsrc(x.slots), (rt * N + n0 + i) * 16, 0, 16);   // aux 16 = sc1
  }
#ifdef P3D_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (i == 0 && tix < 2048) g_p3d_trace[16384 + tix * 8 + 2] = wall_clock64();
#endif
}

// Wave 0, all 64 lanes: lanes with `mine` publish their column's pair (one-wave form, WK = 1).
__device__ __forceinline__ void p3d_xchg_put(const XchgSite& x, int N, int rt, int col, bool mine, float a0, float b0,
                                             unsigned tag) {
  if (mine) {
    const u32x4_t v = {__float_as_uint(a0), tag, __float_as_uint(b0), tag};
    __builtin_amdgcn_raw_buffer_store_b128(v, p3d_rsrc(x.near), (rt * N + col) * 16, 0, 0);     // plain
    __builtin_amdgcn_raw_buffer_store_b128(v, p3d_rsrc(x.slots), (rt * N + col) * 16, 0, 16);   // aux 16 = sc1
  }
}

// Wave 0, all 64 lanes: every lane collects the R pairs of column `col` (a[t], b[t], t < R)
// once all R tags match (independent work of the caller can sit between put and get).
// NR: a compile-time bound on R.  Every sweep issues its NR loads unconditionally (entries past
// R re-read entry R - 1) and only then tests them: a load behind a runtime `t < R` branch made the
// compiler wait for each load on its own (vmcnt(0) per entry: R dependent round trips per sweep,
// ~3 us per exchange at R = 4), a straight run waits once per sweep.
// Entries t0 .. t0 + NR - 1 (those < R) into a[t], b[t] (t relative to t0).
template <int NR>
__device__ __forceinline__ void p3d_xchg_get_n(const XchgSite& x, int N, int R, int col, unsigned tag,
                                               float (&a)[NR], float (&b)[NR], int trace_rt, int t0 = 0) {
  const __amdgpu_buffer_rsrc_t rn = p3d_rsrc(x.near), rs = p3d_rsrc(x.slots);
#ifdef P3D_TRACE
  const int tix = (col >> 4) + (N >> 4) * trace_rt;
  if ((threadIdx.x & 63) == 0 && tix < 2048) g_p3d_trace[16384 + tix * 8 + 0] = wall_clock64();
  int sweeps = 0, far = 0;
#else
  (void)trace_rt;
#endif
  bool got[NR];
#pragma unroll
  for (int t = 0; t < NR; ++t) got[t] = t0 + t >= R;
  for (int spin = 0;; ++spin) {
    const bool far_sweep = (spin & 7) == 7;   // every 8th sweep: a sibling on another XCD (sc1 copy)
    const __amdgpu_buffer_rsrc_t rr = far_sweep ? rs : rn;
    u32x4_t v[NR];
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      const int e = t0 + t < R ? t0 + t : R - 1;
      v[t] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rr, (e * N + col) * 16, 0, 16));
    }
    bool ok = true;
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      const bool hit = !got[t] & (v[t].y == tag) & (v[t].w == tag);
      a[t] = hit ? __uint_as_float(v[t].x) : a[t];
      b[t] = hit ? __uint_as_float(v[t].z) : b[t];
      got[t] = got[t] | hit;
      ok &= got[t];
    }
#ifdef P3D_TRACE
    ++sweeps;
    far += far_sweep;
#endif
    if (__all(ok)) break;
    if (spin > P3D_XCHG_SPIN) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#ifdef P3D_TRACE
  if ((threadIdx.x & 63) == 0 && tix < 2048) {
    g_p3d_trace[16384 + tix * 8 + 3] = wall_clock64();
    g_p3d_trace[16384 + tix * 8 + 4] = sweeps;
    g_p3d_trace[16384 + tix * 8 + 5] = far;
  }
#endif
}

// The combination after the swap, over NR slots (NR = 4 for B <= 64: the combine loops then
// run 4 iterations, not 16 guarded ones -- 16 guarded Chan terms, each with its divide, had
// cost ~0.5 us per forward launch).  Forward: the batch mean / variance (Chan, row-tile order);
// backward: sum g, sum g xhat (row-tile order).  Same association as the split kernels.
// CH < NR (16-wave kernels, see p3d_xchg_sums): two passes over the entries in rounds of CH -- the
// sum (then the mean), then the Chan terms -- the same association as one pass over all NR.  The
// second pass re-reads entries that are already tagged (a slot is re-tagged only by the next launch
// of the site, stream-ordered behind this one): its sweeps match at once.
template <int NR, int CH = NR>
__device__ __forceinline__ void p3d_xchg_moments(const XchgSite& x, int N, int R, int col, unsigned tag, int rt,
                                                 int M, float& mean, float& var) {
  static_assert(NR % CH == 0, "p3d_xchg_moments: NR must be a multiple of CH");
  const float fm = (float)M;
  if constexpr (CH == NR) {
    float st[NR], qt[NR];
    p3d_xchg_get_n<NR>(x, N, R, col, tag, st, qt, rt);
    float S = 0.f;
#pragma unroll
    for (int t = 0; t < NR; ++t)
      if (t < R) S += st[t];
    mean = S / fm;
    float M2 = 0.f;
#pragma unroll
    for (int t = 0; t < NR; ++t)
      if (t < R) M2 += p3d_chan_term(st[t], qt[t], min(16, M - 16 * t), mean);
    var = M2 / fm;
  } else {
    float S = 0.f;
#pragma unroll
    for (int c0 = 0; c0 < NR; c0 += CH) {
      if (c0 >= R) break;
      float st[CH], qt[CH];
      p3d_xchg_get_n<CH>(x, N, R, col, tag, st, qt, rt, c0);
#pragma unroll
      for (int t = 0; t < CH; ++t)
        if (c0 + t < R) S += st[t];
    }
    mean = S / fm;
    float M2 = 0.f;
#pragma unroll
    for (int c0 = 0; c0 < NR; c0 += CH) {
      if (c0 >= R) break;
      float st[CH], qt[CH];
      p3d_xchg_get_n<CH>(x, N, R, col, tag, st, qt, rt, c0);
#pragma unroll
      for (int t = 0; t < CH; ++t)
        if (c0 + t < R) M2 += p3d_chan_term(st[t], qt[t], min(16, M - 16 * (c0 + t)), mean);
    }
    var = M2 / fm;
  }
}
// CH < NR: the entries in rounds of CH, each round summed (in row-tile order, so the same bits)
// before the next is fetched -- 16-wave kernels have 128 registers per lane, and 16 entries held
// at once spilled 64 of them to scratch (round 5, tools/kdev.hip).
template <int NR, int CH = NR>
__device__ __forceinline__ void p3d_xchg_sums(const XchgSite& x, int N, int R, int col, unsigned tag, int rt,
                                              float& sa, float& sb) {
  static_assert(NR % CH == 0, "p3d_xchg_sums: NR must be a multiple of CH");
  sa = 0.f;
  sb = 0.f;
#pragma unroll
  for (int c0 = 0; c0 < NR; c0 += CH) {
    if (c0 >= R) break;                                   // (wave-uniform)
    float at[CH], bt[CH];
    p3d_xchg_get_n<CH>(x, N, R, col, tag, at, bt, rt, c0);
#pragma unroll
    for (int t = 0; t < CH; ++t)
      if (c0 + t < R) { sa += at[t]; sb += bt[t]; }
  }
}

// Row tile 0 of column tile ct, after its swap: the tile's next launch gets a new tag.
__device__ __forceinline__ void p3d_xchg_done(const XchgSite& x, int ct, int rt) {
  if (rt == 0 && (threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(x.epoch + ct * P3D_XCHG_EPOCH_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
