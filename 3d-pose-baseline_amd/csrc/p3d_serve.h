// p3d_serve.h -- persistent XCD-local inference of the pose-lifting network at batch 64.
//
// The reference evaluates as a sequence of independent batch-64 steps
// (src/predict_3dpose.py:352-444 calling LinearModel.step, src/linear_model.py:203-245).
// Run as one kernel chain per step (k_fwd, six launches), a step is bound by per-launch
// fixed costs (dispatch, operand latency, drain: ~4.5 us per layer for 0.85 us of MFMA
// work).  k_serve instead keeps the whole network of a step inside ONE XCD:
//
//   * grid = one 512-thread workgroup per CU.  Each workgroup reads its XCD id
//     (s_getreg HW_REG_XCC_ID) and joins that XCD's group (census: one returning atomic);
//     a one-time fan-in waits until every workgroup is resident and the census is final.
//   * the groups take the launch's batch-64 steps round-robin (step b -> group b % ngroups);
//     a group runs its steps one after another, every layer of a step spread over its ~32
//     CUs: unit u = 64 rows x 32 output columns (column tiles 2u, 2u+1).  The contraction
//     of a unit is split over the 8 waves (2 column tiles x 4 K-quarters), each wave
//     running four row tiles with a register ring of operand fragments loaded straight
//     from L2 (fragment-major 1 KB tiles, p3d_kernels.h: every operand byte is loaded once
//     per CU, no LDS staging); the K-quarter partials meet in LDS and are summed in fixed
//     order.  The product is transposed, so the epilogue (max-norm scale, bias, eval BN,
//     ReLU, residual) works on float4s and stores whole 1 KB tiles.
//   * layer -> layer hand-off stays inside the XCD's L2: producers store plainly (the L1 is
//     write-through), drain (s_waitcnt vmcnt(0)) and publish a per-member phase flag (plain
//     store: it lands in the same L2); consumers poll the members' flags and read the
//     activations with sc1 loads (L1 bypass, served by the shared L2).  Grouping by the
//     XCD id read from the hardware -- not by blockIdx -- is what makes that hand-off valid.
//   * the next layer's weight fragments (which do not depend on the hand-off) are loaded
//     into the ring between the drain and the flag poll, so their latency hides under the
//     barrier; bias / BN / residual / W4 operands are loaded before the contraction.
//   * the output layer (N = 48) is fused into the last hidden layer's epilogue: every unit
//     multiplies its 64 x 32 slice of the block output by the matching 32 rows of W4 and
//     stores a 64 x 48 partial; the next phase (the next step's input layer) sums the
//     partials in fixed unit order (deterministic) and writes y = sum / maxnorm + b4.
//
// Phases per step: input layer (+ the previous step's output reduction), then the 2N
// hidden layers, one group barrier after each.  Results are those of a batch-64 forward
// (eval BN, keep_prob 1), deterministic and independent of where the workgroups land.
#pragma once
#include "p3d_kernels.h"

#define P3D_SERVE_MAXL 16          // input + 2*blocks + output layers
// layers whose epilogue constants k_serve5 keeps in LDS (input + hidden): 15, or 9 (N <= 4
// blocks) for the 8-column-tile form, whose K-combine buffer takes 128 KB
#ifndef P3D_SERVE_IN_EARLY
#define P3D_SERVE_IN_EARLY 0       // next step's input-layer operands requested after the K-combine
#endif
#ifndef P3D_S4_RE                  // 8-column-tile form (SPLIT 4, UPM 4) variants
#define P3D_S4_RE 2                // output-reduction elements per lane
#endif
#ifndef P3D_S4_WOPIPE
#define P3D_S4_WOPIPE 0            // next unit's output-layer operands during this unit's partial
#endif
#ifndef P3D_S4_INPIPE
#define P3D_S4_INPIPE 0            // next unit's input-layer operands during this unit's layer
#endif
#define P3D_SERVE_ECL(NC) ((NC) >= 8 ? 9 : P3D_SERVE_MAXL - 1)
// sync words: [32 x] census counter of XCD x (a 128-B line each: the 32 arrivals of an XCD
// serialise on their own line, the 8 XCDs' in parallel -- one counter for all 256 workgroups
// serialised 256 atomics, ~9.6 us per launch), [P3D_SERVE_FLAG0 + 64 g + r] flag of member r
// of group g
#define P3D_SERVE_FLAG0 256
#define P3D_SERVE_SYNC_WORDS (P3D_SERVE_FLAG0 + 64 * 64)   // flags of up to 64 groups (k_serve6 S <= 8)
// the model's serve sync allocation: k_serve6 banks 0 / 1 (group flags), the k_serve5 bank, then
// k_serve6's 64 per-group-slot epoch words (bank = epoch & 1)
#define P3D_SERVE_SYNC_ALL (3 * P3D_SERVE_SYNC_WORDS + 64)
#define P3D_SERVE_GROUPS 32        // XCD groups (k_serve5 SPLIT = 4: four per XCD)
#define P3D_SERVE6_ROWS 4096       // k_serve6: rows in flight (8 S groups x 16 RT rows) its slabs hold
#define P3D_SERVE_SPIN (1 << 22)   // bounded spins (~0.5 s): a stuck group reports instead of hanging
#ifndef P3D_SERVE_SLICE_WAIT       // k_serve5: each wave waits only for the members its K slice reads
#define P3D_SERVE_SLICE_WAIT 1
#endif
#ifndef P3D_SERVE_PREFETCH_B       // request the next layer's weight fragments inside the barrier
#define P3D_SERVE_PREFETCH_B 1
#endif
#ifndef P3D_SERVE_EPI_EARLY        // bias / BN / residual / W4 operands requested before the contraction
#define P3D_SERVE_EPI_EARLY 1
#endif
#ifndef P3D_SERVE_RV_LATE          // k_serve5: residual operands requested after the contraction
#define P3D_SERVE_RV_LATE 1
#endif

// Phase timestamps for development (-DP3D_TRACE, tools/trace_serve.py): workgroup rank 0
// (and rank 1) of every XCD group, first 8 local steps, up to 8 stamps per phase (0 begin,
// 1 compute done, 2 barrier passed, 3 contraction done, 4 K-partials combined) into
// g_p3d_trace (p3d_kernels.h).
#ifdef P3D_TRACE
#define P3D_SERVE_TR(xcc, r, jl, ph) \
  (((r) < 2 && (jl) < 8 && (ph) < 16) ? g_p3d_trace + 8192 + (r) * 8192 + ((((xcc) * 8 + (jl)) * 16 + (ph)) * 8) : nullptr)
#define P3D_SERVE_STAMP(tr, k)                                  \
  do {                                                          \
    if ((tr) && threadIdx.x == 0) (tr)[k] = wall_clock64();     \
  } while (0)
#else
#define P3D_SERVE_TR(xcc, r, jl, ph) ((unsigned long long*)nullptr)
#define P3D_SERVE_STAMP(tr, k) do { (void)(tr); } while (0)
#endif

struct ServeLayer {
  const float* Wf;     // packed forward weight [N, K] (ngK = K/16 groups per column tile)
  const float* bias;
  const float* gamma; const float* beta; const float* mmean; const float* mvar;
  const float* wsq;    // max-norm ||W||^2 or null
};

struct ServeArgs {
  const float* x;      // [M, K0] row-major network input
  float* y;            // [M, ND] row-major output
  int64_t M;           // rows; step b covers rows [64b, 64b + 64)
  int nb;              // steps = ceil(M / 64)
  int L, K0, ND, nblk; // linear_size, input_size (<= 64), output_size (<= 64), residual blocks
  int bn, residual; float eps;
  float* act;          // [8][3][64 * L] packed activations per XCD group
  float* part;         // [groups][2][L/16][4 * NDT * 256] output partials per XCD group (step parity)
  unsigned* sync;      // k_serve5: its P3D_SERVE_SYNC_WORDS, zeroed before every launch; k_serve6: bank 0
                       // of two consecutive banks (the launch picks one by *epoch)
  int* err;            // host-visible (pinned) error word: 1 = a bounded spin ran out, 2 = a placement
                       // the launch was not sized for
  unsigned* epoch;     // k_serve6: per group slot (<= 64) its epoch word (bank = epoch & 1)
  int delay, delay_xcc;  // k_serve6 test hook (P3D_SERVE_TEST_DELAY): the workgroups on XCD delay_xcc start late
  int census_extra;    // test hook: k_serve5's census waits for this many workgroups beyond the grid; k_serve6 takes it as a placement failure
  int max_groups;      // steps are dealt over at most this many XCD groups (others idle)
  int split;           // k_serve6: groups per XCD (1..4)
  const float* ecg;    // k_serve6: epilogue constants per layer and 16-column tile (k_serve_prep)
  // fused MSE (p3d_serve_mse, k_serve6 only; tgt == nullptr: off): targets [M, ND] row-major, one
  // squared-error partial per output tile (lpart), an arrival counter (lcnt, zero between launches)
  // and the loss word mean((y - t)^2) the last arriving tile writes (src/linear_model.py:129)
  const float* tgt;
  float* lpart;
  unsigned* lcnt;
  float* loss;
  // p3d_serve_mse_sync: host-visible completion word (pinned, coherent; null: off) and the call's
  // sequence number, stored by the last arriving tile once every output row and the loss are
  // system-visible (each tile's wave fences its own rows at system scope before it arrives)
  unsigned* hflag;
  unsigned hseq;
  ServeLayer ly[P3D_SERVE_MAXL];
};


// Census (thread 0 of every workgroup): the XCD id read from the hardware, the workgroup's
// rank within its XCD (one returning atomic on that XCD's counter), then a wait until the
// eight counters sum to the grid (every workgroup resident, every count final).  sh[0] = XCD,
// sh[1] = rank, sh[8 + x] = workgroups on XCD x, sh[2] = 1 if the wait timed out or an XCD
// holds more than maxn workgroups (the flag barriers poll one lane per member).  In two
// halves, so a kernel can do independent work between its arrival and the wait.
__device__ __forceinline__ void p3d_serve_census_arrive(unsigned* sync, int* sh) {
  if (threadIdx.x == 0) {
    unsigned xr;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xr));
    const int xcc = (int)(xr & 7u);
    sh[0] = xcc;
    sh[1] = (int)__hip_atomic_fetch_add(sync + 32 * xcc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
}
__device__ __forceinline__ void p3d_serve_census_wait(const ServeArgs& p, unsigned* sync, int* sh, int maxn) {
  if (threadIdx.x == 0) {
    int bad = 0, spin = 0;
    unsigned c[8];
    const unsigned expect = gridDim.x + (unsigned)p.census_extra;
    while (true) {
      unsigned tot = 0;
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        c[x] = __hip_atomic_load(sync + 32 * x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tot += c[x];
      }
      if (tot >= expect) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spin > P3D_SERVE_SPIN) { bad = 1; break; }
    }
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      sh[8 + x] = (int)c[x];
      if ((int)c[x] > maxn) bad = 1;   // judged on every XCD's count: all workgroups decide alike
    }
    if (bad) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    sh[2] = bad;
  }
  __syncthreads();
}
__device__ __forceinline__ void p3d_serve_census(const ServeArgs& p, int* sh, int maxn) {
  p3d_serve_census_arrive(p.sync, sh);
  p3d_serve_census_wait(p, p.sync, sh, maxn);
}

// ---- register ring -------------------------------------------------------------------
// The unit's contraction (64 rows x 32 columns x L) is split over the 8 waves along K.
//   KS = 8: wave w owns k-groups [w*ngL/8, (w+1)*ngL/8) of all 4 row tiles x 2 column
//           tiles: per k-group 4 A + 2 B fragments for 32 MFMAs, every operand byte loaded
//           once per CU (384 KB per layer at L = 1024).
//   KS = 4: wave (kq, ct) owns k-groups [kq*ngL/4, ..) of the 4 row tiles of column tile
//           ct: 4 A + 1 B per 16 MFMAs, A loaded by both waves of a K-quarter.
template <int DEPTH, int KS>
struct ServeRingA {
  f32x4 a[DEPTH][4];            // activation fragments of the four row tiles
};
template <int DEPTH, int KS>
struct ServeRingB {
  f32x4 b[DEPTH][KS / 4];       // weight fragments of this wave's column tile(s)
};

template <int KS>
__device__ __forceinline__ int p3d_ring_gb(int ngL) {
  const int w = threadIdx.x >> 6;
  return KS == 8 ? (ngL * w) >> 3 : (ngL * (w >> 1)) >> 2;
}

// wave's first weight fragment: column tile 2u (KS = 8) or 2u + ct (KS = 4)
template <int KS>
__device__ __forceinline__ const f32x4* p3d_ring_bptr(const float* Wf, int u, int ngL) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ct0 = KS == 8 ? 0 : (w & 1);
  return (const f32x4*)Wf + ((int64_t)(2 * u + ct0) * ngL + p3d_ring_gb<KS>(ngL)) * 64 + lane;
}

template <int DEPTH, int KS>
__device__ __forceinline__ void p3d_ring_load_b(ServeRingB<DEPTH, KS>& R, const float* Wf, int u, int ngL) {
  const f32x4* pb = p3d_ring_bptr<KS>(Wf, u, ngL);
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int c = 0; c < KS / 4; ++c) R.b[d][c] = pb[(c * ngL + d) * 64];
}

template <int DEPTH, int KS>
__device__ __forceinline__ void p3d_ring_load_a(ServeRingA<DEPTH, KS>& R, const float* A, int ngL) {
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t ra = p3d_rsrc(A);
  const int aoff0 = (p3d_ring_gb<KS>(ngL) * 64 + lane) * 16, rstride = ngL * 1024;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int t = 0; t < 4; ++t) R.a[d][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + d * 1024);
}

// The unit's contraction, the ring's first DEPTH k-groups already requested.  The wave's
// ngL/KS k-groups are a multiple of DEPTH (host): straight-line rounds, so the compiler
// tracks the ring's loads exactly (vmcnt(N) waits, no drain at a loop head).  Returns this
// wave's tile (row tile w >> 1, column tile 2u + (w & 1)) in the transposed layout, its
// KS K-slice partials summed in slice order (deterministic).
template <int DEPTH, int KS>
__device__ __forceinline__ f32x4 p3d_ring_run(ServeRingA<DEPTH, KS>& RA, ServeRingB<DEPTH, KS>& RB, const float* A,
                                              const float* Wf, int u, int ngL, f32x4* red, unsigned long long* tr) {
  constexpr int NC = KS / 4;     // column tiles per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kq = KS == 8 ? w : (w >> 1), ct0 = KS == 8 ? 0 : (w & 1);
  const int ng = ngL / KS;
  const __amdgpu_buffer_rsrc_t ra = p3d_rsrc(A);
  const int aoff0 = (p3d_ring_gb<KS>(ngL) * 64 + lane) * 16, rstride = ngL * 1024;
  const f32x4* pb = p3d_ring_bptr<KS>(Wf, u, ngL);
  f32x4 acc[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[c][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#ifndef P3D_SERVE_DIAG_A   // diagnostic builds (tools/trace_serve.py): re-read early k-groups
#define P3D_SERVE_DIAG_A(g) (g)
#endif
#ifndef P3D_SERVE_DIAG_B
#define P3D_SERVE_DIAG_B(g) (g)
#endif
  for (int g0 = 0; g0 < ng - DEPTH; g0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[c][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(RB.b[d][c][e], RA.a[d][t][e], acc[c][t], 0, 0, 0);
      const int gn = g0 + DEPTH + d;
#pragma unroll
      for (int t = 0; t < 4; ++t) RA.a[d][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + P3D_SERVE_DIAG_A(gn) * 1024);
#pragma unroll
      for (int c = 0; c < NC; ++c) RB.b[d][c] = pb[(c * ngL + P3D_SERVE_DIAG_B(gn)) * 64];
      // keep the refill of slot d here, ahead of slot d+1's MFMAs: left alone the scheduler
      // sinks every refill to the end of the round, exposing the full load latency there
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[c][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(RB.b[d][c][e], RA.a[d][t][e], acc[c][t], 0, 0, 0);
  P3D_SERVE_STAMP(tr, 3);
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t) red[((kq * 4 + t) * 2 + ct0 + c) * 64 + lane] = acc[c][t];
  __syncthreads();
  P3D_SERVE_STAMP(tr, 4);
  f32x4 s = red[w * 64 + lane];   // slice 0, tile (w >> 1, w & 1)
#pragma unroll
  for (int k = 1; k < KS; ++k) s += red[(k * 8 + w) * 64 + lane];
  __syncthreads();
  return s;
}

// ---- epilogue: lane (j, q) of the tile holds row 16rt + j, columns n0 .. n0+3 ---------
struct ServeEpi {
  f32x4 b, g, be, mu, va;
  float mx;
};

// Requested before the contraction; the BN factors are formed after it (forming them here
// would make the wave wait for these loads -- and, vmcnt being in order, for every ring load
// issued before them -- before its first MFMA: measured +2.2 us per layer).
__device__ __forceinline__ ServeEpi p3d_epi_load(const ServeLayer& ly, int n0, int bn, float eps) {
  (void)eps;
  ServeEpi e;
  e.mx = ly.wsq ? *ly.wsq : 1.0f;   // ||W||^2 here; maxnorm = max(sqrt(.), 1) in the apply
  e.b = *(const f32x4*)(ly.bias + n0);
  e.g = e.be = e.mu = e.va = f32x4{0.f, 0.f, 0.f, 0.f};
  if (bn) {
    e.g = *(const f32x4*)(ly.gamma + n0); e.be = *(const f32x4*)(ly.beta + n0);
    e.mu = *(const f32x4*)(ly.mmean + n0); e.va = *(const f32x4*)(ly.mvar + n0);
  }
  return e;
}

// Same arithmetic as k_gemm_f32's / k_fwd's epilogue: z = acc / maxnorm + b;
// y = relu(z * inv + (beta - mean * inv)), inv = gamma / sqrt(var + eps).
__device__ __forceinline__ f32x4 p3d_epi_apply(const ServeEpi& ep, f32x4 acc, bool wsq, int bn, float eps) {
  f32x4 o;
  const float mx = fmaxf(sqrtf(ep.mx), 1.0f);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float z = (wsq ? acc[e] / mx : acc[e]) + ep.b[e];
    if (bn) {
      const float inv = (1.0f / sqrtf(ep.va[e] + eps)) * ep.g[e];
      const float shift = ep.be[e] - ep.mu[e] * inv;
      o[e] = fmaxf(z * inv + shift, 0.0f);
    } else {
      o[e] = fmaxf(z, 0.0f);
    }
  }
  return o;
}

// W4 fragments (k-group ctg, output tiles o) for the fused output layer
template <int NDT>
__device__ __forceinline__ void p3d_wo_load(const ServeLayer& lo, int ctg, int ngL, f32x4 (&wo)[NDT]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 0; o < NDT; ++o) wo[o] = *(const f32x4*)(lo.Wf + ((int64_t)(o * ngL + ctg) * 64 + lane) * 4);
}

// Output-layer partial of one unit: y (this wave's tile, A-fragment of k-group ctg) times
// W4 rows 16ctg.. -> NDT 16x16 tiles; the two waves of a row tile combine through LDS
// (wave ct = 1 hands over, ct = 0 adds in fixed order and stores).  All waves call it.
template <int NDT>
__device__ __forceinline__ void p3d_serve_partial(const f32x4 (&wo)[NDT], f32x4 yv, int rt, int ct, f32x4* xch,
                                                  float* pdst) {
  const int lane = threadIdx.x & 63;
  f32x4 acc[NDT];
#pragma unroll
  for (int o = 0; o < NDT; ++o) {
    acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[o] = __builtin_amdgcn_mfma_f32_16x16x4f32(yv[e], wo[o][e], acc[o], 0, 0, 0);
  }
  if (ct == 1) {
#pragma unroll
    for (int o = 0; o < NDT; ++o) xch[(rt * NDT + o) * 64 + lane] = acc[o];
  }
  __syncthreads();
  if (ct == 0) {
#pragma unroll
    for (int o = 0; o < NDT; ++o) {
      const f32x4 v = acc[o] + xch[(rt * NDT + o) * 64 + lane];
      *(f32x4*)(pdst + ((rt * NDT + o) * 64 + lane) * 4) = v;
    }
  }
  __syncthreads();
}

// Output of one step from its partials: y[row, col] = (sum_u part[u]) / maxnorm + b4.
// Partial element e4 = (tile (rt, o), lane (i, q)) holds rows 16rt + 4q + r, column 16o + i.
// This workgroup handles its share [r/n, (r+1)/n) of the float4 elements.
// y[row, col] = sum / maxnorm + b4 for partial element e4 of the step at row0
template <int NDT>
// Stores this lane's 4 outputs; returns their squared error against the lane's 4 targets tv
// (p3d_serve_load_tgt, requested ahead of the tile's contraction: they may live in host memory) --
// 0 without targets.
__device__ __forceinline__ float p3d_serve_store_out(const ServeArgs& p, const ServeLayer& lo, f32x4 sum, int e4,
                                                     int64_t row0, f32x4 tv = f32x4{0.f, 0.f, 0.f, 0.f}) {
  const int tile = e4 >> 6, ln = e4 & 63, rt = tile / NDT, o = tile % NDT;
  const int col = 16 * o + (ln & 15), q = ln >> 4;
  if (col >= p.ND) return 0.0f;
  const float mx = lo.wsq ? fmaxf(sqrtf(*lo.wsq), 1.0f) : 1.0f;
  const float bb = lo.bias[col];
  float se = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t row = row0 + 16 * rt + 4 * q + k;
    if (row < p.M) {
      const float yv = (lo.wsq ? sum[k] / mx : sum[k]) + bb;
      p.y[row * p.ND + col] = yv;
      const float d = yv - tv[k];
      se = __builtin_fmaf(d, d, se);
    }
  }
  return p.tgt ? se : 0.0f;
}
// The targets of this lane's 4 outputs of output element e4 (rows past the end / columns past
// output_size: 0, unused)
template <int NDT>
__device__ __forceinline__ f32x4 p3d_serve_load_tgt(const ServeArgs& p, int e4, int64_t row0) {
  const int tile = e4 >> 6, ln = e4 & 63, rt = tile / NDT, o = tile % NDT;
  const int col = 16 * o + (ln & 15), q = ln >> 4;
  f32x4 tv = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t row = row0 + 16 * rt + 4 * q + k;
    if (col < p.ND && row < p.M) tv[k] = p.tgt[row * p.ND + col];
  }
  return tv;
}

// Fused MSE, one output tile's share (a whole wave; wave-uniform call): the lanes' squared errors
// summed in a fixed butterfly, stored as tile gtile's partial (write-through), then one arrival on
// the launch's counter.  The wave whose arrival is the last sums every tile's partial in a fixed
// order (lane l: tiles l, l + 64, ...; then the same butterfly) and writes mean = sum / (M ND); it
// resets the counter for the next launch (stream-ordered behind this one).  Same bits for the same
// launch shape; tiles past the last row (a pair unit past the end) do not arrive.
// HF: the form may carry the host completion word (p3d_serve_mse_sync; not the pair form, whose
// register budget has no room for the fence path -- that form's sync call waits on the stream).
template <bool HF>
__device__ __forceinline__ void p3d_serve_loss_tile(const ServeArgs& p, float se, int64_t gtile, int64_t ntiles) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) se += __shfl_xor(se, o, 64);
  if (gtile >= ntiles) return;
  if (HF && p.hflag) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // this wave's rows (host memory): system-visible
  unsigned v = 0;
  if (lane == 0) {
    __hip_atomic_store(p.lpart + gtile, se, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    v = __hip_atomic_fetch_add(p.lcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  v = __shfl(v, 0, 64);
  if ((int64_t)v + 1 != ntiles) return;
  float t = 0.0f;
  for (int64_t i = lane; i < ntiles; i += 64) t += __hip_atomic_load(p.lpart + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
  if (lane == 0) {
    *p.loss = t / (float)(p.M * p.ND);
    __hip_atomic_store(p.lcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (HF && p.hflag)   // every tile arrived after its fence: rows + loss are the host's once it reads hseq
      __hip_atomic_store(p.hflag, p.hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The units' partials of one element are summed as 4 consecutive slices (slice sums in unit
// order, then the slices in order) -- the association k_serve5's split reduction uses (one
// slice per wave: exactly the units that wave's producers wrote), so every path gives the
// same bits.  This workgroup handles elements [E4*r/n, E4*(r+1)/n).
template <int NDT>
__device__ __forceinline__ void p3d_serve_reduce(const ServeArgs& p, const ServeLayer& lo, const float* pb, int U,
                                                 int64_t row0, int r, int n) {
  constexpr int E4 = 4 * NDT * 64;
  const int s = (int)(((int64_t)E4 * r) / n), e = (int)(((int64_t)E4 * (r + 1)) / n);
  const __amdgpu_buffer_rsrc_t rs = p3d_rsrc(pb);
  for (int e4 = s + (int)threadIdx.x; e4 < e; e4 += (int)blockDim.x) {
    f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < 4; ++sl) {
      const int ub = (U * sl) >> 2, ue = (U * (sl + 1)) >> 2;
      if (ub == ue) continue;
      f32x4 ss = p3d_ld_sc1(rs, (ub * E4 + e4) * 16);
      for (int u = ub + 1; u < ue; ++u) ss += p3d_ld_sc1(rs, (u * E4 + e4) * 16);
      sum += ss;
    }
    (void)p3d_serve_store_out<NDT>(p, lo, sum, e4, row0);
  }
}

// Phase 0 of a step: the input layer (K0 = input_size, A straight from the row-major
// input; or, with no blocks, the output partials) and the previous step's output
// reduction, the first unit's operands requested before the reduction.  Inlined by
// default; as a call (-DP3D_SERVE_PHASE0_CALL=1) its registers do not crowd the hidden
// layers' register ring (inlined, deeper rings than 2 spill inside the ring).
#ifndef P3D_SERVE_PHASE0_CALL
#define P3D_SERVE_PHASE0_CALL 0
#endif
#if P3D_SERVE_PHASE0_CALL
#define P3D_SERVE_P0_ATTR __noinline__
#else
#define P3D_SERVE_P0_ATTR __forceinline__
#endif
template <int NDT>
__device__ P3D_SERVE_P0_ATTR void p3d_serve_phase0(const ServeArgs& p, int r, int n, int64_t row0, bool lastp,
                                              int64_t prev_row0, const float* prev_part, float* pdst, float* act,
                                              f32x4* xch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, rt = w >> 1, ct = w & 1;
  const int ngL = p.L >> 4, U = p.L >> 5, ngK0 = p.K0 >> 4;
  constexpr int PT = 4 * NDT * 256;
  const ServeLayer& li = p.ly[0];
  const ServeLayer& lo = p.ly[2 * p.nblk + 1];
  const bool wsq_any = li.wsq != nullptr;
  for (int u = r; u < U || u == r; u += n) {
    const bool has = u < U;
    const int ctg = 2 * u + ct, n0 = 16 * ctg + 4 * (lane >> 4);
    f32x4 xa[4], wb[4], wo[NDT];
    ServeEpi ep;
    if (has) {
      int64_t rowc = row0 + 16 * rt + (lane & 15);
      rowc = rowc < p.M ? rowc : p.M - 1;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        if (g < ngK0) {
          xa[g] = *(const f32x4*)(p.x + rowc * p.K0 + 16 * g + 4 * (lane >> 4));
          wb[g] = *(const f32x4*)(li.Wf + ((int64_t)(ctg * ngK0 + g) * 64 + lane) * 4);
        }
      ep = p3d_epi_load(li, n0, p.bn, p.eps);
      if (lastp) p3d_wo_load<NDT>(lo, ctg, ngL, wo);
    }
    if (u == r && prev_row0 >= 0) p3d_serve_reduce<NDT>(p, lo, prev_part, U, prev_row0, r, n);
    if (!has) break;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (g < ngK0)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[g][e], xa[g][e], acc, 0, 0, 0);
    const f32x4 yv = p3d_epi_apply(ep, acc, wsq_any, p.bn, p.eps);
    if (lastp) p3d_serve_partial<NDT>(wo, yv, rt, ct, xch, pdst + (int64_t)u * PT);
    else *(f32x4*)(act + ((int64_t)(rt * ngL + ctg) * 64 + lane) * 4) = yv;
  }
}

template <int DEPTH, int NDT, int KS>
__global__ __launch_bounds__(512) void k_serve(ServeArgs p) {
  __shared__ __attribute__((aligned(16))) f32x4 red[KS * 8 * 64];    // K-slice partials (32 / 64 KB)
  __shared__ __attribute__((aligned(16))) f32x4 xch[4 * NDT * 64];   // output-partial exchange
  __shared__ int sh[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rt = w >> 1, ct = w & 1;         // this wave's output tile of a unit
  const int L = p.L, ngL = L >> 4, U = L >> 5, ngK0 = p.K0 >> 4;

  // ---- census: XCD id, rank within the XCD, wait for every workgroup -----------------
  p3d_serve_census(p, sh, 64);
  if (sh[2]) return;
  const int xcc = sh[0], r = sh[1], n = sh[8 + xcc];
  int ng = 0, gi = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x)
    if (sh[8 + x] > 0) { if (x == xcc) gi = ng; ++ng; }
  if (p.max_groups > 0 && ng > p.max_groups) {
    ng = p.max_groups;
    if (gi >= ng) gi = p.nb;   // this group takes no steps
  }
  unsigned* flags = p.sync + P3D_SERVE_FLAG0 + 64 * xcc;
  const int64_t slab = (int64_t)64 * L;
  float* act = p.act + (int64_t)xcc * 3 * slab;
  constexpr int PT = 4 * NDT * 256;          // floats of one unit's partial
  float* part = p.part + (int64_t)xcc * 2 * U * PT;
  const ServeLayer& lo = p.ly[2 * p.nblk + 1];
  const bool wsq_any = p.ly[0].wsq != nullptr;   // max-norm is all layers or none
  const int P = 2 * p.nblk + 1;              // phases per step
  unsigned nsync = 0;
  bool broken = false;
  ServeRingB<DEPTH, KS> RB;
  bool b_ready = false;                      // R.b holds layer ph's first fragments of unit r

  // Group barrier through per-member flags kept in the XCD's L2: drain this workgroup's
  // stores, then (all waves) request the next layer's weight fragments -- independent of
  // the hand-off -- then one lane publishes the phase and wave 0 polls every member's flag
  // (sc1 loads, one lane per member) until all reached it.
  auto group_sync = [&](int next_ph) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ++nsync;
    if (P3D_SERVE_PREFETCH_B && next_ph > 0 && next_ph < P && r < U) {
      p3d_ring_load_b(RB, p.ly[next_ph].Wf, r, ngL);
      b_ready = true;
    }
    if (tid < 64) {
      if (lane == 0) __hip_atomic_store(flags + r, nsync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (!broken) {
        int spin = 0;
        while (true) {
          const unsigned v = lane < n ? __hip_atomic_load(flags + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : nsync;
          if (__all(v >= nsync)) break;
          if (++spin > P3D_SERVE_SPIN) {
            broken = true;
            if (lane == 0) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
        }
      }
    }
    __syncthreads();
  };

  int jl = 0;                                // local step index (partial-buffer parity)
  int64_t prev_row0 = -1;
  for (int b = gi; b < p.nb; b += ng, ++jl) {
    const int64_t row0 = (int64_t)b * 64;
    int cur = 0;                             // buffer holding the current block input
    for (int ph = 0; ph < P; ++ph) {
      unsigned long long* tr = P3D_SERVE_TR(xcc, r, jl, ph);
      P3D_SERVE_STAMP(tr, 0);
      const bool lastp = (ph == P - 1);
      float* pdst = part + (int64_t)(jl & 1) * U * PT;
      if (ph == 0) {
        p3d_serve_phase0<NDT>(p, r, n, row0, lastp, prev_row0, part + (int64_t)((jl - 1) & 1) * U * PT, pdst, act,
                              xch);
      } else {
        // ---- hidden layer ph (block (ph-1)/2, first or second linear) ----------------
        const ServeLayer& ly = p.ly[ph];
        const bool second = ((ph - 1) & 1) == 1;
        const int t1 = (cur + 1) % 3, t2 = (cur + 2) % 3;
        const float* A = act + (second ? t1 : cur) * slab;
        float* Y = act + (second ? t2 : t1) * slab;
        const float* res = (second && p.residual) ? act + cur * slab : nullptr;
        for (int u = r; u < U; u += n) {
          const int ctg = 2 * u + ct, n0 = 16 * ctg + 4 * (lane >> 4);
          const int64_t off = ((int64_t)(rt * ngL + ctg) * 64 + lane) * 4;
          if (!(b_ready && u == r)) p3d_ring_load_b(RB, ly.Wf, u, ngL);
          ServeRingA<DEPTH, KS> RA;
          p3d_ring_load_a(RA, A, ngL);
          ServeEpi ep;
          f32x4 rv = f32x4{0.f, 0.f, 0.f, 0.f}, wo[NDT];
          if (P3D_SERVE_EPI_EARLY) {
            ep = p3d_epi_load(ly, n0, p.bn, p.eps);
            if (res) rv = p3d_ld_sc1(p3d_rsrc(res), (int)(off * 4));
            if (lastp) p3d_wo_load<NDT>(lo, ctg, ngL, wo);
          }
          const f32x4 acc = p3d_ring_run(RA, RB, A, ly.Wf, u, ngL, red, tr);
          if (!P3D_SERVE_EPI_EARLY) {
            ep = p3d_epi_load(ly, n0, p.bn, p.eps);
            if (res) rv = p3d_ld_sc1(p3d_rsrc(res), (int)(off * 4));
            if (lastp) p3d_wo_load<NDT>(lo, ctg, ngL, wo);
          }
          f32x4 yv = p3d_epi_apply(ep, acc, wsq_any, p.bn, p.eps);
          if (res) yv += rv;
          if (lastp) p3d_serve_partial<NDT>(wo, yv, rt, ct, xch, pdst + (int64_t)u * PT);
          else *(f32x4*)(Y + off) = yv;
        }
        b_ready = false;
        if (second) cur = t2;
      }
      P3D_SERVE_STAMP(tr, 1);
      group_sync(ph + 1);
      P3D_SERVE_STAMP(tr, 2);
    }
    prev_row0 = row0;
  }
  if (prev_row0 >= 0) p3d_serve_reduce<NDT>(p, lo, part + (int64_t)((jl - 1) & 1) * U * PT, U, prev_row0, r, n);
}

// =====================================================================================
// k_serve5 (default): 4-wave (256-thread) workgroups, one wave per SIMD, so every wave has
// the full 512-entry register file (arch VGPRs + AGPRs).  Wave w owns K slice w of a unit
// (k-groups [w*ngL/4, (w+1)*ngL/4)) for all 4 row tiles x 2 column tiles: per k-group 4 A +
// 2 B fragments (each operand byte loaded once per CU) for 32 MFMAs on 8 independent
// accumulators, with a DEPTH-deep register ring.  After the K-slice combine (LDS, slice
// order) wave w owns row tile w of both column tiles, so the fused output-layer partial of a
// row tile needs no exchange.  The steps of a group are software-pipelined so a step costs
// only its 2N hidden-layer phases:
//   * the input layer of step b+1 (it depends on nothing of step b) runs in the last
//     hidden phase of step b, after that phase's contraction, into the activation buffer
//     that phase does not touch (buffer rotation c0' = c0 + 2N mod 3); only the group's
//     first step has an input-layer phase of its own;
//   * the output of step b (the sum of its 32 fused output-layer partials) is formed in
//     the first hidden phase of step b+1, after its contraction (split over the workgroup:
//     8 unit slices x 32 elements, combined in LDS in slice order);
//   * every off-contraction load (the next layer's first weight fragments, the next step's
//     inputs and layer-0 operands, the partials) is requested right after the contraction,
//     so its latency hides under the K-combine and the epilogue.
// Needs N >= 1 block (N = 0 runs k_serve).
// =====================================================================================
// SPLIT = 2 / 4: the members of an XCD form SPLIT groups (by rank mod SPLIT) that run
// different steps, each with ~32/SPLIT CUs: a layer's contraction takes SPLIT times as long
// while the per-layer fixed costs (hand-off, operand fill, epilogue) stay, so they weigh less.
// UPM = 2: a workgroup runs its two units of a layer (u, u + n) as ONE contraction of 4
// column tiles: the activation fragments are loaded once for both, one fill, one K-combine
// and one epilogue per phase.  A pair whose second unit does not exist computes a copy of
// the first and stores nothing for it.
template <int DEPTH, int NDT, int SPLIT, int UPM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_serve5(ServeArgs p) {
  constexpr int NC = 2 * UPM;                // column tiles per contraction
  __shared__ __attribute__((aligned(16))) f32x4 red[4 * 4 * NC * 64]; // [slice][rt][ct][lane] (32 / 64 KB)
  // split output reduction: RE elements per lane (a group of 8 members has 96 per workgroup)
  constexpr int RE = UPM >= 4 ? P3D_S4_RE : 1;
  __shared__ __attribute__((aligned(16))) f32x4 rsum[4 * 64 * RE];   // (4 / 8 KB)
  // epilogue constants of this workgroup's first UPM units, per layer 0..2N and column tile:
  // bias[16] | inv[16] = gamma / sqrt(var + eps) | shift[16] = beta - mean * inv, formed once
  // per launch (the sqrt and divide of every epilogue element, and ~80 registers of BN operands
  // held across the contraction, are gone)
  __shared__ __attribute__((aligned(16))) float ec[P3D_SERVE_ECL(NC) * NC * 48];
  __shared__ int sh[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = p.L, ngL = L >> 4, U = L >> 5, ngK0 = p.K0 >> 4;
  const int q4 = 4 * (lane >> 4);

  // ---- census: XCD id, rank within the XCD, wait for every workgroup -----------------
  p3d_serve_census(p, sh, 64);
  if (sh[2]) return;
  const int xcc = sh[0], rx = sh[1], nx = sh[8 + xcc];
  const int half = rx % SPLIT;                          // group = (XCD, rank mod SPLIT)
  const int r = rx / SPLIT;
  const int n = (nx + SPLIT - 1 - half) / SPLIT;
  const int gid = xcc * SPLIT + half;
  int ng = 0, gi = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int h = 0; h < SPLIT; ++h) {
      const int cnt = (sh[8 + x] + SPLIT - 1 - h) / SPLIT;
      if (cnt > 0) { if (x == xcc && h == half) gi = ng; ++ng; }
    }
  if (p.max_groups > 0 && ng > p.max_groups) {
    ng = p.max_groups;
    if (gi >= ng) gi = p.nb;   // this group takes no steps
  }
  unsigned* flags = p.sync + P3D_SERVE_FLAG0 + 64 * gid;
  const int64_t slab = (int64_t)64 * L;
  float* act = p.act + (int64_t)gid * 3 * slab;
  constexpr int PT = 4 * NDT * 256;          // floats of one unit's partial
  constexpr int E4 = 4 * NDT * 64;           // float4 elements of a step's output partial
  float* part = p.part + (int64_t)gid * 2 * U * PT;
  const ServeLayer& li = p.ly[0];
  const ServeLayer& lo = p.ly[2 * p.nblk + 1];
  const bool wsq_any = li.wsq != nullptr;    // max-norm is all layers or none
  const int NH = 2 * p.nblk;                 // hidden layers = phases per step
  unsigned nsync = 0;
  bool broken = false;
  const int gb = (ngL * w) >> 2, gcount = ngL >> 2;   // this wave's K slice
  // this workgroup's share of a step's output elements, split over (slice, element) threads
  const int es = (int)(((int64_t)E4 * r) / n), ecnt = (int)(((int64_t)E4 * (r + 1)) / n) - es;
  const bool split_red = r < U && ecnt <= 64 * RE && U <= 64 / RE;
  const int rsl = w, rei = lane;             // slice = this wave's producers' units

  // Group barrier: drain, one lane publishes this member's phase, then every wave waits only
  // for the members whose output its next contraction reads -- its K slice [gb, gb+gcount)
  // is units [gb/2, (gb+gcount)/2), unit u produced by member u % n -- or for all members
  // (full).  A wave loads another member's bytes only after its own poll has matched them.
  // Write-after-read safety needs no more: a member writes its phase-p output only after its
  // K-combine barrier, i.e. after all four of its waves saw every member finish phase p-1, so
  // every read of the buffer being overwritten (last read in phase p-2 or earlier) is done.
  {
    const int nl = NH + 1;
    for (int idx = tid; idx < nl * NC * 16; idx += 256) {
      const int l = idx / (NC * 16), rem = idx % (NC * 16), cc = rem >> 4, j = rem & 15;
      const int uk = r + (cc >> 1) * n;
      float bb = 0.f, inv = 1.f, shift = 0.f;
      if (uk < U) {
        const ServeLayer& lyc = p.ly[l];
        const int col = 16 * (2 * uk + (cc & 1)) + j;
        bb = lyc.bias[col];
        if (p.bn) {
          inv = (1.0f / sqrtf(lyc.mvar[col] + p.eps)) * lyc.gamma[col];
          shift = lyc.beta[col] - lyc.mmean[col] * inv;
        }
      }
      float* e = ec + (l * NC + cc) * 48;
      e[j] = bb; e[16 + j] = inv; e[32 + j] = shift;
    }
    __syncthreads();
  }
  // epilogue of column tile cc of layer l from the constants: z = acc / maxnorm + b,
  // y = relu(z * inv + shift) -- the arithmetic of p3d_epi_apply
  auto epi_c = [&](int l, int cc, f32x4 acc) -> f32x4 {
    const float* e = ec + (l * NC + cc) * 48 + q4;
    const f32x4 b4 = *(const f32x4*)e, inv4 = *(const f32x4*)(e + 16), sh4 = *(const f32x4*)(e + 32);
    const float mx = wsq_any ? fmaxf(sqrtf(*p.ly[l].wsq), 1.0f) : 1.0f;
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float z = (wsq_any ? acc[k] / mx : acc[k]) + b4[k];
      o[k] = fmaxf(p.bn ? z * inv4[k] + sh4[k] : z, 0.0f);
    }
    return o;
  };

  auto group_sync = [&](bool full) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ++nsync;
    if (tid == 0) __hip_atomic_store(flags + r, nsync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!P3D_SERVE_SLICE_WAIT) full = true;
    const int cnt = full ? n : (gcount >> 1), ub = gb >> 1;
    if (!broken) {
      int spin = 0;
      while (true) {
        const int mem = full ? lane : (ub + lane) % n;
        const unsigned v = lane < cnt ? __hip_atomic_load(flags + mem, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : nsync;
        if (__all(v >= nsync)) break;
        if (++spin > P3D_SERVE_SPIN) {
          broken = true;
          if (lane == 0) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
  };

  // input layer of unit u for the step at row rbase into act buffer cbuf (row tile w, both
  // column tiles); operands as loaded by in_load
  struct InOps { f32x4 xa[4], wb[2][4]; };
  auto in_load_w = [&](int u, InOps& o) {     // the unit's input-layer weight fragments
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (g < ngK0)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          o.wb[c][g] = *(const f32x4*)(li.Wf + ((int64_t)((2 * u + c) * ngK0 + g) * 64 + lane) * 4);
  };
  auto in_load = [&](int u, int64_t rbase, InOps& o) {
    int64_t rowc = rbase + 16 * w + (lane & 15);
    rowc = rowc < p.M ? rowc : p.M - 1;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (g < ngK0) o.xa[g] = *(const f32x4*)(p.x + rowc * p.K0 + 16 * g + q4);
    in_load_w(u, o);
  };
  auto in_finish = [&](int u, const InOps& o, int cbuf) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < 4; ++g)
        if (g < ngK0)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(o.wb[c][g][e], o.xa[g][e], acc, 0, 0, 0);
      const int kk = (u - r) / n;               // which of this workgroup's units
      f32x4 y;
      if (kk < UPM) y = epi_c(0, 2 * kk + c, acc);
      else y = p3d_epi_apply(p3d_epi_load(li, 16 * (2 * u + c) + q4, p.bn, p.eps), acc, wsq_any, p.bn, p.eps);
      *(f32x4*)(act + cbuf * slab + ((int64_t)(w * ngL + 2 * u + c) * 64 + lane) * 4) = y;
    }
  };

  // ring slots prefetched off-contraction (one for the 8-column-tile form: register budget)
  constexpr int PD = UPM >= 4 ? 1 : DEPTH < 2 ? DEPTH : 2;
  // output-layer operands of the fused partial: all units' before the combine, or (8 column
  // tiles, register budget) the first unit's before it and each next unit's while the
  // current one's partial is formed (two units' worth of registers)
  constexpr bool WO_LATE = UPM >= 4;
  constexpr int NWO = WO_LATE ? 2 + 2 * P3D_S4_WOPIPE : NC;
  f32x4 rbp[PD][NC];                         // the next ring's first weight fragments
  bool b_ready = false;
  auto b_prefetch = [&](int layer, int unit) {   // units unit, unit + n (UPM = 2)
    if (unit >= U) return;
#pragma unroll
    for (int k = 0; k < UPM; ++k) {
      const int uk = (unit + k * n < U) ? unit + k * n : unit;
      const f32x4* pbn = (const f32x4*)p.ly[layer].Wf + ((int64_t)(2 * uk) * ngL + gb) * 64 + lane;
#pragma unroll
      for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int c = 0; c < 2; ++c) rbp[d][2 * k + c] = pbn[(c * ngL + d) * 64];
    }
    b_ready = true;
  };

  int jl = 0, c0 = 0;
  int64_t prev_row0 = -1;
  if (gi < p.nb) {                           // the group's first step: its input layer alone
    for (int u = r; u < U; u += n) {
      InOps o;
      in_load(u, (int64_t)gi * 64, o);
      in_finish(u, o, 0);
    }
    b_prefetch(1, r);
    group_sync(false);
  }
  for (int b = gi; b < p.nb; b += ng, ++jl) {
    const int64_t row0 = (int64_t)b * 64;
    const bool has_next = b + ng < p.nb;
    const int c0n = (c0 + 2 * p.nblk) % 3;   // buffer the next step's input layer writes
    int cur = c0;
    float* pdst = part + (int64_t)(jl & 1) * U * PT;
    const float* prev_part = part + (int64_t)((jl - 1) & 1) * U * PT;
    for (int ph = 1; ph <= NH; ++ph) {
      unsigned long long* tr = P3D_SERVE_TR(xcc, r, jl, ph);
      P3D_SERVE_STAMP(tr, 0);
      const bool lastp = (ph == NH);
      const bool red_here = (ph == 1 && prev_row0 >= 0);
      if (red_here && !split_red) p3d_serve_reduce<NDT>(p, lo, prev_part, U, prev_row0, r, n);
      const ServeLayer& ly = p.ly[ph];
      const bool second = ((ph - 1) & 1) == 1;
      const int t1 = (cur + 1) % 3, t2 = (cur + 2) % 3;
      const float* A = act + (second ? t1 : cur) * slab;
      float* Y = act + (second ? t2 : t1) * slab;
      const float* res = (second && p.residual) ? act + cur * slab : nullptr;
      const __amdgpu_buffer_rsrc_t ra = p3d_rsrc(A);
      const int aoff0 = (gb * 64 + lane) * 16, rstride = ngL * 1024;
      for (int u = r; u < U; u += n * UPM) {
        const bool first_u = (u == r);
        int uu[UPM];
        bool uv[UPM];
#pragma unroll
        for (int k = 0; k < UPM; ++k) {
          uv[k] = (u + k * n < U);
          uu[k] = uv[k] ? u + k * n : u;
        }
        const f32x4* pbk[UPM];
#pragma unroll
        for (int k = 0; k < UPM; ++k) pbk[k] = (const f32x4*)ly.Wf + ((int64_t)(2 * uu[k]) * ngL + gb) * 64 + lane;
        f32x4 ra_[DEPTH][4], rb_[DEPTH][NC];
        const bool pre = b_ready;
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
          for (int t = 0; t < 4; ++t) ra_[d][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + d * 1024);
#pragma unroll
          for (int k = 0; k < UPM; ++k)
#pragma unroll
            for (int c = 0; c < 2; ++c)
              rb_[d][2 * k + c] = (pre && d < PD) ? rbp[d < PD ? d : 0][2 * k + c] : pbk[k][(c * ngL + d) * 64];
        }
        b_ready = false;
        f32x4 rv[NC], wo[NWO][NDT];
        auto rv_load = [&]() {                   // residual operands of the epilogue
#pragma unroll
          for (int cc = 0; cc < NC; ++cc) {
            const int col_t = 2 * uu[cc >> 1] + (cc & 1);
            const int64_t off = ((int64_t)(w * ngL + col_t) * 64 + lane) * 4;
            rv[cc] = res ? p3d_ld_sc1(p3d_rsrc(res), (int)(off * 4)) : f32x4{0.f, 0.f, 0.f, 0.f};
          }
        };
        if (!P3D_SERVE_RV_LATE) rv_load();
        f32x4 acc[NC][4];
#pragma unroll
        for (int cc = 0; cc < NC; ++cc)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[cc][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int g0 = 0; g0 < gcount - DEPTH; g0 += DEPTH) {
#pragma unroll
          for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int cc = 0; cc < NC; ++cc)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                  acc[cc][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(rb_[d][cc][e], ra_[d][t][e], acc[cc][t], 0, 0, 0);
            const int gn = g0 + DEPTH + d;
#pragma unroll
            for (int t = 0; t < 4; ++t) ra_[d][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + gn * 1024);
#pragma unroll
            for (int k = 0; k < UPM; ++k)
#pragma unroll
              for (int c = 0; c < 2; ++c) rb_[d][2 * k + c] = pbk[k][(c * ngL + gn) * 64];
            __builtin_amdgcn_sched_barrier(0);   // refill of slot d stays ahead of slot d+1's MFMAs
          }
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc)
#pragma unroll
              for (int t = 0; t < 4; ++t)
                acc[cc][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(rb_[d][cc][e], ra_[d][t][e], acc[cc][t], 0, 0, 0);
        P3D_SERVE_STAMP(tr, 3);
        // ---- off-contraction loads, their latency under the combine and epilogue ----------
        __builtin_amdgcn_sched_barrier(0);
        if (u + n * UPM < U) b_prefetch(ph, u + n * UPM);   // this workgroup's next unit(s)
        else if (!lastp) b_prefetch(ph + 1, r);              // the next layer's first unit(s)
        else if (has_next) b_prefetch(1, r);                 // the next step's first layer
        constexpr int KR = 16 / RE;              // units per slice (U <= 64 / RE)
        f32x4 rpv[RE][KR];
        const bool red_now = red_here && split_red && first_u && rei < ecnt;
        if (red_now) {
          const __amdgpu_buffer_rsrc_t rp = p3d_rsrc(prev_part);
          const int ub = (U * rsl) >> 2, ue = (U * (rsl + 1)) >> 2;
#pragma unroll
          for (int j = 0; j < RE; ++j)
#pragma unroll
            for (int k = 0; k < KR; ++k)
              if (ub + k < ue && rei + 64 * j < ecnt)
                rpv[j][k] = p3d_ld_sc1(rp, ((ub + k) * E4 + es + rei + 64 * j) * 16);
        }
        if (P3D_SERVE_RV_LATE) rv_load();
        if (lastp) {                             // output-layer operands of the fused partial
#pragma unroll
          for (int cc = 0; cc < (WO_LATE ? 2 * P3D_S4_WOPIPE : NC); ++cc)
            p3d_wo_load<NDT>(lo, 2 * uu[cc >> 1] + (cc & 1), ngL, wo[cc]);
        }
        const bool in_now = lastp && has_next;   // the next step's input layer, these units
        __builtin_amdgcn_sched_barrier(0);
        // ---- K-slice combine (LDS), epilogue ----------------------------------------------
#pragma unroll
        for (int cc = 0; cc < NC; ++cc)
#pragma unroll
          for (int t = 0; t < 4; ++t) red[((w * 4 + t) * NC + cc) * 64 + lane] = acc[cc][t];
        if (red_here && split_red && first_u) {
#pragma unroll
          for (int j = 0; j < RE; ++j) {
            f32x4 ss = f32x4{0.f, 0.f, 0.f, 0.f};
            if (red_now && rei + 64 * j < ecnt) {
              const int ub = (U * rsl) >> 2, ue = (U * (rsl + 1)) >> 2;
              if (ub < ue) ss = rpv[j][0];
#pragma unroll
              for (int k = 1; k < KR; ++k)
                if (ub + k < ue) ss += rpv[j][k];
            }
            rsum[rsl * 64 * RE + rei + 64 * j] = ss;
          }
        }
        __syncthreads();
        P3D_SERVE_STAMP(tr, 4);
        // (P3D_SERVE_IN_EARLY) the next step's first input-layer operands requested here, the
        // K-slice accumulators being dead: their latency hides under the epilogue and the
        // fused output-layer partials
        InOps nx_early;
        if (P3D_SERVE_IN_EARLY && UPM < 4 && in_now) in_load(uu[0], row0 + (int64_t)ng * 64, nx_early);
        if (red_here && split_red && first_u && tid < ecnt) {
          f32x4 tot = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int sl = 0; sl < 4; ++sl) tot += rsum[sl * 64 * RE + tid];
          (void)p3d_serve_store_out<NDT>(p, lo, tot, es + tid, prev_row0);
        }
        f32x4 yv[NC];
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) {
          f32x4 sacc = red[((0 * 4 + w) * NC + cc) * 64 + lane];   // slice 0, tile (w, cc)
#pragma unroll
          for (int k = 1; k < 4; ++k) sacc += red[((k * 4 + w) * NC + cc) * 64 + lane];
          if (first_u) yv[cc] = epi_c(ph, cc, sacc);
          else yv[cc] = p3d_epi_apply(p3d_epi_load(ly, 16 * (2 * uu[cc >> 1] + (cc & 1)) + q4, p.bn, p.eps), sacc,
                                      wsq_any, p.bn, p.eps);
          if (res) yv[cc] += rv[cc];
        }
        if (lastp) {
#pragma unroll
          for (int k = 0; k < UPM; ++k) {
            if (!uv[k]) continue;
            if (WO_LATE && P3D_S4_WOPIPE && k + 1 < UPM && uv[k + 1]) {
#pragma unroll
              for (int c = 0; c < 2; ++c)
                p3d_wo_load<NDT>(lo, 2 * uu[k + 1] + c, ngL, wo[P3D_S4_WOPIPE ? 2 * ((k + 1) & 1) + c : c]);
            } else if (WO_LATE && !P3D_S4_WOPIPE) {
#pragma unroll
              for (int c = 0; c < 2; ++c) p3d_wo_load<NDT>(lo, 2 * uu[k] + c, ngL, wo[c]);
            }
#pragma unroll
            for (int o = 0; o < NDT; ++o) {
              f32x4 pacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  pacc = __builtin_amdgcn_mfma_f32_16x16x4f32(yv[2 * k + c][e], wo[WO_LATE ? (P3D_S4_WOPIPE ? 2 * (k & 1) + c : c) : 2 * k + c][o][e], pacc,
                                                              0, 0, 0);
              *(f32x4*)(pdst + (int64_t)uu[k] * PT + ((w * NDT + o) * 64 + lane) * 4) = pacc;
            }
          }
        } else {
#pragma unroll
          for (int cc = 0; cc < NC; ++cc)
            if (uv[cc >> 1])
              *(f32x4*)(Y + ((int64_t)(w * ngL + 2 * uu[cc >> 1] + (cc & 1)) * 64 + lane) * 4) = yv[cc];
        }
        // (requested here, not before the combine: held across it, the operands of both units
        // pushed the kernel past 512 registers -- 200 spills, -18 %)
        // the step's input rows are loaded once for all of this contraction's units; one
        // unit's weights at a time (all of them hoisted together spill)
        if (in_now && UPM >= 4 && P3D_S4_INPIPE) {               // one unit's operands in flight ahead
          InOps nx[2];
          in_load(uu[0], row0 + (int64_t)ng * 64, nx[0]);
#pragma unroll
          for (int k = 0; k < UPM; ++k) {
            __builtin_amdgcn_sched_barrier(0);
            if (k + 1 < UPM && uv[k + 1]) in_load(uu[k + 1], row0 + (int64_t)ng * 64, nx[(k + 1) & 1]);
            if (uv[k]) in_finish(uu[k], nx[k & 1], c0n);
          }
        } else if (in_now) {
          InOps nx;
          if (P3D_SERVE_IN_EARLY && UPM < 4) nx = nx_early;
          else in_load(uu[0], row0 + (int64_t)ng * 64, nx);
          in_finish(uu[0], nx, c0n);
#pragma unroll
          for (int k = 1; k < UPM; ++k)
            if (uv[k]) {
              __builtin_amdgcn_sched_barrier(0);
              in_load_w(uu[k], nx);
              in_finish(uu[k], nx, c0n);
            }
        }
        // red / rsum are rewritten by this workgroup's next contraction; after its last one
        // of the phase the group barrier's workgroup barrier orders the next phase's writes
        if (u + n * UPM < U) __syncthreads();
      }
      if (second) cur = t2;
      P3D_SERVE_STAMP(tr, 1);
      // after a step's last phase the output reduction (next step's first phase, or the final
      // one below) reads every unit's partial -- unless split, when each wave reads exactly
      // its producers' partials
      group_sync(lastp && (!has_next || !split_red));
      P3D_SERVE_STAMP(tr, 2);
    }
    prev_row0 = row0;
    c0 = c0n;
  }
  if (prev_row0 >= 0) p3d_serve_reduce<NDT>(p, lo, part + (int64_t)((jl - 1) & 1) * U * PT, U, prev_row0, r, n);
}
