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
// Why not one persistent chain: the hand-off of a layer's 1024 features from the 64 producing
// workgroups to EVERY consumer costs ~3-4 us inside a launch (price list rows allgather /
// barrier-xcd of MI355X_MICROARCH.md) against ~1.2 us for the dependent kernel boundary between
// short GEMV kernels (row boundary).  Two of the six launches are folded away all the same
// (k_gemv_fold, round 4), where neither costs an all-to-all:
//   * the input layer (K = 32, 128 KB of weights) is recomputed by every workgroup of the first
//     hidden layer: 32 FMAs per feature and row, its weights read from the XCD's L2 beside the
//     hidden layer's own slice; each workgroup writes its own 16 columns of the input layer's
//     output for the residual of layer 2;
//   * the output layer (48 x 1024) is run by ONE extra workgroup of the last hidden layer's launch:
//     it requests its 192 KB of weights at kernel start, then gathers the 64 producers' outputs
//     (a many-to-one hand-off, ~1 us, data-tagged granules as in p3d_xchg.h) and contracts them.
// Both folds keep k_gemv's associations (input layer: the 2-wave split of k_gemv<4, 2, 4>; output
// layer: the 16-wave split of k_gemv<4, 16, 4>), so the folded chain gives the unfolded chain's
// bits (tests/test_gpu_parity.py::test_gemv_small_batch).
#pragma once
#include "p3d_kernels.h"
#include "p3d_xchg.h"

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

// Frame I/O of p3d_lift: the raw 2D rows in, the unNormalizeData'd 3D rows out.
struct GemvFrames {
  const double* raw; int ldraw;                                      // [M][ldraw] float64 (null: off)
  const double* mean2; const double* std2; const int32_t* use2;      // use2: in.K columns of raw
  double* out; int D3;                                               // [M][D3] float64 (null: off)
  const double* mean3; const double* std3; const int32_t* use3;      // use3: out.N columns of out
  // p3d_lift_sync: host-visible completion word (pinned, coherent; null: off), the call's sequence
  // number, a device arrival counter (zero between launches) and the launch's output workgroups
  unsigned* hflag; unsigned* hcnt; unsigned hseq; int hcount;
  // p3d_serve_mse at B <= 4 (null: off): the targets [M][N] row-major, the loss word, and a device
  // scratch of the M N squared differences the last output workgroup reduces as k_mse does
  const float* tgt; float* loss; float* sq;
};

// The arrival of one output workgroup (whole workgroup, uniform call): each thread's host-memory
// stores made system-visible, then one arrival on the counter.  The last arriver resets it, with
// a fused MSE (fr.loss) reduces the squared differences every output workgroup left in fr.sq --
// k_mse's order (p3d_layers.h: 256 slots, one element each at n <= 256, the same halving tree), so
// the loss has p3d_mse's bits -- and stores the call's sequence number into the host word
// (system-scope release; null: no word).  n: the M N squared differences (<= 256: M <= 4, N <= 64).
// The squares are handed over without an acquire on the reading CU (MI355X_MICROARCH.md, sc1 hand-off
// table, first row: sc1 4-B stores, every storing wave's vmcnt(0) before the barrier behind which one
// lane adds to one unsharded counter, the last adder's workgroup loading with sc1 4-B loads after
// that add returned / behind the barrier its wave joins) -- an agent acquire costs ~1.7 us.
__device__ __forceinline__ void p3d_host_arrive(const GemvFrames& fr, int n) {
  __shared__ int last;
  __shared__ float part[256];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // (system scope: no acquire half, no cache invalidate)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the guide's compiler hazard: always explicit)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(fr.hcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool l = (int)prev + 1 == fr.hcount;
    if (l) __hip_atomic_store(fr.hcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (l && !fr.loss && fr.hflag) __hip_atomic_store(fr.hflag, fr.hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    last = l;
  }
  if (!fr.loss) return;
  __syncthreads();
  if (!last) return;   // (uniform)
  const int e = threadIdx.x;   // (the other output workgroups' squares: sc1 loads, see above)
  if (e < 256)
    part[e] = e < n ? __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(fr.sq) + e, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT))
                    : 0.f;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (e < h) part[e] += part[e + h];
    __syncthreads();
  }
  if (e == 0) {
    *fr.loss = part[0] / (float)n;
    if (fr.hflag) __hip_atomic_store(fr.hflag, fr.hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- the layer epilogue of k_fwd for one (row, column) ---------------------------------------
struct GemvEpi {
  float b = 0.f, gam = 1.f, bet = 0.f, mmu = 0.f, mva = 1.f, rv = 0.f, mxv = 1.f;
  uint64_t ctr = 0;
};
__device__ __forceinline__ void p3d_gemv_epi_load(const GemvArgs& p, int row, int cc, GemvEpi& e) {
  e.ctr = p.ctr;
  e.b = p.bias[cc];
  if (p.bn) { e.gam = p.gamma[cc]; e.bet = p.beta[cc]; e.mmu = p.mmean[cc]; e.mva = p.mvar[cc]; }
  if (p.res) e.rv = p.res[p3d_pk(row, cc, (p.N + 15) >> 4)];
  if (p.wsq) e.mxv = *p.wsq;
  if (p.ctr_dev) e.ctr = (uint64_t)*p.ctr_dev;
}
__device__ __forceinline__ float p3d_gemv_epi(const GemvArgs& p, const GemvEpi& e, float zs, int row, int cc) {
  const float mx = p.wsq ? fmaxf(sqrtf(e.mxv), 1.0f) : 1.0f;
  const float z = (p.wsq ? zs / mx : zs) + e.b;
  float y = z;
  if (p.bn) {
    const float inv = (1.0f / sqrtf(e.mva + p.eps)) * e.gam;
    const float shift = e.bet - e.mmu * inv;
    y = z * inv + shift;
  }
  if (p.relu) y = fmaxf(y, 0.0f);
  if (p.keep < 1.0f) y = (y / p.keep) * p3d_dropout_mask(p.keep, p3d_uniform(p.seed, e.ctr, p.site, p.row_off + row, cc));
  if (p.res) y += e.rv;
  return y;
}

// ---- this wave's share of the contraction (k_gemv's chain) -----------------------------------
// acc[r] += sum over groups g in [gb, ge) (ascending), components x..w, of the lane's fragment
// times xat(g, r) = x[r][16g + 4q .. +3]; the first GC fragments arrive preloaded in wf.
template <int MR, int GC, class XAT>
__device__ __forceinline__ void p3d_gemv_chain(const f32x4* pw, int gb, int ge, int M, f32x4 (&wf)[GC], XAT xat,
                                               float (&acc)[MR]) {
  for (int g0 = gb; g0 < ge; g0 += GC) {
    if (g0 != gb) {
#pragma unroll
      for (int j = 0; j < GC; ++j) {
        const int g = g0 + j < ge ? g0 + j : ge - 1;   // (here ge > g0 >= gb: in the slice)
        wf[j] = pw[(int64_t)g * 64];
      }
    }
#pragma unroll
    for (int j = 0; j < GC; ++j) {
      if (g0 + j >= ge) break;
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        if (r >= M) break;
        const f32x4 xv = xat(g0 + j, r);
        float a = acc[r];
        a = fmaf(wf[j].x, xv.x, a);
        a = fmaf(wf[j].y, xv.y, a);
        a = fmaf(wf[j].z, xv.z, a);
        a = fmaf(wf[j].w, xv.w, a);
        acc[r] = a;
      }
    }
  }
}
// Pin values in registers here: the loads that produce them complete at this point and are not
// re-issued later.  (Without it the compiler sank a persistent kernel's weight and epilogue-operand
// loads past its hand-off waits, to the point of use: ~0.6 us of load latency per layer on the
// critical path, 2.7 us for the output layer -- tools/trace_chain.py.)
template <int GC>
__device__ __forceinline__ void p3d_pin(f32x4 (&v)[GC]) {
#pragma unroll
  for (int j = 0; j < GC; ++j) asm volatile("" : "+v"(v[j]));
}
__device__ __forceinline__ void p3d_pin_epi(GemvEpi& e) {
  asm volatile("" : "+v"(e.b), "+v"(e.gam), "+v"(e.bet), "+v"(e.mmu), "+v"(e.mva), "+v"(e.rv), "+v"(e.mxv));
}
// (Loads past the slice's end re-read its last fragment, unused.  A wave's slice is EMPTY when the
// layer has fewer K groups than the workgroup has waves (K < 16 WV, e.g. L < 256 at 16 waves): gb ==
// ge, and the clamp must not step to ge - 1 = gb - 1 -- for wave 0 of tile 0 that is the 1 KB in
// front of the weight buffer, a read outside the allocation.  Clamped to gb, which is < ngK.)
template <int GC>
__device__ __forceinline__ void p3d_gemv_preload(const f32x4* pw, int gb, int ge, f32x4 (&wf)[GC]) {
  const int glast = ge > gb ? ge - 1 : gb;
#pragma unroll
  for (int j = 0; j < GC; ++j) {
    const int g = gb + j < ge ? gb + j : glast;
    wf[j] = pw[(int64_t)g * 64];   // default policy: frame after frame hits the XCD's L2 / MALL
  }
}

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
  GemvEpi e;
  e.ctr = p.ctr;
  if (w == 0 && q < M) p3d_gemv_epi_load(p, q, cc, e);
  // ---- contraction: this wave's K groups, GC fragments in flight per chunk -----------------
  float acc[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) acc[r] = 0.f;
  const f32x4* pw = (const f32x4*)p.Wf + (int64_t)ct * ngK * 64 + lane;
  f32x4 wf[GC];
  p3d_gemv_preload<GC>(pw, gb, ge, wf);
  if (p.xpk)
    p3d_gemv_chain<MR, GC>(pw, gb, ge, M, wf, [&](int g, int r) {
      return *(const f32x4*)(p.X + ((int64_t)g << 8) + ((r + 16 * q) << 2)); }, acc);
  else
    p3d_gemv_chain<MR, GC>(pw, gb, ge, M, wf, [&](int g, int r) {
      return *(const f32x4*)(p.X + (int64_t)r * p.ldx + 16 * g + 4 * q); }, acc);
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
  const float y = p3d_gemv_epi(p, e, zs, q, cc);
  if (!cok) return;
  if (p.ypk) p.Y[p3d_pk(q, col, (p.N + 15) >> 4)] = y;
  else p.Y[(int64_t)q * p.ldy + col] = y;
}

// ---- the folded first / last hidden layers (k_gemv_fold) -------------------------------------
#define P3D_GEMV_FOLD_MAXK 4096   // largest hidden width the fold's LDS image holds
#define P3D_GEMV_FOLD_MAXIN 32    // the input width the input-layer fold takes (HUMAN_2D_SIZE)

struct GemvFold {
  int fin;            // 1: this (first hidden) layer's workgroups compute the input layer themselves
  GemvArgs in;        //    the input layer: X = the user rows (row-major), Y = act[0] (packed) or null
  int fout;           // 1: workgroup gridDim.x - 1 runs the output layer on this layer's outputs
  GemvArgs out;       //    the output layer: Y = the user's y (row-major); X unused
  float* hand;        // this workspace slot's hand-off: [4 rows][N / 2] 16-B granules {a, tag, b, tag}
  unsigned* epoch;    // this slot's epoch word (tag = epoch + 1), advanced by the consumer
  int* err;           // host-visible error word: 1 = the consumer's spin ran out
  GemvFrames fr;      // p3d_lift's output side (fr.out null: off)
};

// The input layer (K = 32) for feature f of row r, as k_gemv<MR, 2, GC> computes it (wave w of
// two contracts group w in one fmaf chain per quarter q; the quarters sum as (a0 + a1) + (a2 + a3),
// the two waves as (0 + t0) + t1); x rows staged in xin.
// (e: the feature's epilogue operands, row-independent -- the input layer has no residual)
__device__ __forceinline__ float p3d_gemv_in_value(const GemvArgs& in, const float (*xin)[P3D_GEMV_FOLD_MAXIN],
                                                   const f32x4 (&wv)[2][4], const GemvEpi& e, int r, int f) {
  float zs = 0.f;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 xv = *(const f32x4*)&xin[r][16 * g + 4 * q];
      float s = 0.f;
      s = fmaf(wv[g][q].x, xv.x, s);
      s = fmaf(wv[g][q].y, xv.y, s);
      s = fmaf(wv[g][q].z, xv.z, s);
      s = fmaf(wv[g][q].w, xv.w, s);
      a[q] = s;
    }
    const float t = (a[0] + a[1]) + (a[2] + a[3]);
    zs += t;
  }
  return p3d_gemv_epi(in, e, zs, r, f);
}
// p3d_normalize's and p3d_unnormalize's element expressions (csrc/p3d_data.h, contraction off)
__device__ __forceinline__ float p3d_norm_in(double x, double mu, double sd) {
#pragma clang fp contract(off)
  return (float)((x - mu) / sd);
}
__device__ __forceinline__ double p3d_unnorm_out(float v, double sd, double mu) {
#pragma clang fp contract(off)
  return (double)v * sd + mu;
}
// the input layer's value from the raw rows, normalised as p3d_normalize rounds them to float32
__device__ __forceinline__ float p3d_gemv_in_value_n(const GemvArgs& in, const GemvFrames& fr, const f32x4 (&wv)[2][4],
                                                     const GemvEpi& e, int r, int f) {
  const double* xr = fr.raw + (int64_t)r * fr.ldraw;
  float zs = 0.f;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 xv;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = fr.use2[16 * g + 4 * q + k];
        xv[k] = p3d_norm_in(xr[d], fr.mean2[d], fr.std2[d]);
      }
      float s = 0.f;
      s = fmaf(wv[g][q].x, xv.x, s);
      s = fmaf(wv[g][q].y, xv.y, s);
      s = fmaf(wv[g][q].z, xv.z, s);
      s = fmaf(wv[g][q].w, xv.w, s);
      a[q] = s;
    }
    const float t = (a[0] + a[1]) + (a[2] + a[3]);
    zs += t;
  }
  return p3d_gemv_epi(in, e, zs, r, f);
}
// The raw rows normalised into LDS by one wave, lane d taking column d of every row (D2 <= 64):
// the rows, the statistics and (separately, scalar) the used-column indices are requested in one
// round, so the indices no longer gate the host-memory row loads (p3d_gemv_in_value_n: a device
// round trip for use2, then the host one).  The caller's wave then reads the staged values by index.
template <int MR>
__device__ __forceinline__ void p3d_gemv_in_stage(const GemvFrames& fr, int M, float (*xn)[64]) {
  const int d = threadIdx.x & 63;
  if (d < fr.ldraw) {
    const double mu = fr.mean2[d], sd = fr.std2[d];
    double xr[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) xr[r] = r < M ? fr.raw[(int64_t)r * fr.ldraw + d] : 0.0;
#pragma unroll
    for (int r = 0; r < MR; ++r) xn[r][d] = p3d_norm_in(xr[r], mu, sd);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// p3d_gemv_in_value_n on the staged values (the same p3d_norm_in values, the same chains)
__device__ __forceinline__ float p3d_gemv_in_value_s(const GemvArgs& in, const GemvFrames& fr, const float (*xn)[64],
                                                     const f32x4 (&wv)[2][4], const GemvEpi& e, int r, int f) {
  float zs = 0.f;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 xv;
#pragma unroll
      for (int k = 0; k < 4; ++k) xv[k] = xn[r][fr.use2[16 * g + 4 * q + k] & 63];   // (indices < D2 <= 64)
      float s = 0.f;
      s = fmaf(wv[g][q].x, xv.x, s);
      s = fmaf(wv[g][q].y, xv.y, s);
      s = fmaf(wv[g][q].z, xv.z, s);
      s = fmaf(wv[g][q].w, xv.w, s);
      a[q] = s;
    }
    const float t = (a[0] + a[1]) + (a[2] + a[3]);
    zs += t;
  }
  return p3d_gemv_epi(in, e, zs, r, f);
}
// the same with x read from in.X (for one feature per lane: no staging)
__device__ __forceinline__ float p3d_gemv_in_value_g(const GemvArgs& in, const f32x4 (&wv)[2][4], const GemvEpi& e,
                                                     int r, int f) {
  const float* xr = in.X + (int64_t)r * in.ldx;
  float zs = 0.f;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 xv = *(const f32x4*)(xr + 16 * g + 4 * q);
      float s = 0.f;
      s = fmaf(wv[g][q].x, xv.x, s);
      s = fmaf(wv[g][q].y, xv.y, s);
      s = fmaf(wv[g][q].z, xv.z, s);
      s = fmaf(wv[g][q].w, xv.w, s);
      a[q] = s;
    }
    const float t = (a[0] + a[1]) + (a[2] + a[3]);
    zs += t;
  }
  return p3d_gemv_epi(in, e, zs, r, f);
}
__device__ __forceinline__ void p3d_gemv_in_weights(const GemvArgs& in, int f, f32x4 (&wv)[2][4]) {
  const f32x4* pw = (const f32x4*)in.Wf + (int64_t)(f >> 4) * 2 * 64 + (f & 15);
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) wv[g][q] = pw[g * 64 + 16 * q];
}
template <int NT>
__device__ __forceinline__ void p3d_gemv_stage_x(const GemvArgs& in, float (*xin)[P3D_GEMV_FOLD_MAXIN]) {
  for (int t = threadIdx.x; t < in.M * P3D_GEMV_FOLD_MAXIN; t += NT)
    xin[t / P3D_GEMV_FOLD_MAXIN][t % P3D_GEMV_FOLD_MAXIN] =
        in.X[(int64_t)(t / P3D_GEMV_FOLD_MAXIN) * in.ldx + t % P3D_GEMV_FOLD_MAXIN];
  __syncthreads();
}

// The whole input layer, rows r < M, into xs[r][feature]; the columns of column tile `own` also to
// in.Y (if set).  The thread's first feature's weights and epilogue operands are requested before
// the x rows are staged (one memory round trip, not two); post() runs once the features are done,
// before the closing barrier (the caller's next requests in flight across it).
template <int MR, int NT, class POST>
__device__ __forceinline__ void p3d_gemv_fold_in(const GemvArgs& in, int own, float* xs, float (*xin)[P3D_GEMV_FOLD_MAXIN],
                                                 POST post) {
  const int M = in.M, N = in.N;
  const int f0 = threadIdx.x;
  f32x4 wv[2][4];
  GemvEpi e;
  if (f0 < N) {
    p3d_gemv_in_weights(in, f0, wv);
    p3d_gemv_epi_load(in, 0, f0, e);
  }
  p3d_gemv_stage_x<NT>(in, xin);
  for (int f = f0; f < N; f += NT) {
    if (f != f0) {
      p3d_gemv_in_weights(in, f, wv);
      p3d_gemv_epi_load(in, 0, f, e);
    }
#pragma unroll 1
    for (int r = 0; r < MR; ++r) {
      if (r >= M) break;
      const float y = p3d_gemv_in_value(in, xin, wv, e, r, f);
      xs[r * N + f] = y;
      if (in.Y && (f >> 4) == own) in.Y[p3d_pk(r, f, N >> 4)] = y;
    }
  }
  post();
  __syncthreads();
}

// One wave: rows r < M, features [16 gb, 16 ge) of a K-wide layer output handed over as granules
// (granule j of row r = features 2j, 2j + 1, at rh + 16 (gbase + r K / 2 + j)) into the wave's own
// columns of xs, each once its tag matches.  No workgroup
// barrier: only this wave reads those columns (k_gemv's K split), so it contracts as soon as its
// own producers have published, whatever the other waves still wait for.
__device__ __forceinline__ void p3d_gemv_gather_wave(__amdgpu_buffer_rsrc_t rh, int gbase, int M, int K, int gb,
                                                     int ge, unsigned tag, float* xs, int* err) {
  const int lane = threadIdx.x & 63, per = 8 * (ge - gb);   // granules per row in the slice
  for (int idx = lane; idx < M * per; idx += 64) {
    const int r = idx / per, j = r * (K >> 1) + 8 * gb + (idx - r * per);
    u32x4_t v;
    for (int spin = 0;; ++spin) {
      v = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rh, (gbase + j) * 16, 0, 16));   // sc1
      if (v.y == tag && v.w == tag) break;
      if (spin > P3D_XCHG_SPIN) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const int k = 2 * (j - r * (K >> 1));
    xs[r * K + k] = __uint_as_float(v.x);
    xs[r * K + k + 1] = __uint_as_float(v.z);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave 0 of a tile's workgroup, all 64 lanes: lane (i even, q < M) stores columns col, col + 1 of
// row q as one sc1 granule {y(col), tag, y(col + 1), tag} at granule gbase + q N / 2 + col / 2.
__device__ __forceinline__ void p3d_gemv_publish(__amdgpu_buffer_rsrc_t rh, int gbase, int M, int N, int col, float y,
                                                 unsigned tag) {
  const int lane = threadIdx.x & 63, i = lane & 15, q = lane >> 4;
  const float y1 = __shfl_down(y, 1, 64);
  if (q < M && (i & 1) == 0 && col < N) {
    const u32x4_t v = {__float_as_uint(y), tag, __float_as_uint(y1), tag};
    __builtin_amdgcn_raw_buffer_store_b128(v, rh, (gbase + q * (N >> 1) + (col >> 1)) * 16, 0, 16);  // sc1
  }
}

// The output layer's column tiles [t0, t0 + NTO) (at most four: N <= 64), by one workgroup: their
// weights first, then the hand-off of the M x K inputs (this launch's other workgroups' outputs)
// into xs, then every tile as k_gemv<MR, WV, GC> computes it (the same K split over the WV waves,
// the same chains and sums).  Which workgroup runs a tile does not change its bits: k_gemv_fold
// gives all of them to one, k_gemv_chain one tile each to three (a workgroup's wave 0 contracting,
// reducing and storing three tiles was 3 us of issue behind the last hand-off; one is 1).  The
// workgroup with t0 = 0 advances the epoch and writes unNormalizeData's unused dimensions.
template <int MR, int WV, int GC, int NTO>
__device__ __forceinline__ void p3d_gemv_fold_out(const GemvFold& f, unsigned tag, float* xs,
                                                  float (*red)[WV][MR][16], int t0) {
  const GemvArgs& o = f.out;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int M = o.M, K = o.K, ngK = K >> 4, nto = (o.N + 15) >> 4;   // nto <= 4
  const int gb = (ngK * w) / WV, ge = (ngK * (w + 1)) / WV;
  const int t1 = t0 + NTO < nto ? t0 + NTO : nto;
  GemvEpi e[NTO];
  f32x4 wf[NTO][GC];
  float tv[NTO];   // fused MSE (k_gemv_chain): the targets, requested with the other epilogue operands
#pragma unroll
  for (int u = 0; u < NTO; ++u) {
    const int t = t0 + u;
    tv[u] = 0.f;
    if (t >= t1) break;
    const int col = 16 * t + i, cc = col < o.N ? col : o.N - 1;
    e[u].ctr = o.ctr;
    if (w == 0 && q < M) p3d_gemv_epi_load(o, q, cc, e[u]);
    if (NTO == 1 && f.fr.tgt && w == 0 && q < M) tv[u] = f.fr.tgt[(int64_t)q * o.N + cc];
    p3d_gemv_preload<GC>((const f32x4*)o.Wf + (int64_t)t * ngK * 64 + lane, gb, ge, wf[u]);
  }
#pragma unroll
  for (int u = 0; u < NTO; ++u) {
    if (t0 + u >= t1) break;
    p3d_pin<GC>(wf[u]);
    p3d_pin_epi(e[u]);
    asm volatile("" : "+v"(tv[u]));
  }
  // unNormalizeData's operands depend on no input: waves 1.. write the unused dimensions
  // ((float) 0 * std + mean) and stage the used columns' index / std / mean in LDS while the
  // producers finish, off the critical path behind the hand-off (registers: no room at 1024 threads)
  __shared__ int od[64];
  __shared__ double osd[64], omu[64];
  if (f.fr.out && w != 0) {
    if (t0 == 0) {
      for (int k = (int)threadIdx.x - 64; k < M * f.fr.D3; k += 64 * (WV - 1)) {
        const int r = k / f.fr.D3, d = k - r * f.fr.D3;
        bool used = false;
        for (int u = 0; u < o.N; ++u) used |= f.fr.use3[u] == d;
        if (!used) f.fr.out[(int64_t)r * f.fr.D3 + d] = p3d_unnorm_out(0.0f, f.fr.std3[d], f.fr.mean3[d]);
      }
    }
    if (w == 1 && lane < o.N) {
      const int d = f.fr.use3[lane];
      od[lane] = d;
      osd[lane] = f.fr.std3[d];
      omu[lane] = f.fr.mean3[d];
    }
  }
  // ---- the hand-off: this launch's other workgroups' outputs ----------------------------------
  p3d_gemv_gather_wave(p3d_rsrc(f.hand), 0, M, K, gb, ge, tag, xs, f.err);
#ifdef P3D_TRACE
  if (threadIdx.x == 0 && blockIdx.x == 0) g_p3d_trace[4] = wall_clock64();
#endif
#pragma unroll
  for (int u = 0; u < NTO; ++u) {
    const int t = t0 + u;
    if (t >= t1) break;
    float acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) acc[r] = 0.f;
    p3d_gemv_chain<MR, GC>((const f32x4*)o.Wf + (int64_t)t * ngK * 64 + lane, gb, ge, M, wf[u],
                           [&](int g, int r) { return *(const f32x4*)&xs[r * K + 16 * g + 4 * q]; }, acc);
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      acc[r] += __shfl_xor(acc[r], 16, 64);
      acc[r] += __shfl_xor(acc[r], 32, 64);
    }
    if (q == 0) {
#pragma unroll
      for (int r = 0; r < MR; ++r) red[u][w][r][i] = acc[r];
    }
  }
#ifdef P3D_TRACE
  if (threadIdx.x == 0 && blockIdx.x == 0) g_p3d_trace[6] = wall_clock64();
#endif
  __syncthreads();
#ifdef P3D_TRACE
  if (threadIdx.x == 0 && blockIdx.x == 0) g_p3d_trace[7] = wall_clock64();
#endif
  // every wave has seen its producers' granules, so every workgroup of the launch has read the
  // epoch (each producer tagged with it): the slot's next launch gets a new tag
  if (threadIdx.x == 0 && t0 == 0) __hip_atomic_fetch_add(f.epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (w == 0 && q < M && q < MR) {
#pragma unroll
    for (int u = 0; u < NTO; ++u) {
      const int t = t0 + u;
      if (t >= t1) break;
      const int col = 16 * t + i;
      float zs = 0.f;
#pragma unroll
      for (int v = 0; v < WV; ++v) zs += red[u][v][q][i];
      const float y = p3d_gemv_epi(o, e[u], zs, q, col < o.N ? col : o.N - 1);
      if (col < o.N) {
        if (o.Y) o.Y[(int64_t)q * o.ldy + col] = y;
        if (f.fr.out) f.fr.out[(int64_t)q * f.fr.D3 + od[col]] = p3d_unnorm_out(y, osd[col], omu[col]);
        if (NTO == 1 && f.fr.tgt) {   // k_mse's element term: d = y - t, d * d
          const float d = y - tv[u];
          __hip_atomic_store(reinterpret_cast<unsigned*>(f.fr.sq) + q * o.N + col, __float_as_uint(d * d),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (sc1: p3d_host_arrive)
        }
      }
    }
  }
  // (frames, the completion word and the fused loss: k_gemv_chain's one-tile form only)
  if (NTO == 1 && (f.fr.hflag || f.fr.loss)) p3d_host_arrive(f.fr, M * o.N);
}

// A hidden layer as k_gemv<MR, WV, GC> (the same bits), with the input layer folded in ahead of it
// (f.fin) and / or the output layer behind it (f.fout: grid N/16 + 1, the last workgroup runs it).
template <int MR, int WV, int GC>
__global__ __launch_bounds__(64 * WV) void k_gemv_fold(GemvArgs p, GemvFold f) {
  __shared__ float xs[MR * P3D_GEMV_FOLD_MAXK];
  __shared__ float red[4][WV][MR][16];
  __shared__ float xin[MR][P3D_GEMV_FOLD_MAXIN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const unsigned tag = f.fout ? __hip_atomic_load(f.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
  if (f.fout && blockIdx.x == gridDim.x - 1) {
    p3d_gemv_fold_out<MR, WV, GC, 4>(f, tag, xs, red, 0);
    return;
  }
  const int ct = blockIdx.x;
  const int ngK = p.K >> 4;
  const int gb = (ngK * w) / WV, ge = (ngK * (w + 1)) / WV;
  const int M = p.M;
  const int col = 16 * ct + i;
  const bool cok = col < p.N;
  const int cc = cok ? col : p.N - 1;
  GemvEpi e;
  e.ctr = p.ctr;
  if (!f.fin && w == 0 && q < M) p3d_gemv_epi_load(p, q, cc, e);
  float acc[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) acc[r] = 0.f;
  const f32x4* pw = (const f32x4*)p.Wf + (int64_t)ct * ngK * 64 + lane;
  f32x4 wf[GC];
  // (with the input layer folded in: requested once that is done -- held in registers across it,
  // 17 of them spill at 1024 threads)
  if (!f.fin) p3d_gemv_preload<GC>(pw, gb, ge, wf);
  if (f.fin) {
    p3d_gemv_fold_in<MR, 64 * WV>(f.in, ct, xs, xin, [&] { p3d_gemv_preload<GC>(pw, gb, ge, wf); });
    if (w == 0 && q < M) p3d_gemv_epi_load(p, q, cc, e);   // (after: fewer registers live across it)
    const int K = p.K;
    p3d_gemv_chain<MR, GC>(pw, gb, ge, M, wf, [&](int g, int r) {
      return *(const f32x4*)&xs[r * K + 16 * g + 4 * q]; }, acc);
  } else {
    p3d_gemv_chain<MR, GC>(pw, gb, ge, M, wf, [&](int g, int r) {
      return *(const f32x4*)(p.X + ((int64_t)g << 8) + ((r + 16 * q) << 2)); }, acc);
  }
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    acc[r] += __shfl_xor(acc[r], 16, 64);
    acc[r] += __shfl_xor(acc[r], 32, 64);
  }
  if (q == 0) {
#pragma unroll
    for (int r = 0; r < MR; ++r) red[0][w][r][i] = acc[r];
  }
  __syncthreads();
  if (w != 0) return;
  float zs = 0.f;
#pragma unroll
  for (int u = 0; u < WV; ++u) zs += red[0][u][q][i];
  const float y = p3d_gemv_epi(p, e, zs, q, cc);   // (lanes q >= M: unused)
  if (!f.fout) {
    if (q < M && cok) p.Y[p3d_pk(q, col, (p.N + 15) >> 4)] = y;
    return;
  }
  p3d_gemv_publish(p3d_rsrc(f.hand), 0, M, p.N, col, y, tag);   // hand-off to the last workgroup
}

// ---- the whole batch <= 4 forward as ONE launch (k_gemv_chain) --------------------------------
// Where every hidden layer's column tiles fit on the device at once (H L / 16 <= CUs: cfg2's four
// 1024-wide layers are exactly 256 workgroups), workgroup (layer l, tile t) requests its 64 KB
// weight slice at kernel start -- all H layers' weights stream in together, not one layer's per
// launch (a k_gemv launch is bound by its 64 CUs' intake of 64 KB each) -- then waits for layer
// l - 1's outputs as data-tagged granules, contracts, and hands its 16 columns on.  The input layer
// (K = 32) is computed by layer 2's workgroups, tile t each, as their first act (hand-off slot 0):
// recomputing all of it in every layer-1 workgroup (k_gemv_fold's way) meant 128 KB of input-layer
// weights per CU, the longest phase of the launch (tools/trace_chain.py).  Its tile is layer 2's
// residual too; later blocks read theirs from layer l - 2's hand-off.  Workgroups 0 .. 2 (layer 1,
// tiles 0 .. 2; idle once their tiles are out) then run an output-layer tile each on the last
// layer's hand-off (p3d_gemv_fold_out), and workgroup 0 advances the slot's epoch: every workgroup
// has read the epoch by then (each published with its tag, and each layer's tiles were all
// gathered by the next layer's).
// Every wait is bounded (err); the launch needs its grid resident (host: H L / 16 <= CUs).  Same
// k_gemv arithmetic throughout, so the same bits as the six launches
// (tests/test_gpu_parity.py::test_gemv_small_batch).
#ifndef P3D_CHAIN_PIN_ARGS
#define P3D_CHAIN_PIN_ARGS 1       // k_gemv_chain's arguments fetched in one round (round 5)
#endif
#define P3D_GEMV_CHAIN_MAXH 8
#define P3D_GEMV_CHAIN_MAXK 2048   // (L = 2048: the second half of each wave's slice requested after the first's FMAs)
struct GemvChain {
  GemvArgs in;                          // layer 0 (X = the user rows, row-major)
  GemvArgs ly[P3D_GEMV_CHAIN_MAXH];     // hidden layers 1 .. H (X, res, Y unused: handed over)
  GemvArgs out;                         // the output layer (Y = the user's y, row-major)
  int H, T;                             // hidden layers; column tiles per layer (L / 16)
  int res;                              // residual blocks: layer l even adds layer l - 2's output
  float* hand;                          // this slot: [H + 1][4 rows][L / 2] 16-B granules (0: the input
                                        // layer's output, l: hidden layer l's)
  unsigned* epoch;                      // this slot's epoch word (tag = epoch + 1)
  int* err;
  GemvFrames fr;                        // p3d_lift: raw 2D rows in (fr.raw), 3D rows out (fr.out)
};

// (Measured and rejected: each wave DMAing its fragments into LDS at kernel start -- layer 1 too,
// ahead of its input layer, with no registers held -- and reading them back for the contraction:
// 17.5 vs 16.3-16.7 us per forward, A/B on one box, profiles/r04_gemv_chain_ab.json.)
template <int MR, int GC>
__global__ __launch_bounds__(1024) void k_gemv_chain(GemvChain c) {
  constexpr int WV = 16;
  __shared__ float xs[MR * P3D_GEMV_CHAIN_MAXK];
  __shared__ float red[4][WV][MR][16];
  __shared__ float xn[MR][64];   // p3d_lift: the normalised raw rows (layer 2's wave 0)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
#ifdef P3D_TRACE   // development builds (tools/trace_chain.py): per workgroup at 8 b: start, input,
                   // contracted, published; workgroup 0 also output gathered (4), end (5),
                   // its output tile contracted (6) and reduced (7)
#define P3D_CH_STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 512) g_p3d_trace[blockIdx.x * 8 + (k)] = wall_clock64(); } while (0)
#else
#define P3D_CH_STAMP(k) do { } while (0)
#endif
  P3D_CH_STAMP(0);
  const unsigned tag = __hip_atomic_load(c.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int b = blockIdx.x, l = 1 + b / c.T, t = b - (l - 1) * c.T;
  // this layer's arguments, read with constant indices only (a runtime index into the argument
  // block would copy it to scratch)
  GemvArgs p = c.ly[0];
#pragma unroll
  for (int k = 1; k < P3D_GEMV_CHAIN_MAXH; ++k)
    if (k == l - 1) p = c.ly[k];
#if P3D_CHAIN_PIN_ARGS
  // (round 5) the layer's arguments and the launch's shared ones fetched in ONE round of scalar
  // loads: left to itself the compiler loaded them where they are used, behind branches on earlier
  // ones -- six dependent scalar-load round trips to the argument segment the host wrote just before
  // the launch (1.4 us to the arguments in hand, profiles/r04_chain_trace_args.json)
  asm volatile("" ::"s"(p.Wf), "s"(p.bias), "s"(p.M), "s"(p.K), "s"(p.N), "s"(p.bn), "s"(p.relu), "s"(p.gamma),
               "s"(p.beta), "s"(p.mmean), "s"(p.mvar), "s"(c.hand), "s"(c.err), "s"(c.res), "s"(c.T),
               "s"(c.in.Wf), "s"(c.in.X), "s"(c.in.bias));
#endif
  const int M = p.M, K = p.K, N = p.N, ngK = K >> 4;
  const int gb = (ngK * w) / WV, ge = (ngK * (w + 1)) / WV;
  const int col = 16 * t + i;
#ifdef P3D_TRACE
  if (b >= 3) P3D_CH_STAMP(5);   // the layer's arguments in hand
#endif
  const __amdgpu_buffer_rsrc_t rh = p3d_rsrc(c.hand);
  const int gpl = 4 * (N >> 1);                  // granules per layer
  // ---- the weight slice, then the epilogue operands (wave 0, lane (i, q) = row q, column col) ---
  // ---- layer 2's wave 0 first computes the input layer's tile t (hand-off slot 0): layer 1's
  // input, and layer 2's own residual when blocks are residual.  Before its weight slice: a wave's
  // loads complete in issue order, so operands requested behind 4 KB of weights wait for them. ----
  const bool second = c.res && l >= 2 && (l & 1) == 0;
  float rv = 0.f;
  if (l == 2 && w == 0) {
    float v0 = 0.f;
    if (c.fr.raw && c.fr.ldraw <= 64) {   // (the weights and epilogue operands requested first)
      f32x4 wv[2][4];
      GemvEpi ei;
      p3d_gemv_in_weights(c.in, col, wv);
      p3d_gemv_epi_load(c.in, 0, col, ei);
      p3d_gemv_in_stage<MR>(c.fr, M, xn);
      if (q < M) v0 = p3d_gemv_in_value_s(c.in, c.fr, xn, wv, ei, q, col);
    } else if (q < M) {
      f32x4 wv[2][4];
      GemvEpi ei;
      p3d_gemv_in_weights(c.in, col, wv);
      p3d_gemv_epi_load(c.in, 0, col, ei);
      v0 = c.fr.raw ? p3d_gemv_in_value_n(c.in, c.fr, wv, ei, q, col) : p3d_gemv_in_value_g(c.in, wv, ei, q, col);
    }
    p3d_gemv_publish(rh, 0, M, N, col, v0, tag);
    rv = v0;
#ifdef P3D_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    P3D_CH_STAMP(4);   // the input layer's tile published
#endif
  }
  const f32x4* pw = (const f32x4*)p.Wf + (int64_t)t * ngK * 64 + lane;
  f32x4 wf[GC];
  p3d_gemv_preload<GC>(pw, gb, ge, wf);
  GemvEpi e;
  e.ctr = p.ctr;
  if (w == 0 && q < M) p3d_gemv_epi_load(p, q, col, e);
  p3d_pin<GC>(wf);   // (every wait below is far longer than these loads)
  p3d_pin_epi(e);
  // ---- the residual tile of later blocks: layer l - 2's hand-off (wave 0) -----------------------
  if (second && l > 2 && w == 0 && q < M) {
    const int off = ((l - 2) * gpl + q * (N >> 1) + (col >> 1)) * 16;
    u32x4_t v = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rh, off, 0, 16));
    for (int spin = 0; !(v.y == tag && v.w == tag); ++spin) {
      if (spin > P3D_XCHG_SPIN) { __hip_atomic_store(c.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); break; }
      __builtin_amdgcn_s_sleep(1);
      v = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rh, off, 0, 16));
    }
    rv = __uint_as_float((i & 1) ? v.z : v.x);
  }
  // ---- this layer's input: layer l - 1's hand-off (slot 0: the input layer) --------------------
  p3d_gemv_gather_wave(rh, (l - 1) * gpl, M, K, gb, ge, tag, xs, c.err);
  P3D_CH_STAMP(1);
  // ---- contraction, quarters, waves (k_gemv) -------------------------------------------------
  float acc[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) acc[r] = 0.f;
  p3d_gemv_chain<MR, GC>(pw, gb, ge, M, wf, [&](int g, int r) {
    return *(const f32x4*)&xs[r * K + 16 * g + 4 * q]; }, acc);
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    acc[r] += __shfl_xor(acc[r], 16, 64);
    acc[r] += __shfl_xor(acc[r], 32, 64);
  }
  if (q == 0) {
#pragma unroll
    for (int r = 0; r < MR; ++r) red[0][w][r][i] = acc[r];
  }
  __syncthreads();
  P3D_CH_STAMP(2);
  if (w == 0) {
    float zs = 0.f;
#pragma unroll
    for (int u = 0; u < WV; ++u) zs += red[0][u][q][i];
    float y = p3d_gemv_epi(p, e, zs, q, col);   // (p.res is null: the residual is added last, as there)
    if (second) y += rv;
    p3d_gemv_publish(rh, l * gpl, M, N, col, y, tag);
#ifdef P3D_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    P3D_CH_STAMP(3);
  }
  if (b >= ((c.out.N + 15) >> 4)) return;
  // ---- workgroups 0 .. N_out / 16 - 1: an output-layer tile each, on the last layer's hand-off ----
  GemvFold f{};
  f.fout = 1;
  f.out = c.out;
  f.hand = c.hand + (int64_t)c.H * gpl * 4;
  f.epoch = c.epoch;
  f.err = c.err;
  f.fr = c.fr;
  p3d_gemv_fold_out<MR, WV, 4, 1>(f, tag, xs, red, b);
  P3D_CH_STAMP(5);
}
