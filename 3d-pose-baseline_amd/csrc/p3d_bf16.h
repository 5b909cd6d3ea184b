// p3d_bf16.h -- bf16 inference path (cfg5 stress config: L = 4096, 4 blocks, B = 1024):
// bf16 weights and activations, fp32 accumulation (v_mfma_f32_16x16x32_bf16), fp32
// bias/BN/ReLU/residual epilogue, activations rounded to bf16 when stored.
//
// bf16 fragment-major packing of an [R, C] matrix (C a multiple of 32): 16x32 tiles of
// 1 KB, tile (rt, g) lane l = i + 16q holding the 8 bf16 of element row 16rt+i,
// columns 32g+8q .. +7 -- the A (or B^T) operand of one 16x16x32 MFMA.  A wave
// instruction moves one whole tile (64 lanes x 16 B), global->LDS via LDS-DMA
// (global_load_lds_dwordx4) and LDS->VGPR via ds_read_b128, both conflict free.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// element offset (bf16 units) of (r, c) in a bf16 packed matrix with ng = C/32 groups
__device__ __host__ __forceinline__ int64_t p3d_pk16(int r, int c, int ng) {
  return (((int64_t)(r >> 4) * ng + (c >> 5)) << 9) + (((r & 15) + ((c & 31) >> 3) * 16) << 3) + (c & 7);
}

__device__ __forceinline__ float p3d_bf2f(unsigned short h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ unsigned short p3d_f2bf(float x) {
  const __bf16 b = (__bf16)x;   // v_cvt_pk_bf16_f32: round to nearest even, NaN-preserving
  return __builtin_bit_cast(unsigned short, b);
}

// Per-column epilogue parameters of an inference layer: y = (acc + b) * inv + shift.
struct Bf16Epi {
  const float* bias;    // [N]
  const float* inv;     // [N] BN eval scale rsqrt(var+eps)*gamma (null: no BN)
  const float* shift;   // [N] beta - mean*inv
  int relu;
};

// =====================================================================================
// Large bf16 GEMM + fused epilogue: Y[M,N] = epi(A[M,K] * W[K,N]) (+ residual)
//   A  : bf16 packed [M, K]          (ngA = K/32)
//   Bt : bf16 packed [N, K] (= W^T)  (ngB = K/32)
//   Y, residual: bf16 packed [M, N]  (ngY = N/32)
// 128x128 tile per 256-thread workgroup, 4 waves of 64x64 (4x4 MFMA 16x16x32 tiles),
// BK = 64 (two k-groups), LDS double buffer filled by LDS-DMA, one barrier per k-step
// plus the one that retires the DMA.  M, N multiples of 128, K a multiple of 32 (BK).
// =====================================================================================
struct GemmBf16Args {
  const unsigned short* A; const unsigned short* Bt; const unsigned short* res; unsigned short* Y;
  int M, N, K;
  Bf16Epi epi;
};

template <int N>
__device__ __forceinline__ void p3d_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// outstanding = number of LDS-DMA instructions this wave may leave in flight
template <int PER, int NST>
__device__ __forceinline__ void p3d_wait_stages(int later_stages) {
  if constexpr (NST >= 4) { if (later_stages >= 3) { p3d_wait_vm<3 * PER>(); return; } }
  if constexpr (NST >= 3) { if (later_stages >= 2) { p3d_wait_vm<2 * PER>(); return; } }
  if (later_stages >= 1) { p3d_wait_vm<PER>(); return; }
  p3d_wait_vm<0>();
}

// LDS fragment read the compiler does not track: hipcc's waitcnt pass merged the two register
// sets of the software pipeline at the loop head and waited lgkmcnt(0) in front of every
// k-group's MFMAs (the group read one step ahead included), exposing the LDS latency each
// group.  With the reads in asm the kernel counts them itself (p3d_wait_lgkm), and the
// sched_barrier keeps the MFMAs behind that wait (cdna_hip_programming.md §5.4 rule 18).
__device__ __forceinline__ bf16x8 p3d_ds_read(const unsigned char* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(uintptr_t)p) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void p3d_wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int BK, int NST>
__global__ __launch_bounds__(256) void k_gemm_bf16(GemmBf16Args p) {
  constexpr int KG = BK / 32;                 // k-groups per stage
  constexpr int STAGE = (8 + 8) * KG * 1024;  // bytes: 8 A tiles + 8 B tiles per k-group
  constexpr int EPI = 128 * 132 * 4;
  constexpr int LDS = (NST * STAGE > EPI) ? NST * STAGE : EPI;
  constexpr int PER = 4 * KG;                 // LDS-DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  // XCD-aware remap: consecutive tile ids (sharing A rows) land on one XCD's L2
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  // grouped order: runs of GM row tiles x all column tiles, so each XCD's contiguous range
  // of 32 tile ids is a GM x (32/GM) block -> its L2 streams GM A row panels + 32/GM B
  // column panels instead of 1 A panel + every B panel (MALL traffic 2.75x lower at cfg5)
  const int tiles_n = p.N / 128, tiles_m = p.M / 128;
  const int GM = (tiles_m % 4 == 0) ? 4 : ((tiles_m % 2 == 0) ? 2 : 1);
  const int grp = tile_id / (GM * tiles_n), in_grp = tile_id % (GM * tiles_n);
  const int mt = grp * GM + (in_grp % GM), nt = in_grp / GM;
  const int ngA = p.K / 32;
  const int nks = p.K / BK;
  const unsigned char* Ag = (const unsigned char*)p.A + (int64_t)(8 * mt) * ngA * 1024;
  const unsigned char* Bg = (const unsigned char*)p.Bt + (int64_t)(8 * nt) * ngA * 1024;

  // each wave DMAs PER of the 16*KG tiles of a stage
  auto issue = [&](int ks, int buf) {
    unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int t = w * PER + c;               // 0 .. 16*KG-1
      const bool isB = t >= 8 * KG;
      const int tt = isB ? t - 8 * KG : t;
      const int j = tt / KG, g = tt % KG;      // row tile j (0..7), k-group g
      const unsigned char* src = (isB ? Bg : Ag) + ((int64_t)j * ngA + ks * KG + g) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(base + t * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

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
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) af[r] = *(const bf16x8*)(base + ((4 * wm + r) * KG + g) * 1024 + lane * 16);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        bfr[c] = *(const bf16x8*)(base + (8 * KG + (4 * wn + c) * KG + g) * 1024 + lane * 16);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[r], bfr[c], acc[r][c], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // ---- epilogue: stage the fp32 tile in LDS (row stride 132), then 16 B packed stores
  float* et = (float*)smem;
  const int i = lane & 15, q = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) et[(64 * wm + 16 * r + 4 * q + e) * 132 + 64 * wn + 16 * c + i] = acc[r][c][e];
  __syncthreads();
  const int ngY = p.N / 32;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int item = it * 256 + tid;        // 32 chunks (8 row tiles x 4 col groups) x 64 lanes
    const int chunk = item >> 6, l = item & 63;
    const int rl = 16 * (chunk >> 2) + (l & 15);      // row within tile
    const int cl = 32 * (chunk & 3) + 8 * (l >> 4);   // first of 8 columns within tile
    const int row = 128 * mt + rl, col = 128 * nt + cl;
    const int64_t off = p3d_pk16(row, col, ngY);
    u16x8 rv;
    if (p.res) rv = *(const u16x8*)(p.res + off);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int n = col + e;
      float z = et[rl * 132 + cl + e] + p.epi.bias[n];
      float y = p.epi.inv ? z * p.epi.inv[n] + p.epi.shift[n] : z;
      if (p.epi.relu) y = fmaxf(y, 0.0f);
      if (p.res) y += p3d_bf2f(rv[e]);
      o[e] = p3d_f2bf(y);
    }
    *(u16x8*)(p.Y + off) = o;
  }
}

// Software-pipelined form of k_gemm_bf16 (same tiles, LDS ring and epilogue): the ds_reads
// of k-group g+1 are issued before the MFMAs of group g (two fragment register sets), and
// the first group of stage s+1 is read right after the one barrier per stage, so LDS
// latency hides behind MFMA work at one wave per SIMD (the k_gemm_bf16 schedule waited
// lgkmcnt(0) in front of every four MFMAs).  One barrier per stage: each wave drains its own
// reads of stage s (lgkmcnt) before it, and the DMA refilling stage s's buffer is issued
// after it.
// DIAG (development ablations, tools/bf16_dev.hip): 1 no MFMA, 2 no LDS-DMA after the
// prologue, 3 no LDS fragment reads after the prologue; 0 = the product kernel.
template <int BK, int NST, int WAVES, bool PRIO = false, int DIAG = 0, bool AR = false>
__global__ __launch_bounds__(64 * WAVES) void k_gemm_bf16p(GemmBf16Args p) {
  constexpr int KG = BK / 32;
  constexpr int STAGE = (8 + 8) * KG * 1024;
  constexpr int EPI = 128 * 132 * 4;
  constexpr int LDS = (NST * STAGE > EPI) ? NST * STAGE : EPI;
  constexpr int PER = 16 * KG / WAVES;            // LDS-DMA instructions per wave per stage
  constexpr int CT = WAVES == 4 ? 4 : 2;          // 16-column MFMA tiles per wave (rows: 4)
  constexpr int WN = 8 / CT;                      // waves along N
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tiles_n = p.N / 128, tiles_m = p.M / 128;
  const int GM = (tiles_m % 4 == 0) ? 4 : ((tiles_m % 2 == 0) ? 2 : 1);
  const int grp = tile_id / (GM * tiles_n), in_grp = tile_id % (GM * tiles_n);
  const int mt = grp * GM + (in_grp % GM), nt = in_grp / GM;
  const int ngA = p.K / 32;
  const int nks = p.K / BK;
  const unsigned char* Ag = (const unsigned char*)p.A + (int64_t)(8 * mt) * ngA * 1024;
  const unsigned char* Bg = (const unsigned char*)p.Bt + (int64_t)(8 * nt) * ngA * 1024;

  auto issue = [&](int ks, int buf) {
    unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int t = w * PER + c;
      const bool isB = t >= 8 * KG;
      const int tt = isB ? t - 8 * KG : t;
      const int j = tt / KG, g = tt % KG;
      const unsigned char* src = (isB ? Bg : Ag) + ((int64_t)j * ngA + ks * KG + g) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(base + t * 1024), 16, 0, 0);
    }
  };
  auto read = [&](int buf, int g, bf16x8 (&af)[4], bf16x8 (&bfr)[CT]) {
    const unsigned char* base = smem + buf * STAGE;
    if constexpr (AR) {
#pragma unroll
      for (int r = 0; r < 4; ++r) af[r] = p3d_ds_read(base + ((4 * wm + r) * KG + g) * 1024 + lane * 16);
#pragma unroll
      for (int c = 0; c < CT; ++c) bfr[c] = p3d_ds_read(base + (8 * KG + (CT * wn + c) * KG + g) * 1024 + lane * 16);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) af[r] = *(const bf16x8*)(base + ((4 * wm + r) * KG + g) * 1024 + lane * 16);
#pragma unroll
      for (int c = 0; c < CT; ++c)
        bfr[c] = *(const bf16x8*)(base + (8 * KG + (CT * wn + c) * KG + g) * 1024 + lane * 16);
    }
  };

  f32x4 acc[4][CT];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < CT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][4], fb[2][CT];

#pragma unroll
  for (int s0 = 0; s0 < NST - 1; ++s0)
    if (s0 < nks) issue(s0, s0);
  {
    const int later = (nks - 1) < (NST - 2) ? (nks - 1) : (NST - 2);
    p3d_wait_stages<PER, NST>(later);
    __builtin_amdgcn_s_barrier();
    read(0, 0, fa[0], fb[0]);
  }
  int cur = 0;
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks % NST;
    if (DIAG != 2 && ks + NST - 1 < nks) issue(ks + NST - 1, (ks + NST - 1) % NST);
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      const int nxt = cur ^ 1;
      if (g + 1 < KG) {
        if (DIAG != 3) read(buf, g + 1, fa[nxt], fb[nxt]);
        if constexpr (AR) p3d_wait_lgkm<4 + CT>();      // this group's reads, not the ones just issued
      } else if (ks + 1 < nks) {
        // stage ks+1 must have landed (counted DMA wait) and every wave must be done
        // reading stage ks before anyone refills it: drain this wave's reads, barrier,
        // then prefetch the first group of stage ks+1
        const int later = (nks - 2 - ks) < (NST - 2) ? (nks - 2 - ks) : (NST - 2);
        if (DIAG == 2) p3d_wait_vm<0>();
        else p3d_wait_stages<PER, NST>(later);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (DIAG != 3) read((ks + 1) % NST, 0, fa[nxt], fb[nxt]);
        if constexpr (AR) __builtin_amdgcn_sched_barrier(0);
      } else {
        if constexpr (AR) p3d_wait_lgkm<0>();
      }
      if (PRIO) __builtin_amdgcn_s_setprio(1);
      if constexpr (DIAG == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" ::"v"(fa[cur][r]));
#pragma unroll
        for (int c = 0; c < CT; ++c) asm volatile("" ::"v"(fb[cur][c]));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < CT; ++c)
            acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(DIAG == 3 ? fa[0][r] : fa[cur][r],
                                                                DIAG == 3 ? fb[0][c] : fb[cur][c], acc[r][c], 0, 0, 0);
      }
      if (PRIO) __builtin_amdgcn_s_setprio(0);
      cur = nxt;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // ---- epilogue (as k_gemm_bf16) ----
  float* et = (float*)smem;
  const int i = lane & 15, q = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        et[(64 * wm + 16 * r + 4 * q + e) * 132 + 16 * CT * wn + 16 * c + i] = acc[r][c][e];
  __syncthreads();
  const int ngY = p.N / 32;
#pragma unroll
  for (int it = 0; it < 2048 / (64 * WAVES); ++it) {
    const int item = it * 64 * WAVES + tid;
    const int chunk = item >> 6, l = item & 63;
    const int rl = 16 * (chunk >> 2) + (l & 15);
    const int cl = 32 * (chunk & 3) + 8 * (l >> 4);
    const int row = 128 * mt + rl, col = 128 * nt + cl;
    const int64_t off = p3d_pk16(row, col, ngY);
    u16x8 rv;
    if (p.res) rv = *(const u16x8*)(p.res + off);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int n = col + e;
      float z = et[rl * 132 + cl + e] + p.epi.bias[n];
      float y = p.epi.inv ? z * p.epi.inv[n] + p.epi.shift[n] : z;
      if (p.epi.relu) y = fmaxf(y, 0.0f);
      if (p.res) y += p3d_bf2f(rv[e]);
      o[e] = p3d_f2bf(y);
    }
    *(u16x8*)(p.Y + off) = o;
  }
}

// (round 5 built two more hidden-layer forms here and measured both slower than k_gemm_bf16p in
// the cfg5 step: k_gemm_bf16s, 256 x 128 tiles with K split over two workgroups meeting in the
// launch, and k_gemm_bf16d, K split over a 128 x 128 tile's 4 waves with operands straight into
// registers; round 6 removed both from the product; the sources stay in the history)

// (the round-3 ablation kernels k_gemm_bf16k / k_gemm_bf16w live in tools/bf16_dev_kernels.h)

// =====================================================================================
// Small-N bf16 layer (output layer, N = 48): register-direct packed operands, 16 waves
// split K (as k_fwd's inference tiling), fp32 row-major output.
// =====================================================================================
struct SmallBf16Args {
  const unsigned short* A; const unsigned short* Bt;  // packed, ng = K/32
  int M, N, K;
  const float* bias;
  float* Y; int64_t ldy;
};

template <int WK>
__global__ __launch_bounds__(64 * WK) void k_out_bf16(SmallBf16Args p) {
  __shared__ f32x4 red[WK - 1][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ct = blockIdx.x, rt = blockIdx.y;
  const int ng = p.K / 32;
  const int gb = (ng * w) / WK, ge = (ng * (w + 1)) / WK;
  const bf16x8* pa = (const bf16x8*)p.A + ((int64_t)rt * ng) * 64 + lane;
  const bf16x8* pb = (const bf16x8*)p.Bt + ((int64_t)ct * ng) * 64 + lane;
  f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  int g = gb;
  for (; g + 1 < ge; g += 2) {
    const bf16x8 a0 = pa[g * 64], b0 = pb[g * 64], a1 = pa[(g + 1) * 64], b1 = pb[(g + 1) * 64];
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc1, 0, 0, 0);
  }
  if (g < ge) acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[g * 64], pb[g * 64], acc0, 0, 0, 0);
  acc0 += acc1;
  if (w > 0) red[w - 1][lane] = acc0;
  __syncthreads();
  if (w > 0) return;
#pragma unroll
  for (int u = 0; u < WK - 1; ++u) acc0 += red[u][lane];
  const int i = lane & 15, q = lane >> 4;
  const int col = 16 * ct + i;
  if (col >= p.N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * rt + 4 * q + r;
    if (row < p.M) p.Y[(int64_t)row * p.ldy + col] = acc0[r] + p.bias[col];
  }
}

// x fp32 row-major [M, 32] -> bf16 packed [Mpad, 32] (one k-group), rows >= M zero
__global__ __launch_bounds__(256) void k_x_to_bf16(const float* __restrict__ x, int M, int K,
                                                   unsigned short* __restrict__ out, int Mpad) {
  const int item = blockIdx.x * 256 + threadIdx.x;   // one 8-element lane slot
  const int ng = K / 32;
  if (item >= (Mpad / 16) * ng * 64) return;
  const int chunk = item >> 6, l = item & 63;
  const int rt = chunk / ng, g = chunk % ng;
  const int row = 16 * rt + (l & 15), c0 = 32 * g + 8 * (l >> 4);
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = row < M ? p3d_f2bf(x[(int64_t)row * K + c0 + e]) : (unsigned short)0;
  *(u16x8*)(out + (int64_t)item * 8) = o;
}

// W fp32 [K, N] (TF layout) -> Wt bf16 packed [NP, K] (rows n, padded to 16, cols k);
// also the per-column BN-eval affine (inv, shift) when gamma is given.
__global__ __launch_bounds__(256) void k_pack_bf16(const float* __restrict__ W, int K, int N,
                                                   unsigned short* __restrict__ out) {
  const int NP = (N + 15) & ~15;
  const int64_t item = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int ng = K / 32;
  if (item >= (int64_t)(NP / 16) * ng * 64) return;
  const int64_t chunk = item >> 6;
  const int l = (int)(item & 63);
  const int nt = (int)(chunk / ng), g = (int)(chunk % ng);
  const int n = 16 * nt + (l & 15), k0 = 32 * g + 8 * (l >> 4);
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = n < N ? p3d_f2bf(W[(int64_t)(k0 + e) * N + n]) : (unsigned short)0;
  *(u16x8*)(out + item * 8) = o;
}

__global__ void k_bn_affine(const float* __restrict__ gamma, const float* __restrict__ beta,
                            const float* __restrict__ mm, const float* __restrict__ mv, float eps, int N,
                            float* __restrict__ inv, float* __restrict__ shift) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const float iv = (1.0f / sqrtf(mv[n] + eps)) * gamma[n];
  inv[n] = iv;
  shift[n] = beta[n] - mm[n] * iv;
}
