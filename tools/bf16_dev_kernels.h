// bf16_dev_kernels.h -- ablation variants of the cfg5 hidden-layer bf16 GEMM (round 3, DESIGN.md
// 5f), kept for tools/bf16_dev.hip only: no dispatch path of libp3d.so uses them.
#pragma once
#include "../3d-pose-baseline_amd/csrc/p3d_bf16.h"

// =====================================================================================
// 128 x 128 tile with the waves splitting K (k_gemm_bf16k): 8 waves = 2 k-groups x 2 x 2 wave
// tiles of 64 x 64; wave (kg, wm, wn) contracts only k-group kg of every 64-deep stage.
// Why: k_gemm_bf16p's 64 x 32 wave tiles read 6 fragments per 8 MFMAs; with the LDS-DMA
// writes that is 256 B/clk per CU at the MFMA rate -- the LDS array, not the MFMA pipes,
// bounds it (ablations in tools/bf16_dev.py: no DMA 28.6 us, no MFMA 31.3, both 38.5 for
// 14-17 us of MFMA work).  64 x 64 wave tiles read 8 fragments per 16 MFMAs: a third fewer
// LDS bytes for the same work.  The two k-group halves meet once, through LDS, at the end
// (kg 1's accumulators added to kg 0's: one fixed association).
// =====================================================================================
template <int NST, int ROT = 0>
__global__ __launch_bounds__(512) void k_gemm_bf16k(GemmBf16Args p) {
  constexpr int KG = 2;
  constexpr int STAGE = (8 + 8) * KG * 1024;       // 32 KB
  constexpr int EPI = 128 * 132 * 4;
  constexpr int LDS = (NST * STAGE > EPI) ? NST * STAGE : EPI;
  constexpr int PER = 16 * KG / 8;                 // LDS-DMA instructions per wave per stage (4)
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = w >> 2, wm = (w >> 1) & 1, wn = w & 1;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tiles_n = p.N / 128, tiles_m = p.M / 128;
  const int GM = (tiles_m % 4 == 0) ? 4 : ((tiles_m % 2 == 0) ? 2 : 1);
  const int grp = tile_id / (GM * tiles_n), in_grp = tile_id % (GM * tiles_n);
  const int mt = grp * GM + (in_grp % GM), nt = in_grp / GM;
  const int ngA = p.K / 32;
  const int nks = p.K / 64;
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
      int kse = ks;
      if constexpr (ROT == 1) { kse += (tile_id >> 5) * (nks >> 3); if (kse >= nks) kse -= nks; }
      if constexpr (ROT == 2) { kse += (bid % 8) * (nks >> 3); if (kse >= nks) kse -= nks; }
      const unsigned char* src = (isB ? Bg : Ag) + ((int64_t)j * ngA + kse * KG + g) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(base + t * 1024), 16, 0, 0);
    }
  };
  auto read = [&](int buf, bf16x8 (&af)[4], bf16x8 (&bfr)[4]) {
    const unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int r = 0; r < 4; ++r) af[r] = *(const bf16x8*)(base + ((4 * wm + r) * KG + kg) * 1024 + lane * 16);
#pragma unroll
    for (int c = 0; c < 4; ++c) bfr[c] = *(const bf16x8*)(base + (8 * KG + (4 * wn + c) * KG + kg) * 1024 + lane * 16);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][4], fb[2][4];

#pragma unroll
  for (int s0 = 0; s0 < NST - 1; ++s0)
    if (s0 < nks) issue(s0, s0);
  {
    const int later = (nks - 1) < (NST - 2) ? (nks - 1) : (NST - 2);
    p3d_wait_stages<PER, NST>(later);
    __builtin_amdgcn_s_barrier();
    read(0, fa[0], fb[0]);
  }
  // two k-steps per trip so the register sets are indexed statically
  auto step = [&](int ks, bf16x8 (&ca)[4], bf16x8 (&cb)[4], bf16x8 (&na)[4], bf16x8 (&nb)[4]) {
    if (ks + NST - 1 < nks) issue(ks + NST - 1, (ks + NST - 1) % NST);
    if (ks + 1 < nks) {
      const int later = (nks - 2 - ks) < (NST - 2) ? (nks - 2 - ks) : (NST - 2);
      p3d_wait_stages<PER, NST>(later);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      read((ks + 1) % NST, na, nb);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[r], cb[c], acc[r][c], 0, 0, 0);
  };
  for (int ks = 0; ks < nks; ks += 2) {
    step(ks, fa[0], fb[0], fa[1], fb[1]);
    if (ks + 1 < nks) step(ks + 1, fa[1], fb[1], fa[0], fb[0]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // ---- combine the k-group halves in LDS, then the epilogue (as k_gemm_bf16p) ----
  float* et = (float*)smem;
  const int i = lane & 15, q = lane >> 4;
  if (kg == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) et[(64 * wm + 16 * r + 4 * q + e) * 132 + 64 * wn + 16 * c + i] = acc[r][c][e];
  }
  __syncthreads();
  if (kg == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float* t = &et[(64 * wm + 16 * r + 4 * q + e) * 132 + 64 * wn + 16 * c + i];
          *t = acc[r][c][e] + *t;
        }
  }
  __syncthreads();
  const int ngY = p.N / 32;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int item = it * 512 + tid;
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

// counted wait for up to 6 stages in flight behind the one about to be read
template <int PER, int NST>
__device__ __forceinline__ void p3d_wait_stages6(int later) {
  static_assert(NST <= 7 && PER * (NST - 2) <= 63, "vmcnt range");
  if constexpr (NST >= 7) { if (later >= 5) { p3d_wait_vm<5 * PER>(); return; } }
  if constexpr (NST >= 6) { if (later >= 4) { p3d_wait_vm<4 * PER>(); return; } }
  if constexpr (NST >= 5) { if (later >= 3) { p3d_wait_vm<3 * PER>(); return; } }
  if constexpr (NST >= 4) { if (later >= 2) { p3d_wait_vm<2 * PER>(); return; } }
  if (later >= 1) { p3d_wait_vm<PER>(); return; }
  p3d_wait_vm<0>();
}

// =====================================================================================
// Split-K form with 128 x 64 wave tiles (k_gemm_bf16w): k_gemm_bf16s's 256 x 128 tile and
// in-launch K-half hand-off, but 4 waves (one per SIMD) of 128 x 64 instead of 8 of 64 x 64.
// LDS budget per 64-deep k-step: the waves read 4 x (8 + 4) fragments per k-group = 96 KB
// (k_gemm_bf16s: 128 KB; the 128 x 128 k_gemm_bf16p: 96 KB for half the MFMA work) and the
// LDS-DMA writes 48 KB, against 1,024 MFMA cycles per SIMD: the LDS array stays below the
// MFMA pipes.  KG k-groups per stage (BK = 32 KG), NST stages in the LDS ring.
// =====================================================================================
template <int KG, int NST>
__global__ __launch_bounds__(256) void k_gemm_bf16w(GemmBf16SplitArgs sa) {
  constexpr int AT = 16, BT = 8;                    // 16-row A tiles, 16-column B tiles per k-group
  constexpr int STAGE = (AT + BT) * KG * 1024;
  constexpr int EPI = 256 * 132 * 4;
  constexpr int LDS = (NST * STAGE > EPI) ? NST * STAGE : EPI;
  constexpr int PER = (AT + BT) * KG / 4;           // LDS-DMA instructions per wave per stage
  static_assert(LDS <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  const GemmBf16Args& p = sa.g;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;                // 2 x 2 waves of 128 x 64
  const int tiles_n = p.N / 128, tiles_m = p.M / 256, T = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const bool reader = bid >= T;
  const int lb = reader ? bid - T : bid;
  const int q8 = T / 8, r8 = T % 8, xcd = lb % 8;
  const int tile_id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + lb / 8;
  const int GM = (tiles_m % 4 == 0) ? 4 : ((tiles_m % 2 == 0) ? 2 : 1);
  const int grp = tile_id / (GM * tiles_n), in_grp = tile_id % (GM * tiles_n);
  const int mt = grp * GM + (in_grp % GM), nt = in_grp / GM;
  const int tile = mt * tiles_n + nt;
  const int ngA = p.K / 32;
  const int nks = p.K / (64 * KG);                  // k-steps per half
  const int ks0 = reader ? 0 : nks;
  unsigned* epoch = sa.sync + tile * 64;
  unsigned* flag = epoch + 32;
  unsigned tag = 0;
  if (tid == 0) tag = __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const unsigned char* Ag = (const unsigned char*)p.A + (int64_t)(16 * mt) * ngA * 1024;
  const unsigned char* Bg = (const unsigned char*)p.Bt + (int64_t)(8 * nt) * ngA * 1024;

  auto issue = [&](int ks, int buf) {
    unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int t = w * PER + c;
      const bool isB = t >= AT * KG;
      const int tt = isB ? t - AT * KG : t;
      const int j = tt / KG, g = tt % KG;
      const unsigned char* src = (isB ? Bg : Ag) + ((int64_t)j * ngA + (ks0 + ks) * KG + g) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(base + t * 1024), 16, 0, 0);
    }
  };
  auto read = [&](int buf, int g, bf16x8 (&af)[8], bf16x8 (&bfr)[4]) {
    const unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int c = 0; c < 4; ++c) bfr[c] = p3d_ds_read(base + (AT * KG + (4 * wn + c) * KG + g) * 1024 + lane * 16);
#pragma unroll
    for (int r = 0; r < 8; ++r) af[r] = p3d_ds_read(base + ((8 * wm + r) * KG + g) * 1024 + lane * 16);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][8], fb[2][4];

#pragma unroll
  for (int s0 = 0; s0 < NST - 1; ++s0)
    if (s0 < nks) issue(s0, s0);
  {
    const int later = (nks - 1) < (NST - 2) ? (nks - 1) : (NST - 2);
    p3d_wait_stages6<PER, NST>(later);
    __builtin_amdgcn_s_barrier();
    read(0, 0, fa[0], fb[0]);
  }
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks % NST;
    if (ks + NST - 1 < nks) issue(ks + NST - 1, (ks + NST - 1) % NST);
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      // (KG even or odd: the register set alternates per k-group; static indices only)
      const int cur = g & 1, nxt = cur ^ 1;
      if (g + 1 < KG) {
        read(buf, g + 1, fa[nxt], fb[nxt]);
        p3d_wait_lgkm<12>();
      } else if (ks + 1 < nks) {
        const int later = (nks - 2 - ks) < (NST - 2) ? (nks - 2 - ks) : (NST - 2);
        p3d_wait_stages6<PER, NST>(later);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        read((ks + 1) % NST, 0, fa[nxt], fb[nxt]);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        p3d_wait_lgkm<0>();
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cur][r], fb[cur][c], acc[r][c], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (KG % 2 == 1) {
        // odd KG: the next k-step's group 0 was read into set nxt; move it to set 0
        if (g + 1 == KG) {
          p3d_wait_lgkm<0>();                       // (the asm reads of set 1 have landed)
#pragma unroll
          for (int r = 0; r < 8; ++r) fa[0][r] = fa[1][r];
#pragma unroll
          for (int c = 0; c < 4; ++c) fb[0][c] = fb[1][c];
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const __amdgpu_buffer_rsrc_t rp = p3d_bf16s_rsrc(sa.part);
  const int pbase = ((tile * 4 + w) * 32) * 1024 + lane * 16;   // byte offset of fragment 0
  if (!reader) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(p3d_u32x4, acc[r][c]), rp, pbase + (r * 4 + c) * 1024, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (w == 0) {
    const unsigned t0 = __builtin_amdgcn_readfirstlane(tag);
    bool ok = false;
    for (int spin = 0; spin < P3D_BF16S_SPIN; ++spin) {
      const unsigned v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == t0) { ok = true; break; }
      __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
      if (!ok) __hip_atomic_store(sa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = acc[r][c] + p3d_bf16s_ld(rp, pbase + (r * 4 + c) * 1024);
  float* et = (float*)smem;
  const int i = lane & 15, q = lane >> 4;
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) et[(128 * wm + 16 * r + 4 * q + e) * 132 + 64 * wn + 16 * c + i] = acc[r][c][e];
  __syncthreads();
  const int ngY = p.N / 32;
#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int item = it * 256 + tid;        // 64 chunks (16 row tiles x 4 col groups) x 64 lanes
    const int chunk = item >> 6, l = item & 63;
    const int rl = 16 * (chunk >> 2) + (l & 15);
    const int cl = 32 * (chunk & 3) + 8 * (l >> 4);
    const int row = 256 * mt + rl, col = 128 * nt + cl;
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

