// p3d_serve6.h -- k_serve6: the persistent XCD-local batch-64 evaluation sized for launches of
// a few dozen steps (the driver's `bench.py --steps 20`).
//
// k_serve5 (p3d_serve.h) is built for throughput over long launches: two 16-CU groups per XCD,
// each running its steps one after another.  With 20 steps per launch that leaves 4 of its 16
// groups running a second step while the other 12 idle: the launch costs two steps of latency
// (8 hidden phases, each ~20 us) for 1.25 steps of work.  The critical path of a launch of nb
// steps is (rounds of steps) x (phases) x (column tiles per CU + fixed cost per phase), so
// k_serve6 takes the groups-per-XCD S as a launch argument, chosen on the host for nb
// (p3d.hip, serve6_split): at nb = 20, S = 3 groups of 11/11/10 CUs run all 20 steps at once,
// each CU contracting <= 7 of a layer's 64 column tiles per phase -- 28 16x16 tiles of K = 1024
// on the critical path and 4 phases, instead of 32 tiles and 8 phases.
//
// One launch per call: the sync words alternate between two banks picked on the device (the
// launch's groups each read their epoch word, use bank epoch & 1, zero their flags of the other for
// the next launch; each group's rank-0 member advances the group's word at its end, when every
// member has provably read it),
// so a launch needs no memset in front and captured graphs replay correctly.  The epilogue
// constants come from a table k_serve_prep forms per parameter version.
//
// What differs from k_serve5 (everything else -- XCD-local groups (k_serve6: placed by the
// dispatcher's round-robin, checked against the hardware XCD id), flag hand-offs in
// the XCD's L2, sc1 reads of other CUs' data, 4-wave K-split contraction with a register ring,
// epilogue constants in LDS, steps pipelined when a group has several -- is the same design):
//   * work is dealt in 16-column tiles, not 32-column units: member r of a group of n owns the
//     contiguous tiles [T r / n, T (r+1) / n) (T = L / 16), i.e. floor or ceil of T / n, and
//     contracts them (all 4 row tiles) as one contraction of NCM tiles (a member with fewer
//     computes a copy of its last tile and stores nothing for it; one with more loops);
//   * the output layer is a phase of its own (round 5; it was fused into the last hidden epilogue
//     as one 64 x 48 partial per column tile, summed by a reduction: 15.7 MB of partials per
//     20-step launch and a full-group wait): its RT x NDT tiles are dealt over the members and
//     contracted like hidden tiles, K split over the 4 waves, slices summed in order -- the
//     association is fixed by the tile, independent of n and S, so every launch shape gives the
//     same bits.
#pragma once
#include "p3d_serve.h"

#ifndef P3D_S6_PIN_ARGS
#define P3D_S6_PIN_ARGS 1          // the prologue's kernel arguments fetched in one round (round 5)
#endif
#ifndef P3D_S6_COMBINE_BATCH
#define P3D_S6_COMBINE_BATCH 1     // the K-combine's LDS reads issued before the first add (round 5)
#endif
#ifndef P3D_S6_OUT_PRE
#define P3D_S6_OUT_PRE 1           // the output layer's first weight fragments requested before the last hand-off
#endif
#ifndef P3D_S6_LATE_EPOCH
#define P3D_S6_LATE_EPOCH 1        // the epoch read off the prologue's critical path (round 5)
#endif


// Timeline stamps for development (-DP3D_TRACE, tools/trace_serve6.py): for every group, its
// rank-0 member (row 0) and its first member with the most tiles (row 1), first step only:
// [0] start, [1] placement, [2] input layer, [3] first hand-off; per hidden phase ph at 8 ph:
// [0] begin, [1] contraction, [2] K-combine, [3] epilogue, [4] hand-off; at 8 (NH + 1): [0]
// the output reduction.  wall_clock64 (100 MHz).
#ifdef P3D_TRACE
#define P3D_S6_STAMP(row, k)                                                              \
  do {                                                                                    \
    if (tr6 && (row) && threadIdx.x == 0) {                                               \
      tr6[(k)] = wall_clock64();                                                          \
      tr6[64 + (k)] = __builtin_amdgcn_s_memtime();                                       \
    }                                                                                     \
  } while (0)
#else
#define P3D_S6_STAMP(row, k) do { } while (0)
#endif

// The epilogue-constant table of the serve launches, formed when the parameters changed (and
// inside every captured graph): bias, inv = gamma / sqrt(var + eps), shift = beta - mean * inv
// -- the arithmetic of every other path -- of every layer 0..2N and column, laid out per
// 16-column tile as k_serve6 keeps them in LDS, so its workgroups copy them with one round of
// loads instead of forming them (five dependent operand loads per element) in every launch.
__global__ __launch_bounds__(256) void k_serve_prep(ServeArgs p, float* ecg) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int L = p.L, nl = 2 * p.nblk + 1;
  if (i >= nl * L) return;
  const int l = i / L, col = i % L, t = col >> 4, j = col & 15;
  const ServeLayer& ly = p.ly[l];
  float inv = 1.f, shift = 0.f;
  if (p.bn) {
    inv = (1.0f / sqrtf(ly.mvar[col] + p.eps)) * ly.gamma[col];
    shift = ly.beta[col] - ly.mmean[col] * inv;
  }
  float* e = ecg + ((int64_t)l * (L >> 4) + t) * 48;
  e[j] = ly.bias[col]; e[16 + j] = inv; e[32 + j] = shift;
  if (col == 0)   // the layer's max-norm divisor max(||W||, 1) (1 without --max_norm)
    ecg[(int64_t)nl * (L >> 4) * 48 + l] = ly.wsq ? fmaxf(sqrtf(*ly.wsq), 1.0f) : 1.0f;
}

// owner of column tile t when T tiles are dealt contiguously over n members
__device__ __forceinline__ int p3d_tile_owner(int t, int n, int T) { return ((t + 1) * n - 1) / T; }

// RT: row tiles per unit.  Rows are independent in evaluation, so the rows of a launch need
// not go in batch-64 steps: a unit of 16 RT rows is what one group runs through all layers.
// RT = 4 is the batch-64 step; RT = 2 half a step (20 steps = 40 units = 5 groups per XCD);
// RT = 6 .. 16 with S = 1 gives each XCD ONE unit of all its rows and all 32 of its CUs, each
// CU 2 of a layer's 64 column tiles for every row tile (20 steps: 160 rows per XCD, RT = 10):
// no group idles, no CU holds more tiles than another, and each weight fragment is read by one
// CU per XCD and serves 10 row tiles (p3d.hip serve6_plan picks the form per launch).
// The epilogue / input-layer work of a chunk, RT x NCM 16 x 16 tiles, is dealt to the waves
// round-robin: unit u = w + 4 j is row tile u / NCM of column tile u % NCM (UMAX per wave).
//
// PAIR (round 5): each group runs TWO units of RT row tiles side by side, alternating their
// phases -- A's phase ph, B's phase ph, A's phase ph + 1, ... -- so the hand-off of one unit runs
// under the other's contraction instead of in front of the next: a member's next contraction
// reads the other unit's previous phase, published a whole contraction earlier.  Per block
// (one unit's phase): the contraction, whose last DEPTH k-groups refill the register ring with
// the next block's first ones (its producers' flags checked a round earlier); partial sums to
// LDS; K-combine, epilogue, stores; the next contraction at once, its ring full.  A block's
// stores are published from inside the next contraction, after its first DEPTH k-groups (a
// vmcnt wait that leaves that contraction's refills in flight), each wave on its own, the fourth
// to arrive (an LDS counter) posting the member's flag -- no barrier, no store round trip and no
// ring fill between contractions.
template <int DEPTH, int NDT, int NCM, int RT = 4, bool PAIR = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_serve6(ServeArgs p) {
  static_assert(RT >= 1 && RT <= 16, "row tiles per unit");
  static_assert(!PAIR || (NCM == 2 && DEPTH == 4), "the pair form: 2 column tiles per member, a 4-deep ring");
  constexpr int ROWS = 16 * RT;              // rows of one unit
  constexpr int UMAX = (RT * NCM + 3) / 4;   // 16 x 16 tiles a wave finishes per chunk
  constexpr int OCH = RT * NCM < 4 ? RT * NCM : 4;   // output tiles per round of the output phase
  // activation ring depth (the wide forms cannot hold both rings DEPTH deep: 4 x 11 fragments
  // spilled 77 registers at NCM = 7, RT = 4)
#ifndef P3D_S6_DA
  // (PAIR: every slot holds both operands -- the ring runs on across blocks)
  constexpr int DA = PAIR ? DEPTH : RT >= 6 ? (DEPTH >= 8 ? 4 : 2) : (NCM >= 7 && DEPTH > 2 ? 2 : DEPTH);
#else
  constexpr int DA = RT >= 6 ? P3D_S6_DA : (NCM >= 7 && DEPTH > 2 ? 2 : DEPTH);   // (development builds)
#endif
#ifndef P3D_S6_PD
  constexpr int PD = NCM <= 4 ? 2 : 1;       // ring slots prefetched off-contraction
#else
  constexpr int PD = P3D_S6_PD;
#endif
  static_assert(!PAIR || DA == DEPTH, "the pair form's ring runs on across blocks: every slot holds both operands");
  // [slice][rt][tile][lane] (PAIR: two of them, alternate blocks)
  __shared__ __attribute__((aligned(16))) f32x4 red[(PAIR ? 2 : 1) * 4 * RT * NCM * 64];
  // epilogue constants of the member's tiles (up to ECT of them), per layer 0..2N:
  // bias | inv | shift, and each layer's max-norm divisor.  Every epilogue reads them from
  // LDS: no global load on a branch of the epilogue, so the compiler's vmcnt waits there stay
  // exact (a load on a not-taken branch had made them wait for every load in flight).
  constexpr int ECT = NCM >= 7 ? NCM : 2 * NCM;
  __shared__ __attribute__((aligned(16))) float ec[(P3D_SERVE_MAXL - 1) * ECT * 48];
  __shared__ float ecm[P3D_SERVE_MAXL];
  __shared__ int sh[32];
  // wave-uniform values the compiler cannot prove uniform (the wave index, everything read
  // from LDS) go through readfirstlane: they end in scalar registers, and
  // buffer loads with a scalar offset need no per-lane waterfall loop
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
#if P3D_S6_PIN_ARGS
  // (round 5) every argument the prologue reads, fetched from the kernel-argument segment at once:
  // left to itself the compiler loaded them where they are used, several behind branches on earlier
  // ones -- a chain of six dependent scalar-load round trips to a segment the host wrote just before
  // the launch (cold in every cache), ~3 us before the first operand request
  asm volatile("" ::"s"(p.split), "s"(p.delay), "s"(p.delay_xcc), "s"(p.census_extra), "s"(p.max_groups),
               "s"(p.nb), "s"(p.L), "s"(p.K0), "s"(p.nblk), "s"(p.M), "s"(p.x), "s"(p.epoch), "s"(p.ecg),
               "s"(p.err), "s"(p.sync), "s"(p.act), "s"(p.ly[0].Wf), "s"(gridDim.x));
#endif
  const int L = p.L, ngL = L >> 4, T = ngL, ngK0 = p.K0 >> 4;
  const int q4 = 4 * (lane >> 4);
  const int S = min(max(p.split, 1), 8);   // (an out-of-range split is reported below, never divided by)
#ifdef P3D_TRACE
  const unsigned long long t_start = wall_clock64();
  unsigned long long* tr6 = nullptr;
#endif

  // ---- placement: XCD id, rank within the XCD ---------------------------------------------
  // The dispatcher deals a launch's workgroups to the 8 XCDs round-robin (consecutive
  // workgroups on consecutive XCDs, from a starting XCD that varies between launches): with
  // grid % 8 == 0 every XCD holds grid / 8 of them, workgroup b being member b / 8 of the XCD
  // its hardware XCC id names -- the placement needs no census.  A grid the host did not size
  // (grid % 8 != 0) or an S out of range sets the error word and fills the output with NaN; a
  // dispatch that broke the pattern leaves some member of a group missing, and a workgroup that
  // is not resident (CUs held by other work) is missing too: the group's bounded hand-off waits
  // (group_sync) find either, and report and poison instead of hanging.  (Round 2's census -- a
  // counter per XCD and a wait for every arrival -- cost ~3-4 us of memory-side round trips at
  // the start of every launch.)
  // The flag words come in two banks used by alternate launches, picked by the device epoch
  // word: this launch zeroes the other bank for the next one (stream order: the launch that
  // used it has completed), so a launch needs no memset in front of it.
  const int nxg = (int)(gridDim.x >> 3);
  unsigned xr;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xr));
  const int xcc = (int)(xr & 7u), rx = (int)(blockIdx.x >> 3);
  unsigned ep = 0;
  if (tid == 0) {
    // test hook (P3D_SERVE_TEST_DELAY): every workgroup of one XCD arrives ~delay x 3.4 us late
    if (p.delay > 0 && xcc == p.delay_xcc)
      for (int i = 0; i < p.delay; ++i) __builtin_amdgcn_s_sleep(127);
    const bool bad = (gridDim.x & 7u) != 0u || p.split < 1 || p.split > 8 || p.census_extra;
    sh[0] = (int)(((unsigned)xcc - blockIdx.x) & 7u);   // (trace: the launch's starting XCD)
    sh[2] = bad ? 1 : 0;
    sh[4] = 0;                               // some wave of this workgroup is broken (group_sync)
    // no epoch word to advance until the first group_sync names one: a workgroup whose group takes
    // no unit never reaches a group_sync, and its end reads this slot (P3D_S6_LATE_EPOCH; a first
    // build left it unset and such a workgroup advanced a word at a stale LDS offset)
    sh[5] = -1;
    sh[6] = 0;                               // PAIR: waves past their store drain (publish counter)
    if (bad) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const int nl_ec = 2 * p.nblk + 1, tot_ec = nl_ec * ECT * 48;
  constexpr int ECN = ((P3D_SERVE_MAXL - 1) * ECT * 48 + 255) / 256;
  // place of this workgroup for XCD counts cnt(x): member r of group gid (gi-th of ng groups
  // taking units), its tiles [t_lo, t_hi)
  auto place = [&](auto cnt, int xcc, int rx, int& r, int& n, int& gid, int& gi, int& ng) {
    const int half = rx % S;
    r = rx / S;
    n = (cnt(xcc) + S - 1 - half) / S;
    gid = xcc * S + half;
    // groups in order of decreasing size (h-major): with fewer units than groups the larger
    // groups -- fewer tiles per member -- take them
    ng = 0;
    gi = 0;
    for (int h = 0; h < S; ++h)
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const int c = (cnt(x) + S - 1 - h) / S;
        if (c > 0) { if (x == xcc && h == half) gi = ng; ++ng; }
      }
    if (p.max_groups > 0 && ng > p.max_groups) {
      ng = p.max_groups;
      if (gi >= ng) gi = p.nb;
    }
    if ((T + n - 1) / n > ECT) gi = -1;      // a placement the host did not size this form for
    // (PAIR: one contraction of 1..NCM tiles per member, and two ring rounds before the last DEPTH
    // k-groups -- a block posts the previous one after the first, checks the next one's producers
    // before the last)
    if (PAIR && ((T + n - 1) / n > NCM || n > T || (T >> 2) < 3 * DEPTH)) gi = -1;
  };
  // first-unit input-layer operands (this wave's tiles) and the epilogue-constant table rows
  f32x4 xa0[UMAX][4], wb0[UMAX][4];
  float vec[ECN], wq = 1.f;
  // Every request unconditional, from a clamped (always valid) address, the unused ones discarded
  // (round 5): behind per-request guards each request sat in a block of its own, and at this
  // kernel's scalar-register pressure the compiler re-fetched the argument words it needed (x, W0,
  // the table) from the argument segment in every block, each with a wait -- ~30 dependent scalar
  // round trips before the last operand request (the trace's 2.7 us from start to placement).
  auto prefetch = [&](int gi_, int tlo, int thi) {
    const int nck = max(min(NCM, thi - tlo), 1);
    // (PAIR: the input operands are requested by its prologue -- held from here they crowded the
    // registers, and the compiler spilled each fragment as it arrived, a serial wait per load)
#pragma unroll
    for (int j = 0; j < (PAIR ? 0 : UMAX); ++j) {
      const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
      int64_t rowc = (int64_t)gi_ * ROWS + 16 * rt + (lane & 15);
      rowc = rowc < p.M ? (rowc > 0 ? rowc : 0) : p.M - 1;
      const int t = min(max(tlo + (cc < nck ? cc : nck - 1), 0), T - 1);
#pragma unroll
      for (int g = 0; g < 2; ++g) {          // K0 <= 32 (the reference's 16 joints x 2): all of it
        const int gg = min(g, ngK0 - 1);   // (g >= ngK0: a copy of the last k-group, never used)
        xa0[j][g] = *(const f32x4*)(p.x + rowc * p.K0 + 16 * gg + q4);
        wb0[j][g] = *(const f32x4*)(p.ly[0].Wf + ((int64_t)(t * ngK0 + gg) * 64 + lane) * 4);
      }
      if (ngK0 > 2) {                        // (one uniform branch for K0 in (32, 64])
#pragma unroll
        for (int g = 2; g < 4; ++g) {
          const int gg = min(g, ngK0 - 1);
          xa0[j][g] = *(const f32x4*)(p.x + rowc * p.K0 + 16 * gg + q4);
          wb0[j][g] = *(const f32x4*)(p.ly[0].Wf + ((int64_t)(t * ngK0 + gg) * 64 + lane) * 4);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < ECN; ++k) {
      const int idx = tid + 256 * k, idc = idx < tot_ec ? idx : 0;
      const int l = idc / (ECT * 48), rem = idc % (ECT * 48), cs = rem / 48, j = rem % 48;
      const float e = p.ecg[((int64_t)l * T + min(tlo + cs, T - 1)) * 48 + j];
      vec[k] = idx < tot_ec ? e : 0.f;
    }
    const float e = p.ecg[(int64_t)nl_ec * T * 48 + (tid < nl_ec ? tid : 0)];
    wq = tid < nl_ec ? e : 1.f;
  };
  // (unconditional: placement under a guard made the compiler keep its results in a form that cost
  // the main loop 52 AGPRs of its allocation and ~20 us per launch; gid is only used to address
  // memory where the launch is placeable)
  int r, n, gid, gi, ng;
  const bool placeable = (gridDim.x & 7u) == 0u && p.split >= 1 && p.split <= 8;
  place([&](int) { return nxg; }, xcc, rx, r, n, gid, gi, ng);
  // The group's epoch word (one per group slot; bank = epoch & 1).  Every member reads it at its
  // start; the group's rank-0 member advances it at the END of its work, by which time every
  // member has read it: rank 0's four waves read the whole K of every hidden layer, i.e. waited
  // for a flag of every member of the group, which each posted after its read.  A late member --
  // or a whole group dispatched late -- reads the epoch its own group is on.  (Round 3 kept one
  // word for the launch, advanced by workgroup 0 at its end: a whole group dispatched after
  // workgroup 0 had finished -- an idle one at max_groups = 1 -- read the advanced epoch, ran on the
  // other bank and left its flags there for the next launch; one launch-wide arrival counter
  // instead cost 2-3 us per launch: 256 returning atomics on one word, serialised.)
#if P3D_S6_LATE_EPOCH
  // (round 5) the epoch is needed first at the input layer's hand-off: read behind the first
  // unit's operands, kept by thread 0 until the first group_sync parks it in LDS -- its memory
  // round trip (the word was last written by an atomic) overlaps the constants and the input
  // layer instead of holding a barrier in front of them
  prefetch(gi, (T * r) / n, (T * (r + 1)) / n);
  if (tid == 0 && placeable) ep = __hip_atomic_load(p.epoch + gid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  if (tid == 0 && placeable) ep = __hip_atomic_load(p.epoch + gid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the first unit's input-layer operands and the epilogue constants in flight with the epoch read
  prefetch(gi, (T * r) / n, (T * (r + 1)) / n);
  if (tid == 0) {
    sh[3] = (int)(ep & 1u);
    // the epoch word this workgroup advances at its end (-1: none), parked in LDS: kept in
    // registers across the whole launch it cost the main loop its register allocation (222 vs
    // 166 AGPRs, 134 vs 113 us per launch)
    sh[5] = (placeable && r == 0 && gi >= 0 && gi < p.nb) ? gid : -1;
  }
  __syncthreads();
#endif
#ifdef P3D_TRACE
  if (tid == 0 && blockIdx.x < 1024) {     // per workgroup: start, placement known, XCD | rank
    g_p3d_trace[16384 + blockIdx.x * 4 + 0] = t_start;
    g_p3d_trace[16384 + blockIdx.x * 4 + 1] = wall_clock64();
    g_p3d_trace[16384 + blockIdx.x * 4 + 2] = wall_clock64();
    g_p3d_trace[16384 + blockIdx.x * 4 + 3] = (unsigned long long)(xcc | (rx << 8) | (sh[0] << 16));
  }
#endif
  // the group's flags in the other bank, zeroed for the group's next launch (every member the same
  // 64 words; nothing of this launch uses that bank).  Invariant: at the start of a launch the bank
  // of a group slot's epoch holds zeros (an idle group posts nothing and does not advance).
  unsigned* flags = nullptr;                 // this launch's bank (bind_bank)
  auto bind_bank = [&]() {                   // after a barrier that published sh[3]
    const int bank = __builtin_amdgcn_readfirstlane(sh[3]);
    flags = p.sync + bank * P3D_SERVE_SYNC_WORDS + P3D_SERVE_FLAG0 + 64 * gid;
    if (placeable && tid < 64) p.sync[(bank ^ 1) * P3D_SERVE_SYNC_WORDS + P3D_SERVE_FLAG0 + 64 * gid + tid] = 0u;
  };
#if !P3D_S6_LATE_EPOCH
  bind_bank();
#endif
  const bool bad_launch = (gridDim.x & 7u) != 0u || p.split < 1 || p.split > 8 || p.census_extra;
  if (bad_launch) {
    // a placement this launch cannot use: no row of it is computed by this workgroup; it fills
    // a stripe of the output with NaN, so a caller who skips p3d_serve_check / p3d_error_flags
    // never reads a stale or unwritten row as a result (the error word is set)
    const float qnan = __builtin_nanf("");
    for (int64_t e = (int64_t)blockIdx.x * 256 + tid; e < p.M * p.ND; e += (int64_t)gridDim.x * 256) p.y[e] = qnan;
  } else {
  if (gi < 0) {                              // a placement the host did not size this form for:
    if (tid == 0) __hip_atomic_store(p.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    gi = p.nb;                               // the whole group reports instead of computing
  }
  const int64_t slab = (int64_t)ROWS * L;
  // slabs 0..2: the hidden layers' rotation; slab 3: the last hidden layer's output, the output
  // layer's input (the next step's input layer writes the slab of the rotation the last phase reads
  // nothing from, so the last phase's output needs a fourth)
  // (PAIR: unit B's four slabs follow unit A's)
  float* act = p.act + (int64_t)gid * (PAIR ? 8 : 4) * slab;
  const ServeLayer& li = p.ly[0];
  const ServeLayer& lo = p.ly[2 * p.nblk + 1];
  const bool wsq_any = li.wsq != nullptr;
  const int NH = 2 * p.nblk;
  unsigned nsync = 0;
  bool broken = false;
  const int gb = (ngL * w) >> 2, gcount = ngL >> 2;      // this wave's K slice (k-groups)
  const int t_lo = (T * r) / n, t_hi = (T * (r + 1)) / n; // this member's column tiles
#ifdef P3D_TRACE
  {
    const int ncmax = (T + n - 1) / n;
    const bool row1 = (t_hi - t_lo == ncmax) && (t_lo == 0 || (T * (r - 1)) / n + ncmax != t_lo);
    if (r == 0 || row1) tr6 = g_p3d_trace + (gid * 2 + (r == 0 ? 0 : 1)) * 128;
    if (tr6 && tid == 0) { tr6[0] = t_start; tr6[1] = wall_clock64(); }
  }
#endif

  bool trs = true;                           // stamping this step (the group's first)
  // input layer of the chunk at c0 for the unit at rbase: this wave's tiles (unit j: row tile
  // (w + 4 j) / NCM, column tile c0 + (w + 4 j) % NCM), both operands of each per k-group
  auto in_issue = [&](int64_t rbase, int c0, f32x4 (&xa)[UMAX][4], f32x4 (&wb)[UMAX][4]) {
    const int nck = min(NCM, t_hi - c0);
#pragma unroll
    for (int j = 0; j < UMAX; ++j) {
      const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
      int64_t rowc = rbase + 16 * rt + (lane & 15);
      rowc = rowc < p.M ? rowc : p.M - 1;
      const int t = c0 + (cc < nck ? cc : nck - 1);
#pragma unroll
      for (int g = 0; g < 2; ++g) {          // (as in prefetch)
        const int gg = min(g, ngK0 - 1);
        xa[j][g] = *(const f32x4*)(p.x + rowc * p.K0 + 16 * gg + q4);
        wb[j][g] = *(const f32x4*)(li.Wf + ((int64_t)(t * ngK0 + gg) * 64 + lane) * 4);
      }
      if (ngK0 > 2) {
#pragma unroll
        for (int g = 2; g < 4; ++g) {
          const int gg = min(g, ngK0 - 1);
          xa[j][g] = *(const f32x4*)(p.x + rowc * p.K0 + 16 * gg + q4);
          wb[j][g] = *(const f32x4*)(li.Wf + ((int64_t)(t * ngK0 + gg) * 64 + lane) * 4);
        }
      }
    }
  };
  {   // epilogue constants of this member's tiles -- bias, inv = gamma / sqrt(var + eps),
      // shift = beta - mean * inv (the arithmetic of every other path), each layer's max-norm
      // divisor -- copied from the table k_serve_prep forms once per parameter version
#pragma unroll
    for (int k = 0; k < ECN; ++k)
      if (tid + 256 * k < tot_ec) ec[tid + 256 * k] = vec[k];
    if (tid < nl_ec) ecm[tid] = wq;
    __syncthreads();
  }
  P3D_S6_STAMP(trs, 4);
  // epilogue of tile t (chunk position cc) of layer l: z = acc / maxnorm + b, relu(z * inv + shift)
  // acc already divided by the max-norm divisor (maxnorm_div, a uniform branch of its own:
  // a per-element select made every epilogue run the division sequence)
  auto epi_c = [&](const f32x4& b4, const f32x4& inv4, const f32x4& sh4, f32x4 acc) -> f32x4 {
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float z = acc[k] + b4[k];
      o[k] = fmaxf(p.bn ? z * inv4[k] + sh4[k] : z, 0.0f);
    }
    return o;
  };
  auto epi_t = [&](int l, int cs, f32x4 acc) -> f32x4 {   // cs = tile - t_lo < ECT
    const float* e = ec + (l * ECT + cs) * 48 + q4;
    return epi_c(*(const f32x4*)e, *(const f32x4*)(e + 16), *(const f32x4*)(e + 32), acc);
  };
  auto maxnorm_div = [&](int l, f32x4& acc) {
    const float mx = ecm[l];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = acc[k] / mx;
  };

  // Group barrier (as k_serve5): drain, publish this member's phase, then each wave waits for
  // the members that produced its K slice (tiles [gb, gb + gcount)) -- or all members (full)
  // A member whose wait ran out is `broken`: it publishes its phases with the poison bit, every
  // member that reads a poisoned flag becomes broken too, and broken members store NaN instead
  // of their output elements -- rows of a unit whose hand-offs failed never carry wrong values.
  auto group_sync = [&](bool full, bool wait = true) {   // (PAIR: posts without the wait too)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (broken) sh[4] = 1;
#if P3D_S6_LATE_EPOCH
    const bool first = flags == nullptr;
    if (first && tid == 0) {
      sh[3] = (int)(ep & 1u);
      // the epoch word this workgroup advances at its end (-1: none), parked in LDS: kept in
      // registers across the whole launch it cost the main loop its register allocation (222 vs
      // 166 AGPRs, 134 vs 113 us per launch)
      sh[5] = (placeable && r == 0 && gi >= 0 && gi < p.nb) ? gid : -1;
    }
    __syncthreads();
    if (first) bind_bank();
#else
    __syncthreads();
#endif
    broken = broken || sh[4] != 0;           // workgroup-wide from here (monotonic)
    ++nsync;
    if (tid == 0)
      __hip_atomic_store(flags + r, nsync | (broken ? 0x80000000u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int m0 = full ? 0 : p3d_tile_owner(gb, n, T);
    const int cnt = full ? n : p3d_tile_owner(gb + gcount - 1, n, T) - m0 + 1;
    if (wait && !broken) {
      int spin = 0;
      while (true) {
        const unsigned v = lane < cnt ? __hip_atomic_load(flags + m0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : nsync;
        if (__all((v & 0x7fffffffu) >= nsync)) {
          if (__any(v & 0x80000000u)) broken = true;
          break;
        }
        if (++spin > P3D_SERVE_SPIN) {
          broken = true;
          if (lane == 0) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    asm volatile("" ::: "memory");           // (the producers' data is read after the relaxed flag check)
  };

  // input layer (K0 = input_size <= 64) of the member's tiles for the rows of the step at
  // rbase, row tile w, into act buffer cbuf: the rows loaded once, then every tile's weight
  // fragments requested before the first MFMA (one round of load latency, not one per tile)
  // (round 5: the wave's tiles contracted side by side -- one block per k-group, the tiles' MFMA
  // chains interleaved instead of one tile's 8 dependent MFMAs after another's -- and their epilogue
  // constants requested before the first MFMA; every tile's sum in the same order: the same bits)
  auto in_compute = [&](int c0, const f32x4 (&xa)[UMAX][4], const f32x4 (&wb)[UMAX][4], float* dst) {
    const int nck = min(NCM, t_hi - c0);
    f32x4 acc[UMAX], ce[UMAX][3];
#pragma unroll
    for (int j = 0; j < UMAX; ++j) {
      acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int u = min(w + 4 * j, RT * NCM - 1), cc = u % NCM;
      const int t = c0 + (cc < nck ? cc : nck - 1);
      const float* e = ec + (0 * ECT + (t - t_lo)) * 48 + q4;
#pragma unroll
      for (int k = 0; k < 3; ++k) ce[j][k] = *(const f32x4*)(e + 16 * k);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (g < ngK0)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < UMAX; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[j][g][e], xa[j][g][e], acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < UMAX; ++j) {
      const int u = w + 4 * j, rt = u / NCM, cc = u % NCM;
      if (u >= RT * NCM || cc >= nck) continue;
      const int t = c0 + cc;
      if (wsq_any) maxnorm_div(0, acc[j]);
      const f32x4 y = epi_c(ce[j][0], ce[j][1], ce[j][2], acc[j]);
      *(f32x4*)(dst + ((int64_t)(rt * ngL + t) * 64 + lane) * 4) = y;
    }
  };
  auto in_layer = [&](int64_t rbase, float* dst, int cfrom) {
    for (int c0 = cfrom; c0 < t_hi; c0 += NCM) {
      f32x4 xa[UMAX][4], wb[UMAX][4];
      in_issue(rbase, c0, xa, wb);
      in_compute(c0, xa, wb, dst);
    }
  };

  const float qnan = __builtin_nanf("");
  // The output phase's first weight fragments (the member's first output tile, the first 2 OGH
  // k-groups of this wave's K slice): they depend on nothing of the step, so the last hidden phase
  // requests them after its epilogue stores, and their memory round trip runs under the hand-off
  // (whose drain waits for them with the stores) instead of after it.  Requested whether or not the
  // member has an output tile (a valid tile's address then): a fixed number of loads.
  constexpr int OGH = 8;
  f32x4 ow0[OGH], ow1[OGH];
  auto out_wpre = [&]() {
    const int oo = (((PAIR ? 2 : 1) * RT * NDT * r) / n) % NDT;
    const __amdgpu_buffer_rsrc_t r4 = p3d_rsrc(lo.Wf);
#pragma unroll
    for (int g = 0; g < OGH; ++g) {
      ow0[g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r4, ((oo * ngL + gb + min(g, gcount - 1)) * 64 + lane) * 16, 0, 0));
      ow1[g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r4, ((oo * ngL + gb + min(OGH + g, gcount - 1)) * 64 + lane) * 16, 0, 0));
    }
  };
  // The output layer of the step at orow0 (round 5: its own phase instead of per-tile partials
  // summed by a reduction): the unit's RT x NDT output tiles are dealt contiguously over the
  // members; each tile is contracted over K = L as every hidden tile is -- wave w the k-groups of
  // its K slice, one MFMA chain in k-group order (A = the last hidden layer's output fragment, B =
  // the W4 fragment), then the four slices summed in slice order -- so the association is fixed by
  // the tile and every launch form gives the same bits.  Reads slab 3 after the last phase's
  // hand-off (this wave's K-slice producers); nothing is written but y.
#ifdef P3D_TRACE   // output-phase detail, every workgroup (tools/trace_serve6.py): 21504 + 4 b + k
#define P3D_S6_OSTAMP(k)                                                                               \
  do {                                                                                                 \
    if (tid == 0 && blockIdx.x < 1024) g_p3d_trace[21504 + blockIdx.x * 4 + (k)] = wall_clock64();     \
  } while (0)
#else
#define P3D_S6_OSTAMP(k) do { } while (0)
#endif
  // (PAIR: both units' tiles, A's then B's, dealt over the members as one list)
  auto out_phase = [&](int64_t orow0, int64_t orow1) {
    constexpr int OT = RT * NDT, OTT = PAIR ? 2 * OT : OT;
    const int o_lo = (OTT * r) / n, o_hi = (OTT * (r + 1)) / n;
    P3D_S6_OSTAMP(0);
    const __amdgpu_buffer_rsrc_t ryA = p3d_rsrc(act + 3 * slab), r4 = p3d_rsrc(lo.Wf);
    const __amdgpu_buffer_rsrc_t ryB = p3d_rsrc(act + (PAIR ? 7 : 3) * slab);
    for (int c0 = o_lo; c0 < o_hi; c0 += OCH) {
      const int nt = min(OCH, o_hi - c0);
      // fused MSE (p3d_serve_mse): wave w's tile's targets requested before the contraction (they
      // may be in host memory: a PCIe round trip hidden under the tile's ~2 us of work)
      f32x4 tv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p.tgt && w < nt) {
        const bool tb = PAIR && c0 + w >= OT;
        tv = p3d_serve_load_tgt<NDT>(p, (tb ? c0 + w - OT : c0 + w) * 64 + lane, tb ? orow1 : orow0);
      }
      f32x4 oacc[OCH];
#pragma unroll
      for (int j = 0; j < OCH; ++j) oacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < OCH; ++j) {
        if (j >= nt) break;                    // (workgroup-uniform)
        const bool tb = PAIR && c0 + j >= OT;    // (workgroup-uniform)
        const int tile = tb ? c0 + j - OT : c0 + j, ort = tile / NDT, oo = tile % NDT;
        const __amdgpu_buffer_rsrc_t ry = tb ? ryB : ryA;
        // the K slice in halves of 8 k-groups, both halves' fragments requested before the first
        // MFMA (32 loads at L = 1024: the hidden rings are dead here; two 8-entry arrays stay in
        // registers where one 16-entry array went to scratch)
        constexpr int GH = OGH;
        auto ld_half = [&](int gs, f32x4 (&av)[GH], f32x4 (&wv)[GH], bool wpre) {
#pragma unroll
          for (int g = 0; g < GH; ++g) {
            const int gg = gb + min(gs + g, gcount - 1);
            av[g] = p3d_ld_sc1(ry, ((ort * ngL + gg) * 64 + lane) * 16);
            if (!wpre)
              wv[g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r4, ((oo * ngL + gg) * 64 + lane) * 16, 0, 0));
          }
        };
        auto mma_half = [&](int gs, const f32x4 (&av)[GH], const f32x4 (&wv)[GH]) {
#pragma unroll
          for (int g = 0; g < GH; ++g) {
            if (gs + g >= gcount) break;
#pragma unroll
            for (int e = 0; e < 4; ++e) oacc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g][e], wv[g][e], oacc[j], 0, 0, 0);
          }
        };
        for (int g0 = 0; g0 < gcount; g0 += 2 * GH) {
          f32x4 a0[GH], w0[GH], a1[GH], w1[GH];
          // the member's first tile: its first 2 GH weight fragments came with the last hand-off
          const bool wpre = P3D_S6_OUT_PRE && c0 == o_lo && j == 0 && g0 == 0;
          if (wpre) {
#pragma unroll
            for (int g = 0; g < GH; ++g) { w0[g] = ow0[g]; w1[g] = ow1[g]; }
          }
          ld_half(g0, a0, w0, wpre);
          ld_half(g0 + GH, a1, w1, wpre);
          mma_half(g0, a0, w0);
          mma_half(g0 + GH, a1, w1);
        }
      }
#pragma unroll
      for (int j = 0; j < OCH; ++j)
        if (j < nt) red[(w * OCH + j) * 64 + lane] = oacc[j];   // (only the round's live tiles)
      if (c0 == o_lo) P3D_S6_OSTAMP(1);
      __syncthreads();
      if (w < nt) {                            // wave j sums tile j's four slices in slice order
        f32x4 sl[4];                           // (all four requested before the first add)
#pragma unroll
        for (int k = 0; k < 4; ++k) sl[k] = red[(k * OCH + w) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        f32x4 tot = sl[0];
#pragma unroll
        for (int k = 1; k < 4; ++k) tot += sl[k];
        if (broken) tot = f32x4{qnan, qnan, qnan, qnan};
        const bool tb = PAIR && c0 + w >= OT;
        const int tile = tb ? c0 + w - OT : c0 + w;
        const int64_t orow = tb ? orow1 : orow0;
        const float se = p3d_serve_store_out<NDT>(p, lo, tot, tile * 64 + lane, orow, tv);
        if (p.tgt)                             // fused MSE (p3d_serve_mse): this tile's share
          p3d_serve_loss_tile<!PAIR>(p, se, (orow >> 4) * NDT + tile, ((p.M + 15) >> 4) * NDT);
      }
      if (c0 == o_lo) P3D_S6_OSTAMP(2);
      __syncthreads();                         // red is rewritten next (next round / phase)
    }
  };

  f32x4 rbp[PD][NCM];                        // the next ring's first weight fragments
  auto b_prefetch = [&](int layer, int c0) {   // c0 < t_hi
    const int nck = min(NCM, t_hi - c0);
#pragma unroll
    for (int cc = 0; cc < NCM; ++cc) {
      const int t = c0 + (cc < nck ? cc : nck - 1);
      const f32x4* pbn = (const f32x4*)p.ly[layer].Wf + ((int64_t)t * ngL + gb) * 64 + lane;
#pragma unroll
      for (int d = 0; d < PD; ++d) rbp[d][cc] = pbn[d * 64];
    }
  };

  if constexpr (!PAIR) {
  int c0b = 0;
  if (gi < p.nb) {                           // the group's first step: its input layer alone
    if (t_lo < t_hi) in_compute(t_lo, xa0, wb0, act);
    P3D_S6_STAMP(trs, 5);
    in_layer((int64_t)gi * ROWS, act, t_lo + NCM);
    P3D_S6_STAMP(trs, 2);
    if (t_lo < t_hi) b_prefetch(1, t_lo);
    group_sync(false);
    P3D_S6_STAMP(trs, 3);
  }
  for (int b = gi; b < p.nb; b += ng) {
    const int64_t row0 = (int64_t)b * ROWS;
    const bool has_next = b + ng < p.nb;
    const int c0n = (c0b + 2 * p.nblk) % 3;  // buffer the next step's input layer writes
    int cur = c0b;
    for (int ph = 1; ph <= NH; ++ph) {
      P3D_S6_STAMP(trs, 8 * ph);
      const bool lastp = (ph == NH);
      const ServeLayer& ly = p.ly[ph];
      const bool second = ((ph - 1) & 1) == 1;
      const int t1 = (cur + 1) % 3, t2 = (cur + 2) % 3;
      const float* A = act + (second ? t1 : cur) * slab;
      float* Y = act + (lastp ? 3 : (second ? t2 : t1)) * slab;
      const float* res = (second && p.residual) ? act + cur * slab : nullptr;
      const __amdgpu_buffer_rsrc_t ra = p3d_rsrc(A);
      const int aoff0 = (gb * 64 + lane) * 16, rstride = ngL * 1024;
      for (int c0 = t_lo; c0 < t_hi; c0 += NCM) {
        const bool first_c = (c0 == t_lo);
        const int nck = min(NCM, t_hi - c0);
        // weight fragments through a buffer resource: one lane offset, tile / k-group offsets
        // scalar (tile cc's fragments at (c0 + cc) ngL + gb + g; a copy of the last past nck)
        const __amdgpu_buffer_rsrc_t rw = p3d_rsrc(ly.Wf);
        const int voff = lane * 16;
        int toff[NCM];
#pragma unroll
        for (int cc = 0; cc < NCM; ++cc) toff[cc] = ((c0 + (cc < nck ? cc : nck - 1)) * ngL + gb) * 1024;
        auto ldb = [&](int cc, int g) -> f32x4 {
          return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, voff, toff[cc] + g * 1024, 0));
        };
        // register ring: weight fragments DEPTH k-groups ahead, activations DA ahead (the
        // weights stream from MALL/HBM, the activations are L2 hits; the wide forms cannot hold
        // both DEPTH deep: 4 x 11 fragments spilled 77 registers at NCM = 7)
        f32x4 ra_[DA][RT], rb_[DEPTH][NCM];
        // the first PD weight slots were requested off the previous contraction (b_prefetch
        // runs before every contraction); a compile-time split keeps the number of loads in
        // flight static, so the compiler's vmcnt waits stay exact
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
          if (d < DA)
#pragma unroll
            for (int t = 0; t < RT; ++t) ra_[d % DA][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + d * 1024);
#pragma unroll
          for (int cc = 0; cc < NCM; ++cc) rb_[d][cc] = d < PD ? rbp[d < PD ? d : 0][cc] : ldb(cc, d);
        }
#ifdef P3D_TRACE   // (trace builds: the ring's first operands in hand -- the phase-start bubble)
        if (trs && first_c) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          P3D_S6_STAMP(true, 8 * ph + 7);
        }
#endif
        f32x4 acc[NCM][RT];
#pragma unroll
        for (int cc = 0; cc < NCM; ++cc)
#pragma unroll
          for (int t = 0; t < RT; ++t) acc[cc][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        auto mfmas = [&](int d) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int cc = 0; cc < NCM; ++cc)
#pragma unroll
              for (int t = 0; t < RT; ++t)
                acc[cc][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(rb_[d][cc][e], ra_[d % DA][t][e], acc[cc][t], 0, 0, 0);
        };
        for (int g0 = 0; g0 < gcount - DEPTH; g0 += DEPTH) {
#pragma unroll
          for (int d = 0; d < DEPTH; ++d) {
            mfmas(d);
            const int ga = g0 + d + DA, gn = g0 + DEPTH + d;
#pragma unroll
            for (int t = 0; t < RT; ++t) ra_[d % DA][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + ga * 1024);
#pragma unroll
            for (int cc = 0; cc < NCM; ++cc) rb_[d][cc] = ldb(cc, gn);
            __builtin_amdgcn_sched_barrier(0);   // refill of slot d stays ahead of slot d+1's MFMAs
          }
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {        // the last DEPTH k-groups
          mfmas(d);
          if (d + DA < DEPTH) {
            const int ga = gcount - DEPTH + d + DA;
#pragma unroll
            for (int t = 0; t < RT; ++t) ra_[d % DA][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + ga * 1024);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        // ---- off-contraction loads, their latency under the combine and epilogue ----------
        __builtin_amdgcn_sched_barrier(0);
        P3D_S6_STAMP(trs && first_c, 8 * ph + 1);
        // the epilogue's operands first (vmcnt waits are in order: the epilogue then waits for
        // them only, not for the next ring's weights behind them)
        // requested unconditionally (the residual operands from A where there is no residual):
        // conditional loads would make the compiler's vmcnt waits conservative, i.e. wait for the
        // next ring's weights behind them as well
        f32x4 rv[UMAX];
        const __amdgpu_buffer_rsrc_t rr = p3d_rsrc(res ? res : A);
#pragma unroll
        for (int j = 0; j < UMAX; ++j) {
          const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
          const int t = c0 + (cc < nck ? cc : nck - 1);
          rv[j] = p3d_ld_sc1(rr, (int)(((int64_t)(rt * ngL + t) * 64 + lane) * 16));
        }
        // the next contraction's first weight slots: this member's next chunk, the next
        // layer, or the next step's first layer (requested even after a group's last step:
        // a fixed number of loads keeps the vmcnt waits exact)
        {
          const bool more = c0 + NCM < t_hi;
          b_prefetch(more ? ph : (!lastp ? ph + 1 : 1), more ? c0 + NCM : t_lo);
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- K-slice combine (LDS), epilogue ----------------------------------------------
#pragma unroll
        for (int cc = 0; cc < NCM; ++cc)
#pragma unroll
          for (int t = 0; t < RT; ++t) red[((w * RT + t) * NCM + cc) * 64 + lane] = acc[cc][t];
        __syncthreads();
        P3D_S6_STAMP(trs && first_c, 8 * ph + 2);
        f32x4 sacc[UMAX];                      // K slices summed in slice order, this wave's tiles
#if P3D_S6_COMBINE_BATCH
        {
          // (round 5) every slice of every tile of the wave, and the tiles' epilogue constants,
          // requested before the first add: left to itself the scheduler interleaved each read with
          // the adds that consume it -- 15 dependent LDS round trips per phase (0.9 us in the trace)
          f32x4 part[UMAX][4], ce[UMAX][3];
#pragma unroll
          for (int j = 0; j < UMAX; ++j) {
            const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
#pragma unroll
            for (int k = 0; k < 4; ++k) part[j][k] = red[((k * RT + rt) * NCM + cc) * 64 + lane];
            const int t = c0 + (cc < nck ? cc : nck - 1);
            const float* e = ec + (ph * ECT + (t - t_lo)) * 48 + q4;
#pragma unroll
            for (int k = 0; k < 3; ++k) ce[j][k] = *(const f32x4*)(e + 16 * k);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < UMAX; ++j) {
            sacc[j] = part[j][0];              // slice 0, tile (rt, cc), then 1, 2, 3
#pragma unroll
            for (int k = 1; k < 4; ++k) sacc[j] += part[j][k];
          }
          P3D_S6_STAMP(trs && first_c, 8 * ph + 5);
          if (wsq_any)
#pragma unroll
            for (int j = 0; j < UMAX; ++j) maxnorm_div(ph, sacc[j]);
#pragma unroll
          for (int j = 0; j < UMAX; ++j) {
            const int u = w + 4 * j, rt = u / NCM, cc = u % NCM;
            if (u >= RT * NCM || cc >= nck) continue;
            const int t = c0 + cc;
            f32x4 yv = epi_c(ce[j][0], ce[j][1], ce[j][2], sacc[j]);
            if (res) yv += rv[j];
            *(f32x4*)(Y + ((int64_t)(rt * ngL + t) * 64 + lane) * 4) = yv;
          }
        }
#else
#pragma unroll
        for (int j = 0; j < UMAX; ++j) {
          const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
          sacc[j] = red[((0 * RT + rt) * NCM + cc) * 64 + lane];   // slice 0, tile (rt, cc)
#pragma unroll
          for (int k = 1; k < 4; ++k) sacc[j] += red[((k * RT + rt) * NCM + cc) * 64 + lane];
        }
        P3D_S6_STAMP(trs && first_c, 8 * ph + 5);
        if (wsq_any)
#pragma unroll
          for (int j = 0; j < UMAX; ++j) maxnorm_div(ph, sacc[j]);
#pragma unroll
        for (int j = 0; j < UMAX; ++j) {
          const int u = w + 4 * j, rt = u / NCM, cc = u % NCM;
          if (u >= RT * NCM || cc >= nck) continue;
          const int t = c0 + cc;
          f32x4 yv = epi_t(ph, t - t_lo, sacc[j]);
          if (res) yv += rv[j];
          *(f32x4*)(Y + ((int64_t)(rt * ngL + t) * 64 + lane) * 4) = yv;
        }
#endif
        P3D_S6_STAMP(trs && first_c, 8 * ph + 6);
        // red / rsum are rewritten by this member's next contraction of the phase
        if (c0 + NCM < t_hi) __syncthreads();
      }
      // the next step's input layer (it depends on nothing of this step) in the last phase
      if (lastp && has_next) in_layer(row0 + (int64_t)ng * ROWS, act + c0n * slab, t_lo);
      if (P3D_S6_OUT_PRE && lastp) out_wpre();
      if (lastp) P3D_S6_OSTAMP(3);
      P3D_S6_STAMP(trs, 8 * ph + 3);
      if (second) cur = t2;
      // every phase's hand-off: each wave waits for the members whose output its K slice reads
      // (after the last phase: the output layer's input, slab 3, and the next step's input layer)
      group_sync(false);
      P3D_S6_STAMP(trs, 8 * ph + 4);
    }
    out_phase(row0, 0);                      // this step's output layer
#ifdef P3D_TRACE
    if (trs && tr6 && tid == 0) tr6[8 * (NH + 1)] = wall_clock64();
    if (tid == 0 && blockIdx.x < 1024) g_p3d_trace[20480 + blockIdx.x] = wall_clock64();   // every member's end
#endif
    trs = false;
    c0b = c0n;
  }
  } else {
  // ---- PAIR: units b (A, slabs 0..3) and b + ng (B, slabs 4..7), phases alternating --------
  // (a unit past the last row -- an odd count of units -- runs on clamped rows and stores nothing)
  const int m0 = p3d_tile_owner(gb, n, T);
  const int cntw = p3d_tile_owner(gb + gcount - 1, n, T) - m0 + 1;
  // group_sync's wait on its own: this wave's K-slice producers have posted `target`
  auto wait_for = [&](unsigned target) {
    if (broken) return;
    int spin = 0;
    while (true) {
      const unsigned v = lane < cntw ? __hip_atomic_load(flags + m0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : target;
      if (__all((v & 0x7fffffffu) >= target)) {
        if (__any(v & 0x80000000u)) broken = true;
        break;
      }
      if (++spin > P3D_SERVE_SPIN) {
        broken = true;
        if (lane == 0) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    asm volatile("" ::: "memory");           // (as in group_sync)
  };
  // this wave's share of a member's post, after its stores are acknowledged (the caller's vmcnt
  // wait): the fourth wave to count posts the member's flag
  auto post_wave = [&]() {
    ++nsync;
    if (lane == 0) {
      const int old = __hip_atomic_fetch_add(&sh[6], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((old & 3) == 3)
        __hip_atomic_store(flags + r, nsync | (broken ? 0x80000000u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };
  // block s: unit s & 1, hidden phase s / 2 + 1; its operand / output / residual slabs
  auto slabs = [&](int s, const float*& A, float*& Y, const float*& res) {
    const int ph = (s >> 1) + 1, cur = (2 * ((ph - 1) >> 1)) % 3, t1 = (cur + 1) % 3, t2 = (cur + 2) % 3;
    const bool second = ((ph - 1) & 1) == 1;
    float* base = act + (s & 1) * 4 * slab;
    A = base + (second ? t1 : cur) * slab;
    Y = base + (ph == NH ? 3 : (second ? t2 : t1)) * slab;
    res = (second && p.residual) ? base + cur * slab : nullptr;
  };
  const int nck = max(min(NCM, t_hi - t_lo), 1);
  const int aoff0 = (gb * 64 + lane) * 16, rstride = ngL * 1024, voff = lane * 16;
  int toff[NCM];
#pragma unroll
  for (int cc = 0; cc < NCM; ++cc) toff[cc] = ((t_lo + (cc < nck ? cc : nck - 1)) * ngL + gb) * 1024;
  f32x4 ra_[DA][RT], rb_[DEPTH][NCM];        // the register ring, loaded for the next block ahead
  auto ring_load = [&](int layer, const float* A) {
    const __amdgpu_buffer_rsrc_t ra = p3d_rsrc(A), rw = p3d_rsrc(p.ly[layer].Wf);
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (d < DA)
#pragma unroll
        for (int t = 0; t < RT; ++t) ra_[d][t] = p3d_ld_sc1(ra, aoff0 + t * rstride + d * 1024);
#pragma unroll
      for (int cc = 0; cc < NCM; ++cc)
        rb_[d][cc] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, voff, toff[cc] + d * 1024, 0));
      // slot order kept: the first MFMAs wait for slot 0 only (the scheduler had issued a slot-0
      // fragment last, and the contraction then waited for every request in flight)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // Every memory request of a block is unconditional (the last block requests a ring it does not
  // use, every wave stores all its epilogue tiles -- a clamped duplicate where it has fewer, the
  // same bits), and the previous block's post sits in a peeled first ring round: requests on
  // branches left the compiler's vmcnt accounting at a merge it resolved with full drains (the
  // first build waited for everything in flight before every contraction and every store).
  for (int b = gi; b < p.nb; b += 2 * ng) {
    const int64_t rowA = (int64_t)b * ROWS, rowB = (int64_t)(b + ng) * ROWS;
    // input layers: both units' operands requested at once; A's computed and posted (the first post
    // binds the bank), then B's computed while A's producers' posts arrive -- B's input layer is
    // posted by block 0's in-contraction post (its stores precede block 0's ring requests, so that
    // post's counted wait finds them acknowledged), which block 1 (B's first hidden phase) waits for.
    // (Round 5 computed both and posted them together: B's input layer sat on the path to the first
    // contraction.)
    {
      f32x4 xa[UMAX][4], wa[UMAX][4], xb[UMAX][4], wbb[UMAX][4];
      in_issue(rowA, t_lo, xa, wa);
      in_issue(rowB, t_lo, xb, wbb);
      in_compute(t_lo, xa, wa, act);
      P3D_S6_STAMP(trs, 5);
      group_sync(false, false);
      in_compute(t_lo, xb, wbb, act + 4 * slab);
      P3D_S6_STAMP(trs, 2);
    }
    wait_for(nsync);                         // A's input layer from this wave's K-slice producers
    P3D_S6_STAMP(trs, 3);
    {
      const float *A0, *r0;
      float* Y0;
      slabs(0, A0, Y0, r0);
      ring_load(1, A0);
    }
    // The epilogue of block sp: its K slices (red buffer sp & 1) and its tiles' constants requested
    // (epi_rd), then summed in slice order, finished with the residual operands rv and stored (epi_st)
    f32x4 part[UMAX][4], ce[UMAX][3], rv[UMAX];
    auto epi_rd = [&](int sp) {
      const int php = (sp >> 1) + 1;
      const f32x4* rdp = red + (sp & 1) * (4 * RT * NCM * 64);
#pragma unroll
      for (int j = 0; j < UMAX; ++j) {
        const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
#pragma unroll
        for (int k = 0; k < 4; ++k) part[j][k] = rdp[((k * RT + rt) * NCM + cc) * 64 + lane];
        const int t = t_lo + (cc < nck ? cc : nck - 1);
        const float* e = ec + (php * ECT + (t - t_lo)) * 48 + q4;
#pragma unroll
        for (int k = 0; k < 3; ++k) ce[j][k] = *(const f32x4*)(e + 16 * k);
      }
    };
    auto epi_st = [&](int sp) {
      const int php = (sp >> 1) + 1;
      const float *Ap, *resp;
      float* Yp;
      slabs(sp, Ap, Yp, resp);
      f32x4 sacc[UMAX];
#pragma unroll
      for (int j = 0; j < UMAX; ++j) {
        sacc[j] = part[j][0];                // slice 0, tile (rt, cc), then 1, 2, 3
#pragma unroll
        for (int k = 1; k < 4; ++k) sacc[j] += part[j][k];
      }
      if (wsq_any)
#pragma unroll
        for (int j = 0; j < UMAX; ++j) maxnorm_div(php, sacc[j]);
#pragma unroll
      for (int j = 0; j < UMAX; ++j) {
        // (a wave with fewer tiles, or a member with fewer than NCM, stores a clamped duplicate:
        // the same tile's sum from the same LDS slices and constants, i.e. the same bits)
        const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
        const int t = t_lo + (cc < nck ? cc : nck - 1);
        f32x4 yv = epi_c(ce[j][0], ce[j][1], ce[j][2], sacc[j]);
        if (resp) yv += rv[j];
        *(f32x4*)(Yp + ((int64_t)(rt * ngL + t) * 64 + lane) * 4) = yv;
      }
    };
    // Block s.  The register ring runs on across blocks: the last DEPTH k-groups refill their slots
    // with the NEXT block's first DEPTH k-groups (the other unit's previous phase, posted about a
    // contraction ago, its producers' flags checked one round earlier), so a block starts with its
    // ring full and the boundary between contractions is the K-combine and epilogue alone.  (A first
    // form requested the next ring after the contraction: 28 requests per wave in a burst, the
    // CU's address path busy ~1 us between contractions.)
    for (int s = 0; s < 2 * NH; ++s) {
      const int ph = (s >> 1) + 1;
      const ServeLayer& ly = p.ly[ph];
      const float *A, *res;
      float* Y;
      slabs(s, A, Y, res);
      const __amdgpu_buffer_rsrc_t ra = p3d_rsrc(A), rw = p3d_rsrc(ly.Wf);
      P3D_S6_STAMP(trs, 8 + 4 * s);
      f32x4 acc[NCM][RT];
#pragma unroll
      for (int cc = 0; cc < NCM; ++cc)
#pragma unroll
        for (int t = 0; t < RT; ++t) acc[cc][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto mfmas = [&](int d) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int cc = 0; cc < NCM; ++cc)
#pragma unroll
            for (int t = 0; t < RT; ++t)
              acc[cc][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(rb_[d][cc][e], ra_[d][t][e], acc[cc][t], 0, 0, 0);
      };
      // slot d refilled with k-group g of the operands (ra2, rw2): exactly kSlotLoads vector loads
      // (the post's counted wait below depends on that number)
      constexpr int kSlotLoads = RT + NCM;
      auto refill = [&](int d, const __amdgpu_buffer_rsrc_t& ra2, const __amdgpu_buffer_rsrc_t& rw2, int g) {
        static_assert(kSlotLoads == RT + NCM, "one load per row tile and one per column tile");
#pragma unroll
        for (int t = 0; t < RT; ++t) ra_[d][t] = p3d_ld_sc1(ra2, aoff0 + t * rstride + g * 1024);
#pragma unroll
        for (int cc = 0; cc < NCM; ++cc)
          rb_[d][cc] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw2, voff, toff[cc] + g * 1024, 0));
      };
      auto round = [&](int g0) {             // DEPTH k-groups, each slot refilled DEPTH ahead
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
          mfmas(d);
          refill(d, ra, rw, g0 + DEPTH + d);
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      round(0);
      // the previous block's post (block 0: nothing new -- one post per block): its stores were issued
      // before this round's DEPTH (RT + NCM) refills, so a wait down to that many leaves the refills in
      // flight (vmcnt retires in issue order) and finds the stores acknowledged.  This holds only while
      // at least that many vector-memory operations follow the stores in the code the compiler emits:
      // the "s_nop 5" marks the wait so that tests/test_kernel_resources.py can count them in the
      // built ISA -- fewer would let the flag overtake the stores
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_nop 5" ::"n"(DEPTH * kSlotLoads) : "memory");
      post_wave();
      __builtin_amdgcn_sched_barrier(0);
      for (int g0 = DEPTH; g0 < gcount - 2 * DEPTH; g0 += DEPTH) round(g0);
      // the next block's producers (the other unit's previous phase; the last block: its own unit's,
      // there too): flags requested a round ahead of the check
      const unsigned fl = __hip_atomic_load(flags + m0 + min(lane, cntw - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_sched_barrier(0);
      round(gcount - 2 * DEPTH);
      if (!broken) {
        if (__any(fl & 0x80000000u)) broken = true;
        else if (!__all((fl & 0x7fffffffu) >= nsync)) wait_for(nsync);
      }
      // (the flags are relaxed atomics: nothing in the memory model keeps the compiler from hoisting
      // the next block's operand loads above the check -- this does; the hardware issues them after
      // the flag values are in hand)
      asm volatile("" ::: "memory");
      // this block's residual operands, then the last DEPTH k-groups, each slot refilled with the
      // next block's (the last block: its own again, unused)
      const __amdgpu_buffer_rsrc_t rr = p3d_rsrc(res ? res : A);
#pragma unroll
      for (int j = 0; j < UMAX; ++j) {
        const int u = min(w + 4 * j, RT * NCM - 1), rt = u / NCM, cc = u % NCM;
        const int t = t_lo + (cc < nck ? cc : nck - 1);
        rv[j] = p3d_ld_sc1(rr, (int)(((int64_t)(rt * ngL + t) * 64 + lane) * 16));
      }
      {
        const int sn = min(s + 1, 2 * NH - 1);
        const float *An, *rn;
        float* Yn;
        slabs(sn, An, Yn, rn);
        const __amdgpu_buffer_rsrc_t ran = p3d_rsrc(An), rwn = p3d_rsrc(p.ly[(sn >> 1) + 1].Wf);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
          mfmas(d);
          refill(d, ran, rwn, d);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      P3D_S6_STAMP(trs, 8 + 4 * s + 1);
      f32x4* rd = red + (s & 1) * (4 * RT * NCM * 64);
#pragma unroll
      for (int cc = 0; cc < NCM; ++cc)
#pragma unroll
        for (int t = 0; t < RT; ++t) rd[((w * RT + t) * NCM + cc) * 64 + lane] = acc[cc][t];
      if (broken) sh[4] = 1;
      __syncthreads();
      broken = broken || sh[4] != 0;
      P3D_S6_STAMP(trs, 8 + 4 * s + 2);
      epi_rd(s);
      __builtin_amdgcn_sched_barrier(0);
      epi_st(s);
      P3D_S6_STAMP(trs, 8 + 4 * s + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    post_wave();                             // the last block's, at once
    if (P3D_S6_OUT_PRE) out_wpre();
    wait_for(nsync);                         // both units' last hidden layers (slabs 3, 7)
    out_phase(rowA, rowB);
#ifdef P3D_TRACE
    if (trs && tr6 && tid == 0) tr6[8 * (NH + 1)] = wall_clock64();
    if (tid == 0 && blockIdx.x < 1024) g_p3d_trace[20480 + blockIdx.x] = wall_clock64();   // every member's end
#endif
    trs = false;
  }
  }
  if (tid == 0 && sh[5] >= 0)   // (every member has read the epoch by now: see its read)
    __hip_atomic_fetch_add(p.epoch + sh[5], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
