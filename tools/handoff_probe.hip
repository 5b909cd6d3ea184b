// handoff_probe.hip -- what a layer boundary costs at batch 64 on MI355X, measured (VERDICT r5
// items 3 and 6: "measure the 64 KB cross-XCD hand-off on the box with a micro-kernel").
//
// Geometry of a batch-64 layer spread over the whole chip (the column split the verdict names, and
// the per-layer k_fwd launches): 256 workgroups of 256 threads, workgroup b owns output tile (row
// tile r = b / 64, column tile c = b % 64) of 16 x 16 floats (1 KB).  The next layer's tile (r, c')
// needs ALL 64 tiles of row tile r (64 KB) -- produced by 64 workgroups that the round-robin
// dispatcher spreads over all 8 XCDs (b % 8 = c % 8).  Each of a consumer's 4 waves takes 16 of the
// producers' tiles (its K quarter: 16 KB) into registers, as a contraction would.
//
//   chain   ONE launch of P phases: per phase each workgroup polls its 64 producers' flags (wave w its
//           16, relaxed agent-scope sc1 loads), loads the 64 KB with sc1 buffer loads, sums it, stores
//           its own tile (sc1 stores), drains (vmcnt 0), barrier, lane 0 publishes its flag.  Phase
//           times from s_memrealtime stamps (100 MHz) of every workgroup.
//   flags   the same chain without payload (flags only): the signalling floor.
//   launch  P dependent launches of one phase each (plain loads of the previous launch's tiles):
//           the kernel-boundary form, timed with events over the P launches.
//   empty   P dependent launches that load nothing: the boundary alone.
// Prints one JSON line of per-phase microseconds (medians over phases 2 .. P-1).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int NWG = 256, NC = 64, TILE = 256;   // floats per 16 x 16 tile

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ f32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, off, 0, 16);
}

// act: [2 banks][4 row tiles][64 column tiles][256]; flags: [NWG] phase counters (start at 0)
template <bool PAYLOAD>
__global__ __launch_bounds__(256) void k_chain(float* act, unsigned* flags, int P, unsigned long long* stamps,
                                               int* err) {
  const int b = blockIdx.x, r = b / NC, c = b % NC;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ f32x4 part[4][64];
  const __amdgpu_buffer_rsrc_t ra = rsrc(act);
  if (tid == 0) stamps[(size_t)b * (P + 1)] = __builtin_amdgcn_s_memrealtime();
  f32x4 v = {1.f, 1.f, 1.f, 1.f};
  for (int p = 0; p < P; ++p) {
    const int bank_in = (p + 1) & 1, bank_out = p & 1;
    if (p > 0) {
      // wave w waits for producers (r, 16 w + i), i = lane < 16
      const int pc = 16 * w + (lane & 15);
      long spins = 0;
      while (true) {
        const unsigned f = __hip_atomic_load(flags + r * NC + pc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all(f >= (unsigned)p)) break;
        if (++spins > 20000000) { if (lane == 0) err[0] = 1; break; }
      }
      asm volatile("" ::: "memory");
      if (PAYLOAD) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, t[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
          t[i] = ld_sc1(ra, (((bank_in * 4 + r) * NC + 16 * w + i) * TILE + 4 * lane) * 4);
#pragma unroll
        for (int i = 0; i < 16; ++i) s += t[i];
        v = s;
      }
    }
    part[w][lane] = v;
    __syncthreads();
    if (w == 0) {
      const f32x4 o = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
      if (PAYLOAD) st_sc1(ra, (((bank_out * 4 + r) * NC + c) * TILE + 4 * lane) * 4, o * 0.25f);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(flags + b, (unsigned)(p + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0) stamps[(size_t)b * (P + 1) + p + 1] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
  }
}

// one phase as its own launch: load the row's 64 KB the previous launch stored, store this tile
template <bool PAYLOAD>
__global__ __launch_bounds__(256) void k_step(float* act, int p) {
  const int b = blockIdx.x, r = b / NC, c = b % NC;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ f32x4 part[4][64];
  const int bank_in = (p + 1) & 1, bank_out = p & 1;
  f32x4 s = {1.f, 1.f, 1.f, 1.f};
  if (PAYLOAD) {
    const f32x4* a = (const f32x4*)act;
    f32x4 t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = a[(((bank_in * 4 + r) * NC + 16 * w + i) * TILE) / 4 + lane];
    s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) s += t[i];
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0) {
    const f32x4 o = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    if (PAYLOAD) ((f32x4*)act)[(((bank_out * 4 + r) * NC + c) * TILE) / 4 + lane] = o * 0.25f;
  }
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

template <bool PAYLOAD>
static int run_chain(float* act, unsigned* flags, unsigned long long* stamps, int* err, int P, double* out) {
  CHECK(hipMemset(flags, 0, NWG * sizeof(unsigned)));
  CHECK(hipMemset(err, 0, sizeof(int)));
  CHECK(hipDeviceSynchronize());
  k_chain<PAYLOAD><<<NWG, 256>>>(act, flags, P, stamps, err);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  int e = 0;
  CHECK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
  if (e) { fprintf(stderr, "chain: a wait timed out\n"); return 1; }
  std::vector<unsigned long long> h((size_t)NWG * (P + 1));
  CHECK(hipMemcpy(h.data(), stamps, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  // phase p's end on the chip = the latest workgroup's stamp; per-phase time = difference of ends
  std::vector<double> ph;
  unsigned long long prev = 0;
  for (int p = 0; p <= P; ++p) {
    unsigned long long mx = 0;
    for (int b = 0; b < NWG; ++b) mx = std::max(mx, h[(size_t)b * (P + 1) + p]);
    if (p >= 3 && p < P) ph.push_back((double)(mx - prev) / 100.0);   // 100 MHz -> us
    prev = mx;
  }
  *out = median(ph);
  return 0;
}

template <bool PAYLOAD>
static int run_launches(float* act, int P, double* out) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int p = 0; p < 20; ++p) k_step<PAYLOAD><<<NWG, 256>>>(act, p);
  CHECK(hipEventRecord(e0, 0));
  for (int p = 0; p < P; ++p) k_step<PAYLOAD><<<NWG, 256>>>(act, p);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  *out = 1000.0 * ms / P;
  return 0;
}

int main() {
  const int P = 200;
  float* act;
  unsigned* flags;
  unsigned long long* stamps;
  int* err;
  CHECK(hipMalloc(&act, 2 * 4 * NC * TILE * sizeof(float)));
  CHECK(hipMemset(act, 0, 2 * 4 * NC * TILE * sizeof(float)));
  CHECK(hipMalloc(&flags, NWG * sizeof(unsigned)));
  CHECK(hipMalloc(&stamps, (size_t)NWG * (P + 1) * sizeof(unsigned long long)));
  CHECK(hipMalloc(&err, sizeof(int)));
  std::vector<double> chain, flags_only, launch, empty;
  for (int rep = 0; rep < 5; ++rep) {
    double a, b2, c2, d;
    if (run_chain<true>(act, flags, stamps, err, P, &a)) return 1;
    if (run_chain<false>(act, flags, stamps, err, P, &b2)) return 1;
    if (run_launches<true>(act, P, &c2)) return 1;
    if (run_launches<false>(act, P, &d)) return 1;
    chain.push_back(a); flags_only.push_back(b2); launch.push_back(c2); empty.push_back(d);
  }
  printf("{\"probe\": \"batch-64 layer boundary, 256 WGs, 64 KB per consumer from 64 producers on 8 XCDs\", "
         "\"in_launch_handoff_us\": %.3f, \"in_launch_flags_only_us\": %.3f, \"launch_boundary_with_64KB_us\": %.3f, "
         "\"launch_boundary_empty_us\": %.3f, \"reps\": 5, \"phases\": %d}\n",
         median(chain), median(flags_only), median(launch), median(empty), P);
  return 0;
}
