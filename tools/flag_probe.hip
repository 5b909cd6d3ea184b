// flag_probe.hip -- how soon the host can use a kernel's result written straight into pinned host
// memory (round 6, VERDICT r5 item 7: the drop-in API's per-call host share).
//
// A kernel of G workgroups (1 or 256); each writes 1 KB of output rows into pinned host memory
// (hipHostMalloc default flags, as torch's pin_memory), makes them system-visible (release fence
// at system scope), and counts itself in on a device word; the last arriver resets the counter and
// stores the call's sequence number into a pinned, coherent flag word (system-scope release).
//   sync         launch + hipStreamSynchronize (the runtime's completion path)
//   flag         launch + a host spin on the flag word, then (untimed) hipStreamSynchronize
//   flag_chain   launch + spin, back to back with no stream synchronize between calls
// Each case checks that every output row holds the call's values once the host has seen the flag.
// Prints one JSON line of medians (us) over 400 calls after 100 warm-up calls.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_rows(float* hout, unsigned* cnt, unsigned* flag, unsigned seq, int fence) {
  hout[(size_t)blockIdx.x * 256 + threadIdx.x] = (float)(seq + threadIdx.x);
  if (fence) __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float* hout;
  unsigned *flag, *cnt;
  CHECK(hipHostMalloc((void**)&hout, 256 * 256 * sizeof(float), hipHostMallocDefault));
  CHECK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent));
  CHECK(hipMalloc((void**)&cnt, 64));
  CHECK(hipMemset(cnt, 0, 64));
  *(volatile unsigned*)flag = 0;
  unsigned seq = 0;
  int bad = 0;
  printf("{");
  const char* sep = "";
  for (int G : {1, 256}) {
    for (int mode = 0; mode < 3; ++mode) {
      std::vector<double> ts;
      for (int it = 0; it < 500; ++it) {
        ++seq;
        const double t0 = now_us();
        hipLaunchKernelGGL(k_rows, dim3(G), dim3(256), 0, st, hout, cnt, flag, seq, 1);
        if (mode == 0) {
          CHECK(hipStreamSynchronize(st));
        } else {
          long spins = 0;
          while (*(volatile unsigned*)flag != seq) {
            if (++spins > 200000000L) { fprintf(stderr, "flag never arrived\n"); return 2; }
          }
        }
        const double t1 = now_us();
        for (int r = 0; r < G * 256; r += 97)
          if (((volatile float*)hout)[r] != (float)(seq + (r & 255))) ++bad;
        if (mode == 1) CHECK(hipStreamSynchronize(st));
        if (it >= 100) ts.push_back(t1 - t0);
      }
      CHECK(hipStreamSynchronize(st));
      std::sort(ts.begin(), ts.end());
      static const char* names[3] = {"sync", "flag", "flag_chain"};
      printf("%s\"%s_g%d\": [%.2f, %.2f, %.2f]", sep, names[mode], G, ts[ts.size() / 2], ts[ts.size() / 10],
             ts[ts.size() * 9 / 10]);
      sep = ", ";
    }
  }
  printf(", \"stale_rows_seen\": %d}\n", bad);
  CHECK(hipHostFree(hout));
  CHECK(hipHostFree(flag));
  CHECK(hipFree(cnt));
  return bad ? 3 : 0;
}
