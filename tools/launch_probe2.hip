// launch_probe2.hip -- where a kernel launch's host enqueue time goes (round 6): the serve launch
// enqueues in ~2.8 us where an empty kernel takes ~0.9 us (-DP3D_HOSTPROF segments, r06_t15), with
// the same argument block in device memory either way (a 0.5 KB block measured like the 1.1 KB one).
// Median host time of one enqueue (the stream synchronised, untimed, before each) for kernels that
// differ in one property at a time: static LDS (0 / 93 KB), argument block (8 B / 1 KB), register
// budget (a 64-register vs a 512-register kernel), and the launch API (<<<>>> vs hipModuleLaunchKernel
// on a function handle resolved once, arguments as one buffer).  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big { int v[256]; };

__global__ __launch_bounds__(256) void k_small(int* out) { if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1; }
__global__ __launch_bounds__(256) void k_bigarg(Big a, int* out) { if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = a.v[255]; }
__global__ __launch_bounds__(256) void k_lds(int* out) {
  __shared__ float s[93 * 256];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (int)s[5];
}
// many live registers: a long dependent chain the compiler cannot shorten
__global__ __launch_bounds__(256) void k_regs(const float* in, float* out) {
  float r[120];
#pragma unroll
  for (int i = 0; i < 120; ++i) r[i] = in[(threadIdx.x + 64 * i) & 4095];
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < 120; ++i) { acc = __builtin_fmaf(acc, r[i], r[(i + k) % 120]); r[i] += acc; }
  if (acc == 12345.f) out[threadIdx.x] = acc;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double med(hipStream_t st, F launch) {
  std::vector<double> ts;
  for (int i = 0; i < 330; ++i) {
    (void)hipStreamSynchronize(st);
    const double t0 = now_us();
    launch();
    const double t1 = now_us();
    if (i >= 30) ts.push_back(t1 - t0);
  }
  (void)hipStreamSynchronize(st);
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* out;
  float *fin, *fout;
  CHECK(hipMalloc(&out, 1024));
  CHECK(hipMalloc(&fin, 4096 * 4));
  CHECK(hipMalloc(&fout, 4096 * 4));
  CHECK(hipMemset(fin, 0, 4096 * 4));
  Big big{};
  const dim3 g(256), b(256);
  const double small = med(st, [&] { k_small<<<g, b, 0, st>>>(out); });
  const double bigarg = med(st, [&] { k_bigarg<<<g, b, 0, st>>>(big, out); });
  const double lds = med(st, [&] { k_lds<<<g, b, 0, st>>>(out); });
  const double regs = med(st, [&] { k_regs<<<g, b, 0, st>>>(fin, fout); });
  hipFunction_t fb;
  CHECK(hipGetFuncBySymbol(&fb, reinterpret_cast<const void*>(&k_bigarg)));
  struct { Big a; int* o; } kb{big, out};
  size_t kbs = sizeof(kb);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &kb, HIP_LAUNCH_PARAM_BUFFER_SIZE, &kbs, HIP_LAUNCH_PARAM_END};
  const double bigarg_mod = med(st, [&] { (void)hipModuleLaunchKernel(fb, 256, 1, 1, 256, 1, 1, 0, st, nullptr, extra); });
  hipFunction_t fs;
  CHECK(hipGetFuncBySymbol(&fs, reinterpret_cast<const void*>(&k_small)));
  void* sargs[] = {&out};
  const double small_mod = med(st, [&] { (void)hipModuleLaunchKernel(fs, 256, 1, 1, 256, 1, 1, 0, st, sargs, nullptr); });
  printf("{\"small\": %.2f, \"bigarg_1kb\": %.2f, \"lds_93kb\": %.2f, \"regs\": %.2f, \"bigarg_module_launch\": %.2f, "
         "\"small_module_launch\": %.2f}\n", small, bigarg, lds, regs, bigarg_mod, small_mod);
  return 0;
}
