// dispatch_probe.hip -- is the 4-stream batch-64 inference bound by kernel dispatch?
// Replays, on S concurrent streams, HIP graphs of G back-to-back null kernels shaped like the
// hidden layer's launch (256 workgroups x 512 threads) and prints the aggregate time per kernel.
// Build: hipcc --offload-arch=gfx950 -O3 tools/dispatch_probe.hip -o tools/dispatch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <chrono>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(512) void knull(float* y) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && y[0] == 12345.f) y[0] = 0;
}

// a kernel that spins ~us microseconds per workgroup (s_sleep), to see overlap of busy kernels
__global__ __launch_bounds__(512) void kspin(float* y, int iters) {
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(16);
  if (threadIdx.x == 0 && blockIdx.x == 0 && y[0] == 12345.f) y[0] = 0;
}

int main(int argc, char** argv) {
  const int G = 60, REPS = 50;
  float* y;
  CK(hipMalloc(&y, 1024));
  CK(hipMemset(y, 0, 1024));
  std::vector<hipStream_t> st(16);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (auto& s : st) { hipLaunchKernelGGL(knull, dim3(1), dim3(64), 0, s, y); }
  CK(hipDeviceSynchronize());
  for (int kind = 0; kind < 3; ++kind) {
    const int spin = kind == 0 ? 0 : kind == 1 ? 4 : 10;
    const int maps[7][8] = {{0}, {0, 1}, {0, 1, 2, 3}, {4, 5, 6, 7}, {0, 2, 4, 6}, {1, 3, 5, 7}, {0, 1, 2, 3, 4, 5, 6, 7}};
    const int nmap[7] = {1, 2, 4, 4, 4, 4, 8};
    for (int mi = 0; mi < 7; ++mi) {
      const int S = nmap[mi];
      std::vector<hipGraphExec_t> ex(S);
      std::vector<hipStream_t> ss(S);
      for (int s = 0; s < S; ++s) ss[s] = st[maps[mi][s]];
      for (int s = 0; s < S; ++s) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(ss[s], hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < G; ++k) {
          if (spin) hipLaunchKernelGGL(kspin, dim3(256), dim3(512), 0, ss[s], y, spin);
          else hipLaunchKernelGGL(knull, dim3(256), dim3(512), 0, ss[s], y);
        }
        CK(hipStreamEndCapture(ss[s], &g));
        CK(hipGraphInstantiate(&ex[s], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
      for (int w = 0; w < 3; ++w)
        for (int s = 0; s < S; ++s) CK(hipGraphLaunch(ex[s], ss[s]));
      CK(hipDeviceSynchronize());
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      auto t0 = std::chrono::steady_clock::now();
      for (int r = 0; r < REPS; ++r)
        for (int s = 0; s < S; ++s) CK(hipGraphLaunch(ex[s], ss[s]));
      CK(hipDeviceSynchronize());
      auto t1 = std::chrono::steady_clock::now();
      const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
      printf("kernel=%s spin=%2d map=%d streams=%d  aggregate %.3f us/kernel  (per stream %.3f us/kernel)\n",
             spin ? "spin" : "null", spin, mi, S, us / (REPS * G * S), us / (REPS * G));
      for (auto& e : ex) CK(hipGraphExecDestroy(e));
    }
  }
  return 0;
}
