// Dev probe: how long does a kernel's first read of its arguments take, against a read of the same
// words from a device-memory global?  Each kernel stamps the 100 MHz wall clock at entry, after one
// scalar load of an argument word, and after one scalar load of a device-global word; between probe
// launches a streaming kernel sweeps 512 MB so no cache holds either word.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/kernarg_probe tools/kernarg_probe.hip && /tmp/kernarg_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

struct Args {
  const int* p;
  int a[30];
  unsigned long long* out;
};

__device__ Args g_args;   // the same block, in device memory

__device__ __forceinline__ unsigned long long p_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned p_sload(const void* base, int off_words) {
  unsigned v;
  const unsigned* p = (const unsigned*)base + off_words;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}

template <int which>
__global__ void k_probe(Args args) {
  const unsigned long long t0 = p_now();
  const void* ka = (const void*)(const char*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned v;
  unsigned long long t1, t2;
  // word 9 of the argument block (args.a[7]) / of the device-global copy, in the stated order
  if (which == 0) {
    v = p_sload(ka, 9);
    t1 = p_now();
    v += p_sload(&g_args, 9);
    t2 = p_now();
  } else {
    v = p_sload(&g_args, 9);
    t1 = p_now();
    v += p_sload(ka, 9);
    t2 = p_now();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    unsigned long long* o = args.out;
    o[0] = t1 - t0;
    o[1] = t2 - t1;
    o[2] = v;
  }
}

__global__ void k_sweep(float4* buf, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) buf[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

int main() {
  unsigned long long* out;
  hipMalloc(&out, 64);
  float4* buf;
  const size_t n = (512u << 20) / sizeof(float4);
  hipMalloc(&buf, n * sizeof(float4));
  Args a{};
  for (int i = 0; i < 30; ++i) a.a[i] = i;
  a.out = out;
  hipMemcpyToSymbol(HIP_SYMBOL(g_args), &a, sizeof(a));
  for (int which = 0; which < 2; ++which) {
    for (int cold = 0; cold < 2; ++cold) {
      std::vector<double> d1, d2;
      for (int r = 0; r < 40; ++r) {
        if (cold) k_sweep<<<2048, 256>>>(buf, n);
        if (which == 0) k_probe<0><<<1, 64>>>(a);
        else k_probe<1><<<1, 64>>>(a);
        unsigned long long h[3];
        hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
        if (r >= 4) { d1.push_back(h[0] / 100.0); d2.push_back(h[1] / 100.0); }
      }
      std::sort(d1.begin(), d1.end());
      std::sort(d2.begin(), d2.end());
      printf("{\"first\": \"%s\", \"cold\": %d, \"first_read_us_median\": %.2f, \"second_read_us_median\": %.2f, "
             "\"first_p10\": %.2f, \"first_p90\": %.2f}\n",
             which == 0 ? "kernarg" : "device_global", cold, d1[d1.size() / 2], d2[d2.size() / 2], d1[d1.size() / 10],
             d1[d1.size() * 9 / 10]);
    }
  }
  hipFree(buf);
  hipFree(out);
  return 0;
}
