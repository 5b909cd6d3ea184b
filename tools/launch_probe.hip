// launch_probe.hip -- host enqueue cost of a kernel launch vs the size of its argument struct
// (the k_serve6 launch passes ~1 KB: ServeArgs with 16 ServeLayer records).  Prints the median
// host time of one <<<>>> enqueue, and of enqueue + hipStreamSynchronize, for 64 B, 256 B and
// 1 KB argument structs, 256 x 256 threads, each kernel reading one word of its arguments; the
// round trip waits with hipDeviceSynchronize (torch.cuda.synchronize), under each schedule flag.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <vector>

template <int BYTES>
struct Args { int v[BYTES / 4]; };

template <int BYTES>
__global__ void k_probe(Args<BYTES> a, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = a.v[BYTES / 4 - 1];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int BYTES>
static void run(hipStream_t st, int* out) {
  Args<BYTES> a{};
  a.v[BYTES / 4 - 1] = BYTES;
  for (int i = 0; i < 200; ++i) k_probe<BYTES><<<256, 256, 0, st>>>(a, out);
  (void)hipStreamSynchronize(st);
  std::vector<double> enq, rt;
  for (int i = 0; i < 200; ++i) {
    (void)hipStreamSynchronize(st);
    const double t0 = now_us();
    k_probe<BYTES><<<256, 256, 0, st>>>(a, out);
    const double t1 = now_us();
    (void)hipDeviceSynchronize();
    const double t2 = now_us();
    enq.push_back(t1 - t0);
    rt.push_back(t2 - t0);
  }
  std::sort(enq.begin(), enq.end());
  std::sort(rt.begin(), rt.end());
  printf("{\"arg_bytes\": %d, \"enqueue_us_median\": %.2f, \"launch_sync_us_median\": %.2f}\n", BYTES, enq[100],
         rt[100]);
}

int main(int argc, char** argv) {
  // argv[1]: device schedule flag set before the runtime initialises the device
  // (auto = HIP's default, spin = hipDeviceScheduleSpin, yield, block = BlockingSync)
  const char* mode = argc > 1 ? argv[1] : "auto";
  unsigned fl = hipDeviceScheduleAuto;
  if (!strcmp(mode, "spin")) fl = hipDeviceScheduleSpin;
  else if (!strcmp(mode, "yield")) fl = hipDeviceScheduleYield;
  else if (!strcmp(mode, "block")) fl = hipDeviceScheduleBlockingSync;
  if (hipSetDeviceFlags(fl) != hipSuccess) printf("{\"warning\": \"hipSetDeviceFlags failed\"}\n");
  printf("{\"schedule\": \"%s\"}\n", mode);
  hipStream_t st;
  int* out;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  (void)hipMalloc(&out, 64);
  run<64>(st, out);
  run<256>(st, out);
  run<1024>(st, out);
  run<64>(st, out);
  (void)hipFree(out);
  (void)hipStreamDestroy(st);
  return 0;
}
