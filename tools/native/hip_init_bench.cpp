// Where a fresh process's HIP start-up goes (the odh-gpu-probe init container pays it per pod):
// exec → main, hipGetDeviceCount (ROCr/HSA init + topology), hipSetDevice, hipFree(0) (context),
// first hipMalloc of the probe's 256 MiB, first kernel launch (code object load), teardown.
//
//   hipcc -O2 tools/native/hip_init_bench.cpp -lhsa-runtime64 -o /tmp/hib && ODH_T0_NS=$(date +%s%N) /tmp/hib
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>

__global__ void touch(int* p) { p[threadIdx.x] = threadIdx.x; }

static double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

int main() {
  const double t_main = now_ms();
  const char* t0s = std::getenv("ODH_T0_NS");
  const double t_exec = t0s ? t_main - std::strtod(t0s, nullptr) / 1e6 : -1.0;
  // ODH_HSA_FIRST=1: initialise the ROCr (HSA) runtime on its own first, so device_count_ms
  // is what HIP (rocclr) adds on top of it
  double d_hsa = -1.0;
  if (std::getenv("ODH_HSA_FIRST")) {
    double th = now_ms();
    if (hsa_init() != HSA_STATUS_SUCCESS) {
      std::printf("{\"error\":\"hsa_init\"}\n");
      return 2;
    }
    d_hsa = now_ms() - th;
  }
  int n = 0;
  double t = now_ms();
  hipError_t e = hipGetDeviceCount(&n);
  const double d_count = now_ms() - t;
  if (e != hipSuccess || n == 0) {
    std::printf("{\"error\":\"%s\"}\n", hipGetErrorString(e));
    return 2;
  }
  t = now_ms();
  (void)hipSetDevice(0);
  const double d_set = now_ms() - t;
  t = now_ms();
  (void)hipFree(nullptr);
  const double d_ctx = now_ms() - t;
  void* buf = nullptr;
  t = now_ms();
  (void)hipMalloc(&buf, 256ull << 20);
  const double d_malloc = now_ms() - t;
  int* p = nullptr;
  (void)hipMalloc(&p, 256 * sizeof(int));
  t = now_ms();
  touch<<<1, 64>>>(p);
  (void)hipDeviceSynchronize();
  const double d_launch = now_ms() - t;
  t = now_ms();
  touch<<<1, 64>>>(p);
  (void)hipDeviceSynchronize();
  const double d_launch2 = now_ms() - t;
  t = now_ms();
  (void)hipFree(buf);
  (void)hipFree(p);
  const double d_free = now_ms() - t;
  std::printf("{\"devices\":%d,\"hsa_init_ms\":%.2f,\"exec_ms\":%.2f,\"device_count_ms\":%.2f,\"set_device_ms\":%.2f,\"context_ms\":%.2f,"
              "\"malloc_256mib_ms\":%.2f,\"first_launch_ms\":%.2f,\"second_launch_ms\":%.3f,\"free_ms\":%.2f,"
              "\"main_to_here_ms\":%.2f}\n",
              n, d_hsa, t_exec, d_count, d_set, d_ctx, d_malloc, d_launch, d_launch2, d_free, now_ms() - t_main);
  std::fflush(stdout);
  if (std::getenv("ODH_FAST_EXIT")) std::_Exit(0);  // skip the runtime's exit-time teardown
  return 0;
}
