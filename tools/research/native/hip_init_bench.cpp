// Where a fresh process's HIP start-up goes (the odh-gpu-probe init container pays it per pod):
// exec → main, hipGetDeviceCount (ROCr/HSA init + topology), hipSetDevice, hipFree(0) (context),
// first hipMalloc of the probe's 256 MiB, first kernel launch (code object load), teardown.
// The last field, end_ns (CLOCK_REALTIME), lets the spawner time the process exit itself
// (tools/hip_exit_ab.py: reaped - end_ns).
//
//   ODH_NO_GPU=1       no HIP call at all (the bare exec + exit of a HIP-linked binary)
//   ODH_HSA_ONLY=1     hsa_init only, then exit
//   ODH_MALLOC_MIB=N   size of the first hipMalloc (default 256)
//   ODH_NO_FREE=1      exit with the buffers still allocated
//   ODH_FAST_EXIT=1    std::_Exit (skip the runtime's exit-time teardown)
//
//   hipcc -O2 tools/native/hip_init_bench.cpp -lhsa-runtime64 -o /tmp/hib && ODH_T0_NS=$(date +%s%N) /tmp/hib
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>

__global__ void touch(int* p) { p[threadIdx.x] = threadIdx.x; }

static long long now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

static int leave(int rc) {
  std::fflush(stdout);
  if (std::getenv("ODH_FAST_EXIT")) std::_Exit(rc);  // skip the runtime's exit-time teardown
  return rc;
}

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
  if (std::getenv("ODH_NO_GPU")) {
    std::printf("{\"exec_ms\":%.2f,\"end_ns\":%lld}\n", t_exec, now_ns());
    return leave(0);
  }
  double d_hsa = -1.0;
  if (std::getenv("ODH_HSA_FIRST") || std::getenv("ODH_HSA_ONLY")) {
    double th = now_ms();
    if (hsa_init() != HSA_STATUS_SUCCESS) {
      std::printf("{\"error\":\"hsa_init\"}\n");
      return 2;
    }
    d_hsa = now_ms() - th;
    if (std::getenv("ODH_HSA_ONLY")) {
      std::printf("{\"exec_ms\":%.2f,\"hsa_init_ms\":%.2f,\"end_ns\":%lld}\n", t_exec, d_hsa, now_ns());
      return leave(0);
    }
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
  const char* mib = std::getenv("ODH_MALLOC_MIB");
  (void)hipMalloc(&buf, (mib ? std::strtoull(mib, nullptr, 10) : 256ull) << 20);
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
  if (!std::getenv("ODH_NO_FREE")) {
    (void)hipFree(buf);
    (void)hipFree(p);
  }
  const double d_free = now_ms() - t;
  std::printf("{\"devices\":%d,\"hsa_init_ms\":%.2f,\"exec_ms\":%.2f,\"device_count_ms\":%.2f,\"set_device_ms\":%.2f,\"context_ms\":%.2f,"
              "\"malloc_256mib_ms\":%.2f,\"first_launch_ms\":%.2f,\"second_launch_ms\":%.3f,\"free_ms\":%.2f,"
              "\"main_to_here_ms\":%.2f,\"end_ns\":%lld}\n",
              n, d_hsa, t_exec, d_count, d_set, d_ctx, d_malloc, d_launch, d_launch2, d_free, now_ms() - t_main,
              now_ns());
  return leave(0);
}
