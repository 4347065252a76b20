// Probe: can a stream wait (hipStreamWaitValue32) on a counter that a RUNNING kernel on another
// stream increments, and does the waiting stream proceed before that kernel ends?
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/probe_waitvalue tools/probe_waitvalue.hip && /tmp/probe_waitvalue
// Stream A: a kernel whose waves spin for ~2 ms and bump the counter half-way.  Stream B: wait for
// counter >= n_waves, then a small kernel stamping the time, then a device-to-host copy.  Prints
// when B's work ran relative to A's kernel.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                    \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

__device__ unsigned long long now_ns() { return wall_clock64() * 10ull; }  // 100 MHz constant clock

__global__ void spinner(unsigned* ctr, unsigned long long* stamps, unsigned long long spin_ns) {
  // (bump at spin_ns / 2 after the wave's start)
  const unsigned long long t0 = now_ns();
  bool bumped = false;
  while (now_ns() - t0 < spin_ns) {
    if (!bumped && now_ns() - t0 > spin_ns / 2) {
      bumped = true;
      if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (old + 1u == gridDim.x) stamps[2] = now_ns();  // the last bump
      }
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) stamps[0] = now_ns();  // (one wave's end)
}

__global__ void stamp(unsigned long long* stamps) {
  if (threadIdx.x == 0) stamps[1] = now_ns();
}

int main() {
  int dev = 0, can = 0;
  CK(hipSetDevice(dev));
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev));
  std::printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
  unsigned* ctr = nullptr;
  CK(hipExtMallocWithFlags((void**)&ctr, 8, hipMallocSignalMemory));
  unsigned long long* stamps = nullptr;
  CK(hipMalloc(&stamps, 64));
  CK(hipMemset(stamps, 0, 64));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  const int waves = 256;
  std::vector<char> host(8 << 20);
  char* dbuf = nullptr;
  CK(hipMalloc(&dbuf, host.size()));
  for (int rep = 0; rep < 8; ++rep) {
    CK(hipStreamWriteValue32(a, ctr, 0, 0));
    CK(hipStreamSynchronize(a));
    hipEvent_t ea0, ea1, eb1;
    CK(hipEventCreate(&ea0));
    CK(hipEventCreate(&ea1));
    CK(hipEventCreate(&eb1));
    auto h0 = std::chrono::steady_clock::now();
    CK(hipEventRecord(ea0, a));
    hipLaunchKernelGGL(spinner, dim3(waves), dim3(64), 0, a, ctr, stamps, 2000000ull + 150000ull * rep);
    CK(hipGetLastError());
    CK(hipEventRecord(ea1, a));
    CK(hipStreamWaitValue32(b, ctr, (uint32_t)waves, hipStreamWaitValueGte, 0xffffffffu));
    hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, b, stamps);
    CK(hipMemcpyAsync(host.data(), dbuf, host.size(), hipMemcpyDeviceToHost, b));
    CK(hipEventRecord(eb1, b));
    CK(hipStreamSynchronize(b));
    auto hb = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(a));
    auto ha = std::chrono::steady_clock::now();
    float ms_a = 0, ms_b = 0;
    CK(hipEventElapsedTime(&ms_a, ea0, ea1));
    CK(hipEventElapsedTime(&ms_b, ea0, eb1));
    unsigned long long st[3];
    CK(hipMemcpy(st, stamps, 24, hipMemcpyDeviceToHost));
    unsigned cv = 0;
    CK(hipMemcpy(&cv, ctr, 4, hipMemcpyDeviceToHost));
    std::printf("rep %d: kernel A %.3f ms; B (wait, stamp, 8 MB D2H) done at %.3f ms; stamp kernel ran %.3f ms "
                "before A's wave 0 ended, %.4f ms after the last bump; host saw B %.3f ms, A %.3f ms; counter %u\n",
                rep, ms_a, ms_b, ((double)st[0] - (double)st[1]) * 1e-6, ((double)st[1] - (double)st[2]) * 1e-6,
                std::chrono::duration<double, std::milli>(hb - h0).count(),
                std::chrono::duration<double, std::milli>(ha - h0).count(), cv);
  }
  std::printf("OK\n");
  return 0;
}
