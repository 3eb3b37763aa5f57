// launch_probe.hip -- what a synchronous frame (start + wait) costs on top of
// the kernel, by launch and completion mechanism (VERDICT r04
// item 3).  A "frame" here is one launch of a kernel whose duration is set by
// a spin on s_memrealtime (the RT frame's ~18 us), over the RT kernel's grid
// (16 384 one-wave workgroups of 128 threads -> 8 192 blocks).  Each mode
// runs N synchronous frames (issue, then wait for completion, then the next)
// and prints the median host time per frame, the host time of the issue call
// alone, and the median device duration (event-timed, separate run).
//   ext_events   hipExtModuleLaunchKernel with start/stop events on the
//                dispatch packet, hipEventQuery spin      (the r04 driver)
//   plain_query  hipModuleLaunchKernel, hipStreamQuery spin
//   plain_sync   hipModuleLaunchKernel, hipStreamSynchronize
//   marker       hipModuleLaunchKernel + hipEventRecord (no timing), hipEventQuery spin
//   writevalue   hipModuleLaunchKernel + hipStreamWriteValue32 to pinned host
//                memory, spin on that word
//   tail_kernel  hipModuleLaunchKernel + a one-wave kernel storing a nonce to
//                pinned host memory (system scope), spin on that word
//   lastwave     the kernel's own waves count down a device counter (one
//                atomic per workgroup); the workgroup that ends it stores the
//                nonce to pinned host memory; spin on that word
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// every wave spins until `ticks` (100 MHz) have passed since its start
__global__ void __launch_bounds__(128) frame_kernel(uint32_t ticks, uint32_t* counter, uint32_t* host_word,
                                                    uint32_t nonce, uint32_t nblocks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((uint32_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  if (counter) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t left = atomicSub(counter, 1u);
      if (left == 1u) {
        __atomic_store_n(counter, nblocks, __ATOMIC_RELAXED);  // re-armed for the next frame
        __hip_atomic_store(host_word, nonce, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

__global__ void tail_kernel(uint32_t* host_word, uint32_t nonce) {
  if (threadIdx.x == 0) __hip_atomic_store(host_word, nonce, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int frames = argc > 1 ? std::atoi(argv[1]) : 400;
  const uint32_t ticks = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1200;  // 12 us of spin per wave
  const uint32_t nblocks = 8192, block = 128;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t *host_word = nullptr, *dev_word = nullptr, *counter = nullptr;
  CK(hipHostMalloc((void**)&host_word, 64, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&dev_word, host_word, 0));
  CK(hipMalloc((void**)&counter, 64));
  CK(hipMemcpy(counter, &nblocks, 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1, mk;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&mk, hipEventDisableTiming));
  volatile uint32_t* hw = host_word;
  uint32_t nonce = 0;
  const char* modes[] = {"ext_events", "plain_query", "plain_sync", "marker", "writevalue", "tail_kernel", "lastwave"};
  // device duration of one frame (events around 50 back-to-back frames)
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(frame_kernel, dim3(nblocks), dim3(block), 0, s, ticks, nullptr, nullptr, 0u, nblocks);
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(frame_kernel, dim3(nblocks), dim3(block), 0, s, ticks, nullptr, nullptr, 0u, nblocks);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::printf("{\"frame_kernel_us_back_to_back\": %.2f, \"frames\": %d", ms * 1000.0 / 50, frames);
  for (int m = 0; m < 7; ++m) {
    std::vector<double> tot, iss;
    for (int i = 0; i < frames + 20; ++i) {
      ++nonce;
      const double t0 = now_us();
      uint32_t* ctr = m == 6 ? counter : nullptr;
      switch (m) {
        case 0:
          hipExtLaunchKernelGGL(frame_kernel, dim3(nblocks), dim3(block), 0, s, e0, e1, 0, ticks, ctr, dev_word,
                                nonce, nblocks);
          break;
        default:
          hipLaunchKernelGGL(frame_kernel, dim3(nblocks), dim3(block), 0, s, ticks, ctr, dev_word, nonce, nblocks);
          break;
      }
      if (m == 3) CK(hipEventRecord(mk, s));
      if (m == 4) CK(hipStreamWriteValue32(s, dev_word, nonce, 0));
      if (m == 5) hipLaunchKernelGGL(tail_kernel, dim3(1), dim3(64), 0, s, dev_word, nonce);
      const double t1 = now_us();
      switch (m) {
        case 0: while (hipEventQuery(e1) == hipErrorNotReady) {} break;
        case 1: while (hipStreamQuery(s) == hipErrorNotReady) {} break;
        case 2: CK(hipStreamSynchronize(s)); break;
        case 3: while (hipEventQuery(mk) == hipErrorNotReady) {} break;
        default:
          while (*hw != nonce) {
            if (now_us() - t1 > 1e6) { std::fprintf(stderr, "mode %s: no completion word\n", modes[m]); std::exit(3); }
          }
          break;
      }
      const double t2 = now_us();
      if (i >= 20) { tot.push_back(t2 - t0); iss.push_back(t1 - t0); }
    }
    CK(hipStreamSynchronize(s));
    std::printf(", \"%s\": {\"frame_us\": %.2f, \"issue_us\": %.2f}", modes[m], median(tot), median(iss));
  }
  std::printf("}\n");
  return 0;
}
