// aql_probe_kernel.hip -- launch_probe.hip's frame and tail kernels as one code
// object for aql_probe.cpp (HSA loader + direct AQL packets, and HIP modules)
#include <hip/hip_runtime.h>
#include <stdint.h>

// every wave spins until `ticks` (100 MHz) have passed since its start
extern "C" __global__ void __launch_bounds__(128) aql_frame_kernel(uint32_t ticks, uint32_t* counter,
                                                                  uint32_t* host_word, uint32_t nonce,
                                                                  uint32_t nblocks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((uint32_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  (void)counter; (void)host_word; (void)nonce; (void)nblocks;
}

extern "C" __global__ void aql_tail_kernel(uint32_t* host_word, uint32_t nonce) {
  if (threadIdx.x == 0) __hip_atomic_store(host_word, nonce, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
