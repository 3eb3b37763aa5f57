// pmc_probe.hip -- known-byte probes for calibrating rocprofv3's FETCH_SIZE /
// WRITE_SIZE against the access widths the RT kernels use (VERDICT r02 item
// 1; the MI355X guide calibrates FETCH_SIZE only for 16-B/lane streaming
// reads (x2) and WRITE_SIZE only for 16-B/lane streaming stores).
//
// Each probe touches exactly `bytes` distinct bytes once per launch, with the
// RT kernels' instruction forms:
//   store4   buffer_store_dword, 4 B per lane, 64 lanes = 256 contiguous bytes
//            (the framebuffer store, rt_trace.h store_pixel)
//   store16  buffer_store_dwordx4, 16 B per lane (the guide's calibrated form)
//   load16   buffer_load_dwordx4, 16 B per lane (the guide's calibrated form)
//   sload64  s_load_dwordx16, one 64-B record per wave-load (the packet walks'
//            node / record loads through the scalar cache)
// Every kernel is launched `reps` times; scripts/pmc_calibrate.py divides the
// per-dispatch counters by the known bytes.  Vector stores only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)0xffffffffu, 0x00020000);
}

extern "C" __global__ void __launch_bounds__(256) probe_store4(uint32_t* dst, uint32_t words) {
  const auto r = rsrc(dst);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < words; i += gridDim.x * 256)
    __builtin_amdgcn_raw_buffer_store_b32(i * 2654435761u, r, 4u * i, 0, 0);
}

extern "C" __global__ void __launch_bounds__(256) probe_store16(uint32_t* dst, uint32_t words) {
  const auto r = rsrc(dst);
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; 4 * i < words; i += gridDim.x * 256) {
    const u4 v = {i, i + 1, i + 2, i + 3};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, 16u * i, 0, 0);
  }
}

extern "C" __global__ void __launch_bounds__(256) probe_load16(const uint32_t* src, uint32_t words,
                                                               uint32_t* sink) {
  const auto r = rsrc((void*)src);
  uint32_t acc = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; 4 * i < words; i += gridDim.x * 256) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, 16u * i, 0, 0);
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x * 256 + threadIdx.x] = acc;  // keeps the loads
}

// one 64-B record per wave-load through the scalar cache: wave w of the grid
// reads records w, w + waves, ...
extern "C" __global__ void __launch_bounds__(256) probe_sload64(const uint32_t* src, uint32_t words,
                                                                uint32_t* sink) {
  const uint32_t waves = gridDim.x * 4, wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t base = (uint64_t)src;
  uint32_t acc = 0;
  for (uint32_t rec = wv; 16 * rec < words; rec += waves) {
    const uint32_t o = (uint32_t)__builtin_amdgcn_readfirstlane(64u * rec);
    typedef uint32_t u16v __attribute__((ext_vector_type(16)));
    const u16v v = *(const __attribute__((address_space(4))) u16v*)(base + o);
#pragma unroll
    for (int k = 0; k < 16; ++k) acc ^= v[k];
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const uint64_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 4;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  const uint32_t words = (uint32_t)(mib * (1u << 20) / 4);
  uint32_t *a = nullptr, *b = nullptr, *c = nullptr, *sink = nullptr;
  CHECK(hipMalloc(&a, (size_t)words * 4));  // store4 target
  CHECK(hipMalloc(&c, (size_t)words * 4));  // store16 target
  CHECK(hipMalloc(&b, (size_t)words * 4));  // load source
  CHECK(hipMalloc(&sink, 1u << 22));
  CHECK(hipMemset(b, 1, (size_t)words * 4));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const dim3 grid(cus * 4), block(256);
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(probe_store4, grid, block, 0, 0, a, words);
    hipLaunchKernelGGL(probe_store16, grid, block, 0, 0, c, words);
    hipLaunchKernelGGL(probe_load16, grid, block, 0, 0, b, words, sink);
    hipLaunchKernelGGL(probe_sload64, grid, block, 0, 0, b, words, sink);
  }
  CHECK(hipDeviceSynchronize());
  std::printf("{\"bytes\": %llu, \"reps\": %d}\n", (unsigned long long)words * 4ull, reps);
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(c));
  CHECK(hipFree(sink));
  return 0;
}
