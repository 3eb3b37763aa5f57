// frame_assemble.hip -- rank 0's frame assembly for the multi-GPU RT path
// (include/rt_shard.h).  HBM-bound copy: 4 B read + 4 B
// written per pixel, no index array.  Each thread moves 4 horizontally
// adjacent pixels: 16 B of one 128-B tile row of the gathered buffer to 16 B
// of one image row, so both sides are coalesced (a wave covers two whole
// tile rows on the read side and 1 KiB of one image row on the write side).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_shard.h"

namespace {

constexpr uint32_t kTile = 32, kThreads = 256;

__global__ __launch_bounds__(kThreads) void frame_assemble(
    uint32_t* __restrict__ img, const uint32_t* __restrict__ recv, uint32_t width,
    uint32_t height, uint32_t world, uint64_t per_rank, uint32_t tiles_x, uint32_t quads_x) {
  const uint64_t q = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint32_t y = (uint32_t)(q / quads_x);
  if (y >= height) return;
  const uint32_t x = (uint32_t)(q - (uint64_t)y * quads_x) * 4u;
  const uint32_t t = (y / kTile) * tiles_x + x / kTile;
  const uint32_t r = t % world, lt = t / world;
  const uint64_t src = (uint64_t)r * per_rank + (uint64_t)lt * (kTile * kTile) +
                       (y % kTile) * kTile + (x % kTile);
  const uint64_t dst = (uint64_t)y * width + x;
  if ((width & 3u) == 0u) {  // 16-B aligned rows: one dwordx4 each way
    *reinterpret_cast<uint4*>(img + dst) = *reinterpret_cast<const uint4*>(recv + src);
  } else {
    for (uint32_t k = 0; k < 4u && x + k < width; ++k) img[dst + k] = recv[src + k];
  }
}

}  // namespace

extern "C" int rt_frame_assemble(uint32_t* image, const uint32_t* recv, uint32_t width,
                                 uint32_t height, uint32_t world, uint64_t slots_per_rank,
                                 void* stream) {
  if (!image || !recv || width == 0 || height == 0 || world == 0 || slots_per_rank % 1024u)
    return -1;
  const uint32_t tiles_x = (width + kTile - 1) / kTile, tiles_y = (height + kTile - 1) / kTile;
  const uint64_t local0 = ((uint64_t)tiles_x * tiles_y + world - 1) / world;  // rank 0's tiles
  if (slots_per_rank < local0 * kTile * kTile) return -1;
  const uint32_t quads_x = (width + 3u) / 4u;
  const uint64_t threads = (uint64_t)quads_x * height;
  const uint64_t blocks = (threads + kThreads - 1) / kThreads;
  if (blocks > 0x7fffffffull) return -1;
  hipLaunchKernelGGL(frame_assemble, dim3((uint32_t)blocks), dim3(kThreads), 0,
                     (hipStream_t)stream, image, recv, width, height, world, slots_per_rank,
                     tiles_x, quads_x);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
