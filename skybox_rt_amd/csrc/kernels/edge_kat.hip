// edge_kat.hip -- the rasterizer's coverage predicate (gfx::covers, the one
// raster_kernel.hip and the RT kernels' primary tests use) over a pixel
// window, for known-answer tests: the RTL raster slice's
// (hw/unit_tests/raster_unit/raster_slice/testbench.cpp:53-66 with
// golden_data/test_data.txt; tests/test_gpu_edge_kat.py).  Thread per pixel.
#include <hip/hip_runtime.h>

#include "gfx_device.h"

typedef struct {
  int32_t edges[9];    // (a, b, c) per edge, Q15.16 as the primitive records hold them
  uint32_t x0, y0;     // window origin (pixels)
  uint32_t w, h;       // window size
  uint32_t pad;
  uint64_t out_addr;   // uint32 [w * h]: bit 31 covered | the three edge values' sign bits
  uint64_t vals_addr;  // int32 [w * h * 3]: the edge values
} edge_kat_arg_t;

static __device__ __forceinline__ void kernel_body(const vx_task_t& task, edge_kat_arg_t* a) {
  const uint32_t i = task.blockIdx.x, j = task.blockIdx.y;
  int32_t e[3];
  const bool in = gfx::covers(a->edges, a->x0 + i, a->y0 + j, e);
  const uint32_t k = j * a->w + i;
  vx_ptr<uint32_t>(a->out_addr)[k] = (in ? 0x80000000u : 0u) | ((uint32_t)e[0] >> 31) |
                                     (((uint32_t)e[1] >> 31) << 1) | (((uint32_t)e[2] >> 31) << 2);
  int32_t* v = vx_ptr<int32_t>(a->vals_addr);
  v[3 * k] = e[0];
  v[3 * k + 1] = e[1];
  v[3 * k + 2] = e[2];
}

VX_MAIN(edge_kat_arg_t, arg, 256) {
  const uint32_t grid[3] = {arg->w, arg->h, 1};
  return vx_spawn_threads(2, grid, (const uint32_t*)nullptr,
                          [](const vx_task_t& t, edge_kat_arg_t* a) { kernel_body(t, a); }, arg);
}
