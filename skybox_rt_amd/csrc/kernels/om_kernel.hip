// om_kernel.hip -- the render-output (OM) regression app's kernel on gfx950
// (tests/regression/om/kernel.cpp:16-40): every pixel of a W x H frame goes
// through the output merger once, with the colour / depth words of the
// kernel argument, the task's alpha ramp when blending, and the OM state the
// host configured through the VX_DCR_OM_* registers (om/main.cpp:153-190).
//
// The reference deals rows to num_tasks tasks (tile_height = ceil(H /
// num_tasks) rows each, alpha = task * 255 / tile_height) and each task walks
// its rows pixel by pixel through vx_om (sim/simx/om_unit.cpp:55-80).  Here a
// task is a pixel (2-D vx_spawn_threads grid W x H: a wave covers 64
// consecutive pixels of a row, so every depth / colour access is one
// coalesced 256-B wave access); the reference's task of the pixel's row,
// y / tile_height, is recomputed where the alpha ramp needs it.  Every pixel
// is written by exactly one thread, so the OM's read-modify-write needs no
// ordering.  The OM configuration is read from the DCR mirror (scalar
// constant loads), with the stencil face chosen by `backface` as the
// hardware unit does (om_unit.cpp:28-49, graphics.cpp:534-620).
#include <hip/hip_runtime.h>

#include "gfx_device.h"
#include "rt_common.h"
#include "vx_spawn.h"

// kernel_arg_t of tests/regression/om/common.h (same layout: 5 words + 3 bools)
typedef struct {
  uint32_t num_tasks;
  uint32_t dst_width;
  uint32_t dst_height;
  uint32_t color;
  uint32_t depth;
  bool backface;
  bool blend_enable;
  bool use_sw;
} om_arg_t;

namespace {

// OutputMerger / DepthTencil / Blender ::configure from the DCR words
__device__ __forceinline__ rt_omstate_t om_state(bool backface) {
  rt_omstate_t s;
  const uint32_t sh = backface ? 16u : 0u;
  s.depth_func = vx_dcr(VX_DCR_OM_DEPTH_FUNC);
  s.depth_writemask = vx_dcr(VX_DCR_OM_DEPTH_WRITEMASK) & 1u;
  s.depth_test_on = !((s.depth_func == VX_OM_DEPTH_FUNC_ALWAYS) && !s.depth_writemask);
  s.stencil_func = (vx_dcr(VX_DCR_OM_STENCIL_FUNC) >> sh) & 0xffffu;
  s.stencil_zpass = (vx_dcr(VX_DCR_OM_STENCIL_ZPASS) >> sh) & 0xffffu;
  s.stencil_zfail = (vx_dcr(VX_DCR_OM_STENCIL_ZFAIL) >> sh) & 0xffffu;
  s.stencil_fail = (vx_dcr(VX_DCR_OM_STENCIL_FAIL) >> sh) & 0xffffu;
  s.stencil_ref = (vx_dcr(VX_DCR_OM_STENCIL_REF) >> sh) & 0xffffu;
  s.stencil_mask = (vx_dcr(VX_DCR_OM_STENCIL_MASK) >> sh) & 0xffffu;
  s.stencil_writemask = (vx_dcr(VX_DCR_OM_STENCIL_WRITEMASK) >> sh) & 0xffffu;
  s.stencil_on = !((s.stencil_func == VX_OM_DEPTH_FUNC_ALWAYS) &&
                   (s.stencil_zpass == VX_OM_STENCIL_OP_KEEP) &&
                   (s.stencil_zfail == VX_OM_STENCIL_OP_KEEP));
  const uint32_t mode = vx_dcr(VX_DCR_OM_BLEND_MODE), func = vx_dcr(VX_DCR_OM_BLEND_FUNC);
  s.blend_mode_rgb = mode & 0xffffu;
  s.blend_mode_a = mode >> 16;
  s.blend_src_rgb = func & 0xffu;
  s.blend_src_a = (func >> 8) & 0xffu;
  s.blend_dst_rgb = (func >> 16) & 0xffu;
  s.blend_dst_a = (func >> 24) & 0xffu;
  s.blend_const = vx_dcr(VX_DCR_OM_BLEND_CONST);
  s.logic_op = vx_dcr(VX_DCR_OM_LOGIC_OP);
  s.blend_on = !((s.blend_mode_rgb == VX_OM_BLEND_MODE_ADD) && (s.blend_mode_a == VX_OM_BLEND_MODE_ADD) &&
                 (s.blend_src_rgb == VX_OM_BLEND_FUNC_ONE) && (s.blend_src_a == VX_OM_BLEND_FUNC_ONE) &&
                 (s.blend_dst_rgb == VX_OM_BLEND_FUNC_ZERO) && (s.blend_dst_a == VX_OM_BLEND_FUNC_ZERO));
  const uint32_t wm = vx_dcr(VX_DCR_OM_CBUF_WRITEMASK) & 0xfu;
  s.cbuf_writemask = ((wm >> 0) & 1u) * 0x000000ffu | ((wm >> 1) & 1u) * 0x0000ff00u |
                     ((wm >> 2) & 1u) * 0x00ff0000u | ((wm >> 3) & 1u) * 0xff000000u;
  s.color_read = wm != 0xfu;
  s.color_write = wm != 0u;
  s.prim_offset = s.prim_count = 0;
  return s;
}

__device__ __forceinline__ void om_pixel(const vx_task_t& t, om_arg_t* a) {
  const vx_arena A = vx_arena::get();
  const uint32_t x = t.blockIdx.x, y = t.blockIdx.y;
  // om/kernel.cpp:35-38 (per launch) and :17-23 (the task of row y)
  const uint32_t tile_h = (a->dst_height + a->num_tasks - 1) / a->num_tasks;
  const float alpha_step = 255.0f / (float)tile_h;
  const uint32_t task = y / tile_h;
  const uint32_t alpha = a->blend_enable ? (uint32_t)((float)task * alpha_step) : 0xffu;
  const uint32_t color = (alpha << 24) | (a->color & 0x00ffffffu);
  const rt_omstate_t s = om_state(a->backface);
  // read what the unit reads (om_unit.cpp:84-101), merge, write what it writes
  const uint32_t zo = (vx_dcr(VX_DCR_OM_ZBUF_ADDR) << 6) + y * vx_dcr(VX_DCR_OM_ZBUF_PITCH) + 4u * x;
  const uint32_t co = (vx_dcr(VX_DCR_OM_CBUF_ADDR) << 6) + y * vx_dcr(VX_DCR_OM_CBUF_PITCH) + 4u * x;
  const bool need_ds = s.depth_test_on || s.stencil_on;
  const bool need_c = s.color_write && (s.color_read || s.blend_on);
  const uint32_t ds0 = need_ds ? A.ld_u32(zo) : 0u;
  uint32_t ds = ds0, c = need_c ? A.ld_u32(co) : 0u;
  const bool passed = gfx::om_write(s, c, ds, color, a->depth);
  if (need_ds && ds != ds0) A.st_u32(zo, ds);
  if (s.color_write && passed) A.st_u32(co, c);
}

}  // namespace

VX_MAIN(om_arg_t, arg, 256) {
  const uint32_t grid[2] = {arg->dst_width, arg->dst_height};
  return vx_spawn_threads(2u, grid, (const uint32_t*)nullptr,
                          [](const vx_task_t& t, om_arg_t* a) { om_pixel(t, a); }, arg);
}
