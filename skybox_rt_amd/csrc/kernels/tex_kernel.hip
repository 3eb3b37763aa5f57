// tex_kernel.hip -- the reference's texture regression kernel
// (tests/regression/tex/kernel.cpp) on gfx950: every destination pixel
// samples the texture through TextureSampler::read (graphics.cpp:253-314,
// restated in gfx_device.h) -- point, bilinear, or bilinear at lod and lod+1
// blended by `frac` (kernel.cpp:83-100) -- in any of the 7 texel formats and
// 3 wrap modes.  Pixel-exact with the reference's tex goldens through the
// oracle (oracle/tex.c).
//
// MI355X mapping: a byte-moving kernel, bound by HBM (4 B written per pixel;
// texels are read once from HBM and then hit L2/MALL).  A task is 4
// consecutive pixels of a row: one 16-B utab load, 4 samples, one 16-B
// buffer store, so a wave writes 1 KiB contiguous; 256-thread workgroups,
// the oversubscribed vx_spawn grid balances the rows.
#include <hip/hip_runtime.h>

#include "gfx_device.h"
#include "tex_common.h"
#include "vx_spawn.h"

namespace {

struct TexFrame {
  vx_arena A;
  uint32_t dst, utab, vtab, width, qpr, frac, filter;
  gfx::DcState s0, s1;  // sampler state at lod and at lod + 1 (trilinear)
};

__device__ __forceinline__ gfx::DcState lod_state(const tex_kernel_arg_t* a, uint32_t lod) {
  gfx::DcState s;
  s.flags = 0;
  s.logw = (int32_t)a->logw - (int32_t)lod > 0 ? a->logw - lod : 0u;
  s.logh = (int32_t)a->logh - (int32_t)lod > 0 ? a->logh - lod : 0u;
  s.format = a->format;
  s.filter = a->filter ? VX_TEX_FILTER_BILINEAR : VX_TEX_FILTER_POINT;
  s.wrapu = a->wrap;
  s.wrapv = a->wrap;
  s.stride = a->format == VX_TEX_FORMAT_A8R8G8B8 ? 4u
             : (a->format == VX_TEX_FORMAT_L8 || a->format == VX_TEX_FORMAT_A8) ? 1u : 2u;
  s.tex_off = (uint32_t)a->tex_addr + a->mipoff[lod];
  return s;
}

__device__ __forceinline__ uint32_t tex_pixel(const TexFrame& F, int32_t u, int32_t v) {
  const uint32_t t0 = gfx::tex_read(F.A, F.s0, u, v);
  if (F.filter != 2) return t0;
  const uint32_t t1 = gfx::tex_read(F.A, F.s1, u, v);
  // Unpack8888 / Lerp8888 / Pack8888 (graphics.h:72-86)
  const uint32_t cl = gfx::lerp8888(t0 & 0x00ff00ffu, t1 & 0x00ff00ffu, F.frac);
  const uint32_t ch = gfx::lerp8888((t0 >> 8) & 0x00ff00ffu, (t1 >> 8) & 0x00ff00ffu, F.frac);
  return (ch << 8) | cl;
}

}  // namespace

VX_MAIN(tex_kernel_arg_t, arg, TEX_BLOCK_THREADS) {
  TexFrame F;
  F.A = vx_arena::get();
  F.dst = (uint32_t)arg->dst_addr;
  F.utab = (uint32_t)arg->utab_addr;
  F.vtab = (uint32_t)arg->vtab_addr;
  F.width = arg->dst_width;
  F.qpr = (arg->dst_width + TEX_PIXELS_PER_TASK - 1) / TEX_PIXELS_PER_TASK;
  F.frac = arg->frac;
  F.filter = arg->filter;
  F.s0 = lod_state(arg, arg->lod);
  F.s1 = lod_state(arg, arg->lod + 1 < VX_TEX_LOD_MAX ? arg->lod + 1 : VX_TEX_LOD_MAX);
  const bool vec = (F.width % TEX_PIXELS_PER_TASK) == 0;
  uint32_t pixels = 0;
  const int rc = vx_spawn_tasks(
      arg->num_tasks,
      [&](const vx_task_t& task, const tex_kernel_arg_t*) {
        const uint32_t y = task.task_id / F.qpr;
        const uint32_t x0 = (task.task_id - y * F.qpr) * TEX_PIXELS_PER_TASK;
        const int32_t v = (int32_t)F.A.ld_u32(F.vtab + 4u * y);
        const uint4 u = F.A.ld_u4(F.utab + 4u * x0);
        const uint32_t c0 = tex_pixel(F, (int32_t)u.x, v), c1 = tex_pixel(F, (int32_t)u.y, v);
        const uint32_t c2 = tex_pixel(F, (int32_t)u.z, v), c3 = tex_pixel(F, (int32_t)u.w, v);
        const uint32_t o = F.dst + 4u * (y * F.width + x0);
        if (vec) {
          __builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) uint32_t){c0, c1, c2, c3},
                                                 F.A.r, o, 0, 0);
          pixels += 4;
        } else {
          const uint32_t c[4] = {c0, c1, c2, c3};
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            if (x0 + j < F.width) {
              F.A.st_u32(o + 4u * j, c[j]);
              ++pixels;
            }
        }
      },
      arg);
  vx_mpm_add(TEX_MPM_USER + TEX_STAT_PIXELS, pixels);
  return rc;
}
