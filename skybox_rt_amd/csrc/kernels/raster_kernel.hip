// raster_kernel.hip -- the reference's draw3d hot path itself on gfx950
// (the full raster-parity pipeline): per drawcall,
// tile binning, homogeneous fixed-point edge functions, the draw3d shader
// (fixed-point interpolation, R5G6B5/... bilinear sampler) and the output
// merger (depth/stencil test, blending, write masks), pixel-exact with the
// reference's golden images through the oracle (oracle/raster.c).
//
// MI355X mapping: one 256-thread workgroup per 32x32 raster tile (the
// reference's RASTER_TILE_LOGSIZE = 5 unit), each thread owning one 2x2 quad
// (the reference's stamp, graphics.cpp:840, kernel.cpp:73-79).  A pixel's
// colour and depth/stencil words stay in the owning thread's registers for
// the whole frame -- initialised to draw3d's clear values, written once -- so the order-dependent OM
// semantics of the reference (per-tile ascending primitive order,
// gpu_sw.h:38-61; drawcalls in order, draw3d/main.cpp:179) hold trivially.
// Binning (gfxutil.cpp:237-271) happens in the workgroup: each chunk of 256
// primitives is bbox-tested against the tile in parallel and compacted in
// order (ballot + mbcnt + a 4-wave prefix in LDS) into the tile's list; the
// listed primitives' records are wave-uniform and come in through the scalar
// cache.  One launch renders every drawcall of the frame.
#include <hip/hip_runtime.h>

#include "gfx_device.h"
#include "rt_common.h"
#include "vx_spawn.h"

#define RS_BLOCK 256

namespace {

constexpr int kWaves = RS_BLOCK / 64;

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

struct RsLds {
  uint32_t list[RS_BLOCK];   // the tile's primitives (global pids) of one chunk, in order
  uint32_t wave_n[kWaves];
};

struct Frame {
  vx_arena A;
  uint32_t prims, dcs, oms, bbox, cbuf, zbuf;
  uint32_t width, height, tiles_x, num_dc, clear_color, clear_depth;
};

__device__ __forceinline__ rt_omstate_t load_om(const vx_arena& A, uint32_t off) {
  rt_omstate_t s;
  uint32_t* w = reinterpret_cast<uint32_t*>(&s);
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // all 32 words (128 B)
    const uint4 v = A.sld_u4(off + 16 * i);
    w[4 * i + 0] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
  return s;
}

// the frame's drawcalls over one tile; col/ds = this thread's quad
__device__ __forceinline__ void render_tile(const Frame& F, uint32_t tile, RsLds& L, uint32_t col[4],
                                            uint32_t ds[4], uint32_t& frags) {
  const uint32_t tx = tile % F.tiles_x, ty = tile / F.tiles_x;
  const uint32_t x0 = tx << RT_TILE_LOG, y0 = ty << RT_TILE_LOG;
  const uint32_t q = threadIdx.x;
  const uint32_t qx = x0 + 2u * (q & 15u), qy = y0 + 2u * (q >> 4);
  const uint32_t w = threadIdx.x >> 6;
  for (uint32_t d = 0; d < F.num_dc; ++d) {
    const rt_omstate_t om = load_om(F.A, F.oms + 128u * d);
    const gfx::DcState st = gfx::load_dcstate<true>(F.A, F.dcs + 64u * d);
    for (uint32_t base = 0; base < om.prim_count; base += RS_BLOCK) {
      // bin: which primitives of this chunk touch the tile (bbox, pixels)
      const uint32_t i = base + threadIdx.x;
      bool ov = false;
      uint32_t g = 0;
      if (i < om.prim_count) {
        g = om.prim_offset + i;
        const uint2 bb = make_uint2(F.A.ld_u32(F.bbox + 8u * g), F.A.ld_u32(F.bbox + 8u * g + 4));
        const uint32_t bx0 = bb.x & 0xffffu, bx1 = bb.x >> 16, by0 = bb.y & 0xffffu, by1 = bb.y >> 16;
        ov = bx0 < bx1 && bx0 < x0 + 32u && bx1 > x0 && by0 < y0 + 32u && by1 > y0;
      }
      const uint64_t m = __ballot(ov);
      if (lane_id() == 0) L.wave_n[w] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t pre = 0, n = 0;
#pragma unroll
      for (int k = 0; k < kWaves; ++k) {
        const uint32_t c = L.wave_n[k];
        pre += (uint32_t)k < w ? c : 0u;
        n += c;
      }
      if (ov) {
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        L.list[pre + r] = g;
      }
      __syncthreads();
      // rasterize the listed primitives in order
      for (uint32_t k = 0; k < n; ++k) {
        const uint32_t pg = L.list[k];
        gfx::Prim p;
        gfx::load_prim<true>(F.A, F.prims + 128u * pg, p);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t x = qx + (j & 1u), y = qy + (j >> 1);
          const int32_t e0 = gfx::edge_eval(p.edge(0), x, y);
          const int32_t e1 = gfx::edge_eval(p.edge(1), x, y);
          const int32_t e2 = gfx::edge_eval(p.edge(2), x, y);
          // inclusive coverage, no top-left rule, viewport scissor
          // (graphics.cpp:813-825)
          if (x < F.width && y < F.height && e0 >= 0 && e1 >= 0 && e2 >= 0) {
            uint32_t z;
            const uint32_t c = gfx::shade_edges(F.A, p, st, e0, e1, e2, &z);
            gfx::om_write(om, col[j], ds[j], c, z);
            ++frags;
          }
        }
      }
      __syncthreads();  // the list is rebuilt for the next chunk
    }
  }
}

__device__ __forceinline__ void flush(int slot, uint32_t v) { vx_mpm_add(RT_MPM_USER + slot, v); }

}  // namespace

VX_MAIN(rt_kernel_arg_t, arg, RS_BLOCK) {
  __shared__ RsLds s_rs;
  Frame F;
  F.A = vx_arena::get();
  F.prims = (uint32_t)arg->prims_addr;
  F.dcs = (uint32_t)arg->dcs_addr;
  F.oms = (uint32_t)arg->oms_addr;
  F.bbox = (uint32_t)arg->bbox_addr;
  F.cbuf = (uint32_t)arg->cbuf_addr;
  F.zbuf = (uint32_t)arg->zbuf_addr;
  F.width = arg->width;
  F.height = arg->height;
  F.tiles_x = arg->tiles_x;
  F.num_dc = arg->num_drawcalls;
  F.clear_color = arg->clear_color;
  F.clear_depth = 0xffffffffu;
  uint32_t frags = 0, pixels = 0;
  uint32_t col[4], ds[4], qx = 0, qy = 0;
  // task = one 2x2 quad (the reference's stamp); a workgroup step = one tile
  const int rc = vx_spawn_tasks_block(
      arg->num_tasks,
      [&](const vx_task_t& task, bool valid, const Frame* f) {
        const uint32_t tile = task.blockIdx.x / RS_BLOCK, q = task.blockIdx.x % RS_BLOCK;
        qx = ((tile % f->tiles_x) << RT_TILE_LOG) + 2u * (q & 15u);
        qy = ((tile / f->tiles_x) << RT_TILE_LOG) + 2u * (q >> 4);
        // the frame starts from draw3d's clears (main.cpp:478-490: colour
        // 0xff000000, depth/stencil 0xffffffff), fused here: no read-back
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t px = qx + (j & 1u), py = qy + (j >> 1);
          col[j] = f->clear_color;
          ds[j] = f->clear_depth;
          pixels += valid && px < f->width && py < f->height;
        }
      },
      [&](uint32_t step, const Frame* f) {
        render_tile(*f, step, s_rs, col, ds, frags);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {  // ... and written once
          const uint32_t px = qx + (j & 1u), py = qy + (j >> 1);
          if (px < f->width && py < f->height) {
            const uint32_t o = 4u * (py * f->width + px);
            f->A.st_u32(f->cbuf + o, col[j]);
            f->A.st_u32(f->zbuf + o, ds[j]);
          }
        }
      },
      &F);
  flush(RT_STAT_PRIMARY, pixels);
  flush(RT_STAT_SHADED, frags);
  return rc;
}
