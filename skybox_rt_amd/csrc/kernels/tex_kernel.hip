// tex_kernel.hip -- the reference's texture regression kernel
// (tests/regression/tex/kernel.cpp) on gfx950: every destination pixel
// samples the texture through TextureSampler::read (graphics.cpp:253-314,
// restated in gfx_device.h) -- point, bilinear, or bilinear at lod and lod+1
// blended by `frac` (kernel.cpp:83-100) -- in any of the 7 texel formats and
// 3 wrap modes.  Pixel-exact with the reference's tex goldens through the
// oracle (oracle/tex.c).
//
// MI355X mapping: a byte-moving kernel, bound by HBM (4 B written per pixel;
// texels are read once from HBM and then hit L2/MALL).  A wave owns a
// group of 64*K pixels of a row (tex_common.h): lane l samples pixels l,
// l+64, ..., so each load/store instruction covers 64 consecutive pixels
// (per-lane runs of consecutive pixels made every instruction span K cache
// lines per lane and ran 2x slower), and the K samples of a lane are
// independent; 256-thread workgroups, the oversubscribed vx_spawn grid
// balances the groups.  The loop is
// specialised per texel format and filter (21 instances): with the stride
// and unpacking known at compile time a task's 4-32 texel loads are all
// issued before the first is consumed (a runtime format switch put a branch
// -- and an s_waitcnt vmcnt(0) -- after every load).
#include <hip/hip_runtime.h>

#include "gfx_device.h"
#include "tex_common.h"
#include "vx_spawn.h"

namespace {

struct TexLod {
  uint32_t base, logw, logh;  // mip level byte offset in the arena, log2 dims
};

struct TexFrame {
  vx_arena A;
  uint32_t dst, utab, vtab, width, gpr, frac, wrap;
  TexLod l0, l1;  // sampled level and the next one (trilinear)
};

template <typename P>
__device__ __forceinline__ TexLod lod_of(P a, uint32_t lod) {
  TexLod l;
  l.logw = (int32_t)a->logw - (int32_t)lod > 0 ? a->logw - lod : 0u;
  l.logh = (int32_t)a->logh - (int32_t)lod > 0 ? a->logh - lod : 0u;
  l.base = (uint32_t)a->tex_addr + a->mipoff[lod];
  return l;
}

template <uint32_t FMT>
constexpr uint32_t stride_of() {
  return FMT == VX_TEX_FORMAT_A8R8G8B8 ? 4u
         : (FMT == VX_TEX_FORMAT_L8 || FMT == VX_TEX_FORMAT_A8) ? 1u : 2u;
}

template <uint32_t FMT>
__device__ __forceinline__ uint32_t fetch(const vx_arena& A, uint32_t base, uint32_t idx) {
  constexpr uint32_t S = stride_of<FMT>();
  if constexpr (S == 4) return A.ld_u32(base + 4u * idx);
  else if constexpr (S == 2) return A.ld_u16(base + 2u * idx);
  else return A.ld_u8(base + idx);
}

// TextureWrap (graphics.cpp:35-53), branch-free over the wave-uniform mode
__device__ __forceinline__ uint32_t wrap_of(int32_t d, uint32_t wrap) {
  const int32_t MASK = (1 << VX_TEX_FXD_FRAC) - 1;
  int32_t clamp = d & -(int32_t)(d >= 0);
  clamp |= (MASK - clamp) >> 31;
  const int32_t mirror = d ^ ((int32_t)((uint32_t)d << (31 - VX_TEX_FXD_FRAC)) >> 31);
  const int32_t r = wrap == VX_TEX_WRAP_REPEAT ? d : wrap == VX_TEX_WRAP_MIRROR ? mirror : clamp;
  return (uint32_t)(r & MASK);
}

// TexAddressPoint / TexAddressLinear (graphics.cpp:124-186), split into the
// row part (from v: the same for every lane of a wave, which owns pixels of
// one row -- computed once, in scalar registers) and the column part (u)
struct Row {
  uint32_t r0, r1, beta;  // texel index of row y0 / y1, vertical blend weight
};
__device__ __forceinline__ Row point_row(const TexLod& L, uint32_t wrap, int32_t v) {
  Row r;
  r.r0 = (wrap_of(v, wrap) >> (VX_TEX_FXD_FRAC - L.logh)) << L.logw;
  r.r1 = r.r0;
  r.beta = 0;
  return r;
}
__device__ __forceinline__ Row linear_row(const TexLod& L, uint32_t wrap, int32_t v) {
  const int32_t dyh = ((1 << VX_TEX_FXD_FRAC) >> 1) >> L.logh;
  const uint32_t v0 = wrap_of((int32_t)((uint32_t)v - (uint32_t)dyh), wrap);
  const uint32_t v1 = wrap_of((int32_t)((uint32_t)v + (uint32_t)dyh), wrap);
  const uint32_t shv = VX_TEX_FXD_FRAC - L.logh;
  const uint32_t y0s = (v0 << 8) >> shv;
  Row r;
  r.r0 = (y0s >> 8) << L.logw;
  r.r1 = (v1 >> shv) << L.logw;
  r.beta = y0s & 0xff;
  return r;
}
struct Taps {
  uint32_t i00, i01, i10, i11, alpha, beta;
};
__device__ __forceinline__ uint32_t point_index(const TexLod& L, uint32_t wrap, int32_t u,
                                                const Row& R) {
  return (wrap_of(u, wrap) >> (VX_TEX_FXD_FRAC - L.logw)) + R.r0;
}
__device__ __forceinline__ Taps linear_taps(const TexLod& L, uint32_t wrap, int32_t u, const Row& R) {
  const int32_t dxh = ((1 << VX_TEX_FXD_FRAC) >> 1) >> L.logw;
  const uint32_t u0 = wrap_of((int32_t)((uint32_t)u - (uint32_t)dxh), wrap);
  const uint32_t u1 = wrap_of((int32_t)((uint32_t)u + (uint32_t)dxh), wrap);
  const uint32_t shu = VX_TEX_FXD_FRAC - L.logw;
  const uint32_t x0s = (u0 << 8) >> shu;
  const uint32_t x0 = x0s >> 8, x1 = u1 >> shu;
  Taps t;
  t.i00 = x0 + R.r0;
  t.i01 = x1 + R.r0;
  t.i10 = x0 + R.r1;
  t.i11 = x1 + R.r1;
  t.alpha = x0s & 0xff;
  t.beta = R.beta;
  return t;
}

// TexFilterPoint / TexFilterLinear (graphics.cpp:188-240)
template <uint32_t FMT>
__device__ __forceinline__ uint32_t filter_point(uint32_t t) {
  uint32_t l, h;
  gfx::unpack8888(FMT, t, &l, &h);
  return (h << 8) | l;
}
template <uint32_t FMT>
__device__ __forceinline__ uint32_t filter_linear(uint32_t t00, uint32_t t01, uint32_t t10,
                                                  uint32_t t11, uint32_t alpha, uint32_t beta) {
  uint32_t c0l, c0h, c1l, c1h, c2l, c2h, c3l, c3h;
  gfx::unpack8888(FMT, t00, &c0l, &c0h);
  gfx::unpack8888(FMT, t01, &c1l, &c1h);
  gfx::unpack8888(FMT, t10, &c2l, &c2h);
  gfx::unpack8888(FMT, t11, &c3l, &c3h);
  const uint32_t c01l = gfx::lerp8888(c0l, c1l, alpha), c01h = gfx::lerp8888(c0h, c1h, alpha);
  const uint32_t c23l = gfx::lerp8888(c2l, c3l, alpha), c23h = gfx::lerp8888(c2h, c3h, alpha);
  const uint32_t cl = gfx::lerp8888(c01l, c23l, beta), ch = gfx::lerp8888(c01h, c23h, beta);
  return (ch << 8) | cl;
}

// K pixels of one lane at one level: every texel load is issued before any
// is consumed (straight-line code, compile-time format and filter)
template <uint32_t FMT, bool LINEAR, uint32_t K>
__device__ __forceinline__ void sample(const TexFrame& F, const TexLod& L, const int32_t* u,
                                       int32_t v, uint32_t* c) {
  if constexpr (!LINEAR) {
    const Row R = point_row(L, F.wrap, v);
    uint32_t t[K];
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) t[j] = fetch<FMT>(F.A, L.base, point_index(L, F.wrap, u[j], R));
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) c[j] = filter_point<FMT>(t[j]);
  } else {
    const Row R = linear_row(L, F.wrap, v);
    Taps k[K];
    uint32_t t[K][4];
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) {
      k[j] = linear_taps(L, F.wrap, u[j], R);
      t[j][0] = fetch<FMT>(F.A, L.base, k[j].i00);
      t[j][1] = fetch<FMT>(F.A, L.base, k[j].i01);
      t[j][2] = fetch<FMT>(F.A, L.base, k[j].i10);
      t[j][3] = fetch<FMT>(F.A, L.base, k[j].i11);
    }
#pragma unroll
    for (uint32_t j = 0; j < K; ++j)
      c[j] = filter_linear<FMT>(t[j][0], t[j][1], t[j][2], t[j][3], k[j].alpha, k[j].beta);
  }
}

// kernel.cpp:83-112 for one task: pixels x0 + lane + 64 j (j < K) of a row
template <uint32_t FMT, uint32_t FILT>
__device__ __forceinline__ uint32_t run_task(const TexFrame& F, uint32_t task_id) {
  constexpr uint32_t K = TEX_PPT(FILT);
  // the group (and so the row) is the wave's: task ids of a chunk are the 64
  // consecutive ids of one group (num_tasks is a multiple of 64)
  const uint32_t grp = __builtin_amdgcn_readfirstlane(task_id >> 6), lane = task_id & 63u;
  const uint32_t y = grp / F.gpr;
  const uint32_t x0 = (grp - y * F.gpr) * TEX_GROUP(FILT) + lane;
  const int32_t v = (int32_t)F.A.sld<uint32_t>(F.vtab + 4u * y);
  int32_t u[K];
#pragma unroll
  for (uint32_t j = 0; j < K; ++j) u[j] = (int32_t)F.A.ld_u32(F.utab + 4u * (x0 + 64u * j));
  uint32_t c[K];
  sample<FMT, FILT != 0, K>(F, F.l0, u, v, c);
  if constexpr (FILT == 2) {
    uint32_t c1[K];
    sample<FMT, true, K>(F, F.l1, u, v, c1);
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) {  // Unpack8888 / Lerp8888 / Pack8888 (graphics.h:72-86)
      const uint32_t cl = gfx::lerp8888(c[j] & 0x00ff00ffu, c1[j] & 0x00ff00ffu, F.frac);
      const uint32_t ch =
          gfx::lerp8888((c[j] >> 8) & 0x00ff00ffu, (c1[j] >> 8) & 0x00ff00ffu, F.frac);
      c[j] = (ch << 8) | cl;
    }
  }
  const uint32_t o = F.dst + 4u * (y * F.width + x0);
  uint32_t n = 0;
#pragma unroll
  for (uint32_t j = 0; j < K; ++j)
    if (x0 + 64u * j < F.width) {
      F.A.st_u32(o + 256u * j, c[j]);
      ++n;
    }
  return n;
}

template <uint32_t FMT, uint32_t FILT>
__device__ __forceinline__ uint32_t run(const TexFrame& F, uint32_t num_tasks,
                                     const tex_kernel_arg_t* arg) {
  uint32_t pixels = 0;
  vx_spawn_tasks(
      num_tasks,
      [&](const vx_task_t& task, const tex_kernel_arg_t*) { pixels += run_task<FMT, FILT>(F, task.task_id); },
      arg);
  return pixels;
}

// TEX_FILTER: the filter this image is built for (one image per filter, so
// that the point and bilinear loops are not held to the trilinear loop's
// register budget); the host loads tex_kernel_f<filter>.vxbin
#ifndef TEX_FILTER
#define TEX_FILTER 0
#endif

template <uint32_t FMT>
__device__ __forceinline__ uint32_t by_filter(const TexFrame& F, uint32_t filter, uint32_t n,
                                              const tex_kernel_arg_t* arg) {
  (void)filter;  // the host launches the image matching arg->filter
  return run<FMT, TEX_FILTER>(F, n, arg);
}

}  // namespace

VX_MAIN(tex_kernel_arg_t, argp, TEX_BLOCK_THREADS) {
  // the argument block through the scalar cache (s_load), not flat loads
  const auto* arg = (const __attribute__((address_space(4))) tex_kernel_arg_t*)argp;
  TexFrame F;
  F.A = vx_arena::get();
  F.dst = (uint32_t)arg->dst_addr;
  F.utab = (uint32_t)arg->utab_addr;
  F.vtab = (uint32_t)arg->vtab_addr;
  F.width = arg->dst_width;
  F.gpr = (arg->dst_width + TEX_GROUP(TEX_FILTER) - 1) / TEX_GROUP(TEX_FILTER);
  F.frac = arg->frac;
  F.wrap = arg->wrap;
  F.l0 = lod_of(arg, arg->lod);
  F.l1 = lod_of(arg, arg->lod + 1 < VX_TEX_LOD_MAX ? arg->lod + 1 : VX_TEX_LOD_MAX);
  const uint32_t n = arg->num_tasks, f = arg->filter;
  uint32_t pixels;
  switch (arg->format) {  // one specialisation per texel format x filter
    case VX_TEX_FORMAT_A8R8G8B8: pixels = by_filter<VX_TEX_FORMAT_A8R8G8B8>(F, f, n, argp); break;
    case VX_TEX_FORMAT_R5G6B5: pixels = by_filter<VX_TEX_FORMAT_R5G6B5>(F, f, n, argp); break;
    case VX_TEX_FORMAT_A1R5G5B5: pixels = by_filter<VX_TEX_FORMAT_A1R5G5B5>(F, f, n, argp); break;
    case VX_TEX_FORMAT_A4R4G4B4: pixels = by_filter<VX_TEX_FORMAT_A4R4G4B4>(F, f, n, argp); break;
    case VX_TEX_FORMAT_A8L8: pixels = by_filter<VX_TEX_FORMAT_A8L8>(F, f, n, argp); break;
    case VX_TEX_FORMAT_L8: pixels = by_filter<VX_TEX_FORMAT_L8>(F, f, n, argp); break;
    default: pixels = by_filter<VX_TEX_FORMAT_A8>(F, f, n, argp); break;
  }
  vx_mpm_add(TEX_MPM_USER + TEX_STAT_PIXELS, pixels);
  return 0;
}
