// gfx_device.h -- device library standing in for the Skybox fixed-function
// texture and shading path, for HIP kernel programs.
//
// The reference executes these in hardware units driven by vx_tex / vx_om
// (sim/simx/tex_unit.cpp, om_unit.cpp) or in the software fallback
// (draw3d/gpu_sw.h); the arithmetic lives in sim/common/graphics.cpp and the
// draw3d shader macros (draw3d/kernel.cpp:16-79).  Restated here as inline
// device functions with bit-identical integer/float behaviour (pinned through
// the oracle, which matches the reference's golden images exactly).  Records
// are fetched from the arena with buffer loads (vx_arena) into registers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "VX_types.h"
#include "rt_common.h"
#include "vx_spawn.h"

namespace gfx {

// rt_dcstate_t in registers
struct DcState {
  uint32_t flags, logw, logh, format, filter, wrapu, wrapv, stride, tex_off;
};

// SCALAR = true: `off` is wave-uniform and the record lands in SGPRs
template <bool SCALAR = false>
__device__ __forceinline__ DcState load_dcstate(const vx_arena& A, uint32_t off) {
  const uint4 a = SCALAR ? A.sld_u4(off) : A.ld_u4(off);
  const uint4 b = SCALAR ? A.sld_u4(off + 16) : A.ld_u4(off + 16);
  const uint4 c = SCALAR ? A.sld_u4(off + 32) : A.ld_u4(off + 32);
  DcState s;
  s.flags = a.x; s.logw = a.y; s.logh = a.z; s.format = a.w;
  s.filter = b.x; s.wrapu = b.y; s.wrapv = b.z; s.stride = b.w;
  s.tex_off = c.x;  // tex_addr low word: arena offsets are < 4 GiB
  return s;
}

// rt_prim_t in registers (32 words: edges 0-8, attribs 9-29, dc 30)
struct Prim {
  int32_t w[32];
  __device__ __forceinline__ const int32_t* edge(int i) const { return &w[3 * i]; }
  __device__ __forceinline__ const int32_t* attr(int k) const { return &w[9 + 3 * k]; }
  __device__ __forceinline__ uint32_t dc() const { return (uint32_t)w[30]; }
};

template <bool SCALAR = false>
__device__ __forceinline__ void load_prim(const vx_arena& A, uint32_t off, Prim& p) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 v = SCALAR ? A.sld_u4(off + 16 * i) : A.ld_u4(off + 16 * i);
    p.w[4 * i + 0] = (int32_t)v.x; p.w[4 * i + 1] = (int32_t)v.y;
    p.w[4 * i + 2] = (int32_t)v.z; p.w[4 * i + 3] = (int32_t)v.w;
  }
}

// TFixed<F> <- float on the device: RISC-V fcvt.w.s (rtz, saturating,
// NaN -> INT_MAX) semantics, as the reference's shader runs on RISC-V cores.
__device__ __forceinline__ int32_t fx_from_float_dev(float f, int frac) {
  const float x = f * (float)(1u << frac);
  if (x != x) return INT32_MAX;
  if (x >= 2147483648.0f) return INT32_MAX;
  if (x < -2147483648.0f) return INT32_MIN;
  return (int32_t)x;
}
__device__ __forceinline__ float fx_to_float(int32_t d, int frac) {
  return (float)d * (1.0f / (float)(1u << frac));
}

// TextureWrap (graphics.cpp:35-53) for TFixed<23>
__device__ __forceinline__ int32_t tex_wrap(int32_t d, uint32_t wrap) {
  const int32_t MASK = (1 << VX_TEX_FXD_FRAC) - 1;
  int32_t ret;
  if (wrap == VX_TEX_WRAP_REPEAT) {
    ret = d;
  } else if (wrap == VX_TEX_WRAP_MIRROR) {
    ret = d ^ ((int32_t)((uint32_t)d << (31 - VX_TEX_FXD_FRAC)) >> 31);
  } else {
    ret = d & -(int32_t)(d >= 0);
    ret |= ((MASK - ret) >> 31);
  }
  return ret & MASK;
}

// Unpack8888 per format (graphics.cpp:72-122)
__device__ __forceinline__ void unpack8888(uint32_t format, uint32_t t, uint32_t* lo, uint32_t* hi) {
  uint32_t r, g, b, a;
  switch (format) {
  case VX_TEX_FORMAT_R5G6B5:
    r = ((t >> 8) & 0xf8) | ((t >> 13) & 0x07);
    g = ((t >> 3) & 0xfc) | ((t >> 9) & 0x03);
    b = ((t << 3) & 0xf8) | ((t >> 2) & 0x07);
    a = 0xff;
    break;
  case VX_TEX_FORMAT_A1R5G5B5:
    r = ((t >> 7) & 0xf8) | ((t >> 12) & 0x07);
    g = ((t >> 2) & 0xf8) | ((t >> 7) & 0x07);
    b = ((t << 3) & 0xf8) | ((t >> 2) & 0x07);
    a = (uint32_t)(((int32_t)(t << 16)) >> 31) & 0xff;
    break;
  case VX_TEX_FORMAT_A4R4G4B4:
    r = ((t >> 4) & 0xf0) | ((t >> 8) & 0x0f);
    g = ((t >> 0) & 0xf0) | ((t >> 4) & 0x0f);
    b = ((t << 4) & 0xf0) | ((t >> 0) & 0x0f);
    a = ((t >> 8) & 0xf0) | ((t >> 12) & 0x0f);
    break;
  case VX_TEX_FORMAT_A8L8:
    r = t & 0xff; g = r; b = r; a = (t >> 8) & 0xff;
    break;
  case VX_TEX_FORMAT_L8:
    r = t & 0xff; g = r; b = r; a = 0xff;
    break;
  case VX_TEX_FORMAT_A8:
    r = 0xff; g = 0xff; b = 0xff; a = t & 0xff;
    break;
  default:
    r = (t >> 16) & 0xff; g = (t >> 8) & 0xff; b = t & 0xff; a = t >> 24;
    break;
  }
  *lo = (r << 16) + b;
  *hi = (a << 16) + g;
}

__device__ __forceinline__ uint32_t lerp8888(uint32_t a, uint32_t b, uint32_t f) {
  const uint32_t p = a * (0xff - f) + b * f + 0x00800080u;   // graphics.h:82-86
  const uint32_t q = (p >> 8) & 0x00ff00ffu;
  return ((p + q) >> 8) & 0x00ff00ffu;
}

__device__ __forceinline__ uint32_t fetch_texel(const vx_arena& A, uint32_t base, uint32_t idx,
                                                uint32_t stride) {
  if (stride == 2) return A.ld_u16(base + 2 * idx);
  if (stride == 4) return A.ld_u32(base + 4 * idx);
  return A.ld_u8(base + idx);
}

// TextureSampler::read, lod 0 (graphics.cpp:253-314)
__device__ __forceinline__ uint32_t tex_read(const vx_arena& A, const DcState& s, int32_t u,
                                             int32_t v) {
  const uint32_t logw = s.logw, logh = s.logh, fmt = s.format, stride = s.stride;
  if (s.filter == VX_TEX_FILTER_BILINEAR) {
    const int32_t half = (1 << VX_TEX_FXD_FRAC) >> 1;
    const int32_t dxh = half >> logw, dyh = half >> logh;
    const uint32_t u0 = (uint32_t)tex_wrap((int32_t)((uint32_t)u - (uint32_t)dxh), s.wrapu);
    const uint32_t u1 = (uint32_t)tex_wrap((int32_t)((uint32_t)u + (uint32_t)dxh), s.wrapu);
    const uint32_t v0 = (uint32_t)tex_wrap((int32_t)((uint32_t)v - (uint32_t)dyh), s.wrapv);
    const uint32_t v1 = (uint32_t)tex_wrap((int32_t)((uint32_t)v + (uint32_t)dyh), s.wrapv);
    const uint32_t shu = VX_TEX_FXD_FRAC - logw, shv = VX_TEX_FXD_FRAC - logh;
    const uint32_t x0s = (u0 << 8) >> shu, y0s = (v0 << 8) >> shv;
    const uint32_t x0 = x0s >> 8, y0 = y0s >> 8, x1 = u1 >> shu, y1 = v1 >> shv;
    const uint32_t t00 = fetch_texel(A, s.tex_off, x0 + (y0 << logw), stride);
    const uint32_t t01 = fetch_texel(A, s.tex_off, x1 + (y0 << logw), stride);
    const uint32_t t10 = fetch_texel(A, s.tex_off, x0 + (y1 << logw), stride);
    const uint32_t t11 = fetch_texel(A, s.tex_off, x1 + (y1 << logw), stride);
    const uint32_t alpha = x0s & 0xff, beta = y0s & 0xff;
    uint32_t c0l, c0h, c1l, c1h, c2l, c2h, c3l, c3h;
    unpack8888(fmt, t00, &c0l, &c0h);
    unpack8888(fmt, t01, &c1l, &c1h);
    const uint32_t c01l = lerp8888(c0l, c1l, alpha), c01h = lerp8888(c0h, c1h, alpha);
    unpack8888(fmt, t10, &c2l, &c2h);
    unpack8888(fmt, t11, &c3l, &c3h);
    const uint32_t c23l = lerp8888(c2l, c3l, alpha), c23h = lerp8888(c2h, c3h, alpha);
    const uint32_t cl = lerp8888(c01l, c23l, beta), ch = lerp8888(c01h, c23h, beta);
    return (ch << 8) | cl;
  }
  const uint32_t uu = (uint32_t)tex_wrap(u, s.wrapu), vv = (uint32_t)tex_wrap(v, s.wrapv);
  const uint32_t x = uu >> (VX_TEX_FXD_FRAC - logw), y = vv >> (VX_TEX_FXD_FRAC - logh);
  uint32_t cl, ch;
  unpack8888(fmt, fetch_texel(A, s.tex_off, x + (y << logw), stride), &cl, &ch);
  return (ch << 8) | cl;
}

// imadd (draw3d/kernel.cpp:48-51) and INTERPOLATE (:56-59)
__device__ __forceinline__ int32_t imadd24(int32_t a, int32_t b, int32_t c) {
  const int32_t p = (int32_t)(((int64_t)a * (int64_t)b) >> 24);
  return (int32_t)((uint32_t)p + (uint32_t)c);
}
__device__ __forceinline__ int32_t interp(const int32_t* at, int32_t dx, int32_t dy) {
  return imadd24(at[1], dy, imadd24(at[0], dx, at[2]));
}
__device__ __forceinline__ uint32_t mul8(int32_t d, uint32_t c) {
  return (((uint32_t)d * c) >> 24) & 0xff;
}

// edge value a*x + b*y + c with int32 wrap (graphics.cpp:640-642)
__device__ __forceinline__ int32_t edge_eval(const int32_t* e, uint32_t x, uint32_t y) {
  return (int32_t)((uint32_t)e[0] * x + (uint32_t)e[1] * y + (uint32_t)e[2]);
}

// The shader's tail from Q.24 barycentric weights dx (vertex 0), dy (vertex 1):
// INTERPOLATE / TEXTURING / MODULATE (draw3d/kernel.cpp:48-79).  Path-trace
// bounce hits enter here with MT barycentrics (oracle/gfx.c orc_shade_weights).
__device__ __forceinline__ uint32_t shade_weights(const vx_arena& A, const Prim& p,
                                                  const DcState& s, int32_t dx, int32_t dy) {
  int32_t cr = 1 << 24, cg = 1 << 24, cb = 1 << 24, ca = 1 << 24;
  if (s.flags & RT_DC_COLOR) {
    cr = interp(p.attr(1), dx, dy);
    cg = interp(p.attr(2), dx, dy);
    cb = interp(p.attr(3), dx, dy);
    ca = interp(p.attr(4), dx, dy);
  }
  if (s.flags & RT_DC_TEX) {
    const int32_t u = interp(p.attr(5), dx, dy);
    const int32_t v = interp(p.attr(6), dx, dy);
    const uint32_t tc = tex_read(A, s, u >> 1, v >> 1);  // TFixed<24> -> TFixed<23>
    if (s.flags & RT_DC_MODULATE) {
      return (mul8(ca, tc >> 24) << 24) | (mul8(cr, (tc >> 16) & 0xff) << 16) |
             (mul8(cg, (tc >> 8) & 0xff) << 8) | mul8(cb, tc & 0xff);
    }
    return tc;
  }
  return (mul8(ca, 255) << 24) | (mul8(cr, 255) << 16) | (mul8(cg, 255) << 8) | mul8(cb, 255);
}

// draw3d shader for one fragment at pixel (x, y) of primitive p
// (draw3d/kernel.cpp:232-279; GRADIENTS_SW reinterprets Q15.16 as Q7.24).
__device__ __forceinline__ uint32_t shade(const vx_arena& A, const Prim& p, const DcState& s,
                                          uint32_t x, uint32_t y) {
  const int32_t F0 = edge_eval(p.edge(0), x, y);
  const int32_t F1 = edge_eval(p.edge(1), x, y);
  const int32_t F2 = edge_eval(p.edge(2), x, y);
  const float f0 = fx_to_float(F0, 24), f1 = fx_to_float(F1, 24), f2 = fx_to_float(F2, 24);
  const float r = 1.0f / (f0 + f1 + f2);
  return shade_weights(A, p, s, fx_from_float_dev(r * f0, 24), fx_from_float_dev(r * f1, 24));
}

}  // namespace gfx
