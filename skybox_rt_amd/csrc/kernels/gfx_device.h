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
  uint4 a, b, c;
  if constexpr (SCALAR) {  // one pointer: merged wide s_loads
    uint4 w[3];
    A.sld_u4n<3>(off, w);
    a = w[0]; b = w[1]; c = w[2];
  } else {
    a = A.ld_u4(off); b = A.ld_u4(off + 16); c = A.ld_u4(off + 32);
  }
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
  uint4 sw[SCALAR ? 8 : 1];
  if constexpr (SCALAR) A.sld_u4n<8>(off, sw);  // two s_load_dwordx16
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint4 v;
    if constexpr (SCALAR) v = sw[i]; else v = A.ld_u4(off + 16 * i);
    p.w[4 * i + 0] = (int32_t)v.x; p.w[4 * i + 1] = (int32_t)v.y;
    p.w[4 * i + 2] = (int32_t)v.z; p.w[4 * i + 3] = (int32_t)v.w;
  }
}

// TFixed<F> <- float on the device: RISC-V fcvt.w.s (rtz, saturating,
// NaN -> INT_MAX) semantics, as the reference's shader runs on RISC-V cores.
// Branch-free (no exec-mask branches per call): the value clamped into
// [-2^31, 2^31 - 128] (the largest float below 2^31) converts exactly as the
// in-range branch did; out-of-range and NaN inputs are then selected.
__device__ __forceinline__ int32_t fx_from_float_dev(float f, int frac) {
  const float x = f * (float)(1u << frac);
  const int32_t r = (int32_t)fminf(fmaxf(x, -2147483648.0f), 2147483520.0f);  // NaN -> -2^31
  return (x >= 2147483648.0f || x != x) ? INT32_MAX : r;
}
__device__ __forceinline__ float fx_to_float(int32_t d, int frac) {
  return (float)d * (1.0f / (float)(1u << frac));
}

// TextureWrap (graphics.cpp:35-53) for TFixed<23>; the three modes
// computed and selected (a wave-uniform mode: no branch per call)
__device__ __forceinline__ int32_t tex_wrap(int32_t d, uint32_t wrap) {
  const int32_t MASK = (1 << VX_TEX_FXD_FRAC) - 1;
  const int32_t mir = d ^ ((int32_t)((uint32_t)d << (31 - VX_TEX_FXD_FRAC)) >> 31);
  int32_t clp = d & -(int32_t)(d >= 0);
  clp |= ((MASK - clp) >> 31);
  const int32_t ret = wrap == VX_TEX_WRAP_REPEAT ? d : (wrap == VX_TEX_WRAP_MIRROR ? mir : clp);
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

// TextureSampler::read, lod 0 (graphics.cpp:253-314), for one texel format
// known at compile time: its stride (setup.cpp FormatStride) and unpack
// (unpack8888's case) are straight-line code, so a shade makes one format
// switch (tex_read) instead of one per texel fetch and unpack
template <uint32_t FMT>
__device__ __forceinline__ uint32_t fmt_fetch(const vx_arena& A, uint32_t base, uint32_t idx) {
  if constexpr (FMT == VX_TEX_FORMAT_A8R8G8B8) return A.ld_u32(base + 4 * idx);
  else if constexpr (FMT == VX_TEX_FORMAT_L8 || FMT == VX_TEX_FORMAT_A8) return A.ld_u8(base + idx);
  else return A.ld_u16(base + 2 * idx);
}
template <uint32_t FMT>
__device__ __forceinline__ uint32_t tex_read_fmt(const vx_arena& A, const DcState& s, int32_t u, int32_t v) {
  const uint32_t logw = s.logw, logh = s.logh;
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
    const uint32_t t00 = fmt_fetch<FMT>(A, s.tex_off, x0 + (y0 << logw));
    const uint32_t t01 = fmt_fetch<FMT>(A, s.tex_off, x1 + (y0 << logw));
    const uint32_t t10 = fmt_fetch<FMT>(A, s.tex_off, x0 + (y1 << logw));
    const uint32_t t11 = fmt_fetch<FMT>(A, s.tex_off, x1 + (y1 << logw));
    const uint32_t alpha = x0s & 0xff, beta = y0s & 0xff;
    uint32_t c0l, c0h, c1l, c1h, c2l, c2h, c3l, c3h;
    unpack8888(FMT, t00, &c0l, &c0h);
    unpack8888(FMT, t01, &c1l, &c1h);
    const uint32_t c01l = lerp8888(c0l, c1l, alpha), c01h = lerp8888(c0h, c1h, alpha);
    unpack8888(FMT, t10, &c2l, &c2h);
    unpack8888(FMT, t11, &c3l, &c3h);
    const uint32_t c23l = lerp8888(c2l, c3l, alpha), c23h = lerp8888(c2h, c3h, alpha);
    const uint32_t cl = lerp8888(c01l, c23l, beta), ch = lerp8888(c01h, c23h, beta);
    return (ch << 8) | cl;
  }
  const uint32_t uu = (uint32_t)tex_wrap(u, s.wrapu), vv = (uint32_t)tex_wrap(v, s.wrapv);
  const uint32_t x = uu >> (VX_TEX_FXD_FRAC - logw), y = vv >> (VX_TEX_FXD_FRAC - logh);
  uint32_t cl, ch;
  unpack8888(FMT, fmt_fetch<FMT>(A, s.tex_off, x + (y << logw)), &cl, &ch);
  return (ch << 8) | cl;
}
// any format: the record's own stride and the generic unpack (formats past
// the seven named ones)
__device__ __forceinline__ uint32_t tex_read_any(const vx_arena& A, const DcState& s, int32_t u,
                                                 int32_t v);
__device__ __forceinline__ uint32_t tex_read(const vx_arena& A, const DcState& s, int32_t u,
                                             int32_t v) {
  if (s.stride == 4 - 2 * (s.format != VX_TEX_FORMAT_A8R8G8B8) -
                     (s.format == VX_TEX_FORMAT_L8 || s.format == VX_TEX_FORMAT_A8)) {
    switch (s.format) {
    case VX_TEX_FORMAT_A8R8G8B8: return tex_read_fmt<VX_TEX_FORMAT_A8R8G8B8>(A, s, u, v);
    case VX_TEX_FORMAT_R5G6B5: return tex_read_fmt<VX_TEX_FORMAT_R5G6B5>(A, s, u, v);
    case VX_TEX_FORMAT_A1R5G5B5: return tex_read_fmt<VX_TEX_FORMAT_A1R5G5B5>(A, s, u, v);
    case VX_TEX_FORMAT_A4R4G4B4: return tex_read_fmt<VX_TEX_FORMAT_A4R4G4B4>(A, s, u, v);
    case VX_TEX_FORMAT_A8L8: return tex_read_fmt<VX_TEX_FORMAT_A8L8>(A, s, u, v);
    case VX_TEX_FORMAT_L8: return tex_read_fmt<VX_TEX_FORMAT_L8>(A, s, u, v);
    case VX_TEX_FORMAT_A8: return tex_read_fmt<VX_TEX_FORMAT_A8>(A, s, u, v);
    default: break;
    }
  }
  return tex_read_any(A, s, u, v);
}
__device__ __forceinline__ uint32_t tex_read_any(const vx_arena& A, const DcState& s, int32_t u,
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
// the rasterizer's coverage of pixel (x, y): all three edge values >= 0
// (inclusive, no top-left rule, graphics.cpp:813-825); the values to `e`
__device__ __forceinline__ bool covers(const int32_t* edges, uint32_t x, uint32_t y, int32_t e[3]) {
  e[0] = edge_eval(edges, x, y);
  e[1] = edge_eval(edges + 3, x, y);
  e[2] = edge_eval(edges + 6, x, y);
  return e[0] >= 0 && e[1] >= 0 && e[2] >= 0;
}

// The shader's tail from Q.24 barycentric weights dx (vertex 0), dy (vertex 1):
// INTERPOLATE / TEXTURING / MODULATE (draw3d/kernel.cpp:48-79).  Path-trace
// bounce hits enter here with MT barycentrics (oracle/gfx.c orc_shade_weights).
__device__ __forceinline__ uint32_t shade_weights(const vx_arena& A, const Prim& p,
                                                  const DcState& s, int32_t dx, int32_t dy,
                                                  uint32_t* depth = nullptr) {
  if (depth) *depth = (s.flags & RT_DC_DEPTH) ? (uint32_t)interp(p.attr(0), dx, dy) : 0u;
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
// ... from the three raw Q15.16 edge values at the fragment (GRADIENTS_SW,
// draw3d/kernel.cpp:37-44); *depth = interpolated Q7.24 z word
__device__ __forceinline__ uint32_t shade_edges(const vx_arena& A, const Prim& p, const DcState& s,
                                                int32_t F0, int32_t F1, int32_t F2,
                                                uint32_t* depth = nullptr) {
  const float f0 = fx_to_float(F0, 24), f1 = fx_to_float(F1, 24), f2 = fx_to_float(F2, 24);
  const float r = 1.0f / (f0 + f1 + f2);
  return shade_weights(A, p, s, fx_from_float_dev(r * f0, 24), fx_from_float_dev(r * f1, 24),
                       depth);
}
__device__ __forceinline__ uint32_t shade(const vx_arena& A, const Prim& p, const DcState& s,
                                          uint32_t x, uint32_t y) {
  return shade_edges(A, p, s, edge_eval(p.edge(0), x, y), edge_eval(p.edge(1), x, y),
                     edge_eval(p.edge(2), x, y));
}

// ---- output merger: graphics.cpp:320-636 + gpu_sw.h:100-168 (oracle/gfx.c
// orc_om_write), for a pixel whose colour and depth/stencil words live in
// registers of the thread that owns the pixel ----
__device__ __forceinline__ bool om_compare(uint32_t func, uint32_t a, uint32_t b) {
  switch (func) {
  case VX_OM_DEPTH_FUNC_NEVER: return false;
  case VX_OM_DEPTH_FUNC_LESS: return a < b;
  case VX_OM_DEPTH_FUNC_EQUAL: return a == b;
  case VX_OM_DEPTH_FUNC_LEQUAL: return a <= b;
  case VX_OM_DEPTH_FUNC_GREATER: return a > b;
  case VX_OM_DEPTH_FUNC_NOTEQUAL: return a != b;
  case VX_OM_DEPTH_FUNC_GEQUAL: return a >= b;
  default: return true;
  }
}
__device__ __forceinline__ uint32_t om_stencil_op(uint32_t op, uint32_t ref, uint32_t val) {
  switch (op) {
  case VX_OM_STENCIL_OP_ZERO: return 0;
  case VX_OM_STENCIL_OP_REPLACE: return ref;
  case VX_OM_STENCIL_OP_INCR: return (val < 0xff) ? (val + 1) : val;
  case VX_OM_STENCIL_OP_DECR: return (val > 0) ? (val - 1) : val;
  case VX_OM_STENCIL_OP_INVERT: return ~val;
  case VX_OM_STENCIL_OP_INCR_WRAP: return (val + 1) & 0xff;
  case VX_OM_STENCIL_OP_DECR_WRAP: return (val - 1) & 0xff;
  default: return val;
  }
}
__device__ __forceinline__ uint32_t div255(int x) { return (uint32_t)((x + (x >> 8)) >> 8); }
struct Argb {
  uint32_t a, r, g, b;
};
__device__ __forceinline__ Argb argb(uint32_t v) { return {v >> 24, (v >> 16) & 0xff, (v >> 8) & 0xff, v & 0xff}; }
__device__ __forceinline__ Argb mk(uint32_t a, uint32_t r, uint32_t g, uint32_t b) {
  return {a & 0xff, r & 0xff, g & 0xff, b & 0xff};
}
__device__ __forceinline__ Argb blend_factor(uint32_t f, Argb s, Argb d, Argb c) {
  switch (f) {
  case VX_OM_BLEND_FUNC_ZERO: return mk(0, 0, 0, 0);
  case VX_OM_BLEND_FUNC_ONE: return mk(0xff, 0xff, 0xff, 0xff);
  case VX_OM_BLEND_FUNC_SRC_RGB: return s;
  case VX_OM_BLEND_FUNC_ONE_MINUS_SRC_RGB: return mk(0xff - s.a, 0xff - s.r, 0xff - s.g, 0xff - s.b);
  case VX_OM_BLEND_FUNC_DST_RGB: return d;
  case VX_OM_BLEND_FUNC_ONE_MINUS_DST_RGB: return mk(0xff - d.a, 0xff - d.r, 0xff - d.g, 0xff - d.b);
  case VX_OM_BLEND_FUNC_SRC_A: return mk(s.a, s.a, s.a, s.a);
  case VX_OM_BLEND_FUNC_ONE_MINUS_SRC_A: return mk(0xff - s.a, 0xff - s.a, 0xff - s.a, 0xff - s.a);
  case VX_OM_BLEND_FUNC_DST_A: return mk(d.a, d.a, d.a, d.a);
  case VX_OM_BLEND_FUNC_ONE_MINUS_DST_A: return mk(0xff - d.a, 0xff - d.a, 0xff - d.a, 0xff - d.a);
  case VX_OM_BLEND_FUNC_CONST_RGB: return c;
  case VX_OM_BLEND_FUNC_ONE_MINUS_CONST_RGB: return mk(0xff - c.a, 0xff - c.r, 0xff - c.g, 0xff - c.b);
  case VX_OM_BLEND_FUNC_CONST_A: return mk(c.a, c.a, c.a, c.a);
  case VX_OM_BLEND_FUNC_ONE_MINUS_CONST_A: return mk(0xff - c.a, 0xff - c.r, 0xff - c.g, 0xff - c.b);
  case VX_OM_BLEND_FUNC_ALPHA_SAT: {
    const uint32_t f2 = s.a < (0xff - d.a) ? s.a : (0xff - d.a);
    return mk(0xff, f2, f2, f2);
  }
  default: return mk(0, 0, 0, 0);
  }
}
__device__ __forceinline__ uint32_t logic_op(uint32_t op, uint32_t s, uint32_t d) {
  switch (op) {
  case 0: return 0; case 1: return s & d; case 2: return s & ~d; case 3: return s;
  case 4: return ~s & d; case 5: return d; case 6: return s ^ d; case 7: return s | d;
  case 8: return ~(s | d); case 9: return ~(s ^ d); case 10: return ~d;
  case 11: return s | ~d; case 12: return ~s; case 13: return ~s | d;
  case 14: return ~(s & d); default: return 0xffffffffu;
  }
}
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ Argb blend_mode(uint32_t mode, uint32_t lop, Argb src, Argb dst, Argb s,
                                           Argb d, uint32_t srcv, uint32_t dstv) {
  switch (mode) {
  case VX_OM_BLEND_MODE_SUB:
    return mk(div255(imax((int)(src.a * s.a) - (int)(dst.a * d.a) + 0x80, 0)),
              div255(imax((int)(src.r * s.r) - (int)(dst.r * d.r) + 0x80, 0)),
              div255(imax((int)(src.g * s.g) - (int)(dst.g * d.g) + 0x80, 0)),
              div255(imax((int)(src.b * s.b) - (int)(dst.b * d.b) + 0x80, 0)));
  case VX_OM_BLEND_MODE_REV_SUB:
    return mk(div255(imax((int)(dst.a * d.a) - (int)(src.a * s.a) + 0x80, 0)),
              div255(imax((int)(dst.r * d.r) - (int)(src.r * s.r) + 0x80, 0)),
              div255(imax((int)(dst.g * d.g) - (int)(src.g * s.g) + 0x80, 0)),
              div255(imax((int)(dst.b * d.b) - (int)(src.b * s.b) + 0x80, 0)));
  case VX_OM_BLEND_MODE_MIN:
    return mk(imin(src.a, dst.a), imin(src.r, dst.r), imin(src.g, dst.g), imin(src.b, dst.b));
  case VX_OM_BLEND_MODE_MAX:
    return mk(imax(src.a, dst.a), imax(src.r, dst.r), imax(src.g, dst.g), imax(src.b, dst.b));
  case VX_OM_BLEND_MODE_LOGICOP:
    return argb(logic_op(lop, srcv, dstv));
  default:  // ADD
    return mk(div255(imin((int)(src.a * s.a + dst.a * d.a) + 0x80, 0xFF00)),
              div255(imin((int)(src.r * s.r + dst.r * d.r) + 0x80, 0xFF00)),
              div255(imin((int)(src.g * s.g + dst.g * d.g) + 0x80, 0xFF00)),
              div255(imin((int)(src.b * s.b + dst.b * d.b) + 0x80, 0xFF00)));
  }
}

// OutputMerger::write on register-resident pixel state (color, ds =
// stencil << 24 | depth); returns whether the depth/stencil test passed
__device__ __forceinline__ bool om_write(const rt_omstate_t& s, uint32_t& cbuf, uint32_t& ds_buf,
                                         uint32_t color, uint32_t depth) {
  const bool depth_on = s.depth_test_on != 0, stencil_on = s.stencil_on != 0;
  const bool blend_on = s.blend_on != 0;
  const uint32_t dst_ds = (depth_on || stencil_on) ? ds_buf : 0u;
  const uint32_t dst_color = (s.color_write && (s.color_read || blend_on)) ? cbuf : 0u;
  bool passed = true;
  uint32_t ds = 0;
  if (depth_on || stencil_on) {  // DepthTencil::test (graphics.cpp:564-596)
    const uint32_t depth_val = dst_ds & VX_OM_DEPTH_MASK;
    const uint32_t stencil_val = dst_ds >> VX_OM_DEPTH_BITS;
    const uint32_t depth_ref = depth & VX_OM_DEPTH_MASK;
    const uint32_t ref_m = s.stencil_ref & s.stencil_mask;
    const uint32_t val_m = stencil_val & s.stencil_mask;
    uint32_t op;
    passed = om_compare(s.stencil_func, ref_m, val_m);
    if (passed) {
      passed = om_compare(s.depth_func, depth_ref, depth_val);
      op = passed ? s.stencil_zpass : s.stencil_zfail;
    } else {
      op = s.stencil_fail;
    }
    const uint32_t sres = om_stencil_op(op, s.stencil_ref, stencil_val);
    ds = (sres << VX_OM_DEPTH_BITS) | depth_ref;
  }
  if (blend_on && passed) {  // Blender (graphics.cpp:622-636)
    const Argb src = argb(color), dst = argb(dst_color), cst = argb(s.blend_const);
    const Argb s_rgb = blend_factor(s.blend_src_rgb, src, dst, cst);
    const Argb s_a = blend_factor(s.blend_src_a, src, dst, cst);
    const Argb d_rgb = blend_factor(s.blend_dst_rgb, src, dst, cst);
    const Argb d_a = blend_factor(s.blend_dst_a, src, dst, cst);
    const Argb rgb = blend_mode(s.blend_mode_rgb, s.logic_op, src, dst, s_rgb, d_rgb, color, dst_color);
    const Argb a = blend_mode(s.blend_mode_a, s.logic_op, src, dst, s_a, d_a, color, dst_color);
    color = (a.a << 24) | (rgb.r << 16) | (rgb.g << 8) | rgb.b;
  }
  const uint32_t ds_wm = ((depth_on && passed && s.depth_writemask) ? VX_OM_DEPTH_MASK : 0u) |
                         (stencil_on ? (s.stencil_writemask << VX_OM_DEPTH_BITS) : 0u);
  if (ds_wm != 0) ds_buf = (dst_ds & ~ds_wm) | (ds & ds_wm);
  if (s.color_write && passed) cbuf = (dst_color & ~s.cbuf_writemask) | (color & s.cbuf_writemask);
  return passed;
}

}  // namespace gfx
