/*
 * gfx.h -- shared pieces of the oracle's restatement of the reference's
 * fixed-point graphics arithmetic.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Every function cites the reference file:line it restates.  Where the
 * reference calls into the un-vendored cocogfx submodule (TFixed, ClipToHDC,
 * ClipToScreen, CGLTrace enums), the semantics are inferred and then pinned by
 * the golden images in tests/golden/ (tests/test_oracle_goldens.py).
 */
#ifndef ORACLE_GFX_H
#define ORACLE_GFX_H

#include <math.h>
#include <stdint.h>
#include "oracle.h"

/* ---- VX constants: hw/rtl/VX_types.vh:304-423 --------------------------- */
enum {
  VX_TEX_FORMAT_A8R8G8B8 = 0, VX_TEX_FORMAT_R5G6B5 = 1, VX_TEX_FORMAT_A1R5G5B5 = 2,
  VX_TEX_FORMAT_A4R4G4B4 = 3, VX_TEX_FORMAT_A8L8 = 4, VX_TEX_FORMAT_L8 = 5,
  VX_TEX_FORMAT_A8 = 6
};
enum { VX_TEX_FILTER_POINT = 0, VX_TEX_FILTER_BILINEAR = 1 };
enum { VX_TEX_WRAP_CLAMP = 0, VX_TEX_WRAP_REPEAT = 1, VX_TEX_WRAP_MIRROR = 2 };
enum {
  VX_OM_DEPTH_FUNC_ALWAYS = 0, VX_OM_DEPTH_FUNC_NEVER = 1, VX_OM_DEPTH_FUNC_LESS = 2,
  VX_OM_DEPTH_FUNC_LEQUAL = 3, VX_OM_DEPTH_FUNC_EQUAL = 4, VX_OM_DEPTH_FUNC_GEQUAL = 5,
  VX_OM_DEPTH_FUNC_GREATER = 6, VX_OM_DEPTH_FUNC_NOTEQUAL = 7
};
enum {
  VX_OM_STENCIL_OP_KEEP = 0, VX_OM_STENCIL_OP_ZERO = 1, VX_OM_STENCIL_OP_REPLACE = 2,
  VX_OM_STENCIL_OP_INCR = 3, VX_OM_STENCIL_OP_DECR = 4, VX_OM_STENCIL_OP_INVERT = 5,
  VX_OM_STENCIL_OP_INCR_WRAP = 6, VX_OM_STENCIL_OP_DECR_WRAP = 7
};
enum {
  VX_OM_BLEND_MODE_ADD = 0, VX_OM_BLEND_MODE_SUB = 1, VX_OM_BLEND_MODE_REV_SUB = 2,
  VX_OM_BLEND_MODE_MIN = 3, VX_OM_BLEND_MODE_MAX = 4, VX_OM_BLEND_MODE_LOGICOP = 5
};
enum {
  VX_OM_BLEND_FUNC_ZERO = 0, VX_OM_BLEND_FUNC_ONE = 1, VX_OM_BLEND_FUNC_SRC_RGB = 2,
  VX_OM_BLEND_FUNC_ONE_MINUS_SRC_RGB = 3, VX_OM_BLEND_FUNC_DST_RGB = 4,
  VX_OM_BLEND_FUNC_ONE_MINUS_DST_RGB = 5, VX_OM_BLEND_FUNC_SRC_A = 6,
  VX_OM_BLEND_FUNC_ONE_MINUS_SRC_A = 7, VX_OM_BLEND_FUNC_DST_A = 8,
  VX_OM_BLEND_FUNC_ONE_MINUS_DST_A = 9, VX_OM_BLEND_FUNC_CONST_RGB = 10,
  VX_OM_BLEND_FUNC_ONE_MINUS_CONST_RGB = 11, VX_OM_BLEND_FUNC_CONST_A = 12,
  VX_OM_BLEND_FUNC_ONE_MINUS_CONST_A = 13, VX_OM_BLEND_FUNC_ALPHA_SAT = 14
};
#define VX_OM_DEPTH_BITS   24
#define VX_OM_DEPTH_MASK   0x00ffffffu
#define VX_OM_STENCIL_MASK 0xffu
#define VX_TEX_FXD_FRAC    23   /* VX_TEX_DIM_BITS + VX_TEX_SUBPIXEL_BITS */

/* ---- cocogfx CGLTrace enums (inferred; pinned by goldens) ---------------
 * compare / stencil-op / blend-op: declaration order = the case order of
 * gfxutil.cpp:296-346 (GL order; depth_func 1 = LESS in tekkaman/box,
 * 3 = LEQUAL in evilskull; blend 4/5 = SRC_ALPHA/ONE_MINUS_SRC_ALPHA).
 * pixel formats: 3 = A8L8 and 4 = R5G6B5 (2 B/texel), 5 = A8R8G8B8 (4 B/texel).
 * filter: NEAREST = 1 (tekkaman min=1, mag=2).  address: WRAP = 0.
 * envmode: MODULATE = 3 (model texels x grey vertex colour).  The last three are settled by tekkaman_ref_128. */
#define CGL_COMPARE_NEVER 0
#define CGL_FILTER_NEAREST 1
#define CGL_ADDRESS_WRAP 0
#define CGL_ENVMODE_MODULATE 3

static inline uint32_t cgl_to_vx_compare(int c) {   /* gfxutil.cpp:296-311 toVXCompare */
  static const uint32_t m[8] = {VX_OM_DEPTH_FUNC_NEVER, VX_OM_DEPTH_FUNC_LESS,
    VX_OM_DEPTH_FUNC_EQUAL, VX_OM_DEPTH_FUNC_LEQUAL, VX_OM_DEPTH_FUNC_GREATER,
    VX_OM_DEPTH_FUNC_NOTEQUAL, VX_OM_DEPTH_FUNC_GEQUAL, VX_OM_DEPTH_FUNC_ALWAYS};
  return (c >= 0 && c < 8) ? m[c] : VX_OM_DEPTH_FUNC_ALWAYS;
}
static inline uint32_t cgl_to_vx_stencil_op(int c) { /* gfxutil.cpp:313-326 toVXStencilOp */
  static const uint32_t m[6] = {VX_OM_STENCIL_OP_KEEP, VX_OM_STENCIL_OP_REPLACE,
    VX_OM_STENCIL_OP_INCR, VX_OM_STENCIL_OP_DECR, VX_OM_STENCIL_OP_ZERO,
    VX_OM_STENCIL_OP_INVERT};
  return (c >= 0 && c < 6) ? m[c] : VX_OM_STENCIL_OP_KEEP;
}
static inline uint32_t cgl_to_vx_blend(int c) {      /* gfxutil.cpp:328-346 toVXBlendFunc */
  static const uint32_t m[11] = {VX_OM_BLEND_FUNC_ZERO, VX_OM_BLEND_FUNC_ONE,
    VX_OM_BLEND_FUNC_SRC_RGB, VX_OM_BLEND_FUNC_ONE_MINUS_SRC_RGB,
    VX_OM_BLEND_FUNC_SRC_A, VX_OM_BLEND_FUNC_ONE_MINUS_SRC_A,
    VX_OM_BLEND_FUNC_DST_A, VX_OM_BLEND_FUNC_ONE_MINUS_DST_A,
    VX_OM_BLEND_FUNC_DST_RGB, VX_OM_BLEND_FUNC_ONE_MINUS_DST_RGB,
    VX_OM_BLEND_FUNC_ALPHA_SAT};
  return (c >= 0 && c < 11) ? m[c] : VX_OM_BLEND_FUNC_ONE;
}
static inline int cgl_to_vx_format(int f) {          /* gfxutil.cpp:280-294 toVXFormat */
  switch (f) {
  case 1: return VX_TEX_FORMAT_A8;
  case 2: return VX_TEX_FORMAT_L8;
  case 3: return VX_TEX_FORMAT_A8L8;
  case 4: return VX_TEX_FORMAT_R5G6B5;
  case 5: return VX_TEX_FORMAT_A8R8G8B8;   /* 4 B/texel in the traces */
  default: return VX_TEX_FORMAT_A8R8G8B8;
  }
}
static inline uint32_t vx_format_stride(int f) {     /* graphics.cpp:55-70 */
  switch (f) {
  case VX_TEX_FORMAT_A8R8G8B8: return 4;
  case VX_TEX_FORMAT_L8: case VX_TEX_FORMAT_A8: return 1;
  default: return 2;
  }
}

/* ---- cocogfx TFixed<F> conversions -------------------------------------- */
/* float -> TFixed<F>: data = (int32)(f * 2^F), truncation toward zero.
 * Host-side (x86 cvttss2si) semantics for out-of-range values. */
static inline int32_t fx_from_float_host(float f, int frac) {
  float x = f * (float)(1u << frac);
  if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT32_MIN;
  return (int32_t)x;
}
/* Device-side (RISC-V fcvt.w.s, rtz) semantics: saturating, NaN -> INT_MAX. */
static inline int32_t fx_from_float_dev(float f, int frac) {
  float x = f * (float)(1u << frac);
  if (x != x) return INT32_MAX;
  if (x >= 2147483648.0f) return INT32_MAX;
  if (x < -2147483648.0f) return INT32_MIN;
  return (int32_t)x;
}
/* TFixed<F> -> float: data * 2^-F (int->float rounding, then exact scale) */
static inline float fx_to_float(int32_t d, int frac) {
  return (float)d * (1.0f / (float)(1u << frac));
}

/* ---- draw3d state derived from a drawcall (draw3d/main.cpp:216-344) ----- */
typedef struct {
  /* kernel_arg flags (main.cpp:336-344) */
  int depth_enabled, color_enabled, tex_enabled, tex_modulate;
  /* texture DCRs (main.cpp:286-331) */
  const uint8_t* tex_base;
  uint32_t tex_logw, tex_logh, tex_format, tex_filter, tex_wrapu, tex_wrapv;
  /* OM DCR derived state (graphics.cpp:534-620, gpu_sw.h:78-98) */
  uint32_t depth_func, depth_writemask;
  int depth_test_on, stencil_on, blend_on;
  uint32_t stencil_func, stencil_zpass, stencil_zfail, stencil_fail;
  uint32_t stencil_ref, stencil_mask, stencil_writemask;
  uint32_t blend_mode_rgb, blend_mode_a, blend_src_rgb, blend_src_a;
  uint32_t blend_dst_rgb, blend_dst_a, blend_const, logic_op;
  uint32_t cbuf_writemask;   /* expanded byte mask */
  int color_read, color_write;
} orc_dcstate_t;

void orc_dcstate_init(orc_dcstate_t* s, const orc_scene_t* scene,
                      const orc_drawcall_t* dc);

/* draw3d shader for one fragment (draw3d/kernel.cpp:232-279 with the
 * FIXEDPOINT_RASTERIZER macros at :46-79): F = raw Q15.16 edge values.
 * Returns ARGB8888; *depth = interpolated Q7.24 z raw word. */
uint32_t orc_shade(const orc_dcstate_t* s, const orc_rast_prim_t* p,
                   int32_t F0, int32_t F1, int32_t F2, uint32_t* depth);

/* The same shader from explicit Q.24 barycentric weights dx (vertex 0) and
 * dy (vertex 1) -- the INTERPOLATE/TEXTURING/MODULATE tail of
 * draw3d/kernel.cpp:48-79; used for path-trace bounce hits. */
uint32_t orc_shade_weights(const orc_dcstate_t* s, const orc_rast_prim_t* p,
                           int32_t dx, int32_t dy, uint32_t* depth);

/* the masked 24-bit depth word of a fragment with edge values F0..F2 */
uint32_t orc_vis_depth(const orc_rast_prim_t* p, int32_t F0, int32_t F1, int32_t F2);

/* primary visibility of one primitive at W x H (oracle/vis.c): covered-pixel
 * rectangle (x0 | x1 << 16, y0 | y1 << 16, inclusive; empty 0x0000ffff) and
 * depth-word lower bound */
typedef struct {
  uint32_t rx, ry, zmin;
  int any;
} orc_vis_prim_t;
void orc_vis_prim_compute(const orc_rast_prim_t* p, int ok, const int32_t bbox[4], uint32_t width,
                          uint32_t height, orc_vis_prim_t* out);
/* rt_vnode_t words ([n][16]: rx[4] ry[4] zmin[4] child[4]) over a tree given
 * by child references refs[n][4] (leaf refs index leaf_pids) */
int orc_vis_nodes(const int32_t* refs, uint32_t n, const int32_t* leaf_pids, uint32_t m,
                  const orc_vis_prim_t* by_pid, uint32_t np, uint32_t* vnodes);

/* OutputMerger::write (gpu_sw.h:100-168) on one pixel. Returns 1 if the
 * depth/stencil test passed (and colour was written if enabled). */
int orc_om_write(const orc_dcstate_t* s, uint32_t* cbuf_px, uint32_t* zbuf_px,
                 uint32_t color, uint32_t depth);

/* The OM regression app (tests/regression/om, see gfx.c): unit state from
 * the 18 OM DCR words, and the whole kernel over pre-cleared buffers. */
void orc_om_configure(orc_dcstate_t* s, const uint32_t dcr[18], int backface);
int orc_om_app(uint32_t width, uint32_t height, uint32_t num_tasks, uint32_t color,
               uint32_t depth, int backface, int blend_enable, const uint32_t dcr[18],
               uint32_t* cbuf, uint32_t* zbuf);

/* TextureSampler::read (graphics.cpp:253-314), lod 0. */
uint32_t orc_tex_read(const orc_dcstate_t* s, int32_t u, int32_t v);

/* Edge value a*x + b*y + c with int32 wrap (graphics.cpp:640-642 + the
 * incremental fixed-point adds of renderTile/renderQuad, which are exact). */
static inline int32_t orc_edge_eval(const int32_t e[3], uint32_t x, uint32_t y) {
  return (int32_t)((uint32_t)e[0] * x + (uint32_t)e[1] * y + (uint32_t)e[2]);
}

#endif
