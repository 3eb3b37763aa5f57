/*
 * gfx.c -- oracle restatement of the reference's fixed-point setup, shader,
 * texture sampler and output merger.  TEST INFRASTRUCTURE ONLY (oracle.h).
 */
#include "gfx.h"

#include <string.h>

/* ---- cocogfx ClipToHDC / ClipToScreen (inferred) ------------------------
 * Called by gfxutil.cpp:150-152 / :164-166 with (left,right,top,bottom) =
 * (0,width,0,height): HDC = (x_s*w, y_s*w, z_s*w, w) with
 * x_s = x/w * (r-l)/2 + (r+l)/2 and y measured from `top`, so framebuffer
 * row 0 is NDC y = -1 (confirmed by triangle_ref_8.png: apex at the top of
 * the vertically flipped PNG, draw3d/main.cpp:385-386). */
static void clip_to_hdc(float out[4], const float in[4], float l, float r,
                        float t, float b, float n, float f) {
  const float sx = (r - l) * 0.5f, cx = (r + l) * 0.5f;
  const float sy = (b - t) * 0.5f, cy = (b + t) * 0.5f;
  const float sz = (f - n) * 0.5f, cz = (f + n) * 0.5f;
  out[0] = in[0] * sx + in[3] * cx;
  out[1] = in[1] * sy + in[3] * cy;
  out[2] = in[2] * sz + in[3] * cz;
  out[3] = in[3];
}

static void clip_to_screen(float out[4], const float in[4], float l, float r,
                           float t, float b, float n, float f) {
  const float sx = (r - l) * 0.5f, cx = (r + l) * 0.5f;
  const float sy = (b - t) * 0.5f, cy = (b + t) * 0.5f;
  const float sz = (f - n) * 0.5f, cz = (f + n) * 0.5f;
  const float rhw = 1.0f / in[3];
  out[0] = (in[0] * rhw) * sx + cx;
  out[1] = (in[1] * rhw) * sy + cy;
  out[2] = (in[2] * rhw) * sz + cz;
  out[3] = rhw;
}

/* EdgeEquation, gfxutil.cpp:35-75 (v = HDC x,y,_,w). */
static int edge_equation(float e[3][3], const float* v0, const float* v1,
                         const float* v2) {
  const float a0 = (v1[1] * v2[3]) - (v2[1] * v1[3]);
  const float a1 = (v2[1] * v0[3]) - (v0[1] * v2[3]);
  const float a2 = (v0[1] * v1[3]) - (v1[1] * v0[3]);
  const float b0 = (v2[0] * v1[3]) - (v1[0] * v2[3]);
  const float b1 = (v0[0] * v2[3]) - (v2[0] * v0[3]);
  const float b2 = (v1[0] * v0[3]) - (v0[0] * v1[3]);
  const float c0 = (v1[0] * v2[1]) - (v2[0] * v1[1]);
  const float c1 = (v2[0] * v0[1]) - (v0[0] * v2[1]);
  const float c2 = (v0[0] * v1[1]) - (v1[0] * v0[1]);
  e[0][0] = a0; e[0][1] = b0; e[0][2] = c0;
  e[1][0] = a1; e[1][1] = b1; e[1][2] = c1;
  e[2][0] = a2; e[2][1] = b2; e[2][2] = c2;
  const float det = c0 * v0[3] + c1 * v1[3] + c2 * v2[3];
  if (det < 0) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) e[i][j] *= -1.0f;
  }
  return det != 0;
}

int orc_setup_prim(const float* v, uint32_t width, uint32_t height,
                   float znear, float zfar, orc_rast_prim_t* out,
                   int32_t bbox[4]) {
  const float* p[3] = {v, v + 10, v + 20};
  float ph[3][4], ps[3][4], e[3][3];
  for (int i = 0; i < 3; ++i)
    clip_to_hdc(ph[i], p[i], 0.0f, (float)width, 0.0f, (float)height, znear, zfar);
  memset(out, 0, sizeof(*out));
  if (!edge_equation(e, ph[0], ph[1], ph[2]))
    return 1;                                   /* gfxutil.cpp:155-159 */
  for (int i = 0; i < 3; ++i)
    clip_to_screen(ps[i], p[i], 0.0f, (float)width, 0.0f, (float)height, znear, zfar);
  {                                             /* gfxutil.cpp:168-192 */
    float l = ps[0][0], r = ps[0][0], t = ps[0][1], b = ps[0][1];
    for (int i = 1; i < 3; ++i) {
      l = fminf(l, ps[i][0]); r = fmaxf(r, ps[i][0]);
      t = fminf(t, ps[i][1]); b = fmaxf(b, ps[i][1]);
    }
    int32_t L = (int32_t)floorf(l), R = (int32_t)ceilf(r);
    int32_t T = (int32_t)floorf(t), B = (int32_t)ceilf(b);
    bbox[0] = L > 0 ? L : 0;
    bbox[1] = R < (int32_t)width ? R : (int32_t)width;
    bbox[2] = T > 0 ? T : 0;
    bbox[3] = B < (int32_t)height ? B : (int32_t)height;
  }
  /* half-pixel offset, gfxutil.cpp:211-214 */
  for (int i = 0; i < 3; ++i)
    e[i][2] += e[i][0] * 0.5f + e[i][1] * 0.5f;
  /* EdgeToFixed, gfxutil.cpp:79-96 (called at :217) */
  {
    float m = fabsf(e[0][0]);
    const float c[5] = {fabsf(e[1][0]), fabsf(e[2][0]), fabsf(e[0][1]),
                        fabsf(e[1][1]), fabsf(e[2][1])};
    for (int i = 0; i < 5; ++i) m = (c[i] > m) ? c[i] : m;
    const float scale = 1.0f / m;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        out->edges[i][j] = fx_from_float_host(e[i][j] * scale, 16);
  }
  /* ATTRIBUTE_DELTA, gfxutil.cpp:204-207,224-230: z uses screen z, the rest raw */
  {
    float a[7][3];
    for (int i = 0; i < 3; ++i) {
      a[0][i] = ps[i][2];
      a[1][i] = p[i][4]; a[2][i] = p[i][5]; a[3][i] = p[i][6]; a[4][i] = p[i][7];
      a[5][i] = p[i][8]; a[6][i] = p[i][9];
    }
    for (int k = 0; k < 7; ++k) {
      out->attribs[k][0] = fx_from_float_host(a[k][0] - a[k][2], 24);
      out->attribs[k][1] = fx_from_float_host(a[k][1] - a[k][2], 24);
      out->attribs[k][2] = fx_from_float_host(a[k][2], 24);
    }
  }
  if (bbox[1] <= bbox[0] || bbox[3] <= bbox[2])
    return 2;
  return 0;
}

static uint32_t log2ceil(uint32_t v) {
  uint32_t l = 0;
  while ((1u << l) < v) ++l;
  return l;
}

void orc_dcstate_init(orc_dcstate_t* s, const orc_scene_t* scene,
                      const orc_drawcall_t* dc) {
  memset(s, 0, sizeof(*s));
  /* kernel_arg flags, draw3d/main.cpp:336-344 */
  s->depth_enabled = dc->depth_test;
  s->color_enabled = dc->color_enabled;
  s->tex_enabled = dc->texture_enabled;
  s->tex_modulate = dc->texture_enabled && dc->texture_envmode == CGL_ENVMODE_MODULATE;
  if (s->tex_modulate && !s->color_enabled) s->tex_modulate = 0;
  if (s->tex_enabled && s->color_enabled && !s->tex_modulate) s->color_enabled = 0;
  /* texture DCRs, main.cpp:286-331 (quirks: magfilter tested twice,
   * wrapV taken from addressU) */
  if (dc->texture_enabled && dc->tex_slot >= 0 && dc->tex_slot < scene->num_textures) {
    const orc_texture_t* t = &scene->textures[dc->tex_slot];
    s->tex_base = scene->texels + t->offset;
    s->tex_logw = log2ceil((uint32_t)t->width);
    s->tex_logh = log2ceil((uint32_t)t->height);
    s->tex_format = (uint32_t)cgl_to_vx_format(t->format);
    s->tex_filter = (dc->texture_magfilter != CGL_FILTER_NEAREST) ||
                    (dc->texture_magfilter != CGL_FILTER_NEAREST)
                        ? VX_TEX_FILTER_BILINEAR : VX_TEX_FILTER_POINT;
    s->tex_wrapu = (dc->texture_addressU == CGL_ADDRESS_WRAP) ? 1u : 0u;
    s->tex_wrapv = (dc->texture_addressU == CGL_ADDRESS_WRAP) ? 1u : 0u;
  } else if (s->tex_enabled) {
    s->tex_enabled = 0;  /* no texture bound: the reference would abort */
  }
  /* OM DCRs, main.cpp:223-284, then DepthTencil/Blender::configure
   * (graphics.cpp:534-620) and OutputMerger::configure (gpu_sw.h:78-98) */
  uint32_t depth_func, depth_wm;
  if (dc->depth_test) {
    depth_func = cgl_to_vx_compare(dc->depth_func);
    depth_wm = (uint32_t)dc->depth_writemask & 1u;
  } else {
    depth_func = VX_OM_DEPTH_FUNC_ALWAYS;
    depth_wm = 0;
  }
  uint32_t st_func, st_zpass, st_zfail, st_fail, st_ref, st_mask, st_wm;
  if (dc->stencil_test) {
    st_func = cgl_to_vx_compare(dc->stencil_func);
    /* quirk: ZPASS written twice (zpass then zfail), ZFAIL never written */
    st_zpass = cgl_to_vx_stencil_op(dc->stencil_zfail);
    st_zfail = 0;
    st_fail = cgl_to_vx_stencil_op(dc->stencil_fail);
    st_ref = (uint32_t)dc->stencil_ref;
    st_mask = (uint32_t)dc->stencil_mask;
    st_wm = (uint32_t)dc->stencil_writemask;
  } else {
    st_func = VX_OM_DEPTH_FUNC_ALWAYS;
    st_zpass = VX_OM_STENCIL_OP_KEEP;
    st_zfail = 0;
    st_fail = VX_OM_STENCIL_OP_KEEP;
    st_ref = 0;
    st_mask = VX_OM_STENCIL_MASK;
    st_wm = 0;
  }
  uint32_t blend_mode = (VX_OM_BLEND_MODE_ADD << 16) | VX_OM_BLEND_MODE_ADD, blend_func;
  if (dc->blend_enabled) {
    uint32_t bs = cgl_to_vx_blend(dc->blend_src), bd = cgl_to_vx_blend(dc->blend_dst);
    blend_func = (bd << 24) | (bd << 16) | (bs << 8) | bs;
  } else {
    blend_func = (VX_OM_BLEND_FUNC_ZERO << 24) | (VX_OM_BLEND_FUNC_ZERO << 16) |
                 (VX_OM_BLEND_FUNC_ONE << 8) | VX_OM_BLEND_FUNC_ONE;
  }
  s->depth_func = depth_func;
  s->depth_writemask = depth_wm;
  s->depth_test_on = !((depth_func == VX_OM_DEPTH_FUNC_ALWAYS) && !depth_wm);
  s->stencil_func = st_func & 0xffff;
  s->stencil_zpass = st_zpass & 0xffff;
  s->stencil_zfail = st_zfail & 0xffff;
  s->stencil_fail = st_fail & 0xffff;
  s->stencil_ref = st_ref & 0xffff;
  s->stencil_mask = st_mask & 0xffff;
  s->stencil_writemask = st_wm & 0xffff;
  s->stencil_on = !((s->stencil_func == VX_OM_DEPTH_FUNC_ALWAYS) &&
                    (s->stencil_zpass == VX_OM_STENCIL_OP_KEEP) &&
                    (s->stencil_zfail == VX_OM_STENCIL_OP_KEEP));
  s->blend_mode_rgb = blend_mode & 0xffff;
  s->blend_mode_a = blend_mode >> 16;
  s->blend_src_rgb = blend_func & 0xff;
  s->blend_src_a = (blend_func >> 8) & 0xff;
  s->blend_dst_rgb = (blend_func >> 16) & 0xff;
  s->blend_dst_a = (blend_func >> 24) & 0xff;
  s->blend_const = 0;
  s->logic_op = 0;
  s->blend_on = !((s->blend_mode_rgb == VX_OM_BLEND_MODE_ADD) &&
                  (s->blend_mode_a == VX_OM_BLEND_MODE_ADD) &&
                  (s->blend_src_rgb == VX_OM_BLEND_FUNC_ONE) &&
                  (s->blend_src_a == VX_OM_BLEND_FUNC_ONE) &&
                  (s->blend_dst_rgb == VX_OM_BLEND_FUNC_ZERO) &&
                  (s->blend_dst_a == VX_OM_BLEND_FUNC_ZERO));
  uint32_t wm = dc->color_writemask & 0xf;
  s->cbuf_writemask = ((wm >> 0) & 1) * 0x000000ffu | ((wm >> 1) & 1) * 0x0000ff00u |
                      ((wm >> 2) & 1) * 0x00ff0000u | ((wm >> 3) & 1) * 0xff000000u;
  s->color_read = (wm != 0xf);
  s->color_write = (wm != 0x0);
}

/* ---- texture sampler: graphics.cpp:35-314 ------------------------------- */
static int32_t tex_wrap(int32_t d, uint32_t wrap) {
  const int32_t MASK = (1 << VX_TEX_FXD_FRAC) - 1;
  int32_t ret;
  switch (wrap) {
  case VX_TEX_WRAP_REPEAT: ret = d; break;
  case VX_TEX_WRAP_MIRROR:
    ret = d ^ ((int32_t)((uint32_t)d << (31 - VX_TEX_FXD_FRAC)) >> 31);
    break;
  default: /* CLAMP */
    ret = d & -(int32_t)(d >= 0);
    ret |= ((MASK - ret) >> 31);
    break;
  }
  return ret & MASK;
}

static void unpack8888(uint32_t format, uint32_t texel, uint32_t* lo, uint32_t* hi) {
  uint32_t r, g, b, a;
  switch (format) {
  case VX_TEX_FORMAT_R5G6B5:
    r = ((texel >> 8) & 0xf8) | ((texel >> 13) & 0x07);
    g = ((texel >> 3) & 0xfc) | ((texel >> 9) & 0x03);
    b = ((texel << 3) & 0xf8) | ((texel >> 2) & 0x07);
    a = 0xff;
    break;
  case VX_TEX_FORMAT_A1R5G5B5:
    r = ((texel >> 7) & 0xf8) | ((texel >> 12) & 0x07);
    g = ((texel >> 2) & 0xf8) | ((texel >> 7) & 0x07);
    b = ((texel << 3) & 0xf8) | ((texel >> 2) & 0x07);
    a = (uint32_t)(((int32_t)(texel << 16)) >> 31) & 0xff;
    break;
  case VX_TEX_FORMAT_A4R4G4B4:
    r = ((texel >> 4) & 0xf0) | ((texel >> 8) & 0x0f);
    g = ((texel >> 0) & 0xf0) | ((texel >> 4) & 0x0f);
    b = ((texel << 4) & 0xf0) | ((texel >> 0) & 0x0f);
    a = ((texel >> 8) & 0xf0) | ((texel >> 12) & 0x0f);
    break;
  case VX_TEX_FORMAT_A8L8:
    r = texel & 0xff; g = r; b = r; a = (texel >> 8) & 0xff;
    break;
  case VX_TEX_FORMAT_L8:
    r = texel & 0xff; g = r; b = r; a = 0xff;
    break;
  case VX_TEX_FORMAT_A8:
    r = 0xff; g = 0xff; b = 0xff; a = texel & 0xff;
    break;
  default: /* A8R8G8B8 */
    r = (texel >> 16) & 0xff; g = (texel >> 8) & 0xff; b = texel & 0xff; a = texel >> 24;
    break;
  }
  *lo = (r << 16) + b;
  *hi = (a << 16) + g;
}

static inline uint32_t lerp8888(uint32_t a, uint32_t b, uint32_t f) { /* graphics.h:82-86 */
  uint32_t p = a * (0xff - f) + b * f + 0x00800080u;
  uint32_t q = (p >> 8) & 0x00ff00ffu;
  return ((p + q) >> 8) & 0x00ff00ffu;
}

static inline uint32_t fetch_texel(const uint8_t* base, uint32_t off, uint32_t stride) {
  const uint8_t* p = base + (uint64_t)off * stride;
  switch (stride) {
  case 4: return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
  case 2: return (uint32_t)p[0] | ((uint32_t)p[1] << 8);
  default: return p[0];
  }
}

uint32_t orc_tex_read(const orc_dcstate_t* s, int32_t u, int32_t v) {
  const uint32_t logw = s->tex_logw, logh = s->tex_logh;
  const uint32_t stride = vx_format_stride((int)s->tex_format);
  if (s->tex_filter == VX_TEX_FILTER_BILINEAR) {   /* TexAddressLinear :124-166 */
    const int32_t half = (1 << VX_TEX_FXD_FRAC) >> 1;
    const int32_t dxh = half >> logw, dyh = half >> logh;
    uint32_t u0 = (uint32_t)tex_wrap((int32_t)((uint32_t)u - (uint32_t)dxh), s->tex_wrapu);
    uint32_t u1 = (uint32_t)tex_wrap((int32_t)((uint32_t)u + (uint32_t)dxh), s->tex_wrapu);
    uint32_t v0 = (uint32_t)tex_wrap((int32_t)((uint32_t)v - (uint32_t)dyh), s->tex_wrapv);
    uint32_t v1 = (uint32_t)tex_wrap((int32_t)((uint32_t)v + (uint32_t)dyh), s->tex_wrapv);
    uint32_t shu = VX_TEX_FXD_FRAC - logw, shv = VX_TEX_FXD_FRAC - logh;
    uint32_t x0s = (u0 << 8) >> shu, y0s = (v0 << 8) >> shv;
    uint32_t x0 = x0s >> 8, y0 = y0s >> 8, x1 = u1 >> shu, y1 = v1 >> shv;
    uint32_t t00 = fetch_texel(s->tex_base, x0 + (y0 << logw), stride);
    uint32_t t01 = fetch_texel(s->tex_base, x1 + (y0 << logw), stride);
    uint32_t t10 = fetch_texel(s->tex_base, x0 + (y1 << logw), stride);
    uint32_t t11 = fetch_texel(s->tex_base, x1 + (y1 << logw), stride);
    uint32_t alpha = x0s & 0xff, beta = y0s & 0xff;
    uint32_t c0l, c0h, c1l, c1h, c2l, c2h, c3l, c3h;           /* :188-225 */
    unpack8888(s->tex_format, t00, &c0l, &c0h);
    unpack8888(s->tex_format, t01, &c1l, &c1h);
    uint32_t c01l = lerp8888(c0l, c1l, alpha), c01h = lerp8888(c0h, c1h, alpha);
    unpack8888(s->tex_format, t10, &c2l, &c2h);
    unpack8888(s->tex_format, t11, &c3l, &c3h);
    uint32_t c23l = lerp8888(c2l, c3l, alpha), c23h = lerp8888(c2h, c3h, alpha);
    uint32_t cl = lerp8888(c01l, c23l, beta), ch = lerp8888(c01h, c23h, beta);
    return (ch << 8) | cl;
  } else {                                         /* TexAddressPoint :168-186 */
    uint32_t uu = (uint32_t)tex_wrap(u, s->tex_wrapu);
    uint32_t vv = (uint32_t)tex_wrap(v, s->tex_wrapv);
    uint32_t x = uu >> (VX_TEX_FXD_FRAC - logw), y = vv >> (VX_TEX_FXD_FRAC - logh);
    uint32_t cl, ch;
    unpack8888(s->tex_format, fetch_texel(s->tex_base, x + (y << logw), stride), &cl, &ch);
    return (ch << 8) | cl;
  }
}

/* ---- shader: draw3d/kernel.cpp:16-79 + :232-279 ------------------------- */
static inline int32_t imadd24(int32_t a, int32_t b, int32_t c) {   /* :48-51 */
  int32_t p = (int32_t)(((int64_t)a * (int64_t)b) >> 24);
  return (int32_t)((uint32_t)p + (uint32_t)c);
}
static inline int32_t interp(const int32_t at[3], int32_t dx, int32_t dy) { /* :56-59 */
  int32_t tmp = imadd24(at[0], dx, at[2]);
  return imadd24(at[1], dy, tmp);
}
static inline uint32_t mul8(int32_t d, uint32_t c) {   /* (data*c) >> 24, int32 wrap */
  return (((uint32_t)d * c) >> 24) & 0xff;
}

uint32_t orc_shade(const orc_dcstate_t* s, const orc_rast_prim_t* p,
                   int32_t F0, int32_t F1, int32_t F2, uint32_t* depth) {
  /* GRADIENTS_SW_i: the Q15.16 words are reinterpreted as Q7.24 (:37-44) */
  const float f0 = fx_to_float(F0, 24), f1 = fx_to_float(F1, 24), f2 = fx_to_float(F2, 24);
  const float r = 1.0f / (f0 + f1 + f2);
  const int32_t dx = fx_from_float_dev(r * f0, 24);
  const int32_t dy = fx_from_float_dev(r * f1, 24);
  return orc_shade_weights(s, p, dx, dy, depth);
}

/* the depth word the shader computes (GRADIENTS_SW + INTERPOLATE z,
 * draw3d/kernel.cpp:37-59), masked to VX_OM_DEPTH_BITS: what the depth test
 * compares (graphics.cpp:564-596) */
uint32_t orc_vis_depth(const orc_rast_prim_t* p, int32_t F0, int32_t F1, int32_t F2) {
  const float f0 = fx_to_float(F0, 24), f1 = fx_to_float(F1, 24), f2 = fx_to_float(F2, 24);
  const float r = 1.0f / (f0 + f1 + f2);
  const int32_t dx = fx_from_float_dev(r * f0, 24);
  const int32_t dy = fx_from_float_dev(r * f1, 24);
  return (uint32_t)interp(p->attribs[0], dx, dy) & VX_OM_DEPTH_MASK;
}

uint32_t orc_shade_weights(const orc_dcstate_t* s, const orc_rast_prim_t* p,
                           int32_t dx, int32_t dy, uint32_t* depth) {
  int32_t z = 0, cr = 1 << 24, cg = 1 << 24, cb = 1 << 24, ca = 1 << 24, u = 0, v = 0;
  if (s->depth_enabled) z = interp(p->attribs[0], dx, dy);
  if (s->color_enabled) {
    cr = interp(p->attribs[1], dx, dy);
    cg = interp(p->attribs[2], dx, dy);
    cb = interp(p->attribs[3], dx, dy);
    ca = interp(p->attribs[4], dx, dy);
  }
  if (s->tex_enabled) {
    u = interp(p->attribs[5], dx, dy);
    v = interp(p->attribs[6], dx, dy);
  }
  uint32_t out;
  if (s->tex_enabled) {
    /* TEXTURING: fixeduv_t(u) = TFixed<24> -> TFixed<23> (:14, :152-156) */
    const uint32_t tc = orc_tex_read(s, u >> 1, v >> 1);
    if (s->tex_modulate) {                                 /* MODULATE :61-65 */
      out = (mul8(ca, tc >> 24) << 24) | (mul8(cr, (tc >> 16) & 0xff) << 16) |
            (mul8(cg, (tc >> 8) & 0xff) << 8) | mul8(cb, tc & 0xff);
    } else {                                               /* REPLACE :140-144 */
      out = tc;
    }
  } else {                                                 /* TO_RGBA :67-71 */
    out = (mul8(ca, 255) << 24) | (mul8(cr, 255) << 16) | (mul8(cg, 255) << 8) | mul8(cb, 255);
  }
  *depth = (uint32_t)z;
  return out;
}

/* ---- output merger: graphics.cpp:320-636, gpu_sw.h:100-168 -------------- */
static int do_compare(uint32_t func, uint32_t a, uint32_t b) {
  switch (func) {
  case VX_OM_DEPTH_FUNC_NEVER: return 0;
  case VX_OM_DEPTH_FUNC_LESS: return a < b;
  case VX_OM_DEPTH_FUNC_EQUAL: return a == b;
  case VX_OM_DEPTH_FUNC_LEQUAL: return a <= b;
  case VX_OM_DEPTH_FUNC_GREATER: return a > b;
  case VX_OM_DEPTH_FUNC_NOTEQUAL: return a != b;
  case VX_OM_DEPTH_FUNC_GEQUAL: return a >= b;
  default: return 1;
  }
}
static uint32_t do_stencil_op(uint32_t op, uint32_t ref, uint32_t val) {
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

typedef struct { uint32_t a, r, g, b; } argb_t;
static inline argb_t argb(uint32_t v) {
  argb_t c = {v >> 24, (v >> 16) & 0xff, (v >> 8) & 0xff, v & 0xff};
  return c;
}
static inline argb_t mk(uint32_t a, uint32_t r, uint32_t g, uint32_t b) {
  argb_t c = {a & 0xff, r & 0xff, g & 0xff, b & 0xff};
  return c;
}
static inline uint32_t div255(int x) { return (uint32_t)((x + (x >> 8)) >> 8); }

static argb_t blend_func(uint32_t f, argb_t s, argb_t d, argb_t c) {
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
    uint32_t f2 = s.a < (0xff - d.a) ? s.a : (0xff - d.a);
    return mk(0xff, f2, f2, f2);
  }
  default: return mk(0, 0, 0, 0);
  }
}
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static uint32_t logic_op(uint32_t op, uint32_t s, uint32_t d) {
  switch (op) {
  case 0: return 0; case 1: return s & d; case 2: return s & ~d; case 3: return s;
  case 4: return ~s & d; case 5: return d; case 6: return s ^ d; case 7: return s | d;
  case 8: return ~(s | d); case 9: return ~(s ^ d); case 10: return ~d;
  case 11: return s | ~d; case 12: return ~s; case 13: return ~s | d;
  case 14: return ~(s & d); default: return 0xffffffffu;
  }
}
static argb_t blend_mode(uint32_t mode, uint32_t lop, argb_t src, argb_t dst, argb_t s, argb_t d,
                         uint32_t srcv, uint32_t dstv) {
#define CH(op, x) op
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
  default: /* ADD */
    return mk(div255(imin((int)(src.a * s.a + dst.a * d.a) + 0x80, 0xFF00)),
              div255(imin((int)(src.r * s.r + dst.r * d.r) + 0x80, 0xFF00)),
              div255(imin((int)(src.g * s.g + dst.g * d.g) + 0x80, 0xFF00)),
              div255(imin((int)(src.b * s.b + dst.b * d.b) + 0x80, 0xFF00)));
  }
#undef CH
}

static uint32_t do_blend(const orc_dcstate_t* st, uint32_t srcv, uint32_t dstv) {
  argb_t src = argb(srcv), dst = argb(dstv), cst = argb(st->blend_const);
  argb_t s_rgb = blend_func(st->blend_src_rgb, src, dst, cst);
  argb_t s_a = blend_func(st->blend_src_a, src, dst, cst);
  argb_t d_rgb = blend_func(st->blend_dst_rgb, src, dst, cst);
  argb_t d_a = blend_func(st->blend_dst_a, src, dst, cst);
  argb_t rgb = blend_mode(st->blend_mode_rgb, st->logic_op, src, dst, s_rgb, d_rgb, srcv, dstv);
  argb_t a = blend_mode(st->blend_mode_a, st->logic_op, src, dst, s_a, d_a, srcv, dstv);
  return (a.a << 24) | (rgb.r << 16) | (rgb.g << 8) | rgb.b;
}

int orc_om_write(const orc_dcstate_t* s, uint32_t* cbuf_px, uint32_t* zbuf_px,
                 uint32_t color, uint32_t depth) {
  const int depth_on = s->depth_test_on, stencil_on = s->stencil_on, blend_on = s->blend_on;
  uint32_t dst_ds = 0, dst_color = 0, ds = 0;
  if (depth_on || stencil_on) dst_ds = *zbuf_px;
  if (s->color_write && (s->color_read || blend_on)) dst_color = *cbuf_px;
  int passed = 1;
  if (depth_on || stencil_on) {          /* DepthTencil::test :564-596 */
    const uint32_t depth_val = dst_ds & VX_OM_DEPTH_MASK;
    const uint32_t stencil_val = dst_ds >> VX_OM_DEPTH_BITS;
    const uint32_t depth_ref = depth & VX_OM_DEPTH_MASK;
    const uint32_t ref_m = s->stencil_ref & s->stencil_mask;
    const uint32_t val_m = stencil_val & s->stencil_mask;
    uint32_t op;
    passed = do_compare(s->stencil_func, ref_m, val_m);
    if (passed) {
      passed = do_compare(s->depth_func, depth_ref, depth_val);
      op = passed ? s->stencil_zpass : s->stencil_zfail;
    } else {
      op = s->stencil_fail;
    }
    const uint32_t sres = do_stencil_op(op, s->stencil_ref, stencil_val);
    ds = (sres << VX_OM_DEPTH_BITS) | depth_ref;
  }
  if (blend_on && passed) color = do_blend(s, color, dst_color);
  const uint32_t ds_wm = ((depth_on && passed && s->depth_writemask) ? VX_OM_DEPTH_MASK : 0) |
                         (stencil_on ? (s->stencil_writemask << VX_OM_DEPTH_BITS) : 0);
  if (ds_wm != 0) *zbuf_px = (dst_ds & ~ds_wm) | (ds & ds_wm);
  if (s->color_write && passed)
    *cbuf_px = (dst_color & ~s->cbuf_writemask) | (color & s->cbuf_writemask);
  return passed;
}

/* ---- the render-output regression app (tests/regression/om) -------------
 * OutputMerger / DepthTencil / Blender ::configure from the 18 OM DCR words
 * (dcr[i] = VX_DCR_OM_STATE_BEGIN + i), the stencil face chosen by
 * `backface` (sim/simx/om_unit.cpp:28-49, graphics.cpp:534-620), then the
 * kernel (om/kernel.cpp:16-40): num_tasks tasks of ceil(H / num_tasks) rows,
 * each pixel written once through the unit (om_unit.cpp:55-80) with the
 * colour (alpha = task * 255 / rows when blending) and depth words.  cbuf /
 * zbuf hold the host's clears on entry (om/main.cpp:262-283). */
enum {
  OM_CBUF_WRITEMASK = 2, OM_DEPTH_FUNC = 5, OM_DEPTH_WRITEMASK = 6, OM_STENCIL_FUNC = 7,
  OM_STENCIL_ZPASS = 8, OM_STENCIL_ZFAIL = 9, OM_STENCIL_FAIL = 10, OM_STENCIL_REF = 11,
  OM_STENCIL_MASK = 12, OM_STENCIL_WRITEMASK = 13, OM_BLEND_MODE = 14, OM_BLEND_FUNC = 15,
  OM_BLEND_CONST = 16, OM_LOGIC_OP = 17
};
void orc_om_configure(orc_dcstate_t* s, const uint32_t dcr[18], int backface) {
  const uint32_t sh = backface ? 16u : 0u;
  memset(s, 0, sizeof(*s));
  s->depth_func = dcr[OM_DEPTH_FUNC];
  s->depth_writemask = dcr[OM_DEPTH_WRITEMASK] & 1u;
  s->depth_test_on = !((s->depth_func == VX_OM_DEPTH_FUNC_ALWAYS) && !s->depth_writemask);
  s->stencil_func = (dcr[OM_STENCIL_FUNC] >> sh) & 0xffffu;
  s->stencil_zpass = (dcr[OM_STENCIL_ZPASS] >> sh) & 0xffffu;
  s->stencil_zfail = (dcr[OM_STENCIL_ZFAIL] >> sh) & 0xffffu;
  s->stencil_fail = (dcr[OM_STENCIL_FAIL] >> sh) & 0xffffu;
  s->stencil_ref = (dcr[OM_STENCIL_REF] >> sh) & 0xffffu;
  s->stencil_mask = (dcr[OM_STENCIL_MASK] >> sh) & 0xffffu;
  s->stencil_writemask = (dcr[OM_STENCIL_WRITEMASK] >> sh) & 0xffffu;
  s->stencil_on = !((s->stencil_func == VX_OM_DEPTH_FUNC_ALWAYS) &&
                    (s->stencil_zpass == VX_OM_STENCIL_OP_KEEP) &&
                    (s->stencil_zfail == VX_OM_STENCIL_OP_KEEP));
  s->blend_mode_rgb = dcr[OM_BLEND_MODE] & 0xffffu;
  s->blend_mode_a = dcr[OM_BLEND_MODE] >> 16;
  s->blend_src_rgb = dcr[OM_BLEND_FUNC] & 0xffu;
  s->blend_src_a = (dcr[OM_BLEND_FUNC] >> 8) & 0xffu;
  s->blend_dst_rgb = (dcr[OM_BLEND_FUNC] >> 16) & 0xffu;
  s->blend_dst_a = (dcr[OM_BLEND_FUNC] >> 24) & 0xffu;
  s->blend_const = dcr[OM_BLEND_CONST];
  s->logic_op = dcr[OM_LOGIC_OP];
  s->blend_on = !((s->blend_mode_rgb == VX_OM_BLEND_MODE_ADD) &&
                  (s->blend_mode_a == VX_OM_BLEND_MODE_ADD) &&
                  (s->blend_src_rgb == VX_OM_BLEND_FUNC_ONE) &&
                  (s->blend_src_a == VX_OM_BLEND_FUNC_ONE) &&
                  (s->blend_dst_rgb == VX_OM_BLEND_FUNC_ZERO) &&
                  (s->blend_dst_a == VX_OM_BLEND_FUNC_ZERO));
  {
    const uint32_t wm = dcr[OM_CBUF_WRITEMASK] & 0xfu;
    s->cbuf_writemask = ((wm >> 0) & 1u) * 0x000000ffu | ((wm >> 1) & 1u) * 0x0000ff00u |
                        ((wm >> 2) & 1u) * 0x00ff0000u | ((wm >> 3) & 1u) * 0xff000000u;
    s->color_read = wm != 0xfu;
    s->color_write = wm != 0u;
  }
}

int orc_om_app(uint32_t width, uint32_t height, uint32_t num_tasks, uint32_t color,
               uint32_t depth, int backface, int blend_enable, const uint32_t dcr[18],
               uint32_t* cbuf, uint32_t* zbuf) {
  orc_dcstate_t s;
  uint32_t task, tile_h;
  float alpha_step;
  if (num_tasks == 0) return -1;
  orc_om_configure(&s, dcr, backface);
  tile_h = (height + num_tasks - 1) / num_tasks;          /* kernel.cpp:35-36 */
  alpha_step = 255.0f / (float)tile_h;
  for (task = 0; task < num_tasks; ++task) {               /* kernel_body :16-33 */
    const uint32_t y0 = task * tile_h;
    const uint32_t y1 = (y0 + tile_h < height) ? y0 + tile_h : height;
    const uint32_t alpha = blend_enable ? (uint32_t)((float)task * alpha_step) : 0xffu;
    const uint32_t c = (alpha << 24) | (color & 0x00ffffffu);
    uint32_t x, y;
    if (y0 >= height) break;
    for (y = y0; y < y1; ++y)
      for (x = 0; x < width; ++x)
        orc_om_write(&s, &cbuf[(size_t)y * width + x], &zbuf[(size_t)y * width + x], c, depth);
  }
  return 0;
}
