// setup.cpp -- see setup.h.  Compiled with -ffp-contract=off: the float
// operation order below is part of the bit-exact contract with the reference
// (every product is rounded before it is added, as on the reference's x86
// host build without FMA).
#include "setup.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace rt {
namespace {

// cocogfx TFixed<F>(float) on the host: truncation toward zero; x86
// cvttss2si yields INT_MIN for values out of range.
int32_t FixedHost(float f, int frac) {
  const float x = f * (float)(1u << frac);
  if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT32_MIN;
  return (int32_t)x;
}

// cocogfx ClipToHDC / ClipToScreen with viewport (0, W, 0, H, near, far):
// framebuffer row 0 is NDC y = -1 (draw3d/main.cpp:385-386).
struct Viewport {
  float sx, cx, sy, cy, sz, cz;
};
Viewport MakeViewport(uint32_t w, uint32_t h, float n, float f) {
  const float l = 0.0f, r = (float)w, t = 0.0f, b = (float)h;
  return {(r - l) * 0.5f, (r + l) * 0.5f, (b - t) * 0.5f, (b + t) * 0.5f,
          (f - n) * 0.5f, (f + n) * 0.5f};
}

}  // namespace

uint32_t ToVXCompare(int32_t c) {  // gfxutil.cpp:296-311
  static const uint32_t m[8] = {VX_OM_DEPTH_FUNC_NEVER,    VX_OM_DEPTH_FUNC_LESS,
                                VX_OM_DEPTH_FUNC_EQUAL,    VX_OM_DEPTH_FUNC_LEQUAL,
                                VX_OM_DEPTH_FUNC_GREATER,  VX_OM_DEPTH_FUNC_NOTEQUAL,
                                VX_OM_DEPTH_FUNC_GEQUAL,   VX_OM_DEPTH_FUNC_ALWAYS};
  return (c >= 0 && c < 8) ? m[c] : VX_OM_DEPTH_FUNC_ALWAYS;
}

int32_t ToVXFormat(int32_t f) {  // gfxutil.cpp:280-294
  switch (f) {
  case 1: return VX_TEX_FORMAT_A8;
  case 2: return VX_TEX_FORMAT_L8;
  case 3: return VX_TEX_FORMAT_A8L8;
  case 4: return VX_TEX_FORMAT_R5G6B5;
  default: return VX_TEX_FORMAT_A8R8G8B8;  // 5 in the traces: 4 bytes per texel
  }
}

uint32_t FormatStride(int32_t vx_format) {
  switch (vx_format) {
  case VX_TEX_FORMAT_A8R8G8B8: return 4;
  case VX_TEX_FORMAT_L8:
  case VX_TEX_FORMAT_A8: return 1;
  default: return 2;
  }
}

int PrimSetup(const std::array<Vertex, 3>& v, uint32_t width, uint32_t height, float znear,
              float zfar, rt_prim_t* out) {
  std::memset(out, 0, sizeof(*out));
  const Viewport vp = MakeViewport(width, height, znear, zfar);
  float hx[3], hy[3], hw[3], sz[3];
  for (int i = 0; i < 3; ++i) {
    const float* p = v[i].pos;
    hx[i] = p[0] * vp.sx + p[3] * vp.cx;  // HDC = screen position * w
    hy[i] = p[1] * vp.sy + p[3] * vp.cy;
    hw[i] = p[3];
    const float rhw = 1.0f / p[3];
    sz[i] = (p[2] * rhw) * vp.sz + vp.cz;  // screen z
  }
  // EdgeEquation (gfxutil.cpp:35-75): e_i = q_j x q_k over (x, y, w)
  float e[3][3];
  for (int i = 0; i < 3; ++i) {
    const int j = (i + 1) % 3, k = (i + 2) % 3;
    e[i][0] = (hy[j] * hw[k]) - (hy[k] * hw[j]);
    e[i][1] = (hx[k] * hw[j]) - (hx[j] * hw[k]);
    e[i][2] = (hx[j] * hy[k]) - (hx[k] * hy[j]);
  }
  const float det = e[0][2] * hw[0] + e[1][2] * hw[1] + e[2][2] * hw[2];
  if (det < 0)
    for (auto& row : e)
      for (float& x : row) x *= -1.0f;
  if (det == 0) return kSetupDegenerate;
  for (auto& row : e) row[2] += row[0] * 0.5f + row[1] * 0.5f;  // half-pixel offset
  // EdgeToFixed (gfxutil.cpp:79-96)
  float m = std::fabs(e[0][0]);
  const float c[5] = {std::fabs(e[1][0]), std::fabs(e[2][0]), std::fabs(e[0][1]),
                      std::fabs(e[1][1]), std::fabs(e[2][1])};
  for (float x : c) m = (x > m) ? x : m;
  const float scale = 1.0f / m;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) out->edges[i][j] = FixedHost(e[i][j] * scale, 16);
  // ATTRIBUTE_DELTA (gfxutil.cpp:204-207,224-230): z from screen z, rest raw
  float a[7][3];
  for (int i = 0; i < 3; ++i) {
    a[0][i] = sz[i];
    for (int k = 0; k < 4; ++k) a[1 + k][i] = v[i].color[k];
    a[5][i] = v[i].uv[0];
    a[6][i] = v[i].uv[1];
  }
  for (int k = 0; k < 7; ++k) {
    out->attribs[k][0] = FixedHost(a[k][0] - a[k][2], 24);
    out->attribs[k][1] = FixedHost(a[k][1] - a[k][2], 24);
    out->attribs[k][2] = FixedHost(a[k][2], 24);
  }
  return kSetupOk;
}

rt_dcstate_t DrawcallState(const DrawCall& dc, const Scene& scene) {
  rt_dcstate_t s;
  std::memset(&s, 0, sizeof(s));
  const States& st = dc.states;
  // kernel_arg flags (draw3d/main.cpp:336-344)
  bool depth = st.depth_test != 0, color = st.color_enabled != 0, tex = st.texture_enabled != 0;
  bool modulate = tex && st.texture_envmode == kCglEnvModeModulate;
  if (modulate && !color) modulate = false;
  if (tex && color && !modulate) color = false;
  auto it = scene.textures.find(dc.texture_id);
  if (tex && it == scene.textures.end()) tex = false;
  if (tex) {
    const Texture& t = it->second;
    uint32_t lw = 0, lh = 0;
    while ((1u << lw) < (uint32_t)t.width) ++lw;
    while ((1u << lh) < (uint32_t)t.height) ++lh;
    s.tex_logw = lw;
    s.tex_logh = lh;
    s.tex_format = (uint32_t)ToVXFormat(t.format);
    s.tex_stride = FormatStride((int32_t)s.tex_format);
    // quirks kept: magfilter tested twice, wrapV from addressU (main.cpp:304-308)
    s.tex_filter = (st.texture_magfilter != kCglFilterNearest) ? VX_TEX_FILTER_BILINEAR
                                                              : VX_TEX_FILTER_POINT;
    s.tex_wrapu = (st.texture_addressU == kCglAddressWrap) ? VX_TEX_WRAP_REPEAT : VX_TEX_WRAP_CLAMP;
    s.tex_wrapv = s.tex_wrapu;
  }
  s.flags = (depth ? RT_DC_DEPTH : 0u) | (color ? RT_DC_COLOR : 0u) | (tex ? RT_DC_TEX : 0u) |
            (modulate ? RT_DC_MODULATE : 0u);
  return s;
}

int PrimBBox(const std::array<Vertex, 3>& v, uint32_t width, uint32_t height, rt_bbox_t* out) {
  const Viewport vp = MakeViewport(width, height, 0.0f, 1.0f);
  float l = 0, r = 0, t = 0, b = 0;
  for (int i = 0; i < 3; ++i) {  // ClipToScreen x, y (oracle clip_to_screen)
    const float* p = v[i].pos;
    const float rhw = 1.0f / p[3];
    const float x = (p[0] * rhw) * vp.sx + vp.cx, y = (p[1] * rhw) * vp.sy + vp.cy;
    if (i == 0) {
      l = r = x;
      t = b = y;
    } else {
      l = std::fmin(l, x); r = std::fmax(r, x);
      t = std::fmin(t, y); b = std::fmax(b, y);
    }
  }
  int32_t L = (int32_t)std::floor(l), R = (int32_t)std::ceil(r);
  int32_t T = (int32_t)std::floor(t), B = (int32_t)std::ceil(b);
  L = L > 0 ? L : 0;
  R = R < (int32_t)width ? R : (int32_t)width;
  T = T > 0 ? T : 0;
  B = B < (int32_t)height ? B : (int32_t)height;
  if (R <= L || B <= T) {
    out->x = out->y = 0;
    return kSetupCulled;
  }
  out->x = (uint32_t)L | ((uint32_t)R << 16);
  out->y = (uint32_t)T | ((uint32_t)B << 16);
  return kSetupOk;
}

namespace {
uint32_t ToVXStencilOp(int32_t c) {  // gfxutil.cpp:313-326
  static const uint32_t m[6] = {VX_OM_STENCIL_OP_KEEP, VX_OM_STENCIL_OP_REPLACE,
                                VX_OM_STENCIL_OP_INCR, VX_OM_STENCIL_OP_DECR,
                                VX_OM_STENCIL_OP_ZERO, VX_OM_STENCIL_OP_INVERT};
  return (c >= 0 && c < 6) ? m[c] : VX_OM_STENCIL_OP_KEEP;
}
uint32_t ToVXBlend(int32_t c) {  // gfxutil.cpp:328-346
  static const uint32_t m[11] = {VX_OM_BLEND_FUNC_ZERO, VX_OM_BLEND_FUNC_ONE,
                                 VX_OM_BLEND_FUNC_SRC_RGB, VX_OM_BLEND_FUNC_ONE_MINUS_SRC_RGB,
                                 VX_OM_BLEND_FUNC_SRC_A, VX_OM_BLEND_FUNC_ONE_MINUS_SRC_A,
                                 VX_OM_BLEND_FUNC_DST_A, VX_OM_BLEND_FUNC_ONE_MINUS_DST_A,
                                 VX_OM_BLEND_FUNC_DST_RGB, VX_OM_BLEND_FUNC_ONE_MINUS_DST_RGB,
                                 VX_OM_BLEND_FUNC_ALPHA_SAT};
  return (c >= 0 && c < 11) ? m[c] : VX_OM_BLEND_FUNC_ONE;
}
}  // namespace

rt_omstate_t OmState(const DrawCall& dc) {
  // draw3d/main.cpp:223-284 DCR writes, then DepthTencil / Blender configure
  // (graphics.cpp:534-620) and OutputMerger::configure (gpu_sw.h:78-98)
  rt_omstate_t s;
  std::memset(&s, 0, sizeof(s));
  const States& st = dc.states;
  uint32_t depth_func = VX_OM_DEPTH_FUNC_ALWAYS, depth_wm = 0;
  if (st.depth_test) {
    depth_func = ToVXCompare(st.depth_func);
    depth_wm = (uint32_t)st.depth_writemask & 1u;
  }
  uint32_t sf = VX_OM_DEPTH_FUNC_ALWAYS, szp = VX_OM_STENCIL_OP_KEEP, szf = 0;
  uint32_t sfail = VX_OM_STENCIL_OP_KEEP, sref = 0, smask = VX_OM_STENCIL_MASK, swm = 0;
  if (st.stencil_test) {
    sf = ToVXCompare(st.stencil_func);
    szp = ToVXStencilOp(st.stencil_zfail);  // quirk: ZPASS written twice, ZFAIL never (:251-260)
    szf = 0;
    sfail = ToVXStencilOp(st.stencil_fail);
    sref = (uint32_t)st.stencil_ref;
    smask = (uint32_t)st.stencil_mask;
    swm = (uint32_t)st.stencil_writemask;
  }
  uint32_t blend_func = (VX_OM_BLEND_FUNC_ZERO << 24) | (VX_OM_BLEND_FUNC_ZERO << 16) |
                        (VX_OM_BLEND_FUNC_ONE << 8) | VX_OM_BLEND_FUNC_ONE;
  if (st.blend_enabled) {
    const uint32_t bs = ToVXBlend(st.blend_src), bd = ToVXBlend(st.blend_dst);
    blend_func = (bd << 24) | (bd << 16) | (bs << 8) | bs;
  }
  s.depth_func = depth_func;
  s.depth_writemask = depth_wm;
  s.depth_test_on = !((depth_func == VX_OM_DEPTH_FUNC_ALWAYS) && !depth_wm);
  s.stencil_func = sf & 0xffff;
  s.stencil_zpass = szp & 0xffff;
  s.stencil_zfail = szf & 0xffff;
  s.stencil_fail = sfail & 0xffff;
  s.stencil_ref = sref & 0xffff;
  s.stencil_mask = smask & 0xffff;
  s.stencil_writemask = swm & 0xffff;
  s.stencil_on = !((s.stencil_func == VX_OM_DEPTH_FUNC_ALWAYS) &&
                   (s.stencil_zpass == VX_OM_STENCIL_OP_KEEP) &&
                   (s.stencil_zfail == VX_OM_STENCIL_OP_KEEP));
  s.blend_mode_rgb = VX_OM_BLEND_MODE_ADD;
  s.blend_mode_a = VX_OM_BLEND_MODE_ADD;
  s.blend_src_rgb = blend_func & 0xff;
  s.blend_src_a = (blend_func >> 8) & 0xff;
  s.blend_dst_rgb = (blend_func >> 16) & 0xff;
  s.blend_dst_a = (blend_func >> 24) & 0xff;
  s.blend_const = 0;
  s.logic_op = 0;
  s.blend_on = !((s.blend_src_rgb == VX_OM_BLEND_FUNC_ONE) && (s.blend_src_a == VX_OM_BLEND_FUNC_ONE) &&
                 (s.blend_dst_rgb == VX_OM_BLEND_FUNC_ZERO) && (s.blend_dst_a == VX_OM_BLEND_FUNC_ZERO));
  const uint32_t wm = st.color_writemask & 0xf;
  s.cbuf_writemask = ((wm >> 0) & 1) * 0x000000ffu | ((wm >> 1) & 1) * 0x0000ff00u |
                     ((wm >> 2) & 1) * 0x00ff0000u | ((wm >> 3) & 1) * 0xff000000u;
  s.color_read = wm != 0xf;
  s.color_write = wm != 0x0;
  s.prim_offset = dc.prim_offset;
  s.prim_count = dc.prim_count;
  return s;
}

}  // namespace rt
