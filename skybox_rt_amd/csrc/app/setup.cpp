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

uint32_t ToVXCompare(int32_t c) {
  static const uint32_t m[8] = {VX_OM_DEPTH_FUNC_NEVER,    VX_OM_DEPTH_FUNC_LESS,
                                VX_OM_DEPTH_FUNC_EQUAL,    VX_OM_DEPTH_FUNC_LEQUAL,
                                VX_OM_DEPTH_FUNC_GREATER,  VX_OM_DEPTH_FUNC_NOTEQUAL,
                                VX_OM_DEPTH_FUNC_GEQUAL,   VX_OM_DEPTH_FUNC_ALWAYS};
  return (c >= 0 && c < 8) ? m[c] : VX_OM_DEPTH_FUNC_ALWAYS;
}

int32_t ToVXFormat(int32_t f) {
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
  // EdgeToFixed (gfxutil.cpp:119-136)
  float m = std::fabs(e[0][0]);
  const float c[5] = {std::fabs(e[1][0]), std::fabs(e[2][0]), std::fabs(e[0][1]),
                      std::fabs(e[1][1]), std::fabs(e[2][1])};
  for (float x : c) m = (x > m) ? x : m;
  const float scale = 1.0f / m;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) out->edges[i][j] = FixedHost(e[i][j] * scale, 16);
  // ATTRIBUTE_DELTA (gfxutil.cpp:244-270): z from screen z, rest raw
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

}  // namespace rt
