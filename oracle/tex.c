/* tex.c -- CPU restatement of the reference's texture regression app
 * (tests/regression/tex/main.cpp host + kernel.cpp device), the sampler of
 * SURVEY.md 8(f) rank 3.  TEST INFRASTRUCTURE ONLY (see oracle.h): the
 * product path is skybox_rt_amd/csrc/kernels/tex_kernel.hip behind
 * librtapp's rt_tex_* C-ABI.
 *
 * Pinned: the 16 tex golden images of the reference (tests/golden/tex/:
 * toad_ref_f0..f6 = the 7 texel formats, {soccer,palette4,palette16,
 * palette64}_ref_g0..g2 = point / bilinear / trilinear), which fix the
 * un-vendored cocogfx LoadImage format conversion inferred here: truncation
 * to the channel width, luminance = the red channel, 1-bit alpha = (a != 0).
 * Unpinned: texels of mip levels >= 1 (cocogfx GenerateMipmaps is not
 * vendored and no golden samples them -- at scale 1 the trilinear blend
 * factor is 0); restated as a 2x2 box filter of the decoded level above,
 * truncating, re-encoded with the same conversion. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "gfx.h"
#include "oracle.h"

#define VX_TEX_LOD_MAX 15  /* VX_types.vh:310 (= VX_TEX_DIM_BITS) */

/* cocogfx LoadImage(path, eformat) conversion of one A8R8G8B8 pixel */
uint32_t orc_tex_encode(uint32_t argb, uint32_t format) {
  const uint32_t a = argb >> 24, r = (argb >> 16) & 0xff, g = (argb >> 8) & 0xff, b = argb & 0xff;
  switch (format) {
  case VX_TEX_FORMAT_A8R8G8B8: return argb;
  case VX_TEX_FORMAT_R5G6B5: return ((r >> 3) << 11) | ((g >> 2) << 5) | (b >> 3);
  case VX_TEX_FORMAT_A1R5G5B5:
    return ((a != 0) << 15) | ((r >> 3) << 10) | ((g >> 3) << 5) | (b >> 3);
  case VX_TEX_FORMAT_A4R4G4B4: return ((a >> 4) << 12) | ((r >> 4) << 8) | ((g >> 4) << 4) | (b >> 4);
  case VX_TEX_FORMAT_A8L8: return (a << 8) | r;
  case VX_TEX_FORMAT_L8: return r;
  default: return a;  /* VX_TEX_FORMAT_A8 */
  }
}

static uint32_t tex_stride(uint32_t format) {  /* graphics.cpp:55-70 FormatStride */
  switch (format) {
  case VX_TEX_FORMAT_A8R8G8B8: return 4;
  case VX_TEX_FORMAT_L8:
  case VX_TEX_FORMAT_A8: return 1;
  default: return 2;
  }
}

static uint32_t ld_texel(const uint8_t* p, uint32_t stride) {
  uint32_t t = 0;
  for (uint32_t i = 0; i < stride; ++i) t |= (uint32_t)p[i] << (8 * i);
  return t;
}
static void st_texel(uint8_t* p, uint32_t stride, uint32_t t) {
  for (uint32_t i = 0; i < stride; ++i) p[i] = (uint8_t)(t >> (8 * i));
}

/* decoded A8R8G8B8 of a stored texel: the sampler's Unpack8888 (bit
 * replication) through its point filter */
static uint32_t tex_decode(uint32_t t, uint32_t format) {
  orc_dcstate_t s;
  memset(&s, 0, sizeof(s));
  uint8_t px[4];
  st_texel(px, tex_stride(format), t);
  s.tex_base = px;
  s.tex_format = format;
  s.tex_filter = VX_TEX_FILTER_POINT;
  return orc_tex_read(&s, 0, 0);
}

/* Texture image of `format` with its full mip chain (LoadImage +
 * GenerateMipmaps, tex/main.cpp:173-183).  out may be NULL (size query);
 * mipoff[16] receives the byte offset of every level (0 beyond the chain,
 * as the unwritten MIPOFF DCRs).  Returns the total byte size. */
size_t orc_tex_build(const uint32_t* argb, uint32_t w, uint32_t h, uint32_t format, uint8_t* out,
                     uint32_t* mipoff, uint32_t* levels) {
  const uint32_t stride = tex_stride(format);
  size_t total = 0;
  uint32_t lw = w, lh = h, n = 0;
  for (;;) {
    if (mipoff && n < 16) mipoff[n] = (uint32_t)total;
    total += (size_t)lw * lh * stride;
    ++n;
    if (lw == 1 && lh == 1) break;
    lw = lw > 1 ? lw / 2 : 1;
    lh = lh > 1 ? lh / 2 : 1;
  }
  if (mipoff)
    for (uint32_t i = n; i < 16; ++i) mipoff[i] = 0;
  if (levels) *levels = n;
  if (!out) return total;
  for (uint32_t i = 0; i < w * h; ++i) st_texel(out + (size_t)i * stride, stride, orc_tex_encode(argb[i], format));
  size_t off = 0;
  lw = w; lh = h;
  for (uint32_t l = 1; l < n; ++l) {
    const uint32_t nw = lw > 1 ? lw / 2 : 1, nh = lh > 1 ? lh / 2 : 1;
    const uint8_t* src = out + off;
    uint8_t* dst = out + off + (size_t)lw * lh * stride;
    for (uint32_t y = 0; y < nh; ++y)
      for (uint32_t x = 0; x < nw; ++x) {
        uint32_t sum[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t sx = lw > 1 ? 2 * x + (k & 1) : 0, sy = lh > 1 ? 2 * y + (k >> 1) : 0;
          const uint32_t c = tex_decode(ld_texel(src + ((size_t)sy * lw + sx) * stride, stride), format);
          for (int ch = 0; ch < 4; ++ch) sum[ch] += (c >> (8 * ch)) & 0xff;
        }
        uint32_t c = 0;
        for (int ch = 0; ch < 4; ++ch) c |= (sum[ch] >> 2) << (8 * ch);
        st_texel(dst + ((size_t)y * nw + x) * stride, stride, orc_tex_encode(c, format));
      }
    off += (size_t)lw * lh * stride;
    lw = nw;
    lh = nh;
  }
  return total;
}

static uint32_t log2floor_u(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

/* tex/kernel.cpp main(): lod and blend fraction from the minification */
void orc_tex_lod(uint32_t logw, uint32_t logh, uint32_t dst_w, uint32_t dst_h, uint32_t* lod,
                 uint32_t* frac) {
  const float wr = (float)(1u << logw) / (float)dst_w;
  const float hr = (float)(1u << logh) / (float)dst_h;
  const float mn = fmaxf(wr, hr);
  const int32_t j = fx_from_float_dev(fmaxf(mn, 1.0f), 16);
  uint32_t l = log2floor_u((uint32_t)j) - 16u;
  if (l > VX_TEX_LOD_MAX) l = VX_TEX_LOD_MAX;
  *lod = l;
  *frac = (uint32_t)((j - (int32_t)(1u << (l + 16))) >> (l + 16 - 8));
}

/* TextureSampler::read at a lod (graphics.cpp:253-314) */
static uint32_t sample(const uint8_t* tex, const uint32_t* mipoff, uint32_t logw, uint32_t logh,
                       uint32_t format, uint32_t bilinear, uint32_t wrap, uint32_t lod, int32_t u,
                       int32_t v) {
  orc_dcstate_t s;
  memset(&s, 0, sizeof(s));
  s.tex_base = tex + mipoff[lod];
  s.tex_logw = (uint32_t)((int32_t)logw - (int32_t)lod > 0 ? (int32_t)logw - (int32_t)lod : 0);
  s.tex_logh = (uint32_t)((int32_t)logh - (int32_t)lod > 0 ? (int32_t)logh - (int32_t)lod : 0);
  s.tex_format = format;
  s.tex_filter = bilinear ? VX_TEX_FILTER_BILINEAR : VX_TEX_FILTER_POINT;
  s.tex_wrapu = wrap;
  s.tex_wrapv = wrap;
  return orc_tex_read(&s, u, v);
}

static uint32_t lerp8888_(uint32_t a, uint32_t b, uint32_t f) {  /* graphics.h:82-86 */
  const uint32_t p = a * (0xff - f) + b * f + 0x00800080u;
  const uint32_t q = (p >> 8) & 0x00ff00ffu;
  return ((p + q) >> 8) & 0x00ff00ffu;
}

/* tex/kernel.cpp kernel_body over all num_tasks tasks: dst (dst_w x dst_h
 * ARGB8888, row 0 = top) from the texture.  filter: 0 point, 1 bilinear,
 * 2 bilinear + blend with the next lod (tex/main.cpp -g). */
void orc_tex_render(const uint8_t* tex, const uint32_t* mipoff, uint32_t logw, uint32_t logh,
                    uint32_t format, uint32_t wrap, uint32_t filter, uint32_t dst_w, uint32_t dst_h,
                    uint32_t num_tasks, uint32_t* dst) {
  const uint32_t tile_h = (dst_h + num_tasks - 1) / num_tasks;
  const float dX = 1.0f / (float)dst_w, dY = 1.0f / (float)dst_h;
  uint32_t lod, frac;
  orc_tex_lod(logw, logh, dst_w, dst_h, &lod, &frac);
  const uint32_t lodn = lod + 1 < VX_TEX_LOD_MAX ? lod + 1 : VX_TEX_LOD_MAX;
  for (uint32_t task = 0; task < num_tasks; ++task) {
    const uint32_t y0 = task * tile_h;
    const uint32_t y1 = y0 + tile_h < dst_h ? y0 + tile_h : dst_h;
    float fv = ((float)y0 + 0.5f) * dY;
    for (uint32_t y = y0; y < y1; ++y) {
      float fu = (0.0f + 0.5f) * dX;
      for (uint32_t x = 0; x < dst_w; ++x) {
        const int32_t xu = fx_from_float_dev(fu, VX_TEX_FXD_FRAC);
        const int32_t xv = fx_from_float_dev(fv, VX_TEX_FXD_FRAC);
        uint32_t color;
        if (filter == 2) {
          const uint32_t t0 = sample(tex, mipoff, logw, logh, format, 1, wrap, lod, xu, xv);
          const uint32_t t1 = sample(tex, mipoff, logw, logh, format, 1, wrap, lodn, xu, xv);
          const uint32_t cl = lerp8888_(t0 & 0x00ff00ffu, t1 & 0x00ff00ffu, frac);
          const uint32_t ch = lerp8888_((t0 >> 8) & 0x00ff00ffu, (t1 >> 8) & 0x00ff00ffu, frac);
          color = (ch << 8) | cl;
        } else {
          color = sample(tex, mipoff, logw, logh, format, filter, wrap, lod, xu, xv);
        }
        dst[(size_t)y * dst_w + x] = color;
        fu += dX;
      }
      fv += dY;
    }
  }
}
