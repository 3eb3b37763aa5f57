// tex_app.cpp -- librtapp.so: the texture regression app behind
// include/vx_tex.h (the reference's tests/regression/tex/main.cpp host side,
// kernel.cpp's per-task setup) on the public vortex.h API.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "VX_types.h"
#include "app_util.h"
#include "tex_common.h"
#include "vortex.h"
#include "vortex_hip.h"
#include "vx_rt.h"
#include "vx_tex.h"

namespace {

using rtapp::set_error;

uint32_t stride_of(uint32_t format) {  // graphics.cpp:55-70 FormatStride
  switch (format) {
    case VX_TEX_FORMAT_A8R8G8B8: return 4;
    case VX_TEX_FORMAT_L8:
    case VX_TEX_FORMAT_A8: return 1;
    default: return 2;
  }
}

// LoadImage(path, eformat) conversion from A8R8G8B8 (cocogfx, not vendored;
// the rules are pinned by the reference's toad_ref_f0..f6 goldens)
uint32_t encode(uint32_t argb, uint32_t format) {
  const uint32_t a = argb >> 24, r = (argb >> 16) & 0xff, g = (argb >> 8) & 0xff, b = argb & 0xff;
  switch (format) {
    case VX_TEX_FORMAT_A8R8G8B8: return argb;
    case VX_TEX_FORMAT_R5G6B5: return ((r >> 3) << 11) | ((g >> 2) << 5) | (b >> 3);
    case VX_TEX_FORMAT_A1R5G5B5:
      return (uint32_t(a != 0) << 15) | ((r >> 3) << 10) | ((g >> 3) << 5) | (b >> 3);
    case VX_TEX_FORMAT_A4R4G4B4:
      return ((a >> 4) << 12) | ((r >> 4) << 8) | ((g >> 4) << 4) | (b >> 4);
    case VX_TEX_FORMAT_A8L8: return (a << 8) | r;
    case VX_TEX_FORMAT_L8: return r;
    default: return a;
  }
}

// Unpack8888 of a stored texel back to A8R8G8B8 (graphics.cpp:72-122)
uint32_t decode(uint32_t t, uint32_t format) {
  uint32_t r, g, b, a;
  switch (format) {
    case VX_TEX_FORMAT_A8R8G8B8: return t;
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
      a = (uint32_t)((int32_t)(t << 16) >> 31) & 0xff;
      break;
    case VX_TEX_FORMAT_A4R4G4B4:
      r = ((t >> 4) & 0xf0) | ((t >> 8) & 0x0f);
      g = (t & 0xf0) | ((t >> 4) & 0x0f);
      b = ((t << 4) & 0xf0) | (t & 0x0f);
      a = ((t >> 8) & 0xf0) | ((t >> 12) & 0x0f);
      break;
    case VX_TEX_FORMAT_A8L8: r = g = b = t & 0xff; a = (t >> 8) & 0xff; break;
    case VX_TEX_FORMAT_L8: r = g = b = t & 0xff; a = 0xff; break;
    default: r = g = b = 0xff; a = t & 0xff; break;
  }
  return (a << 24) | (r << 16) | (g << 8) | b;
}

uint32_t load_texel(const uint8_t* p, uint32_t stride) {
  uint32_t t = 0;
  for (uint32_t i = 0; i < stride; ++i) t |= (uint32_t)p[i] << (8 * i);
  return t;
}
void store_texel(uint8_t* p, uint32_t stride, uint32_t t) {
  for (uint32_t i = 0; i < stride; ++i) p[i] = (uint8_t)(t >> (8 * i));
}

// TFixed<F>(float) in the reference's kernel (RISC-V fcvt.w.s: truncating,
// saturating, NaN -> INT_MAX)
int32_t fx_dev(float f, int frac) {
  const float x = f * (float)(1u << frac);
  if (x != x) return INT32_MAX;
  if (x >= 2147483648.0f) return INT32_MAX;
  if (x < -2147483648.0f) return INT32_MIN;
  return (int32_t)x;
}

bool pow2(uint32_t v) { return v && !(v & (v - 1)); }
uint32_t log2u(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

}  // namespace

int rt_tex_build_image(const uint32_t* argb, uint32_t w, uint32_t h, uint32_t format, uint8_t* out,
                       uint64_t* size, uint32_t mipoff[16], uint32_t* levels) {
  if (!argb || !size || !mipoff || w == 0 || h == 0) return set_error("null argument");
  if (format > VX_TEX_FORMAT_A8) return set_error("invalid texture format");
  const uint32_t stride = stride_of(format);
  uint64_t total = 0;
  uint32_t lw = w, lh = h, n = 0;
  for (;;) {  // level sizes: halve each side down to 1x1
    if (n < 16) mipoff[n] = (uint32_t)total;
    total += (uint64_t)lw * lh * stride;
    ++n;
    if (lw == 1 && lh == 1) break;
    lw = std::max(lw / 2, 1u);
    lh = std::max(lh / 2, 1u);
  }
  if (n > VX_TEX_LOD_MAX) return set_error("texture has more mip levels than VX_TEX_LOD_MAX");
  for (uint32_t i = n; i < 16; ++i) mipoff[i] = 0;
  if (levels) *levels = n;
  if (!out) {
    *size = total;
    return 0;
  }
  if (*size < total) return set_error("buffer too small");
  *size = total;
  for (uint64_t i = 0; i < (uint64_t)w * h; ++i) store_texel(out + i * stride, stride, encode(argb[i], format));
  // GenerateMipmaps (cocogfx, not vendored; unpinned): 2x2 box filter of the
  // decoded level above, truncating, re-encoded
  uint64_t off = 0;
  lw = w;
  lh = h;
  for (uint32_t l = 1; l < n; ++l) {
    const uint32_t nw = std::max(lw / 2, 1u), nh = std::max(lh / 2, 1u);
    const uint8_t* src = out + off;
    uint8_t* dst = out + off + (uint64_t)lw * lh * stride;
    for (uint32_t y = 0; y < nh; ++y)
      for (uint32_t x = 0; x < nw; ++x) {
        uint32_t sum[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t sx = lw > 1 ? 2 * x + (k & 1) : 0, sy = lh > 1 ? 2 * y + (k >> 1) : 0;
          const uint32_t c = decode(load_texel(src + ((uint64_t)sy * lw + sx) * stride, stride), format);
          for (int ch = 0; ch < 4; ++ch) sum[ch] += (c >> (8 * ch)) & 0xff;
        }
        uint32_t c = 0;
        for (int ch = 0; ch < 4; ++ch) c |= (sum[ch] >> 2) << (8 * ch);
        store_texel(dst + ((uint64_t)y * nw + x) * stride, stride, encode(c, format));
      }
    off += (uint64_t)lw * lh * stride;
    lw = nw;
    lh = nh;
  }
  return 0;
}

struct rt_tex {
  vx_device_h dev = nullptr;
  vx_buffer_h krnl[3] = {nullptr, nullptr, nullptr}, tex = nullptr, dst = nullptr, utab = nullptr, vtab = nullptr,
              args = nullptr;
  tex_kernel_arg_t arg{};
  rt_tex_stats_t st{};
  bool configured = false;
  vx_hip_last_run_t last_run = nullptr;
  ~rt_tex() {
    for (vx_buffer_h* b : {&krnl[0], &krnl[1], &krnl[2], &tex, &dst, &utab, &vtab, &args}) {
      if (*b) vx_mem_free(*b);
      *b = nullptr;
    }
    if (dev) vx_dev_close(dev);
  }
};

namespace {
int upload(vx_device_h dev, const void* data, uint64_t size, int flags, vx_buffer_h* buf,
           uint64_t* addr) {
  const uint64_t sz = size ? size : 64;
  if (*buf) vx_mem_free(*buf);
  *buf = nullptr;
  if (vx_mem_alloc(dev, sz, flags, buf) != 0) return set_error("vx_mem_alloc failed");
  if (data && size && vx_copy_to_dev(*buf, data, 0, size) != 0)
    return set_error("vx_copy_to_dev failed");
  if (vx_mem_address(*buf, addr) != 0) return set_error("vx_mem_address failed");
  if (*addr + sz > (1ull << 32)) return set_error("buffer beyond the 4 GiB kernel address range");
  return 0;
}
}  // namespace

int rt_tex_create(const char* kernel_dir, rt_tex_h* out) {
  if (!out) return set_error("null argument");
  auto t = std::make_unique<rt_tex>();
  if (vx_dev_open(&t->dev) != 0) {
    t->dev = nullptr;
    return set_error("vx_dev_open failed (no GPU or driver missing)");
  }
  uint64_t isa = 0;
  if (vx_dev_caps(t->dev, VX_CAPS_ISA_FLAGS, &isa) != 0 || !(isa & VX_ISA_EXT_TEX))
    return set_error("texture extension not supported");  // tex/main.cpp:200-206
  const std::string dir = kernel_dir ? kernel_dir : rtapp::library_dir();
  for (int f = 0; f < 3; ++f) {  // one image per filter (-g 0/1/2)
    const std::string path = dir + "/tex_kernel_f" + std::to_string(f) + ".vxbin";
    if (vx_upload_kernel_file(t->dev, path.c_str(), &t->krnl[f]) != 0)
      return set_error("cannot upload kernel " + path);
  }
  t->last_run = (vx_hip_last_run_t)vx_driver_symbol("vx_hip_last_run");
  // the tex app reports its pixel counter (rt_tex_stats): counter rows on
  if (auto sc = (vx_hip_set_counters_t)vx_driver_symbol("vx_hip_set_counters")) sc(t->dev, 1);
  *out = t.release();
  return 0;
}

int rt_tex_free(rt_tex_h t) {
  delete t;
  return 0;
}

int rt_tex_configure(rt_tex_h t, const uint32_t* argb, uint32_t w, uint32_t h,
                     const rt_tex_params_t* p) {
  if (!t || !argb || !p) return set_error("null argument");
  if (!pow2(w) || !pow2(h)) return set_error("only power of two textures supported");
  if (p->format > VX_TEX_FORMAT_A8 || p->wrap > VX_TEX_WRAP_MIRROR || p->filter > 2)
    return set_error("invalid format / wrap / filter");
  t->configured = false;
  tex_kernel_arg_t& a = t->arg;
  std::memset(&a, 0, sizeof(a));
  uint64_t size = 0;
  uint32_t levels = 0;
  if (rt_tex_build_image(argb, w, h, p->format, nullptr, &size, a.mipoff, &levels)) return -1;
  std::vector<uint8_t> texels(size);
  if (rt_tex_build_image(argb, w, h, p->format, texels.data(), &size, a.mipoff, &levels)) return -1;
  // tex/main.cpp:173-190: dst = (uint32_t)(src * scale)
  const uint32_t dw = (uint32_t)((float)w * p->scale), dh = (uint32_t)((float)h * p->scale);
  if (dw == 0 || dh == 0) return set_error("empty destination image");
  if ((uint64_t)dw * dh * 4 >= (1ull << 31)) return set_error("destination image too large");
  uint64_t ncores = 0, nwarps = 0, nthreads = 0;
  vx_dev_caps(t->dev, VX_CAPS_NUM_CORES, &ncores);
  vx_dev_caps(t->dev, VX_CAPS_NUM_WARPS, &nwarps);
  vx_dev_caps(t->dev, VX_CAPS_NUM_THREADS, &nthreads);
  const uint64_t caps_tasks = ncores * nwarps * nthreads;
  const uint32_t ntasks = (uint32_t)std::min<uint64_t>(p->num_tasks ? p->num_tasks : caps_tasks, dh);
  // kernel.cpp main() + kernel_body: lod/frac from the minification and the
  // float coordinates each task walks (fu from x = 0 per row; fv from its
  // first row, tile_height rows per task), replayed once per column / row
  const uint32_t logw = log2u(w), logh = log2u(h);
  {
    const float wr = (float)(1u << logw) / (float)dw, hr = (float)(1u << logh) / (float)dh;
    const int32_t j = fx_dev(std::max(std::max(wr, hr), 1.0f), 16);
    a.lod = std::min<uint32_t>(log2u((uint32_t)j) - 16, VX_TEX_LOD_MAX);
    a.frac = (uint32_t)((j - (int32_t)(1u << (a.lod + 16))) >> (a.lod + 16 - 8));
  }
  const float dX = 1.0f / (float)dw, dY = 1.0f / (float)dh;
  const uint32_t grp = TEX_GROUP(p->filter);
  const uint32_t gpr = (dw + grp - 1) / grp;  // groups per row
  std::vector<int32_t> ut(gpr * grp, 0), vt(dh);
  float fu = (0 + 0.5f) * dX;
  for (uint32_t x = 0; x < dw; ++x, fu += dX) ut[x] = fx_dev(fu, VX_TEX_FXD_FRAC);
  const uint32_t tile_h = (dh + ntasks - 1) / ntasks;
  for (uint32_t y0 = 0; y0 < dh; y0 += tile_h) {
    float fv = ((float)y0 + 0.5f) * dY;
    for (uint32_t y = y0; y < std::min(y0 + tile_h, dh); ++y, fv += dY) vt[y] = fx_dev(fv, VX_TEX_FXD_FRAC);
  }
  // TEX DCRs as tex/main.cpp:233-246 writes them (the kernel reads them from
  // its argument; the DCR writes keep the vortex.h call sequence)
  vx_dcr_write(t->dev, VX_DCR_TEX_STAGE, 0);
  vx_dcr_write(t->dev, VX_DCR_TEX_LOGDIM, (logh << 16) | logw);
  vx_dcr_write(t->dev, VX_DCR_TEX_FORMAT, p->format);
  vx_dcr_write(t->dev, VX_DCR_TEX_WRAP, (p->wrap << 16) | p->wrap);
  vx_dcr_write(t->dev, VX_DCR_TEX_FILTER, p->filter ? VX_TEX_FILTER_BILINEAR : VX_TEX_FILTER_POINT);
  if (upload(t->dev, texels.data(), size, VX_MEM_READ, &t->tex, &a.tex_addr) ||
      upload(t->dev, ut.data(), ut.size() * 4, VX_MEM_READ, &t->utab, &a.utab_addr) ||
      upload(t->dev, vt.data(), vt.size() * 4, VX_MEM_READ, &t->vtab, &a.vtab_addr) ||
      upload(t->dev, nullptr, (uint64_t)dw * dh * 4, VX_MEM_WRITE, &t->dst, &a.dst_addr))
    return -1;
  vx_dcr_write(t->dev, VX_DCR_TEX_ADDR, (uint32_t)(a.tex_addr / 64));
  for (uint32_t i = 0; i < levels; ++i) vx_dcr_write(t->dev, VX_DCR_TEX_MIPOFF(i), a.mipoff[i]);
  a.dst_width = dw;
  a.dst_height = dh;
  a.filter = p->filter;
  a.logw = logw;
  a.logh = logh;
  a.format = p->format;
  a.wrap = p->wrap;
  a.num_tasks = dh * gpr * 64;
  uint64_t args_addr = 0;
  if (upload(t->dev, &a, sizeof(a), VX_MEM_READ, &t->args, &args_addr)) return -1;
  std::memset(&t->st, 0, sizeof(t->st));
  t->st.dst_width = dw;
  t->st.dst_height = dh;
  t->st.lod = a.lod;
  t->st.frac = a.frac;
  t->st.levels = levels;
  t->st.num_tasks = ntasks;
  t->st.texture_bytes = size;
  t->configured = true;
  return 0;
}

int rt_tex_render(rt_tex_h t) {
  if (!t || !t->configured) return set_error("texture app not configured");
  if (vx_start(t->dev, t->krnl[t->arg.filter], t->args) != 0) return set_error("vx_start failed");
  return vx_ready_wait(t->dev, VX_MAX_TIMEOUT) == 0 ? 0 : set_error("vx_ready_wait failed");
}

int rt_tex_stats(rt_tex_h t, rt_tex_stats_t* st) {
  if (!t || !st || !t->configured) return set_error("texture app not configured");
  *st = t->st;
  vx_mpm_query(t->dev, VX_CSR_MPM_BASE + TEX_MPM_USER + TEX_STAT_PIXELS, 0, &st->pixels);
  if (t->last_run) t->last_run(t->dev, &st->kernel_ms, &st->grid, &st->block);
  return 0;
}

int rt_tex_read(rt_tex_h t, uint32_t* out, uint64_t count) {
  if (!t || !out || !t->configured) return set_error("texture app not configured");
  const uint64_t n = (uint64_t)t->arg.dst_width * t->arg.dst_height;
  if (count < n) return set_error("buffer too small");
  return vx_copy_from_dev(out, t->dst, 0, n * 4) == 0 ? 0 : set_error("vx_copy_from_dev failed");
}
