// png.cpp -- see png.h.
#include "png.h"

#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace rt {
namespace {

void put_be32(std::vector<uint8_t>* v, uint32_t x) {
  v->push_back((uint8_t)(x >> 24));
  v->push_back((uint8_t)(x >> 16));
  v->push_back((uint8_t)(x >> 8));
  v->push_back((uint8_t)x);
}
uint32_t get_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

void chunk(std::vector<uint8_t>* out, const char* type, const std::vector<uint8_t>& data) {
  put_be32(out, (uint32_t)data.size());
  const size_t start = out->size();
  out->insert(out->end(), type, type + 4);
  out->insert(out->end(), data.begin(), data.end());
  const uLong crc = crc32(0L, out->data() + start, (uInt)(out->size() - start));
  put_be32(out, (uint32_t)crc);
}

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

}  // namespace

int SavePngARGB(const std::string& path, const uint32_t* argb, uint32_t w, uint32_t h) {
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (w * 4 + 1));
  for (uint32_t y = 0; y < h; ++y) {
    const uint32_t* row = argb + (size_t)(h - 1 - y) * w;  // flip: row 0 is the bottom
    raw.push_back(0);
    for (uint32_t x = 0; x < w; ++x) {
      const uint32_t c = row[x];
      raw.push_back((uint8_t)(c >> 16));
      raw.push_back((uint8_t)(c >> 8));
      raw.push_back((uint8_t)c);
      raw.push_back((uint8_t)(c >> 24));
    }
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return -1;
  z.resize(zlen);
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put_be32(&ihdr, w);
  put_be32(&ihdr, h);
  ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA
  chunk(&png, "IHDR", ihdr);
  chunk(&png, "IDAT", z);
  chunk(&png, "IEND", {});
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return -1;
  const bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
  std::fclose(f);
  return ok ? 0 : -1;
}

int LoadPngARGB(const std::string& path, std::vector<uint32_t>* argb, uint32_t* width,
                uint32_t* height) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return -1;
  std::vector<uint8_t> d;
  uint8_t buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + n);
  std::fclose(f);
  if (d.size() < 8 || std::memcmp(d.data(), "\x89PNG\r\n\x1a\n", 8) != 0) return -1;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = 0, interlace = 0;
  std::vector<uint8_t> idat;
  for (size_t p = 8; p + 12 <= d.size();) {
    const uint32_t len = get_be32(&d[p]);
    if (p + 12 + len > d.size()) return -1;
    const char* type = (const char*)&d[p + 4];
    const uint8_t* data = &d[p + 8];
    if (!std::memcmp(type, "IHDR", 4)) {
      w = get_be32(data);
      h = get_be32(data + 4);
      depth = data[8];
      ctype = data[9];
      interlace = data[12];
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), data, data + len);
    }
    p += 12 + len;
  }
  const int ch = ctype == 6 ? 4 : ctype == 2 ? 3 : 0;
  if (depth != 8 || ch == 0 || interlace != 0 || w == 0 || h == 0) return -1;
  const size_t stride = (size_t)w * ch;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf rl = (uLongf)raw.size();
  if (uncompress(raw.data(), &rl, idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size())
    return -1;
  std::vector<uint8_t> img(stride * h), prev(stride, 0);
  for (uint32_t y = 0; y < h; ++y) {
    const uint8_t ft = raw[y * (stride + 1)];
    const uint8_t* src = &raw[y * (stride + 1) + 1];
    uint8_t* dst = &img[y * stride];
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= (size_t)ch ? dst[x - ch] : 0, b = prev[x], c = x >= (size_t)ch ? prev[x - ch] : 0;
      int v = src[x];
      switch (ft) {
      case 1: v += a; break;
      case 2: v += b; break;
      case 3: v += (a + b) / 2; break;
      case 4: v += paeth(a, b, c); break;
      default: break;
      }
      dst[x] = (uint8_t)v;
    }
    std::memcpy(prev.data(), dst, stride);
  }
  argb->resize((size_t)w * h);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    const uint8_t* p = &img[i * ch];
    const uint32_t a = ch == 4 ? p[3] : 0xff;
    (*argb)[i] = (a << 24) | ((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2];
  }
  *width = w;
  *height = h;
  return 0;
}

int64_t CompareARGB(const uint32_t* a, const uint32_t* b, uint64_t count, int tol) {
  int64_t errors = 0;
  for (uint64_t i = 0; i < count; ++i) {
    int m = 0;
    for (int s = 0; s < 32; s += 8) {
      const int d = std::abs((int)((a[i] >> s) & 0xff) - (int)((b[i] >> s) & 0xff));
      m = d > m ? d : m;
    }
    if (m > tol) ++errors;
  }
  return errors;
}

}  // namespace rt
