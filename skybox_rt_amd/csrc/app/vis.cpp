// vis.cpp -- see vis.h.
#include "vis.h"

#include <algorithm>
#include <cstring>
#include <string>

#include "bvh.h"

namespace rt {
namespace {

constexpr int64_t kQ24 = int64_t(1) << 24;

int64_t FloorDiv(int64_t a, int64_t b) {  // b > 0
  int64_t q = a / b;
  if (a % b != 0 && a < 0) --q;
  return q;
}
int64_t CeilDiv(int64_t a, int64_t b) { return -FloorDiv(-a, b); }  // b > 0

// draw3d's edge value at an integer pixel: a*x + b*y + c in uint32, read as
// int32 (graphics.cpp:640-642)
int32_t EdgeAt(const int32_t* e, uint32_t x, uint32_t y) {
  return (int32_t)((uint32_t)e[0] * x + (uint32_t)e[1] * y + (uint32_t)e[2]);
}

// Lower bound of the masked depth word (Z & 0xffffff) over the covered
// pixels of a primitive whose z attribute is (a0-a2, a1-a2, a2) in Q7.24.
// The shader (draw3d/kernel.cpp:37-59; gfx_device.h shade_edges) computes
// Z = a2 + ((a0 * dx) >> 24) + ((a1 * dy) >> 24) (mod 2^32) with
// dx = fx(r*f0), dy = fx(r*f1), r = 1/(f0+f1+f2), f_i = E_i * 2^-24 >= 0 at a
// covered pixel: dx, dy >= 0 and dx + dy <= 2^24 + 8 (four roundings of at
// most 2^-24 relative each), so a0*dx + a1*dy lies between min and max of
// {0, a0*T, a1*T} (T = 2^24 + 8, the corners of that triangle) and each
// floor loses less than 1.  When [Zlo, Zhi] stays inside one 2^24 period the
// masked word is >= Zlo mod 2^24; otherwise the bound is 0.  The one case
// outside the argument -- all three edge values 0 at a covered pixel, where
// r is infinite and dx = dy = INT32_MAX -- is caught by the caller (bound 0).
uint32_t DepthLowerBound(const int32_t* z) {
  const int64_t T = kQ24 + 8;
  const int64_t p0 = (int64_t)z[0] * T, p1 = (int64_t)z[1] * T;
  const int64_t lo = std::min<int64_t>({0, p0, p1}), hi = std::max<int64_t>({0, p0, p1});
  const int64_t zlo = (int64_t)z[2] + FloorDiv(lo, kQ24) - 4;
  const int64_t zhi = (int64_t)z[2] + FloorDiv(hi, kQ24) + 4;
  if (FloorDiv(zlo, kQ24) != FloorDiv(zhi, kQ24)) return 0;
  return (uint32_t)(zlo - FloorDiv(zlo, kQ24) * kQ24);
}

uint32_t Pack(uint32_t lo, uint32_t hi) { return lo | (hi << 16); }

}  // namespace

VisPrim ComputeVisPrim(const rt_prim_t& p, bool ok, const rt_bbox_t& bb, uint32_t width,
                       uint32_t height) {
  VisPrim v;
  if (!ok) return v;
  const uint32_t L = bb.x & 0xffffu, R = bb.x >> 16, T = bb.y & 0xffffu, B = bb.y >> 16;
  if (R <= L || B <= T) return v;
  // the 32x32 tiles the screen box was binned to (gfxutil.cpp:237-250), clipped
  // to the viewport (graphics.cpp:813-825 scissor)
  const uint32_t X0 = (L >> RT_TILE_LOG) << RT_TILE_LOG;
  const uint32_t X1 = std::min(((R + 31u) >> RT_TILE_LOG) << RT_TILE_LOG, width);
  const uint32_t Y0 = (T >> RT_TILE_LOG) << RT_TILE_LOG;
  const uint32_t Y1 = std::min(((B + 31u) >> RT_TILE_LOG) << RT_TILE_LOG, height);
  const int32_t* e = &p.edges[0][0];
  uint32_t xmin = UINT32_MAX, xmax = 0, ymin = UINT32_MAX, ymax = 0;
  bool all_zero = false;
  for (uint32_t y = Y0; y < Y1; ++y) {
    int64_t lo = X0, hi = (int64_t)X1 - 1, d[3];
    bool exact = true;
    for (int i = 0; i < 3 && exact; ++i) {
      const int64_t a = e[3 * i];
      d[i] = (int64_t)e[3 * i + 1] * y + e[3 * i + 2];
      const int64_t vl = a * X0 + d[i], vr = a * ((int64_t)X1 - 1) + d[i];
      // linear along the row: no int32 wrap between the ends iff none at them
      if (vl < INT32_MIN || vl > INT32_MAX || vr < INT32_MIN || vr > INT32_MAX) {
        exact = false;
        break;
      }
      if (a > 0) lo = std::max(lo, CeilDiv(-d[i], a));
      else if (a < 0) hi = std::min(hi, FloorDiv(d[i], -a));
      else if (d[i] < 0) hi = lo - 1;
    }
    if (!exact) {  // wrapping edge values: pixel by pixel, as the rasterizer does
      for (uint32_t x = X0; x < X1; ++x) {
        const int32_t e0 = EdgeAt(e, x, y), e1 = EdgeAt(e + 3, x, y), e2 = EdgeAt(e + 6, x, y);
        if (e0 < 0 || e1 < 0 || e2 < 0) continue;
        xmin = std::min(xmin, x); xmax = std::max(xmax, x);
        ymin = std::min(ymin, y); ymax = std::max(ymax, y);
        all_zero |= (e0 | e1 | e2) == 0;
      }
      continue;
    }
    if (lo > hi) continue;
    xmin = std::min(xmin, (uint32_t)lo); xmax = std::max(xmax, (uint32_t)hi);
    ymin = std::min(ymin, y); ymax = std::max(ymax, y);
    // a covered pixel where all three edge values are 0 (see DepthLowerBound)
    int k = 0;
    while (k < 3 && e[3 * k] == 0) ++k;
    if (k == 3) {
      all_zero |= d[0] == 0 && d[1] == 0 && d[2] == 0;
    } else if ((-d[k]) % e[3 * k] == 0) {
      const int64_t x = -d[k] / e[3 * k];
      all_zero |= x >= lo && x <= hi && e[0] * x + d[0] == 0 && e[3] * x + d[1] == 0 &&
                  e[6] * x + d[2] == 0;
    }
  }
  if (xmin == UINT32_MAX) return v;
  v.any = true;
  v.rx = Pack(xmin, xmax);
  v.ry = Pack(ymin, ymax);
  v.zmin = all_zero ? 0u : DepthLowerBound(p.attribs[0]);
  return v;
}

rt_vtri_t MakeVisTri(const rt_prim_t& p, const VisPrim& v, int32_t pid) {
  rt_vtri_t t;
  std::memcpy(t.edges, p.edges, sizeof(t.edges));
  t.rx = v.rx;
  t.ry = v.ry;
  t.pid = pid;
  std::memcpy(t.z, p.attribs[0], sizeof(t.z));
  t.zmin = v.zmin;
  return t;
}

namespace {

struct Cover {
  uint32_t x0 = 0xffffu, x1 = 0, y0 = 0xffffu, y1 = 0, zmin = RT_VIS_ZMIN_NONE;
  bool any = false;
  void add(const Cover& c) {
    if (!c.any) return;
    any = true;
    x0 = std::min(x0, c.x0); x1 = std::max(x1, c.x1);
    y0 = std::min(y0, c.y0); y1 = std::max(y1, c.y1);
    zmin = std::min(zmin, c.zmin);
  }
};

// a node's slots in ascending depth bound (stable; empty slots, bound
// RT_VIS_ZMIN_NONE, last): the order the primary walks enter children, so
// the kernels take needed children in slot order with no sort per step
void SortSlots(rt_vnode_t& n) {
  for (int i = 1; i < 4; ++i)
    for (int j = i; j > 0 && n.zmin[j] < n.zmin[j - 1]; --j) {
      std::swap(n.lo[j], n.lo[j - 1]);
      std::swap(n.hi[j], n.hi[j - 1]);
      std::swap(n.zmin[j], n.zmin[j - 1]);
      std::swap(n.child[j], n.child[j - 1]);
    }
}

struct NodeBuilder {
  const std::vector<std::array<int32_t, 4>>& refs;
  const std::vector<int32_t>& pids;
  const std::vector<VisPrim>& by_pid;
  std::vector<rt_vnode_t>* out;
  int err = 0;

  Cover of(int32_t ref, int depth) {
    Cover c;
    if (ref == RT_EMPTY_REF || depth > 64) {
      if (depth > 64) err = -1;
      return c;
    }
    if (ref < 0) {  // leaf: its triangle records
      const uint32_t lr = (uint32_t)ref, first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      for (uint32_t k = first; k < first + count; ++k) {
        if (k >= pids.size() || pids[k] < 0 || (size_t)pids[k] >= by_pid.size()) {
          err = -1;
          return c;
        }
        const VisPrim& v = by_pid[pids[k]];
        if (!v.any) continue;
        Cover t;
        t.any = true;
        t.x0 = v.rx & 0xffffu; t.x1 = v.rx >> 16;
        t.y0 = v.ry & 0xffffu; t.y1 = v.ry >> 16;
        t.zmin = v.zmin;
        c.add(t);
      }
      return c;
    }
    if ((size_t)ref >= refs.size()) {
      err = -1;
      return c;
    }
    rt_vnode_t& n = (*out)[ref];
    for (int i = 0; i < 4; ++i) {
      const Cover k = of(refs[ref][i], depth + 1);
      n.child[i] = k.any ? refs[ref][i] : RT_EMPTY_REF;
      n.lo[i] = k.any ? Pack(k.x0, k.y0) : RT_VIS_EMPTY_RECT;
      n.hi[i] = k.any ? Pack(k.x1, k.y1) : RT_VIS_EMPTY_RECT;
      n.zmin[i] = k.any ? k.zmin : RT_VIS_ZMIN_NONE;
      c.add(k);
    }
    SortSlots(n);
    return c;
  }
};

}  // namespace

int BuildVisNodes(const std::vector<std::array<int32_t, 4>>& refs,
                  const std::vector<int32_t>& leaf_pids, const std::vector<VisPrim>& by_pid,
                  std::vector<rt_vnode_t>* out) {
  out->assign(refs.size(), rt_vnode_t{});
  for (rt_vnode_t& n : *out)
    for (int i = 0; i < 4; ++i) {
      n.lo[i] = n.hi[i] = RT_VIS_EMPTY_RECT;
      n.zmin[i] = RT_VIS_ZMIN_NONE;
      n.child[i] = RT_EMPTY_REF;
    }
  if (refs.empty()) return 0;
  NodeBuilder b{refs, leaf_pids, by_pid, out};
  b.of(0, 0);
  return b.err;
}

int BuildScreenTree(const std::vector<VisPrim>& by_pid, const std::vector<int32_t>& geometry,
                    float depth_scale, std::vector<std::array<int32_t, 4>>* refs,
                    std::vector<int32_t>* leaf_pids, uint32_t* stack4) {
  refs->clear();
  leaf_pids->clear();
  *stack4 = 0;
  std::vector<BuildTri> bt;
  for (int32_t g : geometry) {
    const VisPrim& v = by_pid[g];
    if (!v.any) continue;
    // a degenerate "triangle" spanning the rectangle [x0, x1 + 1) x [y0, y1 + 1)
    // at depth z: its box is the rectangle, so the builder's SAH is on area
    const float z = depth_scale * (float)v.zmin * (1.0f / 16777216.0f);
    BuildTri t;
    t.v[0][0] = (float)(v.rx & 0xffffu); t.v[0][1] = (float)(v.ry & 0xffffu); t.v[0][2] = z;
    t.v[1][0] = (float)((v.rx >> 16) + 1); t.v[1][1] = (float)((v.ry >> 16) + 1); t.v[1][2] = z;
    t.v[2][0] = t.v[0][0]; t.v[2][1] = t.v[0][1]; t.v[2][2] = z;
    t.pid = g;
    bt.push_back(t);
  }
  if (bt.empty()) return 0;
  BvhParams bp;
  bp.f16_boxes = false;
  bp.all_axes = true;
  Bvh b;
  std::string err;
  if (BuildBvhWith(bt, bp, &b, &err) != 0) return -1;
  for (const rt_node4_t& n : b.nodes4) {
    std::array<int32_t, 4> c;
    std::memcpy(c.data(), &n.v[24], 16);
    refs->push_back(c);
  }
  for (const rt_tri_t& t : b.tris) {
    int32_t pid;
    std::memcpy(&pid, &t.v[3], 4);
    leaf_pids->push_back(pid);
  }
  *stack4 = b.stack4;
  return 0;
}

}  // namespace rt
