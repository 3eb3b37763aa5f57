// bvh.cpp -- see bvh.h.
#include "bvh.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace rt {
namespace {

// --- binary16 box planes (rt_node4h_t) ------------------------------------
// The nearest binary16-representable value below (dir < 0) or above
// (dir > 0) x, as a float: x scaled by the binary16 quantum of its binade is
// an exact float, floor/ceil of it is exact, and so is scaling back.  Beyond
// the binary16 range a lower bound saturates to -/+65504 or -inf and an upper
// bound to +/-65504 or +inf -- always outward, so a rounded box contains the
// original one and the slab test (monotone in the planes under round-to-
// nearest arithmetic) accepts every ray the unrounded box accepted.
float HalfRound(float x, int dir) {
  if (std::isnan(x) || std::isinf(x) || x == 0.0f) return x;
  const float kMax = 65504.0f;
  if (x > kMax) return dir < 0 ? kMax : INFINITY;
  if (x < -kMax) return dir < 0 ? -INFINITY : -kMax;
  int e;
  std::frexp(std::fabs(x), &e);                     // |x| in [2^(e-1), 2^e)
  const int q = std::max(e - 1, -14) - 10;          // quantum 2^q (subnormals: 2^-24)
  const float m = std::ldexp(x, -q);                // exact
  const float r = dir < 0 ? std::floor(m) : std::ceil(m);
  const float v = std::ldexp(r, q);                 // exact (|r| <= 2048)
  return v > kMax ? INFINITY : (v < -kMax ? -INFINITY : v);
}

// binary16 encoding of a float that is exactly representable in binary16
uint16_t HalfBits(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  const uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
  const float a = std::fabs(v);
  if (a == 0.0f) return sign;
  if (std::isinf(a)) return (uint16_t)(sign | 0x7c00u);
  int e;
  const float m = std::frexp(a, &e);               // a = m 2^e, m in [0.5, 1)
  if (e - 1 >= -14)
    return (uint16_t)(sign | ((uint32_t)(e - 1 + 15) << 10) |
                      (uint32_t)std::ldexp(2.0f * m - 1.0f, 10));
  return (uint16_t)(sign | (uint32_t)std::ldexp(a, 24));  // subnormal: a = f 2^-24
}

float HalfValue(uint16_t h) {
  const int ex = (h >> 10) & 31, f = h & 1023;
  float v;
  if (ex == 31) v = f ? NAN : INFINITY;
  else if (ex == 0) v = std::ldexp((float)f, -24);
  else v = std::ldexp((float)(1024 + f), ex - 25);
  return (h & 0x8000u) ? -v : v;
}


double g_wside = 1.0;

struct Box {
  float lo[3] = {INFINITY, INFINITY, INFINITY};
  float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const float* p) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  // SAH area; g_wside weighs the faces that extend along w (probe knob)
  double area() const {
    if (lo[0] > hi[0]) return 0.0;
    const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    return 2.0 * (dx * dy + g_wside * (dy * dz + dz * dx));
  }
};

class Builder {
 public:
  Builder(const std::vector<BuildTri>& t, Bvh* out, const BvhParams& bp)
      : t_(t), out_(out), leaf_(bp.leaf_size), bins_(bp.bins), all_axes_(bp.all_axes) {
    box_.resize(t.size());
    cen_.resize(t.size());
    float ext = 0.0f;
    for (size_t i = 0; i < t.size(); ++i) {
      for (int c = 0; c < 3; ++c) {
        box_[i].grow(t[i].v[c]);
        for (int k = 0; k < 3; ++k) ext = std::max(ext, std::fabs(t[i].v[c][k]));
      }
      for (int k = 0; k < 3; ++k) cen_[i][k] = (box_[i].lo[k] + box_[i].hi[k]) * 0.5f;
    }
    pad_ = std::max(ext * (1.0f / 65536.0f), 1e-6f);
    idx_.resize(t.size());
    for (size_t i = 0; i < t.size(); ++i) idx_[i] = (uint32_t)i;
  }

  void run() {
    out_->nodes.clear();
    out_->tris.clear();
    out_->depth = 0;
    out_->leaves = 0;
    if (t_.empty()) return;
    if (t_.size() <= leaf_) {  // root must be internal: leaf + empty child
      out_->nodes.resize(1);
      Box b = range_box(0, (uint32_t)t_.size());
      const int32_t leaf = make_leaf(0, (uint32_t)t_.size());
      set_child(0, 0, b, leaf);
      set_child(0, 1, Box(), RT_EMPTY_REF);
      out_->depth = 1;
      return;
    }
    build(0, (uint32_t)t_.size(), 1);
  }

 private:
  Box range_box(uint32_t b, uint32_t e) const {
    Box r;
    for (uint32_t i = b; i < e; ++i) r.grow(box_[idx_[i]]);
    return r;
  }

  int32_t make_leaf(uint32_t b, uint32_t e) {
    const uint32_t first = (uint32_t)out_->tris.size();
    for (uint32_t i = b; i < e; ++i) {
      const BuildTri& s = t_[idx_[i]];
      rt_tri_t r;
      std::memset(&r, 0, sizeof(r));
      // v0, e1 = v1 - v0, e2 = v2 - v0 in fp32 (same as oracle/rt.c)
      for (int k = 0; k < 3; ++k) {
        r.v[k] = s.v[0][k];
        r.v[4 + k] = s.v[1][k] - s.v[0][k];
        r.v[8 + k] = s.v[2][k] - s.v[0][k];
      }
      std::memcpy(&r.v[3], &s.pid, 4);
      out_->tris.push_back(r);
    }
    ++out_->leaves;
    return (int32_t)(RT_LEAF_FLAG | (first << 4) | (e - b - 1));
  }

  void set_child(uint32_t node, int ch, const Box& b, int32_t ref) {
    rt_node_t& n = out_->nodes[node];
    for (int k = 0; k < 3; ++k) {
      const bool empty = ref == RT_EMPTY_REF;
      n.v[4 * k + 2 * ch + 0] = empty ? 0.0f : b.lo[k] - pad_;
      n.v[4 * k + 2 * ch + 1] = empty ? 0.0f : b.hi[k] + pad_;
    }
    std::memcpy(&n.v[12 + ch], &ref, 4);
  }

  // returns the child reference for range [b, e)
  int32_t build(uint32_t b, uint32_t e, uint32_t depth) {
    const uint32_t n = e - b;
    if (n <= leaf_) return make_leaf(b, e);
    out_->depth = std::max(out_->depth, depth);
    const uint32_t node = (uint32_t)out_->nodes.size();
    out_->nodes.emplace_back();
    std::memset(&out_->nodes[node], 0, sizeof(rt_node_t));
    const uint32_t mid = split(b, e);
    const Box lb = range_box(b, mid), rb = range_box(mid, e);
    const int32_t l = build(b, mid, depth + 1);
    const int32_t r = build(mid, e, depth + 1);
    set_child(node, 0, lb, l);
    set_child(node, 1, rb, r);
    return (int32_t)node;
  }

  // full-sweep SAH (bins == 0): every axis, every split position of the
  // triangles sorted by centroid (ties by index); the range is left sorted
  // along the chosen axis
  uint32_t split_sweep(uint32_t b, uint32_t e) {
    const uint32_t n = e - b;
    std::vector<uint32_t> ord(n);
    std::vector<double> left(n);
    double best = INFINITY;
    int best_axis = -1;
    uint32_t best_nl = 0;
    for (int axis = 0; axis < 3; ++axis) {
      std::copy(idx_.begin() + b, idx_.begin() + e, ord.begin());
      std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
        return cen_[x][axis] < cen_[y][axis] || (cen_[x][axis] == cen_[y][axis] && x < y);
      });
      Box acc;
      for (uint32_t i = 0; i < n; ++i) {
        acc.grow(box_[ord[i]]);
        left[i] = acc.area();
      }
      Box r;
      for (uint32_t i = n; i-- > 1;) {  // right = ord[i..n), left = ord[0..i)
        r.grow(box_[ord[i]]);
        const double c = (double)i * left[i - 1] + (double)(n - i) * r.area();
        if (c < best) { best = c; best_axis = axis; best_nl = i; }
      }
    }
    if (best_axis < 0) return b + n / 2;
    const int axis = best_axis;
    std::sort(idx_.begin() + b, idx_.begin() + e, [&](uint32_t x, uint32_t y) {
      return cen_[x][axis] < cen_[y][axis] || (cen_[x][axis] == cen_[y][axis] && x < y);
    });
    return b + best_nl;
  }

  // binned SAH over centroids (the widest centroid axis, or every axis with
  // all_axes); stable partition
  uint32_t split(uint32_t b, uint32_t e) {
    if (bins_ == 0) return split_sweep(b, e);
    float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = b; i < e; ++i)
      for (int k = 0; k < 3; ++k) {
        cl[k] = std::min(cl[k], cen_[idx_[i]][k]);
        ch[k] = std::max(ch[k], cen_[idx_[i]][k]);
      }
    int wide = 0;
    for (int k = 1; k < 3; ++k)
      if (ch[k] - cl[k] > ch[wide] - cl[wide]) wide = k;
    const uint32_t median = b + (e - b) / 2;
    const uint32_t nb = bins_;
    auto bin_of = [&](uint32_t t, int axis) {
      const float ext = ch[axis] - cl[axis];
      int bi = (int)((cen_[t][axis] - cl[axis]) * ((float)nb / ext));
      return std::min(std::max(bi, 0), (int)nb - 1);
    };
    double best = INFINITY;
    uint32_t best_s = 0;
    int best_axis = -1;
    for (int axis = 0; axis < 3; ++axis) {
      if (!all_axes_ && axis != wide) continue;
      if (!(ch[axis] - cl[axis] > 0.0f)) continue;
      Box bb[kBvhMaxBins];
      uint32_t cnt[kBvhMaxBins] = {};
      for (uint32_t i = b; i < e; ++i) {
        const int bi = bin_of(idx_[i], axis);
        bb[bi].grow(box_[idx_[i]]);
        ++cnt[bi];
      }
      // suffix sweep: right boxes/counts for every split position
      Box rs[kBvhMaxBins];
      uint32_t rc[kBvhMaxBins] = {};
      Box acc;
      uint32_t na = 0;
      for (uint32_t s = nb; s-- > 1;) {
        acc.grow(bb[s]);
        na += cnt[s];
        rs[s] = acc;
        rc[s] = na;
      }
      Box l;
      uint32_t nl = 0;
      for (uint32_t s = 1; s < nb; ++s) {
        l.grow(bb[s - 1]);
        nl += cnt[s - 1];
        if (nl == 0 || rc[s] == 0) continue;
        const double c = nl * l.area() + rc[s] * rs[s].area();
        if (c < best) { best = c; best_s = s; best_axis = axis; }
      }
    }
    if (best_axis < 0) return median;
    auto mid_it = std::stable_partition(idx_.begin() + b, idx_.begin() + e, [&](uint32_t t) {
      return (uint32_t)bin_of(t, best_axis) < best_s;
    });
    return (uint32_t)(mid_it - idx_.begin());
  }

  const std::vector<BuildTri>& t_;
  Bvh* out_;
  std::vector<Box> box_;
  std::vector<std::array<float, 3>> cen_;
  std::vector<uint32_t> idx_;
  float pad_ = 0.0f;
  uint32_t leaf_, bins_;
  bool all_axes_;
};

// Collapse the BVH2 into a BVH4 (W = 4): a node's children are repeatedly
// replaced by the children of its largest-area internal child (in place, so
// the order stays left to right) until it has W or none is internal.  Boxes
// are copied verbatim from the BVH2 nodes that stored them.  Nodes are
// numbered in preorder into nodes4 (rt_node4_t).  (An 8-wide collapse, walked
// by opt-in BVH8 images, measured slower than the BVH4 everywhere in r05 and
// was removed in r06: DESIGN.md 2.8.)
template <int W>
class Collapser {
  static_assert(W == 4, "rt_node4_t: four children per node");
 public:
  explicit Collapser(Bvh* b) : b_(b) {}
  void run() {
    out().clear();
    depth() = 0;
    if (b_->nodes.empty()) {
      stack() = 0;
      return;
    }
    uint32_t st = 0;
    collapse(0, 1, &st);
    stack() = st;
  }

 private:
  std::vector<rt_node4_t>& out() { return b_->nodes4; }
  uint32_t& depth() { return b_->depth4; }
  uint32_t& stack() { return b_->stack4; }
  struct Child {
    float lo[3], hi[3];
    int32_t ref;
  };
  Child child_of(uint32_t n, int ch) const {
    const rt_node_t& nd = b_->nodes[n];
    Child c;
    for (int k = 0; k < 3; ++k) {
      c.lo[k] = nd.v[4 * k + 2 * ch + 0];
      c.hi[k] = nd.v[4 * k + 2 * ch + 1];
    }
    std::memcpy(&c.ref, &nd.v[12 + ch], 4);
    return c;
  }
  static double area(const Child& c) {
    const double dx = (double)c.hi[0] - c.lo[0], dy = (double)c.hi[1] - c.lo[1],
                 dz = (double)c.hi[2] - c.lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
  // returns the BVH4 index of BVH2 node n; *stack = worst-case stack
  // entries needed below (and including) this node
  uint32_t collapse(uint32_t n, uint32_t depth, uint32_t* stack) {
    this->depth() = std::max(this->depth(), depth);
    std::vector<Child> cs;
    for (int ch = 0; ch < 2; ++ch) {
      const Child c = child_of(n, ch);
      if (c.ref != RT_EMPTY_REF) cs.push_back(c);
    }
    while (cs.size() < (size_t)W) {
      int best = -1;
      double ba = -1.0;
      for (size_t i = 0; i < cs.size(); ++i)
        if (cs[i].ref >= 0 && area(cs[i]) > ba) { ba = area(cs[i]); best = (int)i; }
      if (best < 0) break;
      const uint32_t m = (uint32_t)cs[best].ref;
      std::vector<Child> sub;
      for (int ch = 0; ch < 2; ++ch) {
        const Child c = child_of(m, ch);
        if (c.ref != RT_EMPTY_REF) sub.push_back(c);
      }
      cs.erase(cs.begin() + best);
      cs.insert(cs.begin() + best, sub.begin(), sub.end());
    }
    constexpr int H = W / 4;  // rt_node4_t halves per node
    const uint32_t idx = (uint32_t)(out().size() / H);
    out().resize(out().size() + H);
    uint32_t below = 0;
    for (size_t i = 0; i < cs.size(); ++i)
      if (cs[i].ref >= 0) {
        uint32_t st = 0;
        cs[i].ref = (int32_t)collapse((uint32_t)cs[i].ref, depth + 1, &st);
        below = std::max(below, st);
      }
    for (int h = 0; h < H; ++h) {
      rt_node4_t& o = out()[(size_t)idx * H + h];
      std::memset(&o, 0, sizeof(o));
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * h + j;
        const bool used = i < (int)cs.size();
        for (int k = 0; k < 3; ++k) {
          o.v[8 * k + j] = used ? cs[i].lo[k] : 0.0f;
          o.v[8 * k + 4 + j] = used ? cs[i].hi[k] : 0.0f;
        }
        const int32_t ref = used ? cs[i].ref : RT_EMPTY_REF;
        std::memcpy(&o.v[24 + j], &ref, 4);
      }
    }
    // descending into one child pushes at most the other (cs.size() - 1)
    *stack = (uint32_t)(cs.empty() ? 0 : cs.size() - 1) + below;
    return idx;
  }
  Bvh* b_;
};

}  // namespace

int BuildBvh(const std::vector<BuildTri>& tris, Bvh* out, std::string* error) {
  if (out == nullptr) return -1;
  if (tris.size() >= (1u << 26)) {
    if (error) *error = "too many triangles for the 27-bit leaf index";
    return -1;
  }
  BvhParams bp;
  // build knobs for A/B runs (defaults are the measured best)
  if (const char* v = std::getenv("RT_BVH_LEAF")) bp.leaf_size = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RT_BVH_BINS")) bp.bins = (uint32_t)std::atoi(v);
  if (const char* v = std::getenv("RT_BVH_AXES")) bp.all_axes = std::atoi(v) == 3;
  if (const char* v = std::getenv("RT_BVH_F16")) bp.f16_boxes = std::atoi(v) != 0;
  g_wside = std::getenv("RT_BVH_WSIDE") ? std::atof(std::getenv("RT_BVH_WSIDE")) : 1.0;
  return BuildBvhWith(tris, bp, out, error);
}

int BuildBvhWith(const std::vector<BuildTri>& tris, const BvhParams& bp, Bvh* out,
                 std::string* error) {
  if (out == nullptr) return -1;
  if (tris.size() >= (1u << 26)) {
    if (error) *error = "too many triangles for the 27-bit leaf index";
    return -1;
  }
  if (bp.leaf_size < 1 || bp.leaf_size > 4 || bp.bins == 1 || bp.bins > kBvhMaxBins) {
    if (error) *error = "bad BVH build parameters (leaf 1..4, bins 0 (sweep) or 2..64)";
    return -1;
  }
  Builder b(tris, out, bp);
  b.run();
  Collapser<4>(out).run();
  // binary16 box planes: round every BVH4 box outward (RT_BVH_F16=0 keeps
  // the fp32 planes, rt_node4h_t is then not uploaded), pack rt_node4h_t and
  // check that it decodes to exactly rt_node4_t's planes
  out->nodes4h.clear();
  if (bp.f16_boxes) {
    out->nodes4h.resize(out->nodes4.size());
    for (size_t n = 0; n < out->nodes4.size(); ++n) {
      rt_node4_t& o = out->nodes4[n];
      rt_node4h_t& h = out->nodes4h[n];
      for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 4; ++i) {
          float& lo = o.v[8 * k + i];
          float& hi = o.v[8 * k + 4 + i];
          lo = HalfRound(lo, -1);
          hi = HalfRound(hi, +1);
          h.b[8 * k + i] = HalfBits(lo);
          h.b[8 * k + 4 + i] = HalfBits(hi);
          if (HalfValue(h.b[8 * k + i]) != lo || HalfValue(h.b[8 * k + 4 + i]) != hi) {
            if (error) *error = "binary16 box packing mismatch";
            return -1;
          }
        }
      std::memcpy(h.child, &o.v[24], 16);
    }
  }
  if (out->depth > RT_STACK_DEEP) {
    if (error) *error = "BVH deeper than RT_STACK_DEEP";
    return -1;
  }
  return 0;
}

}  // namespace rt
