/* lbvh.c -- CPU restatement of the GPU BVH builder
 * (skybox_rt_amd/csrc/kernels/bvh_build.hip).  TEST INFRASTRUCTURE ONLY
 * (see oracle.h): the tests compare the device-built node and triangle
 * arrays with these bit for bit, and trace frames over them.
 *
 * NO REFERENCE (the reference has no BVH): the
 * algorithm is the linear BVH of Karras 2012 ("Maximizing parallelism in
 * the construction of BVHs, octrees and k-d trees"): 30-bit Morton codes of
 * the triangle centroids normalised to the centroid bounds, sorted stably
 * (= by (code, index)), the binary radix tree over the unique 62-bit keys
 * code << 32 | index, boxes bottom-up; subtrees of <= 4 triangles become
 * leaves.  Parity of the resulting frames is pinned through brute force
 * (any BVH gives the same closest hit); the tree itself is this build's own
 * definition -- "parity unpinned" in the reference sense. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define LEAF_FLAG 0x80000000u
#define EMPTY_REF (-1)
#define LEAF_MAX 4

static void tri_box(const float* v, uint32_t t, float* lo, float* hi) {
  const float* a = v + 9 * (size_t)t;
  for (int k = 0; k < 3; ++k) {
    lo[k] = fminf(fminf(a[k], a[3 + k]), a[6 + k]);
    hi[k] = fmaxf(fmaxf(a[k], a[3 + k]), a[6 + k]);
  }
}

static uint32_t expand10(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

static uint32_t quant(float c, float lo, float hi) {
  const float e = hi - lo;
  const float t = e > 0.0f ? (c - lo) / e : 0.0f;
  const uint32_t q = (uint32_t)(t * 1024.0f);
  return q < 1023u ? q : 1023u;
}

typedef struct {
  uint32_t code, idx;
} kv_t;

static int kv_cmp(const void* x, const void* y) {
  const kv_t* a = (const kv_t*)x;
  const kv_t* b = (const kv_t*)y;
  if (a->code != b->code) return a->code < b->code ? -1 : 1;
  return a->idx < b->idx ? -1 : (a->idx > b->idx);
}

static int delta(const kv_t* k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint64_t a = ((uint64_t)k[i].code << 32) | k[i].idx;
  const uint64_t b = ((uint64_t)k[j].code << 32) | k[j].idx;
  return __builtin_clzll(a ^ b);
}

static void set_child(float* node, int ch, const float* lo, const float* hi, float pad, int32_t ref) {
  const int empty = ref == EMPTY_REF;
  for (int k = 0; k < 3; ++k) {
    node[4 * k + 2 * ch + 0] = empty ? 0.0f : lo[k] - pad;
    node[4 * k + 2 * ch + 1] = empty ? 0.0f : hi[k] + pad;
  }
  memcpy(&node[12 + ch], &ref, 4);
}

int orc_lbvh_build(const float* verts, const float* geom, uint32_t n_, float* nodes, float* tris,
                   uint32_t* depth_out) {
  const int n = (int)n_;
  if (n <= 0) return -1;
  /* bounds: centroids, centroid bounds, max |coordinate| (bvh_build.hip phase_bounds) */
  float* cen = (float*)malloc(sizeof(float) * 3 * (size_t)n);
  float* box = (float*)malloc(sizeof(float) * 6 * 2 * (size_t)n); /* internal [0,n), leaves [n,2n) */
  kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)n);
  int* parent = (int*)malloc(sizeof(int) * 2 * (size_t)n);
  int* child = (int*)malloc(sizeof(int) * 2 * (size_t)n);
  uint32_t* range = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (size_t)n);
  if (!cen || !box || !kv || !parent || !child || !range) return -2;
  float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
  float am = 0.0f;
  for (int t = 0; t < n; ++t) {
    float lo[3], hi[3];
    tri_box(verts, (uint32_t)t, lo, hi);
    for (int k = 0; k < 3; ++k) {
      const float c = (lo[k] + hi[k]) * 0.5f;
      cen[3 * t + k] = c;
      cmin[k] = fminf(cmin[k], c);
      cmax[k] = fmaxf(cmax[k], c);
      am = fmaxf(am, fmaxf(fabsf(lo[k]), fabsf(hi[k])));
    }
  }
  /* Morton codes, sorted by (code, index) = the stable LSD radix sort */
  for (int t = 0; t < n; ++t) {
    kv[t].code = (expand10(quant(cen[3 * t], cmin[0], cmax[0])) << 2) |
                 (expand10(quant(cen[3 * t + 1], cmin[1], cmax[1])) << 1) |
                 expand10(quant(cen[3 * t + 2], cmin[2], cmax[2]));
    kv[t].idx = (uint32_t)t;
  }
  qsort(kv, (size_t)n, sizeof(kv_t), kv_cmp);
  /* binary radix tree (phase_tree) */
  for (int i = 0; i < n - 1; ++i) {
    const int d = (delta(kv, n, i, i + 1) - delta(kv, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(kv, n, i, i - d);
    int lmax = 2;
    while (delta(kv, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
      if (delta(kv, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(kv, n, i, j);
    int s = 0, t = l;
    do {
      t = (t + 1) / 2;
      if (delta(kv, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int g = i + s * d + (d < 0 ? -1 : 0);
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    const int c0 = (lo == g) ? ~g : g, c1 = (hi == g + 1) ? ~(g + 1) : g + 1;
    child[2 * i] = c0;
    child[2 * i + 1] = c1;
    range[2 * i] = (uint32_t)lo;
    range[2 * i + 1] = (uint32_t)hi;
    parent[c0 >= 0 ? c0 : n + ~c0] = i;
    parent[c1 >= 0 ? c1 : n + ~c1] = i;
  }
  parent[0] = -1;
  /* boxes: leaves, then internal nodes children-first (a node's index is
   * not ordered w.r.t. its children's, so recurse from the root) */
  for (int k = 0; k < n; ++k) tri_box(verts, kv[k].idx, &box[6 * (n + k)], &box[6 * (n + k) + 3]);
  if (n >= 2) {
    int* stack = (int*)malloc(sizeof(int) * 2 * (size_t)n);
    unsigned char* seen = (unsigned char*)calloc((size_t)n, 1);
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
      const int p = stack[sp - 1];
      const int c0 = child[2 * p], c1 = child[2 * p + 1];
      if (!seen[p]) {
        seen[p] = 1;
        if (c0 >= 0) stack[sp++] = c0;
        if (c1 >= 0) stack[sp++] = c1;
        continue;
      }
      --sp;
      const float* b0 = &box[6 * (c0 >= 0 ? c0 : n + ~c0)];
      const float* b1 = &box[6 * (c1 >= 0 ? c1 : n + ~c1)];
      for (int k = 0; k < 3; ++k) {
        box[6 * p + k] = fminf(b0[k], b1[k]);
        box[6 * p + 3 + k] = fmaxf(b0[3 + k], b1[3 + k]);
      }
    }
    free(stack);
    free(seen);
  }
  /* emit (phase_emit) */
  const float pad = fmaxf(am * (1.0f / 65536.0f), 1e-6f);
  for (int k = 0; k < n; ++k) memcpy(&tris[12 * (size_t)k], &geom[12 * (size_t)kv[k].idx], 48);
  memset(&tris[12 * (size_t)n], 0, 3 * 48);
  uint32_t depth = 1;
  const int nn = n > 1 ? n - 1 : 1;
  memset(nodes, 0, sizeof(float) * 16 * (size_t)nn);
  if (n <= LEAF_MAX) {
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
      lo[k] = box[6 * n + k];
      hi[k] = box[6 * n + 3 + k];
    }
    for (int q = 1; q < n; ++q)
      for (int k = 0; k < 3; ++k) {
        lo[k] = fminf(lo[k], box[6 * (n + q) + k]);
        hi[k] = fmaxf(hi[k], box[6 * (n + q) + 3 + k]);
      }
    set_child(nodes, 0, lo, hi, pad, (int32_t)(LEAF_FLAG | (uint32_t)(n - 1)));
    set_child(nodes, 1, lo, hi, pad, EMPTY_REF);
  } else {
    for (int i = 0; i < n - 1; ++i) {
      const uint32_t size = range[2 * i + 1] - range[2 * i] + 1;
      if (i != 0 && size <= LEAF_MAX) continue;
      float* nd = &nodes[16 * (size_t)i];
      for (int ch = 0; ch < 2; ++ch) {
        const int c = child[2 * i + ch];
        int32_t ref;
        int bi;
        if (c < 0) {
          ref = (int32_t)(LEAF_FLAG | ((uint32_t)~c << 4));
          bi = n + ~c;
        } else {
          const uint32_t cs = range[2 * c + 1] - range[2 * c] + 1;
          ref = cs <= LEAF_MAX ? (int32_t)(LEAF_FLAG | (range[2 * c] << 4) | (cs - 1)) : c;
          bi = c;
        }
        set_child(nd, ch, &box[6 * bi], &box[6 * bi + 3], pad, ref);
      }
      uint32_t dd = 1;
      for (int p = i; p != 0; p = parent[p]) ++dd;
      if (dd > depth) depth = dd;
    }
  }
  if (depth_out) *depth_out = depth;
  free(cen);
  free(box);
  free(kv);
  free(parent);
  free(child);
  free(range);
  return 0;
}

/* ---- BVH4 collapse (bvh_build.hip phase_collapse) --------------------------
 * Restated top-down: a DFS from the root over internal refs carries each
 * node's depth and the stack its BVH4 ancestors have pushed; the device
 * decides per node by walking parent links instead -- same nodes, same slots,
 * same bound. */
static int ref_of(const float* nd, int ch) {
  int32_t r;
  memcpy(&r, &nd[12 + ch], 4);
  return r;
}

static int collapse_slots(const float* nodes, int i, float* o) {
  int cnt = 0;
  const float* nd = nodes + 16 * (size_t)i;
  for (int ch = 0; ch < 2; ++ch) {
    const int32_t r = ref_of(nd, ch);
    if (r == EMPTY_REF) continue;
    const float* src = nd;
    int g0 = ch, g1 = ch;
    if (r >= 0) { src = nodes + 16 * (size_t)r; g0 = 0; g1 = 1; }
    for (int g = g0; g <= g1; ++g) {
      const int32_t rr = ref_of(src, g);
      if (rr == EMPTY_REF) continue;
      if (o) {
        for (int k = 0; k < 3; ++k) {
          o[8 * k + cnt] = src[4 * k + 2 * g];
          o[8 * k + 4 + cnt] = src[4 * k + 2 * g + 1];
        }
        memcpy(&o[24 + cnt], &rr, 4);
      }
      ++cnt;
    }
  }
  return cnt;
}

int orc_lbvh_collapse4(const float* nodes, uint32_t nn, float* nodes4, uint32_t* stack_out) {
  if (nn == 0) return -1;
  memset(nodes4, 0, sizeof(float) * 32 * (size_t)nn);
  /* explicit DFS stack: (node, depth, pushes of the BVH4 ancestors) */
  int* st = (int*)malloc(sizeof(int) * 3 * (size_t)(nn + 1));
  if (!st) return -2;
  int sp = 0;
  uint32_t worst = 0;
  st[0] = 0; st[1] = 0; st[2] = 0; sp = 1;
  while (sp) {
    --sp;
    const int i = st[3 * sp], d = st[3 * sp + 1], acc = st[3 * sp + 2];
    int acc2 = acc;
    if ((d & 1) == 0) {
      float* o = nodes4 + 32 * (size_t)i;
      const int32_t e = EMPTY_REF;
      for (int q = 0; q < 4; ++q) memcpy(&o[24 + q], &e, 4);
      const int cnt = collapse_slots(nodes, i, o);
      acc2 = acc + (cnt > 0 ? cnt - 1 : 0);
      if ((uint32_t)acc2 > worst) worst = (uint32_t)acc2;
    }
    const float* nd = nodes + 16 * (size_t)i;
    for (int ch = 0; ch < 2; ++ch) {
      const int32_t r = ref_of(nd, ch);
      if (r >= 0 && (uint32_t)r < nn) {
        st[3 * sp] = r; st[3 * sp + 1] = d + 1; st[3 * sp + 2] = acc2;
        ++sp;
      }
    }
  }
  free(st);
  *stack_out = worst;
  return 0;
}

/* ---- binary16 box planes (the kernels' rt_node4h_t) ----------------------
 * Restates app/bvh.cpp HalfRound / HalfBits and the device phase
 * BVHB_HALF (kernels/bvh_build.hip): every plane of a BVH4 node rounded
 * outward to a binary16-representable value (lower planes down, upper planes
 * up; exact scaling by the binade's quantum, floor / ceil, saturating
 * outward past +-65504), the fp32 node rewritten with the rounded values and
 * the 64-B half record emitted (24 halves in rt_node4_t plane order, then
 * the 4 child refs). */
static float half_round(float x, int dir) {
  if (isnan(x) || isinf(x) || x == 0.0f) return x;
  const float kmax = 65504.0f;
  if (x > kmax) return dir < 0 ? kmax : INFINITY;
  if (x < -kmax) return dir < 0 ? -INFINITY : -kmax;
  int e;
  frexpf(fabsf(x), &e);
  int q = e - 1 > -14 ? e - 1 : -14;
  q -= 10;
  const float m = ldexpf(x, -q);
  const float r = dir < 0 ? floorf(m) : ceilf(m);
  const float v = ldexpf(r, q);
  return v > kmax ? INFINITY : (v < -kmax ? -INFINITY : v);
}

static uint16_t half_bits(float v) {
  uint32_t u;
  memcpy(&u, &v, 4);
  const uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
  const float a = fabsf(v);
  if (a == 0.0f) return sign;
  if (isinf(a)) return (uint16_t)(sign | 0x7c00u);
  int e;
  const float m = frexpf(a, &e);
  if (e - 1 >= -14)
    return (uint16_t)(sign | ((uint32_t)(e - 1 + 15) << 10) | (uint32_t)ldexpf(2.0f * m - 1.0f, 10));
  return (uint16_t)(sign | (uint32_t)ldexpf(a, 24));
}

int orc_half4(float* nodes4, uint32_t nn, void* half) {
  uint8_t* out = (uint8_t*)half;
  for (uint32_t i = 0; i < nn; ++i) {
    float* n = nodes4 + 32 * (size_t)i;
    uint16_t b[24];
    for (int k = 0; k < 24; ++k) {
      const int upper = (k & 4) != 0; /* lo.x[4] hi.x[4] lo.y[4] hi.y[4] ... */
      n[k] = half_round(n[k], upper ? 1 : -1);
      b[k] = half_bits(n[k]);
    }
    memcpy(out + 64 * (size_t)i, b, 48);
    memcpy(out + 64 * (size_t)i + 48, &n[24], 16);
  }
  return 0;
}
