/*
 * vis.c -- oracle restatement of the RT kernels' primary-visibility records
 * (skybox_rt_amd/csrc/app/vis.cpp, kernels/rt_common.h "primary
 * visibility").  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The product computes each primitive's covered-pixel rectangle row by row
 * with exact integer arithmetic; here it is found by brute force, by
 * evaluating draw3d's coverage rule at every pixel of every 32x32 tile the
 * primitive was binned to -- the oracle raster's own binning (raster.c,
 * gfxutil.cpp:237-271) and edge test (graphics.cpp:640-642, 813-825).  The
 * depth lower bound is a definition of the RT path (NO REFERENCE), restated
 * from vis.cpp DepthLowerBound; every covered pixel's actual depth word is
 * checked against it in tests/test_vis.py.
 */
#include <stdlib.h>
#include <string.h>

#include "gfx.h"

#define Q24 ((int64_t)1 << 24)

static int64_t floor_div(int64_t a, int64_t b) {  /* b > 0 */
  int64_t q = a / b;
  if (a % b != 0 && a < 0) --q;
  return q;
}

/* vis.cpp DepthLowerBound: Z = a2 + ((a0*dx) >> 24) + ((a1*dy) >> 24) with
 * dx, dy >= 0, dx + dy <= 2^24 + 8 at a covered pixel; bound of Z mod 2^24 */
static uint32_t depth_lower_bound(const int32_t z[3]) {
  const int64_t T = Q24 + 8;
  const int64_t p0 = (int64_t)z[0] * T, p1 = (int64_t)z[1] * T;
  int64_t lo = 0, hi = 0;
  if (p0 < lo) lo = p0;
  if (p1 < lo) lo = p1;
  if (p0 > hi) hi = p0;
  if (p1 > hi) hi = p1;
  const int64_t zlo = (int64_t)z[2] + floor_div(lo, Q24) - 4;
  const int64_t zhi = (int64_t)z[2] + floor_div(hi, Q24) + 4;
  if (floor_div(zlo, Q24) != floor_div(zhi, Q24)) return 0;
  return (uint32_t)(zlo - floor_div(zlo, Q24) * Q24);
}

void orc_vis_prim_compute(const orc_rast_prim_t* p, int ok, const int32_t bb[4], uint32_t width,
                          uint32_t height, orc_vis_prim_t* out) {
  out->rx = out->ry = 0x0000ffffu;
  out->zmin = 0xffffffffu;
  out->any = 0;
  if (!ok) return;
  const uint32_t tx0 = (uint32_t)bb[0] >> 5, tx1 = ((uint32_t)bb[1] + 31) >> 5;
  const uint32_t ty0 = (uint32_t)bb[2] >> 5, ty1 = ((uint32_t)bb[3] + 31) >> 5;
  uint32_t x0 = 0xffffffffu, x1 = 0, y0 = 0xffffffffu, y1 = 0;
  int all_zero = 0;
  for (uint32_t y = ty0 << 5; y < (ty1 << 5) && y < height; ++y)
    for (uint32_t x = tx0 << 5; x < (tx1 << 5) && x < width; ++x) {
      const int32_t e0 = orc_edge_eval(p->edges[0], x, y);
      const int32_t e1 = orc_edge_eval(p->edges[1], x, y);
      const int32_t e2 = orc_edge_eval(p->edges[2], x, y);
      if (e0 < 0 || e1 < 0 || e2 < 0) continue;
      if (x < x0) x0 = x;
      if (x > x1) x1 = x;
      if (y < y0) y0 = y;
      if (y > y1) y1 = y;
      if ((e0 | e1 | e2) == 0) all_zero = 1;
    }
  if (x0 == 0xffffffffu) return;
  out->any = 1;
  out->rx = x0 | (x1 << 16);
  out->ry = y0 | (y1 << 16);
  out->zmin = all_zero ? 0u : depth_lower_bound(p->attribs[0]);
}

int orc_vis_prims(const orc_scene_t* s, uint32_t width, uint32_t height, uint32_t* out) {
  if (!s || !out || width == 0 || height == 0) return -1;
  for (int d = 0; d < s->num_drawcalls; ++d) {
    const orc_drawcall_t* dc = &s->drawcalls[d];
    for (int i = 0; i < dc->prim_count; ++i) {
      const int g = dc->prim_offset + i;
      orc_rast_prim_t rp;
      int32_t bb[4];
      const int ok = orc_setup_prim(s->prim_verts + (size_t)g * 30, width, height, dc->znear,
                                    dc->zfar, &rp, bb) == 0;
      orc_vis_prim_t v;
      orc_vis_prim_compute(&rp, ok, bb, width, height, &v);
      out[3 * g + 0] = v.rx;
      out[3 * g + 1] = v.ry;
      out[3 * g + 2] = v.zmin;
    }
  }
  return 0;
}

/* ---- rt_vnode_t over a tree (vis.cpp BuildVisNodes) --------------------- */
typedef struct {
  uint32_t x0, x1, y0, y1, zmin;
  int any;
} cover_t;

static void cover_add(cover_t* c, const cover_t* k) {
  if (!k->any) return;
  if (!c->any) {
    *c = *k;
    return;
  }
  if (k->x0 < c->x0) c->x0 = k->x0;
  if (k->x1 > c->x1) c->x1 = k->x1;
  if (k->y0 < c->y0) c->y0 = k->y0;
  if (k->y1 > c->y1) c->y1 = k->y1;
  if (k->zmin < c->zmin) c->zmin = k->zmin;
}

typedef struct {
  const int32_t* refs;
  uint32_t n;
  const int32_t* pids;
  uint32_t m;
  const orc_vis_prim_t* by_pid;
  uint32_t np;
  uint32_t* out;
  int err;
} vn_ctx_t;

static cover_t vn_of(vn_ctx_t* c, int32_t ref, int depth) {
  cover_t r;
  memset(&r, 0, sizeof(r));
  if (ref == -1) return r;
  if (depth > 64) { c->err = -1; return r; }
  if (ref < 0) {
    const uint32_t lr = (uint32_t)ref, first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
    for (uint32_t k = first; k < first + count; ++k) {
      if (k >= c->m || c->pids[k] < 0 || (uint32_t)c->pids[k] >= c->np) { c->err = -1; return r; }
      const orc_vis_prim_t* v = &c->by_pid[c->pids[k]];
      if (!v->any) continue;
      cover_t t = {v->rx & 0xffffu, v->rx >> 16, v->ry & 0xffffu, v->ry >> 16, v->zmin, 1};
      cover_add(&r, &t);
    }
    return r;
  }
  if ((uint32_t)ref >= c->n) { c->err = -1; return r; }
  uint32_t* o = c->out + (size_t)ref * 16;
  for (int i = 0; i < 4; ++i) {
    const int32_t cr = c->refs[(size_t)ref * 4 + i];
    const cover_t k = vn_of(c, cr, depth + 1);
    o[i] = k.any ? (k.x0 | (k.x1 << 16)) : 0x0000ffffu;
    o[4 + i] = k.any ? (k.y0 | (k.y1 << 16)) : 0x0000ffffu;
    o[8 + i] = k.any ? k.zmin : 0xffffffffu;
    o[12 + i] = k.any ? (uint32_t)cr : 0xffffffffu;
    cover_add(&r, &k);
  }
  /* slots in ascending depth bound, stable (vis.cpp SortSlots) */
  for (int i = 1; i < 4; ++i)
    for (int j = i; j > 0 && o[8 + j] < o[8 + j - 1]; --j)
      for (int f = 0; f < 16; f += 4) {
        const uint32_t t = o[f + j]; o[f + j] = o[f + j - 1]; o[f + j - 1] = t;
      }
  return r;
}

int orc_vis_nodes(const int32_t* refs, uint32_t n, const int32_t* leaf_pids, uint32_t m,
                  const orc_vis_prim_t* by_pid, uint32_t np, uint32_t* vnodes) {
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 4; ++k) {
      vnodes[i * 16 + k] = vnodes[i * 16 + 4 + k] = 0x0000ffffu;
      vnodes[i * 16 + 8 + k] = vnodes[i * 16 + 12 + k] = 0xffffffffu;
    }
  if (n == 0) return 0;
  vn_ctx_t c = {refs, n, leaf_pids, m, by_pid, np, vnodes, 0};
  vn_of(&c, 0, 0);
  return c.err;
}
