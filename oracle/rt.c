/*
 * rt.c -- oracle restatement of the north-star ray-tracing path:
 * per-pixel primary ray generation, Möller–Trumbore closest hit, screen
 * layers, raster-parity shading of the hit, any-hit shadow rays.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * There is NO reference implementation of this path:
 * parity of the RT-specific parts is unpinned; primary visibility is
 * cross-checked against the raster restatement (raster.c), which is pinned by
 * the reference's golden images.  Anchors used:
 *   - pixel centres / framebuffer orientation: gfxutil.cpp:150-152,164-166,211-214 and
 *     draw3d/main.cpp:385-386 (row 0 = NDC y = -1);
 *   - MT == homogeneous edge functions for eye rays: gfxutil.cpp:35-75;
 *   - inclusive coverage (no top-left rule): graphics.cpp:813-825;
 *   - PRIMARY rays are raster-exact (vis.c; the kernels' trace_primary):
 *     coverage = the Q15.16 edge test inside the binned tiles
 *     (graphics.cpp:813-825, gfxutil.cpp:237-271), closest hit = the depth
 *     test's winner on the 24-bit word (graphics.cpp:564-596, ties to the
 *     first drawn for LESS / last drawn for LEQUAL, gpu_sw.h:46-60), found
 *     by a BVH walk over per-node pixel rectangles + depth bounds;
 *   - SECONDARY rays (shadow, bounce): Möller–Trumbore, closest hit with
 *     ties -> lowest pid (LESS) / highest (LEQUAL);
 *   - layers (depth_test off) painted in order: draw3d/main.cpp:239-242;
 *   - shading of a hit = draw3d shader (kernel.cpp:232-279) evaluated with
 *     the hit primitive's fixed-point edge functions at the pixel centre.
 */
#include <float.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "gfx.h"

/* ---- vector helpers: explicit fmaf, identical op order to the kernel ---- */
static inline void cross3(float r[3], const float a[3], const float b[3]) {
  r[0] = fmaf(a[1], b[2], -(a[2] * b[1]));
  r[1] = fmaf(a[2], b[0], -(a[0] * b[2]));
  r[2] = fmaf(a[0], b[1], -(a[1] * b[0]));
}
static inline float dot3(const float a[3], const float b[3]) {
  return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0]));
}

/* MT with the reference's inclusive coverage: hit iff det != 0, u >= 0,
 * v >= 0, u + v <= det (after sign normalisation) and t > tmin.  The single
 * division is IEEE-correctly-rounded (the kernel uses the same). */
static inline int mt_hit(const float o[3], const float d[3], const float v0[3],
                         const float e1[3], const float e2[3], float tmin, float* t_out) {
  float pvec[3], tvec[3], qvec[3];
  cross3(pvec, d, e2);
  const float det = dot3(e1, pvec);
  tvec[0] = o[0] - v0[0]; tvec[1] = o[1] - v0[1]; tvec[2] = o[2] - v0[2];
  float u = dot3(tvec, pvec);
  cross3(qvec, tvec, e1);
  float v = dot3(d, qvec);
  float adet = det;
  if (det < 0.0f) { adet = -det; u = -u; v = -v; }
  if (!(adet > 0.0f) || u < 0.0f || v < 0.0f || u + v > adet) return 0;
  const float t = dot3(e2, qvec) / det;
  if (!(t > tmin)) return 0;
  *t_out = t;
  return 1;
}

int orc_mt(const float o[3], const float d[3], const float v0[3],
           const float e1[3], const float e2[3], float tmin, float* t_out) {
  return mt_hit(o, d, v0, e1, e2, tmin, t_out);
}

/* ---- scene preparation --------------------------------------------------- */
typedef struct {
  const orc_scene_t* scene;
  const orc_bvh_t* bvh;           /* NULL = brute force */
  orc_rt_params_t p;
  orc_rast_prim_t* rp;            /* [num_prims] setup at W x H */
  int* rp_ok;                     /* non-degenerate */
  int* prim_dc;                   /* drawcall of each prim */
  orc_dcstate_t* dcst;            /* [num_drawcalls] */
  orc_vis_prim_t* vis;            /* [num_prims] primary visibility (vis.c) */
  uint32_t* vnodes;               /* [num vnodes][16] over the primary rays' tree */
  uint32_t* bl_idx;               /* vis_lists: per 8x8 block (first entry, count) */
  uint32_t* bl_ent;               /* per entry: geometry pid, suffix union rx, ry */
  uint32_t bl_nbx;
  uint32_t* sl_idx;               /* shadow_lists: per light-space cell (first entry, count) */
  int32_t* sl_ent;                /* per entry: geometry index (c->geom) */
  float* sl_key;                  /* per entry: its sort key (sl_key) */
  int32_t* vpids;                 /* its leaf records' pids */
  uint32_t num_vnodes;
  int32_t* vhit;                  /* [W*H] primary winner per pixel (packet pre-pass) */
  uint32_t* lcnt;                 /* [W*H] screen layers the pixel's lane tested */
  int next_tile_row;
  float* tri;                     /* [num_prims][9] v0,e1,e2 (clip x,y,w) */
  int32_t* geom;                  /* geometry prim ids, ascending */
  int num_geom;
  int tie_high;                   /* LEQUAL: ties -> highest pid */
  float sx, sy;
  uint32_t* color; int32_t* pid; float* tout;
  orc_rt_counters_t cnt;
  pthread_mutex_t mu;
  int next_row;
} rt_ctx_t;

static int rt_prepare(rt_ctx_t* c, const orc_scene_t* s, const orc_rt_params_t* p) {
  memset(c, 0, sizeof(*c));
  c->scene = s;
  c->p = *p;
  const int np = s->num_prims > 0 ? s->num_prims : 1;
  c->rp = (orc_rast_prim_t*)calloc(np, sizeof(orc_rast_prim_t));
  c->rp_ok = (int*)calloc(np, sizeof(int));
  c->prim_dc = (int*)calloc(np, sizeof(int));
  c->tri = (float*)calloc((size_t)np * 9, sizeof(float));
  c->geom = (int32_t*)calloc(np, sizeof(int32_t));
  c->dcst = (orc_dcstate_t*)calloc(s->num_drawcalls > 0 ? s->num_drawcalls : 1, sizeof(orc_dcstate_t));
  c->vis = (orc_vis_prim_t*)calloc(np, sizeof(orc_vis_prim_t));
  int seen_geom = 0, geom_func = -1;
  for (int d = 0; d < s->num_drawcalls; ++d) {
    const orc_drawcall_t* dc = &s->drawcalls[d];
    orc_dcstate_init(&c->dcst[d], s, dc);
    /* RT-path restrictions (DESIGN.md "Scope"): layers before geometry, one
     * depth function, no blending/stencil, full colour writes. */
    if (dc->blend_enabled || dc->stencil_test || (dc->color_writemask & 0xf) != 0xf) return -2;
    if (dc->depth_test) {
      const uint32_t f = cgl_to_vx_compare(dc->depth_func);
      if (f != VX_OM_DEPTH_FUNC_LESS && f != VX_OM_DEPTH_FUNC_LEQUAL) return -2;
      if (geom_func >= 0 && (int)f != geom_func) return -2;
      if (!(dc->depth_writemask & 1)) return -2;  /* the winner must write its depth */
      geom_func = (int)f;
      seen_geom = 1;
    } else if (seen_geom) {
      return -2;
    }
    for (int i = 0; i < dc->prim_count; ++i) {
      const int g = dc->prim_offset + i;
      const float* v = s->prim_verts + (size_t)g * 30;
      int32_t bb[4];
      const int st = orc_setup_prim(v, p->width, p->height, dc->znear, dc->zfar, &c->rp[g], bb);
      c->rp_ok[g] = st != 1;
      orc_vis_prim_compute(&c->rp[g], st == 0, bb, p->width, p->height, &c->vis[g]);
      c->prim_dc[g] = d;
      float* t = c->tri + (size_t)g * 9;
      /* clip-space (x, y, w) triangle: v0, e1 = v1 - v0, e2 = v2 - v0 */
      t[0] = v[0]; t[1] = v[1]; t[2] = v[3];
      t[3] = v[10] - v[0]; t[4] = v[11] - v[1]; t[5] = v[13] - v[3];
      t[6] = v[20] - v[0]; t[7] = v[21] - v[1]; t[8] = v[23] - v[3];
      /* every depth-tested triangle is geometry: MT rejects degenerate ones
       * (det == 0) by itself, exactly like the kernel */
      if (dc->depth_test) c->geom[c->num_geom++] = g;
    }
  }
  c->tie_high = (geom_func == VX_OM_DEPTH_FUNC_LEQUAL);
  c->sx = 2.0f / (float)p->width;
  c->sy = 2.0f / (float)p->height;
  pthread_mutex_init(&c->mu, NULL);
  return 0;
}

static void rt_release(rt_ctx_t* c) {
  free(c->rp); free(c->rp_ok); free(c->prim_dc); free(c->tri); free(c->geom); free(c->dcst);
  free(c->bl_idx); free(c->bl_ent);
  free(c->sl_idx); free(c->sl_ent); free(c->sl_key);
  free(c->vis); free(c->vnodes); free(c->vpids); free(c->vhit); free(c->lcnt);
  pthread_mutex_destroy(&c->mu);
}

static inline int better(const rt_ctx_t* c, float t, int pid, float bt, int bpid) {
  if (t < bt) return 1;
  if (t == bt) return c->tie_high ? (pid > bpid) : (pid < bpid);
  return 0;
}

/* ---- BVH traversal: restatement of the kernel's loop -------------------- */
#define BVH_EMPTY (-1)
#define BVH_STACK 64

typedef struct { float inv[3], oi[3]; } ray_pre_t;

static inline float safe_dir(float d) {
  return fabsf(d) < 1e-20f ? (d < 0.0f ? -1e-20f : 1e-20f) : d;
}
static inline void ray_pre(ray_pre_t* r, const float o[3], const float d[3]) {
  for (int k = 0; k < 3; ++k) {
    r->inv[k] = 1.0f / safe_dir(d[k]);
    r->oi[k] = o[k] * r->inv[k];
  }
}
/* slab test of child `ch` of a node; returns hit and tnear */
static inline int slab(const float* n, int ch, const ray_pre_t* r, float tmin, float tmax, float* tnear) {
  float lo[3], hi[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = fmaf(n[4 * k + 2 * ch + 0], r->inv[k], -r->oi[k]);
    hi[k] = fmaf(n[4 * k + 2 * ch + 1], r->inv[k], -r->oi[k]);
  }
  const float t0 = fminf(lo[0], hi[0]), t1 = fminf(lo[1], hi[1]), t2 = fminf(lo[2], hi[2]);
  const float u0 = fmaxf(lo[0], hi[0]), u1 = fmaxf(lo[1], hi[1]), u2 = fmaxf(lo[2], hi[2]);
  const float tn = fmaxf(fmaxf(t0, t1), fmaxf(t2, tmin));
  const float tf = fminf(fminf(u0, u1), fminf(u2, tmax));
  *tnear = tn;
  return tn <= tf;
}

static inline int32_t node_ref(const float* n, int ch) {
  int32_t r;
  memcpy(&r, &n[12 + ch], 4);
  return r;
}

/* BVH4 node step (the kernel's rt_trace.h trace(), RT_FLAG_BVH4 branch):
 * slab-test the 4 children, order the hits by tnear with the same 5-exchange
 * sorting network (strict <, misses keyed +inf, hit keys clamped to FLT_MAX),
 * continue with the nearest and push the others farthest first.  Any-hit
 * walks (anyhit) key the hits by slot: fixed slot order (rt_trace.h
 * node4_step `any`, the order of the kernels' shadow packets,
 * occluded_packet).  Returns the next ref, or BVH_EMPTY when nothing was hit. */
static int32_t bvh4_step(const float* n, const ray_pre_t* r, float tmin, float lim, int anyhit,
                         int32_t* stack, int* sp) {
  float key[4];
  int32_t ref[4];
  int cnt = 0;
  for (int i = 0; i < 4; ++i) {
    memcpy(&ref[i], &n[24 + i], 4);
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
      lo[k] = fmaf(n[8 * k + i], r->inv[k], -r->oi[k]);
      hi[k] = fmaf(n[8 * k + 4 + i], r->inv[k], -r->oi[k]);
    }
    const float t0 = fminf(lo[0], hi[0]), t1 = fminf(lo[1], hi[1]), t2 = fminf(lo[2], hi[2]);
    const float u0 = fmaxf(lo[0], hi[0]), u1 = fmaxf(lo[1], hi[1]), u2 = fmaxf(lo[2], hi[2]);
    const float tn = fmaxf(fmaxf(t0, t1), fmaxf(t2, tmin));
    const float tf = fminf(fminf(u0, u1), fminf(u2, lim));
    const int h = ref[i] != BVH_EMPTY && tn <= tf;
    key[i] = h ? (anyhit ? (float)i : fminf(tn, FLT_MAX)) : INFINITY;
    cnt += h;
  }
  static const int net[5][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}};
  for (int e = 0; e < 5; ++e) {
    const int a = net[e][0], b = net[e][1];
    if (key[b] < key[a]) {
      const float tk = key[a]; key[a] = key[b]; key[b] = tk;
      const int32_t tr = ref[a]; ref[a] = ref[b]; ref[b] = tr;
    }
  }
  if (cnt == 0) return BVH_EMPTY;
  for (int i = cnt - 1; i >= 1; --i)
    if (*sp < BVH_STACK) stack[(*sp)++] = ref[i];
  return ref[0];
}

/* closest (anyhit=0) or any (anyhit=1) hit; returns hit pid or -1 */
static int bvh_trace(const rt_ctx_t* c, const float o[3], const float d[3], float tmin,
                     float tmax, int anyhit, int skip_pid, float* t_out,
                     uint64_t* visits, uint64_t* tests) {
  const orc_bvh_t* b = c->bvh;
  if (b->num_nodes <= 0) return -1;
  ray_pre_t rp;
  ray_pre(&rp, o, d);
  int32_t stack[BVH_STACK];
  int sp = 0;
  int32_t ref = 0;
  float bt = tmax;
  int bpid = -1;
  for (;;) {
    if (ref >= 0 && b->num_nodes4 > 0) {
      ++*visits;
      const int32_t nx = bvh4_step(b->nodes4 + (size_t)ref * 32, &rp, tmin, anyhit ? tmax : bt,
                                   anyhit, stack, &sp);
      if (nx != BVH_EMPTY) { ref = nx; continue; }
    } else if (ref >= 0) {
      const float* n = b->nodes + (size_t)ref * 16;
      ++*visits;
      const int32_t c0 = node_ref(n, 0), c1 = node_ref(n, 1);
      float tn0 = 0.0f, tn1 = 0.0f;
      const float lim = anyhit ? tmax : bt;
      const int h0 = (c0 != BVH_EMPTY) && slab(n, 0, &rp, tmin, lim, &tn0);
      const int h1 = (c1 != BVH_EMPTY) && slab(n, 1, &rp, tmin, lim, &tn1);
      if (h0 && h1) {
        int32_t near = c0, far = c1;
        if (!anyhit && tn1 < tn0) { near = c1; far = c0; }  /* any-hit: slot order */
        if (sp < BVH_STACK) stack[sp++] = far;
        ref = near;
        continue;
      } else if (h0) { ref = c0; continue; }
      else if (h1) { ref = c1; continue; }
    } else {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      for (uint32_t k = 0; k < count; ++k) {
        const float* tr = b->tris + (size_t)(first + k) * 12;
        int32_t pid;
        memcpy(&pid, &tr[3], 4);
        ++*tests;
        if (pid == skip_pid) continue;
        /* the BVH supplies structure only; vertices come from the oracle's own
         * setup so a wrong device triangle record cannot hide here */
        const float* tv = c->tri + (size_t)pid * 9;
        float t;
        if (!mt_hit(o, d, tv, tv + 3, tv + 6, tmin, &t)) continue;
        if (anyhit) {
          if (t < tmax) { *t_out = t; return pid; }
          continue;
        }
        if (better(c, t, pid, bt, bpid)) { bt = t; bpid = pid; }
      }
    }
    if (sp == 0) break;
    ref = stack[--sp];
  }
  if (bpid >= 0) *t_out = bt;
  return bpid;
}

/* brute force over the geometry list (ascending pid) */
static int brute_trace(const rt_ctx_t* c, const float o[3], const float d[3], float tmin,
                       float tmax, int anyhit, int skip_pid, float* t_out, uint64_t* tests) {
  float bt = tmax;
  int bpid = -1;
  for (int k = 0; k < c->num_geom; ++k) {
    const int g = c->geom[k];
    ++*tests;
    if (g == skip_pid) continue;
    const float* tr = c->tri + (size_t)g * 9;
    float t;
    if (!mt_hit(o, d, tr, tr + 3, tr + 6, tmin, &t)) continue;
    if (anyhit) {
      if (t < tmax) { *t_out = t; return g; }
      continue;
    }
    if (better(c, t, g, bt, bpid)) { bt = t; bpid = g; }
  }
  if (bpid >= 0) *t_out = bt;
  return bpid;
}

/* ---- primary visibility: restatement of the kernels' trace_primary ------ */
static inline int rect_in(uint32_t r, uint32_t p) { return p >= (r & 0xffffu) && p <= (r >> 16); }

static inline int vis_better(uint32_t z, int pid, uint32_t bz, int bpid, int tie_high) {
  return z < bz || (z == bz && (tie_high ? pid > bpid : (bpid >= 0 && pid < bpid)));
}

/* one candidate primitive at pixel (px, py): draw3d's coverage (the binned
 * rectangle + inclusive edge test) and depth test against (bz, bpid) */
static inline void vis_test(const rt_ctx_t* c, int pid, uint32_t px, uint32_t py, uint32_t* bz,
                            int* bpid) {
  const orc_vis_prim_t* v = &c->vis[pid];
  if (!rect_in(v->rx, px) || !rect_in(v->ry, py) || v->zmin > *bz) return;
  const orc_rast_prim_t* p = &c->rp[pid];
  const int32_t e0 = orc_edge_eval(p->edges[0], px, py);
  const int32_t e1 = orc_edge_eval(p->edges[1], px, py);
  const int32_t e2 = orc_edge_eval(p->edges[2], px, py);
  if (e0 < 0 || e1 < 0 || e2 < 0) return;
  const uint32_t z = orc_vis_depth(p, e0, e1, e2);
  if (vis_better(z, pid, *bz, *bpid, c->tie_high)) { *bz = z; *bpid = pid; }
}

/* rt_vnode_t step (kernels' vnode_step): children whose rectangle holds the
 * pixel and whose depth bound can still win, in slot order -- the slots are
 * stored in ascending depth bound (vis.c / vis.cpp SortSlots) -- the first
 * returned, the others pushed last slot first */
static int32_t vnode_step(const uint32_t* n, uint32_t px, uint32_t py, uint32_t bz,
                          int32_t* stack, int* sp) {
  int idx[4];
  int cnt = 0;
  for (int i = 0; i < 4; ++i) {
    const int h = (int32_t)n[12 + i] != BVH_EMPTY && rect_in(n[i], px) && rect_in(n[4 + i], py) &&
                  n[8 + i] <= bz;
    if (h) idx[cnt++] = i;
  }
  if (cnt == 0) return BVH_EMPTY;
  for (int j = cnt - 1; j >= 1; --j)
    if (*sp < BVH_STACK) stack[(*sp)++] = (int32_t)n[12 + idx[j]];
  return (int32_t)n[12 + idx[0]];
}

static int vis_trace(const rt_ctx_t* c, uint32_t px, uint32_t py, uint64_t* visits, uint64_t* tests) {
  if (c->num_vnodes == 0) return -1;
  int32_t stack[BVH_STACK];
  int sp = 0;
  int32_t ref = 0;
  uint32_t bz = VX_OM_DEPTH_MASK;
  int bpid = -1;
  for (;;) {
    if (ref >= 0) {
      ++*visits;
      const int32_t nx = vnode_step(c->vnodes + (size_t)ref * 16, px, py, bz, stack, &sp);
      if (nx != BVH_EMPTY) { ref = nx; continue; }
    } else {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      for (uint32_t k = 0; k < count; ++k) {
        ++*tests;
        vis_test(c, c->vpids[first + k], px, py, &bz, &bpid);
      }
    }
    if (sp == 0) break;
    ref = stack[--sp];
  }
  return bpid;
}

/* Packet form (the kernels' trace_primary_packet, RT_VIS_PACKET): the
 * wave's pixels walk the tree together -- a child is entered when some
 * lane's pixel lies in its rectangle with a bound that can still beat that
 * lane's best; entered children in slot order (= ascending bound), the
 * first taken, the others pushed last first; every lane tests every leaf primitive of the walk.
 * n lanes at (px[i], py[i]); out[i] = winner.  Visits and tests count once
 * per packet. */
#define PK_LANES 64
static void vis_trace_packet(const rt_ctx_t* c, int n, const uint32_t* px, const uint32_t* py,
                             int32_t* out, uint64_t* visits, uint64_t* tests) {
  uint32_t bz[PK_LANES];
  int bpid[PK_LANES];
  for (int i = 0; i < n; ++i) { bz[i] = VX_OM_DEPTH_MASK; bpid[i] = -1; out[i] = -1; }
  if (c->num_vnodes == 0 || n == 0) return;
  int32_t stack[BVH_STACK];
  int sp = 0;
  int32_t ref = 0;
  for (;;) {
    if (ref >= 0) {
      ++*visits;
      const uint32_t* nd = c->vnodes + (size_t)ref * 16;
      int32_t r[4];
      int cnt = 0;
      for (int k = 0; k < 4; ++k) {  /* needed children in slot order (sorted slots) */
        const int32_t ck = (int32_t)nd[12 + k];
        int need = 0;
        if (ck != BVH_EMPTY)
          for (int i = 0; i < n && !need; ++i)
            need = rect_in(nd[k], px[i]) && rect_in(nd[4 + k], py[i]) && nd[8 + k] <= bz[i];
        if (need) r[cnt++] = ck;
      }
      if (cnt > 0) {
        for (int i = cnt - 1; i >= 1; --i)
          if (sp < BVH_STACK) stack[sp++] = r[i];
        ref = r[0];
        continue;
      }
    } else {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      for (uint32_t k = 0; k < count; ++k) {
        ++*tests;
        for (int i = 0; i < n; ++i) vis_test(c, c->vpids[first + k], px[i], py[i], &bz[i], &bpid[i]);
      }
    }
    if (sp == 0) break;
    ref = stack[--sp];
  }
  for (int i = 0; i < n; ++i) out[i] = bpid[i];
}

/* tile (tx, ty) runs as 32-pixel waves (8x4 half blocks) in the path tracer
 * iff some geometry primitive covers a pixel of it (the host's split rule,
 * rt_app.cpp: tiles any covered-pixel rectangle reaches) */
static int tile_split(const rt_ctx_t* c, uint32_t tx, uint32_t ty) {
  if (!(c->p.flags & ORC_RT_PATH) || c->p.path_queue) return 0;
  const uint32_t x0 = tx * 32, x1 = x0 + 31, y0 = ty * 32, y1 = y0 + 31;
  for (int k = 0; k < c->num_geom; ++k) {
    const orc_vis_prim_t* v = &c->vis[c->geom[k]];
    if (!v->any) continue;
    if ((v->rx & 0xffffu) <= x1 && (v->rx >> 16) >= x0 && (v->ry & 0xffffu) <= y1 && (v->ry >> 16) >= y0)
      return 1;
  }
  return 0;
}

/* Per-8x8-block candidate lists (rt_app.cpp build_block_lists): the
 * geometry primitives whose covered rectangle reaches the block, in
 * ascending (depth bound, geometry index), each with the union rectangle of
 * itself and the entries after it. */
typedef struct { uint32_t zmin, k; } bl_key_t;
static int bl_cmp(const void* a, const void* b) {
  const bl_key_t *x = (const bl_key_t*)a, *y = (const bl_key_t*)b;
  if (x->zmin != y->zmin) return x->zmin < y->zmin ? -1 : 1;
  return x->k < y->k ? -1 : x->k > y->k;
}
static void vis_build_lists(rt_ctx_t* c) {
  const uint32_t nbx = (c->p.width + 7) / 8, nby = (c->p.height + 7) / 8, nb = nbx * nby;
  uint32_t* cnt = (uint32_t*)calloc(nb, sizeof(uint32_t));
  for (int k = 0; k < c->num_geom; ++k) {
    const orc_vis_prim_t* v = &c->vis[c->geom[k]];
    if (!v->any) continue;
    for (uint32_t by = (v->ry & 0xffffu) >> 3; by <= (v->ry >> 16) >> 3 && by < nby; ++by)
      for (uint32_t bx = (v->rx & 0xffffu) >> 3; bx <= (v->rx >> 16) >> 3 && bx < nbx; ++bx) ++cnt[by * nbx + bx];
  }
  c->bl_idx = (uint32_t*)malloc(sizeof(uint32_t) * 2 * nb);
  uint32_t tot = 0;
  for (uint32_t b = 0; b < nb; ++b) { c->bl_idx[2 * b] = tot; c->bl_idx[2 * b + 1] = 0; tot += cnt[b]; }
  bl_key_t* keys = (bl_key_t*)malloc(sizeof(bl_key_t) * (tot ? tot : 1));
  for (int k = 0; k < c->num_geom; ++k) {
    const orc_vis_prim_t* v = &c->vis[c->geom[k]];
    if (!v->any) continue;
    for (uint32_t by = (v->ry & 0xffffu) >> 3; by <= (v->ry >> 16) >> 3 && by < nby; ++by)
      for (uint32_t bx = (v->rx & 0xffffu) >> 3; bx <= (v->rx >> 16) >> 3 && bx < nbx; ++bx) {
        const uint32_t b = by * nbx + bx;
        bl_key_t* e = &keys[c->bl_idx[2 * b] + c->bl_idx[2 * b + 1]++];
        e->zmin = v->zmin;
        e->k = (uint32_t)k;
      }
  }
  c->bl_ent = (uint32_t*)malloc(sizeof(uint32_t) * 3 * (tot ? tot : 1));
  for (uint32_t b = 0; b < nb; ++b) {
    const uint32_t o = c->bl_idx[2 * b], n = c->bl_idx[2 * b + 1];
    qsort(keys + o, n, sizeof(bl_key_t), bl_cmp);
    uint32_t x0 = 0xffffu, x1 = 0, y0 = 0xffffu, y1 = 0;
    for (uint32_t i = n; i-- > 0;) {
      const int32_t pid = c->geom[keys[o + i].k];
      const orc_vis_prim_t* v = &c->vis[pid];
      if ((v->rx & 0xffffu) < x0) x0 = v->rx & 0xffffu;
      if ((v->rx >> 16) > x1) x1 = v->rx >> 16;
      if ((v->ry & 0xffffu) < y0) y0 = v->ry & 0xffffu;
      if ((v->ry >> 16) > y1) y1 = v->ry >> 16;
      c->bl_ent[3 * (o + i)] = (uint32_t)pid;
      c->bl_ent[3 * (o + i) + 1] = x0 | (x1 << 16);
      c->bl_ent[3 * (o + i) + 2] = y0 | (y1 << 16);
    }
  }
  c->bl_nbx = nbx;
  free(keys);
  free(cnt);
}

/* the kernels' block_primary: the wave's block list two entries per round,
 * stopping once no lane's pixel lies in the remaining entries' union with a
 * bound (the next entry's, the smallest left) not above its best depth word;
 * tests count once per wave per entry tested */
static void vis_scan_block(const rt_ctx_t* c, int n, const uint32_t* px, const uint32_t* py,
                           int32_t* out, uint64_t* tests) {
  uint32_t bz[PK_LANES];
  int bpid[PK_LANES];
  for (int i = 0; i < n; ++i) { bz[i] = VX_OM_DEPTH_MASK; bpid[i] = -1; }
  const uint32_t b = (py[0] >> 3) * c->bl_nbx + (px[0] >> 3);
  const uint32_t o = c->bl_idx[2 * b], cnt = c->bl_idx[2 * b + 1];
  for (uint32_t k = 0; k < cnt; k += 2) {
    const uint32_t* e = &c->bl_ent[3 * (o + k)];
    const uint32_t zk = c->vis[e[0]].zmin;
    int go = 0;
    for (int i = 0; i < n && !go; ++i)
      go = rect_in(e[1], px[i]) && rect_in(e[2], py[i]) && zk <= bz[i];
    if (!go) break;
    for (uint32_t j = k; j < k + 2 && j < cnt; ++j) {
      ++*tests;
      const int32_t pid = (int32_t)c->bl_ent[3 * (o + j)];
      for (int i = 0; i < n; ++i) vis_test(c, pid, px[i], py[i], &bz[i], &bpid[i]);
    }
  }
  for (int i = 0; i < n; ++i) out[i] = bpid[i];
}

/* the primary pre-pass over one row of 32x32 tiles: every wave's packet
 * (8x8 blocks, or 8x4 halves in split tiles, the kernels' task_map) */
/* pixels per wave in a split tile: 2^split_log (the kernels' task_map) */
static uint32_t split_pl(const rt_ctx_t* c) { return c->p.split_log ? c->p.split_log : 5u; }
static int tile_waves(const rt_ctx_t* c, int split) { return split ? (int)(1024u >> split_pl(c)) : 16; }

/* the in-image pixels of wave `wv` of tile (tx, ty): an 8x8 block, or in a
 * split tile the 2^split_log-pixel part of one (8x4 halves by default; the
 * kernels' task_map); returns their number */
static int wave_pixels(const rt_ctx_t* c, uint32_t tx, uint32_t ty, int split, int wv, uint32_t* px,
                       uint32_t* py, int32_t* idx) {
  const uint32_t W = c->p.width, H = c->p.height;
  const uint32_t pl = split_pl(c), sub = 6u - pl;
  const int lanes = split ? (1 << pl) : 64;
  int n = 0;
  for (int ln = 0; ln < lanes; ++ln) {
    const uint32_t ti = split ? (((uint32_t)wv >> sub) << 6) + (((uint32_t)wv & ((1u << sub) - 1u)) << pl) +
                                    (uint32_t)ln
                              : ((uint32_t)wv << 6) + (uint32_t)ln;
    const uint32_t blk = ti >> 6, l = ti & 63u;
    const uint32_t x = tx * 32 + (blk & 3u) * 8 + (l & 7u), y = ty * 32 + (blk >> 2) * 8 + (l >> 3);
    if (x >= W || y >= H) continue;
    px[n] = x; py[n] = y; idx[n] = (int32_t)(y * W + x);
    ++n;
  }
  return n;
}

static void vis_tile_row(rt_ctx_t* c, uint32_t ty, orc_rt_counters_t* k) {
  const uint32_t W = c->p.width;
  const uint32_t ntx = (W + 31) / 32;
  uint32_t px[PK_LANES], py[PK_LANES];
  int32_t out[PK_LANES];
  int32_t idx[PK_LANES];
  for (uint32_t tx = 0; tx < ntx; ++tx) {
    const int split = tile_split(c, tx, ty);
    const int waves = tile_waves(c, split);
    for (int wv = 0; wv < waves; ++wv) {
      const int n = wave_pixels(c, tx, ty, split, wv, px, py, idx);
      if (n == 0) continue;
      if (c->bl_idx)
        vis_scan_block(c, n, px, py, out, &k->tri_tests);
      else
        vis_trace_packet(c, n, px, py, out, &k->node_visits, &k->tri_tests);
      for (int i = 0; i < n; ++i) c->vhit[idx[i]] = out[i];
    }
  }
}

static void* vis_worker(void* arg) {
  rt_ctx_t* c = (rt_ctx_t*)arg;
  orc_rt_counters_t k;
  memset(&k, 0, sizeof(k));
  const uint32_t nty = (c->p.height + 31) / 32;
  for (;;) {
    pthread_mutex_lock(&c->mu);
    const int i = c->next_tile_row++;
    pthread_mutex_unlock(&c->mu);
    if ((uint32_t)i >= nty) break;
    vis_tile_row(c, (uint32_t)i, &k);
  }
  pthread_mutex_lock(&c->mu);
  c->cnt.node_visits += k.node_visits;
  c->cnt.tri_tests += k.tri_tests;
  pthread_mutex_unlock(&c->mu);
  return NULL;
}

/* flat list: every geometry primitive, ascending pid */
static int vis_brute(const rt_ctx_t* c, uint32_t px, uint32_t py, uint64_t* tests) {
  uint32_t bz = VX_OM_DEPTH_MASK;
  int bpid = -1;
  for (int k = 0; k < c->num_geom; ++k) {
    ++*tests;
    vis_test(c, c->geom[k], px, py, &bz, &bpid);
  }
  return bpid;
}

/* the primary ray's parameter at the winner's plane: MT's t without the
 * coverage test (the kernels' plane_t) */
static float plane_t(const float o[3], const float d[3], const float* tri) {
  float pvec[3], tvec[3], qvec[3];
  cross3(pvec, d, tri + 6);
  const float det = dot3(tri + 3, pvec);
  tvec[0] = o[0] - tri[0]; tvec[1] = o[1] - tri[1]; tvec[2] = o[2] - tri[2];
  cross3(qvec, tvec, tri + 3);
  return dot3(tri + 6, qvec) / det;
}

static void vis_build_nodes(rt_ctx_t* c) {
  const orc_bvh_t* b = c->bvh;
  if (!b) return;
  uint32_t n, m;
  int32_t *refs, *pids;
  if (b->vis_refs && b->num_vis_nodes > 0) {  /* the product's primary tree */
    n = (uint32_t)b->num_vis_nodes;
    m = (uint32_t)b->num_vis_leaves;
    refs = (int32_t*)malloc(sizeof(int32_t) * 4 * n);
    pids = (int32_t*)malloc(sizeof(int32_t) * (m ? m : 1));
    memcpy(refs, b->vis_refs, sizeof(int32_t) * 4 * n);
    memcpy(pids, b->vis_pids, sizeof(int32_t) * m);
  } else {                                     /* the secondary rays' BVH */
    if (b->num_nodes <= 0) return;
    n = (uint32_t)(b->num_nodes4 > 0 ? b->num_nodes4 : b->num_nodes);
    m = (uint32_t)b->num_tris;
    refs = (int32_t*)malloc(sizeof(int32_t) * 4 * n);
    for (uint32_t i = 0; i < n; ++i)
      for (int k = 0; k < 4; ++k) {
        int32_t r = BVH_EMPTY;
        if (b->num_nodes4 > 0) memcpy(&r, &b->nodes4[(size_t)i * 32 + 24 + k], 4);
        else if (k < 2) memcpy(&r, &b->nodes[(size_t)i * 16 + 12 + k], 4);
        refs[i * 4 + k] = r;
      }
    pids = (int32_t*)malloc(sizeof(int32_t) * (m ? m : 1));
    for (uint32_t k = 0; k < m; ++k) memcpy(&pids[k], &b->tris[(size_t)k * 12 + 3], 4);
  }
  c->vnodes = (uint32_t*)malloc(sizeof(uint32_t) * 16 * n);
  c->vpids = pids;
  c->num_vnodes = n;
  if (orc_vis_nodes(refs, n, pids, m, c->vis, (uint32_t)c->scene->num_prims, c->vnodes) != 0)
    c->num_vnodes = 0;
  free(refs);
}

static inline uint32_t shadow_attenuate(uint32_t c) {
  return (c & 0xff000000u) | ((c >> 1) & 0x007f7f7fu);
}

static uint32_t shade_at(const rt_ctx_t* c, int g, uint32_t x, uint32_t y, orc_rt_counters_t* k) {
  const orc_rast_prim_t* p = &c->rp[g];
  const orc_dcstate_t* st = &c->dcst[c->prim_dc[g]];
  const int32_t e0 = orc_edge_eval(p->edges[0], x, y);
  const int32_t e1 = orc_edge_eval(p->edges[1], x, y);
  const int32_t e2 = orc_edge_eval(p->edges[2], x, y);
  uint32_t z;
  ++k->shaded;
  if (st->tex_enabled)
    k->texel_bytes += (st->tex_filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * vx_format_stride((int)st->tex_format);
  return orc_shade(st, p, e0, e1, e2, &z);
}

/* ---- diffuse path trace -------------------
 * NO REFERENCE: the reference has no lights, normals or materials.  The
 * estimator is the build's own documented choice (DESIGN.md "Path tracing"),
 * restated here op for op as the HIP kernel (kernels/pt_kernel.hip) runs it:
 * at every path vertex one shadow ray to the point light (direct term
 * T * max(0, cos)), then -- for `bounces` segments -- a cosine-weighted bounce
 * about the geometric normal; an escaped ray adds T * ORC_PT_SKY; a bounce hit
 * multiplies T by the draw3d shader's colour at the hit's barycentrics.
 * Only +, -, *, /, sqrt and integer hashing: bit-exact across CPU and GPU. */
static inline uint32_t pcg_hash(uint32_t v) {
  const uint32_t state = v * 747796405u + 2891336453u;
  const uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
  return (word >> 22u) ^ word;
}
static inline uint32_t pt_key(uint32_t seed, uint32_t px, uint32_t v) {
  return pcg_hash(px ^ pcg_hash(seed ^ (0x9E3779B9u * (v + 1u))));
}
static inline float pt_u11(uint32_t h) { return (float)(h >> 8) * 0x1p-23f - 1.0f; }

/* cosine-weighted direction about unit normal n: uniform point in the unit
 * disk by bounded rejection sampling, lifted to the hemisphere (Malley), in
 * the Duff et al. (2017) orthonormal basis of n */
static void pt_bounce_dir(const float n[3], uint32_t key, float dir[3]) {
  float x = 0.0f, y = 0.0f;
  for (uint32_t i = 0; i < ORC_PT_TRIES; ++i) {
    const float a = pt_u11(pcg_hash(key + 2u * i)), b = pt_u11(pcg_hash(key + 2u * i + 1u));
    if (fmaf(a, a, b * b) < 1.0f) { x = a; y = b; break; }
  }
  const float z = sqrtf(1.0f - fmaf(x, x, y * y));
  const float sgn = n[2] >= 0.0f ? 1.0f : -1.0f;
  const float a = -1.0f / (sgn + n[2]);
  const float b = (n[0] * n[1]) * a;
  const float t1[3] = {fmaf(sgn * (n[0] * n[0]), a, 1.0f), sgn * b, -(sgn * n[0])};
  const float t2[3] = {b, fmaf(n[1] * n[1], a, sgn), -n[1]};
  for (int k = 0; k < 3; ++k) dir[k] = fmaf(x, t1[k], fmaf(y, t2[k], z * n[k]));
}

/* unit geometric normal of triangle (v0, e1, e2), facing against din */
static void pt_normal(const float* tri, const float din[3], float n[3]) {
  cross3(n, tri + 3, tri + 6);
  const float len = sqrtf(dot3(n, n));
  n[0] = n[0] / len; n[1] = n[1] / len; n[2] = n[2] / len;
  if (dot3(n, din) > 0.0f) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
}

/* barycentric weights of the MT hit (b1 = vertex 1, b2 = vertex 2): the
 * same numerators as mt_hit, divided by |det| */
static void mt_bary(const float o[3], const float d[3], const float* tri, float* b1, float* b2) {
  float pvec[3], tvec[3], qvec[3];
  cross3(pvec, d, tri + 6);
  const float det = dot3(tri + 3, pvec);
  tvec[0] = o[0] - tri[0]; tvec[1] = o[1] - tri[1]; tvec[2] = o[2] - tri[2];
  float u = dot3(tvec, pvec);
  cross3(qvec, tvec, tri + 3);
  float v = dot3(d, qvec);
  float adet = det;
  if (det < 0.0f) { adet = -det; u = -u; v = -v; }
  *b1 = u / adet;
  *b2 = v / adet;
}

static inline uint32_t pt_to8(float x) {
  return x >= 1.0f ? 255u : (x > 0.0f ? (uint32_t)fmaf(x, 255.0f, 0.5f) : 0u);
}

static int trace_any(const rt_ctx_t* c, const float o[3], const float d[3], float tmin,
                     float tmax, int anyhit, int skip, float* t, orc_rt_counters_t* k) {
  return c->bvh ? bvh_trace(c, o, d, tmin, tmax, anyhit, skip, t, &k->node_visits, &k->tri_tests)
                : brute_trace(c, o, d, tmin, tmax, anyhit, skip, t, &k->tri_tests);
}

static int sl_occluded(const rt_ctx_t* c, const float so[3], const float sd[3], int skip,
                       uint64_t* tests);

static uint32_t path_trace(const rt_ctx_t* c, uint32_t px, const float d0[3], float t0, int g,
                           uint32_t alb0, orc_rt_counters_t* k) {
  const float k255 = 1.0f / 255.0f;
  float T[3] = {(float)((alb0 >> 16) & 0xffu) * k255, (float)((alb0 >> 8) & 0xffu) * k255,
                (float)(alb0 & 0xffu) * k255};
  float L[3] = {0.0f, 0.0f, 0.0f};
  float o[3] = {0.0f, 0.0f, 0.0f}, dir[3] = {d0[0], d0[1], d0[2]};
  float th = t0;
  int pid = g;
  for (uint32_t v = 0;; ++v) {
    float n[3], P[3];
    pt_normal(c->tri + (size_t)pid * 9, dir, n);
    const float tt = th * 0.999755859375f;
    for (int i = 0; i < 3; ++i) P[i] = fmaf(dir[i], tt, o[i]);
    /* direct light: shadow segment P -> light */
    const float sd[3] = {c->p.light[0] - P[0], c->p.light[1] - P[1], c->p.light[2] - P[2]};
    float ts;
    ++k->shadow_rays;
    /* the light-space lists when built (the kernels' occluded_list), else the BVH */
    if (c->sl_idx ? sl_occluded(c, P, sd, pid, &k->tri_tests)
                  : trace_any(c, P, sd, 0.0f, 1.0f, 1, pid, &ts, k) >= 0) {
      ++k->occluded;
    } else {
      const float cosl = dot3(n, sd) / sqrtf(dot3(sd, sd));
      if (cosl > 0.0f)
        for (int i = 0; i < 3; ++i) L[i] = fmaf(T[i], cosl, L[i]);
    }
    if (v == c->p.bounces) break;
    /* bounce */
    float nd[3], nt = 0.0f;
    pt_bounce_dir(n, pt_key(c->p.seed, px, v), nd);
    ++k->bounce_rays;
    const int np = trace_any(c, P, nd, 0.0f, INFINITY, 0, pid, &nt, k);
    if (np < 0) {
      for (int i = 0; i < 3; ++i) L[i] = fmaf(T[i], ORC_PT_SKY, L[i]);
      break;
    }
    float b1, b2;
    mt_bary(P, nd, c->tri + (size_t)np * 9, &b1, &b2);
    const int32_t dx = fx_from_float_dev((1.0f - b1) - b2, 24);
    const int32_t dy = fx_from_float_dev(b1, 24);
    const orc_dcstate_t* st = &c->dcst[c->prim_dc[np]];
    uint32_t z;
    ++k->shaded;
    if (st->tex_enabled)
      k->texel_bytes += (st->tex_filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * vx_format_stride((int)st->tex_format);
    const uint32_t a = orc_shade_weights(st, &c->rp[np], dx, dy, &z);
    T[0] = T[0] * ((float)((a >> 16) & 0xffu) * k255);
    T[1] = T[1] * ((float)((a >> 8) & 0xffu) * k255);
    T[2] = T[2] * ((float)(a & 0xffu) * k255);
    for (int i = 0; i < 3; ++i) { o[i] = P[i]; dir[i] = nd[i]; }
    th = nt;
    pid = np;
  }
  return (alb0 & 0xff000000u) | (pt_to8(L[0]) << 16) | (pt_to8(L[1]) << 8) | pt_to8(L[2]);
}

/* ---- light-space shadow lists (the kernels' occluded_list; built on the
 * device by rt_setup.hip SCOUNT .. SSORT).  Every shadow segment ends at the
 * one point light, so a ray is identified by its direction from the light,
 * u = P - L.  The directions are binned on the 6 faces of a cube around the
 * light (face 2k + (u_k < 0) for the dominant axis k, face coordinates
 * u_i / |u_k|, u_j / |u_k| in [-1, 1], SL_N x SL_N cells); a cell's list holds
 * every geometry triangle whose projection from the light reaches the cell:
 * the triangle clipped to the face's frustum widened by SL_EPS, its projected
 * polygon's box widened by SL_EPS, then a separating-axis test against the
 * cell widened by SL_EPS.  Conservative: a triangle MT accepts for a ray meets
 * the ray's direction, which lies in the ray's cell, and the widening covers
 * fp32 rounding; the lists only narrow the candidates -- a ray's verdict is
 * the brute-force any-hit's.  A cell's list is ordered by (key, geometry
 * index), key = the squared distance from the light to the triangle's
 * bounding box (sl_key: a lower bound of |X - L|^2 over its points); a ray
 * tests its cell's list in that order until the first occluder, or until a
 * record whose key exceeds |L - P|^2 * 1.001 (that triangle has no point on
 * the segment, nor has any after it).  All arithmetic fp32, no
 * contraction, the device's operation order. */
#define SL_N 128
#define SL_EPS (1.0f / 512.0f)
#define SL_CELLS (6 * SL_N * SL_N)
static const int sl_ax[3][2] = {{1, 2}, {0, 2}, {0, 1}};

static int sl_clip_plane(float in[][3], int n, int k, float s, int m, float sg, float out[][3]) {
  const float ke = 1.0f + SL_EPS;
  int o = 0;
  for (int q = 0; q < n; ++q) {
    const float* a = in[q];
    const float* b = in[(q + 1) % n];
    const float da = (s * a[k]) * ke - sg * a[m], db = (s * b[k]) * ke - sg * b[m];
    if (da >= 0.0f) { out[o][0] = a[0]; out[o][1] = a[1]; out[o][2] = a[2]; ++o; }
    if ((da >= 0.0f) != (db >= 0.0f)) {
      const float tq = da / (da - db);
      for (int cc = 0; cc < 3; ++cc) out[o][cc] = a[cc] + (b[cc] - a[cc]) * tq;
      ++o;
    }
  }
  return o;
}

/* triangle t9 (v0, e1, e2) on face f: projected polygon (pu, pv, n) and cell
 * range; returns 0 when the face holds none of it, 2 when the polygon reaches
 * the light (every cell of the face, no separating-axis test) */
static int sl_project(const float* t9, const float L[3], int f, float pu[8], float pv[8], int* n,
                      int rng[4]) {
  const int k = f >> 1, i = sl_ax[k][0], j = sl_ax[k][1];
  const float s = (f & 1) ? -1.0f : 1.0f;
  float A[8][3], B[8][3];
  for (int cc = 0; cc < 3; ++cc) {
    A[0][cc] = t9[cc] - L[cc];
    A[1][cc] = (t9[cc] + t9[3 + cc]) - L[cc];
    A[2][cc] = (t9[cc] + t9[6 + cc]) - L[cc];
  }
  int m = 3;
  m = sl_clip_plane(A, m, k, s, i, 1.0f, B);
  if (m) m = sl_clip_plane(B, m, k, s, i, -1.0f, A);
  if (m) m = sl_clip_plane(A, m, k, s, j, 1.0f, B);
  if (m) m = sl_clip_plane(B, m, k, s, j, -1.0f, A);
  if (!m) return 0;
  const float hn = (float)SL_N * 0.5f;
  for (int q = 0; q < m; ++q)
    if (!(s * A[q][k] > 0.0f)) {
      rng[0] = 0; rng[1] = SL_N - 1; rng[2] = 0; rng[3] = SL_N - 1;
      *n = 0;
      return 2;
    }
  float u0 = 0, u1 = 0, v0 = 0, v1 = 0;
  for (int q = 0; q < m; ++q) {
    const float ck = s * A[q][k];
    pu[q] = A[q][i] / ck;
    pv[q] = A[q][j] / ck;
    if (q == 0 || pu[q] < u0) u0 = pu[q];
    if (q == 0 || pu[q] > u1) u1 = pu[q];
    if (q == 0 || pv[q] < v0) v0 = pv[q];
    if (q == 0 || pv[q] > v1) v1 = pv[q];
  }
  *n = m;
  int x0 = (int)floorf(((u0 - SL_EPS) + 1.0f) * hn), x1 = (int)floorf(((u1 + SL_EPS) + 1.0f) * hn);
  int y0 = (int)floorf(((v0 - SL_EPS) + 1.0f) * hn), y1 = (int)floorf(((v1 + SL_EPS) + 1.0f) * hn);
  if (x0 < 0) x0 = 0;
  if (y0 < 0) y0 = 0;
  if (x1 > SL_N - 1) x1 = SL_N - 1;
  if (y1 > SL_N - 1) y1 = SL_N - 1;
  rng[0] = x0; rng[1] = x1; rng[2] = y0; rng[3] = y1;
  return x0 <= x1 && y0 <= y1;
}

/* separating-axis test of the projected polygon against cell (cx, cy)
 * widened by SL_EPS (the box axes are the cell range's) */
static int sl_cell_meets(const float* pu, const float* pv, int n, int cx, int cy) {
  if (n < 3) return 1;
  const float cw = 2.0f / (float)SL_N;
  const float rx0 = ((float)cx * cw - 1.0f) - SL_EPS, rx1 = ((float)(cx + 1) * cw - 1.0f) + SL_EPS;
  const float ry0 = ((float)cy * cw - 1.0f) - SL_EPS, ry1 = ((float)(cy + 1) * cw - 1.0f) + SL_EPS;
  for (int a = 0; a < n; ++a) {
    const int b = a + 1 < n ? a + 1 : 0;
    const float nx = pv[b] - pv[a], ny = pu[a] - pu[b];
    float p0 = 0, p1 = 0;
    for (int q = 0; q < n; ++q) {
      const float d = nx * pu[q] + ny * pv[q];
      if (q == 0 || d < p0) p0 = d;
      if (q == 0 || d > p1) p1 = d;
    }
    const float c0 = nx * rx0 + ny * ry0, c1 = nx * rx1 + ny * ry0;
    const float c2 = nx * rx0 + ny * ry1, c3 = nx * rx1 + ny * ry1;
    const float r0 = fminf(fminf(c0, c1), fminf(c2, c3)), r1 = fmaxf(fmaxf(c0, c1), fmaxf(c2, c3));
    if (p1 < r0 || p0 > r1) return 0;
  }
  return 1;
}

/* every (cell, geometry index) pair, in (k, face, cy, cx) order: count (ent
 * NULL) or fill at the cells' cursors */
static void sl_pairs(const rt_ctx_t* c, const float L[3], uint32_t* cnt, uint32_t* cur, int32_t* ent) {
  for (int k = 0; k < c->num_geom; ++k) {
    const float* t9 = c->tri + (size_t)c->geom[k] * 9;
    for (int f = 0; f < 6; ++f) {
      float pu[8], pv[8];
      int n = 0, rng[4];
      const int r = sl_project(t9, L, f, pu, pv, &n, rng);
      if (!r) continue;
      for (int cy = rng[2]; cy <= rng[3]; ++cy)
        for (int cx = rng[0]; cx <= rng[1]; ++cx) {
          if (r == 1 && !sl_cell_meets(pu, pv, n, cx, cy)) continue;
          const uint32_t cell = ((uint32_t)f * SL_N + (uint32_t)cy) * SL_N + (uint32_t)cx;
          if (ent) ent[cur[cell]++] = k;
          else ++cnt[cell];
        }
    }
  }
}

/* rt_setup.hip sl_key: squared distance from L to the box of (v0, v0 + e1,
 * v0 + e2) */
static float sl_key(const float* t9, const float L[3]) {
  float s = 0.0f;
  for (int k = 0; k < 3; ++k) {
    const float p = t9[k], q = t9[k] + t9[3 + k], u = t9[k] + t9[6 + k];
    const float lo = fminf(p, fminf(q, u)), hi = fmaxf(p, fmaxf(q, u));
    const float d = L[k] < lo ? lo - L[k] : (L[k] > hi ? L[k] - hi : 0.0f);
    s = s + d * d;
  }
  return s;
}
static const float* sl_sort_keys;
static int sl_cmp(const void* a, const void* b) {
  const int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
  const float kx = sl_sort_keys[x], ky = sl_sort_keys[y];
  if (kx != ky) return kx < ky ? -1 : 1;
  return x < y ? -1 : (x > y ? 1 : 0);
}

static void sl_build(rt_ctx_t* c) {
  uint32_t* cnt = (uint32_t*)calloc(SL_CELLS, sizeof(uint32_t));
  sl_pairs(c, c->p.light, cnt, NULL, NULL);
  c->sl_idx = (uint32_t*)malloc(sizeof(uint32_t) * 2 * SL_CELLS);
  uint32_t* cur = (uint32_t*)malloc(sizeof(uint32_t) * SL_CELLS);
  uint64_t tot = 0;
  for (uint32_t i = 0; i < SL_CELLS; ++i) {
    c->sl_idx[2 * i] = (uint32_t)tot;
    c->sl_idx[2 * i + 1] = cnt[i];
    cur[i] = (uint32_t)tot;
    tot += cnt[i];
  }
  c->sl_ent = (int32_t*)malloc(sizeof(int32_t) * (tot ? tot : 1));
  sl_pairs(c, c->p.light, NULL, cur, c->sl_ent);  /* ascending k within each cell */
  /* then by (key, k): nearest to the light first */
  float* gk = (float*)malloc(sizeof(float) * (c->num_geom ? c->num_geom : 1));
  for (int k = 0; k < c->num_geom; ++k) gk[k] = sl_key(c->tri + (size_t)c->geom[k] * 9, c->p.light);
  sl_sort_keys = gk;
  for (uint32_t i = 0; i < SL_CELLS; ++i)
    if (c->sl_idx[2 * i + 1] > 1)
      qsort(c->sl_ent + c->sl_idx[2 * i], c->sl_idx[2 * i + 1], sizeof(int32_t), sl_cmp);
  c->sl_key = (float*)malloc(sizeof(float) * (tot ? tot : 1));
  for (uint64_t e = 0; e < tot; ++e) c->sl_key[e] = gk[c->sl_ent[e]];
  free(gk);
  free(cnt);
  free(cur);
}

/* the ray's cell: dominant axis of u = -sd (ties to the lower axis) */
static uint32_t sl_cell_of(const float sd[3]) {
  const float u[3] = {-sd[0], -sd[1], -sd[2]};
  int k = 0;
  float m = fabsf(u[0]);
  if (fabsf(u[1]) > m) { k = 1; m = fabsf(u[1]); }
  if (fabsf(u[2]) > m) { k = 2; m = fabsf(u[2]); }
  if (!(m > 0.0f)) return 0;
  const int f = 2 * k + (u[k] < 0.0f ? 1 : 0);
  const float hn = (float)SL_N * 0.5f;
  int cx = (int)floorf((u[sl_ax[k][0]] / m + 1.0f) * hn), cy = (int)floorf((u[sl_ax[k][1]] / m + 1.0f) * hn);
  cx = cx < 0 ? 0 : (cx > SL_N - 1 ? SL_N - 1 : cx);
  cy = cy < 0 ? 0 : (cy > SL_N - 1 ? SL_N - 1 : cy);
  return ((uint32_t)f * SL_N + (uint32_t)cy) * SL_N + (uint32_t)cx;
}

/* any-hit over the ray's cell list (t in (0, 1), skip excluded): 1 = occluded */
static int sl_occluded(const rt_ctx_t* c, const float so[3], const float sd[3], int skip, uint64_t* tests) {
  const uint32_t cell = sl_cell_of(sd);
  const uint32_t o = c->sl_idx[2 * cell], n = c->sl_idx[2 * cell + 1];
  const float lim = (sd[0] * sd[0] + sd[1] * sd[1] + sd[2] * sd[2]) * 1.001f;
  for (uint32_t q = 0; q < n; ++q) {
    if (c->sl_key[o + q] > lim) return 0;  /* this and every later record: off the segment */
    const int g = c->geom[c->sl_ent[o + q]];
    ++*tests;
    const float* t9 = c->tri + (size_t)g * 9;
    float t;
    if (g != skip && mt_hit(so, sd, t9, t9 + 3, t9 + 6, 0.0f, &t) && t < 1.0f) return 1;
  }
  return 0;
}

int orc_shadow_lists(const orc_scene_t* scene, const float light[3], uint32_t* idx, int32_t* ent,
                     uint64_t* total) {
  if (!scene || !light) return -1;
  orc_rt_params_t p;
  memset(&p, 0, sizeof(p));
  p.width = p.height = 64;
  for (int i = 0; i < 3; ++i) p.light[i] = light[i];
  rt_ctx_t c;
  int err = rt_prepare(&c, scene, &p);
  if (err) { rt_release(&c); return err; }
  sl_build(&c);
  const uint64_t tot = (uint64_t)c.sl_idx[2 * (SL_CELLS - 1)] + c.sl_idx[2 * (SL_CELLS - 1) + 1];
  if (idx) memcpy(idx, c.sl_idx, sizeof(uint32_t) * 2 * SL_CELLS);
  if (ent) memcpy(ent, c.sl_ent, sizeof(int32_t) * tot);
  if (total) *total = tot;
  rt_release(&c);
  return 0;
}

static void rt_row(rt_ctx_t* c, uint32_t y, orc_rt_counters_t* k) {
  const orc_scene_t* s = c->scene;
  const uint32_t W = c->p.width;
  for (uint32_t x = 0; x < W; ++x) {
    const float o[3] = {0.0f, 0.0f, 0.0f};
    const float d[3] = {fmaf((float)x + 0.5f, c->sx, -1.0f),
                        fmaf((float)y + 0.5f, c->sy, -1.0f), 1.0f};
    ++k->primary_rays;
    /* primary visibility: the raster's winner at this pixel */
    const int hit = c->vhit ? c->vhit[(uint64_t)y * W + x]
                 : c->bvh ? vis_trace(c, x, y, &k->node_visits, &k->tri_tests)
                          : vis_brute(c, x, y, &k->tri_tests);
    uint32_t col = c->p.clear_color;
    int32_t opid = -1;
    float t = 0.0f;
    if (hit >= 0) {
      ++k->geometry_hits;
      col = shade_at(c, hit, x, y, k);
      opid = hit;
      /* secondary rays start at the winner's plane (none if edge-on) */
      t = plane_t(o, d, c->tri + (size_t)hit * 9);
      const int sec = t > 0.0f && t < INFINITY;
      if (sec && (c->p.flags & ORC_RT_PATH)) {
        col = path_trace(c, y * W + x, d, t, hit, col, k);
      } else if (sec && (c->p.flags & ORC_RT_SHADOWS)) {
        /* origin pulled toward the eye by 2^-12 of t, segment to the light */
        const float tt = t * 0.999755859375f;
        const float so[3] = {d[0] * tt, d[1] * tt, d[2] * tt};
        const float sd[3] = {c->p.light[0] - so[0], c->p.light[1] - so[1], c->p.light[2] - so[2]};
        float ts;
        ++k->shadow_rays;
        const int occ = c->sl_idx ? (sl_occluded(c, so, sd, hit, &k->tri_tests) ? 0 : -1)
                      : c->bvh ? bvh_trace(c, so, sd, 0.0f, 1.0f, 1, hit, &ts, &k->node_visits, &k->tri_tests)
                               : brute_trace(c, so, sd, 0.0f, 1.0f, 1, hit, &ts, &k->tri_tests);
        if (occ >= 0) { ++k->occluded; col = shadow_attenuate(col); }
      }
    } else {
      /* screen layers (depth_test off): painter order, the last drawn
       * (highest) covering pid, by draw3d's coverage rule */
      int lpid = -1;
      uint32_t nl = 0;  /* layers this pixel's lane tests (layer_waves counts per wave) */
      for (int dd = s->num_drawcalls - 1; dd >= 0 && lpid < 0; --dd) {
        const orc_drawcall_t* dc = &s->drawcalls[dd];
        if (dc->depth_test) continue;
        for (int i = dc->prim_count - 1; i >= 0; --i) {
          const int g = dc->prim_offset + i;
          ++nl;
          const orc_vis_prim_t* v = &c->vis[g];
          if (!rect_in(v->rx, x) || !rect_in(v->ry, y)) continue;
          const orc_rast_prim_t* p = &c->rp[g];
          if (orc_edge_eval(p->edges[0], x, y) >= 0 && orc_edge_eval(p->edges[1], x, y) >= 0 &&
              orc_edge_eval(p->edges[2], x, y) >= 0) { lpid = g; break; }
        }
      }
      if (lpid >= 0) { col = shade_at(c, lpid, x, y, k); opid = lpid; }
      c->lcnt[(uint64_t)y * W + x] = nl;
    }
    const uint64_t px = (uint64_t)y * W + x;
    c->color[px] = col;
    if (c->pid) c->pid[px] = opid;
    if (c->tout) c->tout[px] = hit >= 0 ? t : 0.0f;
  }
}

/* Screen-layer records fetched per frame: the kernels' resolve_layers loads
 * layer k once per wave (wave-uniform, scalar cache) while some lane of the
 * wave is still unresolved, so a wave fetches max over its lanes of the
 * layers each lane tests -- counted once per wave, like the block lists' and
 * packet walks' record tests. */
static uint64_t layer_waves(const rt_ctx_t* c) {
  const uint32_t ntx = (c->p.width + 31) / 32, nty = (c->p.height + 31) / 32;
  uint32_t px[PK_LANES], py[PK_LANES];
  int32_t idx[PK_LANES];
  uint64_t tot = 0;
  for (uint32_t ty = 0; ty < nty; ++ty)
    for (uint32_t tx = 0; tx < ntx; ++tx) {
      const int split = tile_split(c, tx, ty);
      for (int wv = 0; wv < tile_waves(c, split); ++wv) {
        const int n = wave_pixels(c, tx, ty, split, wv, px, py, idx);
        uint32_t m = 0;
        for (int i = 0; i < n; ++i) m = c->lcnt[idx[i]] > m ? c->lcnt[idx[i]] : m;
        tot += m;
      }
    }
  return tot;
}

static void* rt_worker(void* arg) {
  rt_ctx_t* c = (rt_ctx_t*)arg;
  orc_rt_counters_t k;
  memset(&k, 0, sizeof(k));
  const uint32_t r0 = c->p.row_begin, r1 = c->p.row_end ? c->p.row_end : c->p.height;
  const uint32_t step = c->p.row_step > 1 ? c->p.row_step : 1;
  for (;;) {
    pthread_mutex_lock(&c->mu);
    const int i = c->next_row++;
    pthread_mutex_unlock(&c->mu);
    const uint64_t y = r0 + (uint64_t)i * step;
    if (y >= r1) break;
    rt_row(c, (uint32_t)y, &k);
  }
  pthread_mutex_lock(&c->mu);
  uint64_t* dst = (uint64_t*)&c->cnt;
  const uint64_t* src = (const uint64_t*)&k;
  for (size_t i = 0; i < sizeof(k) / sizeof(uint64_t); ++i) dst[i] += src[i];
  pthread_mutex_unlock(&c->mu);
  return NULL;
}

static int rt_run(const orc_scene_t* scene, const orc_bvh_t* bvh, const orc_rt_params_t* p,
                  uint32_t* color, int32_t* pid, float* t, orc_rt_counters_t* counters) {
  if (!scene || !p || !color || p->width == 0 || p->height == 0) return -1;
  rt_ctx_t c;
  int err = rt_prepare(&c, scene, p);
  if (err) { rt_release(&c); return err; }
  c.bvh = bvh;
  vis_build_nodes(&c);
  /* (BVH mode only: the flat image's shadow rays test the whole list) */
  if (bvh && p->shadow_lists && (p->flags & (ORC_RT_PATH | ORC_RT_SHADOWS))) sl_build(&c);
  c.color = color; c.pid = pid; c.tout = t;
  c.lcnt = (uint32_t*)calloc((size_t)p->width * p->height, sizeof(uint32_t));
  const uint32_t nt = p->nthreads > 1 ? p->nthreads : 1;
  if (bvh && !p->vis_per_lane && p->row_begin == 0 && p->row_end == 0 && p->row_step <= 1) {
    /* primary visibility as the kernels walk it: one packet per wave */
    c.vhit = (int32_t*)malloc(sizeof(int32_t) * (size_t)p->width * p->height);
    if (p->vis_lists) vis_build_lists(&c);
    c.next_tile_row = 0;
    if (nt == 1) {
      vis_worker(&c);
    } else {
      pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nt);
      for (uint32_t i = 0; i < nt; ++i) pthread_create(&th[i], NULL, vis_worker, &c);
      for (uint32_t i = 0; i < nt; ++i) pthread_join(th[i], NULL);
      free(th);
    }
  }
  if (nt == 1) {
    rt_worker(&c);
  } else {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nt);
    for (uint32_t i = 0; i < nt; ++i) pthread_create(&th[i], NULL, rt_worker, &c);
    for (uint32_t i = 0; i < nt; ++i) pthread_join(th[i], NULL);
    free(th);
  }
  c.cnt.layer_tests = layer_waves(&c);
  if (counters) *counters = c.cnt;
  rt_release(&c);
  return 0;
}

int orc_rt_render_bruteforce(const orc_scene_t* scene, const orc_rt_params_t* p,
                             uint32_t* color, int32_t* pid, float* t,
                             orc_rt_counters_t* counters) {
  return rt_run(scene, NULL, p, color, pid, t, counters);
}

int orc_rt_render_bvh(const orc_scene_t* scene, const orc_bvh_t* bvh,
                      const orc_rt_params_t* p, uint32_t* color, int32_t* pid,
                      float* t, orc_rt_counters_t* counters) {
  if (!bvh) return -1;
  return rt_run(scene, bvh, p, color, pid, t, counters);
}

/* The candidate lists of one shard's 8x8 blocks in the product's layout
 * (rt_common.h rt_bentry_t; the device build rt_setup.hip BCOUNT .. BSORT and
 * the host restatement rt_app.cpp build_block_lists): local block
 * lb = (t / shard_count) * 16 + (by & 3) * 4 + (bx & 3) for the tiles
 * t = (by / 4) * tiles_x + bx / 4 with t % shard_count == shard_index; its
 * list = the full-frame block's (vis_build_lists).  idx [nlb][2] = (first,
 * count); ent [total][4] = (geometry index, union lo = x0 | y0 << 16,
 * hi = x1 | y1 << 16, depth bound); NULL = sizes only. */
int orc_vis_block_lists(const orc_scene_t* scene, uint32_t width, uint32_t height, uint32_t shard_index,
                        uint32_t shard_count, uint32_t* idx, uint32_t* ent, uint64_t* total, uint32_t* nlb) {
  if (!scene || width == 0 || height == 0 || shard_count == 0 || shard_index >= shard_count) return -1;
  orc_rt_params_t p;
  memset(&p, 0, sizeof(p));
  p.width = width;
  p.height = height;
  rt_ctx_t c;
  int err = rt_prepare(&c, scene, &p);
  if (err) { rt_release(&c); return err; }
  vis_build_lists(&c);
  int32_t* kof = (int32_t*)malloc(sizeof(int32_t) * (size_t)(scene->num_prims > 0 ? scene->num_prims : 1));
  for (int k = 0; k < c.num_geom; ++k) kof[c.geom[k]] = k;
  const uint32_t tx = (width + 31) / 32, ty = (height + 31) / 32, nt = tx * ty;
  const uint32_t ltiles = nt > shard_index ? (nt - shard_index + shard_count - 1) / shard_count : 0;
  const uint32_t nbx = (width + 7) / 8, nby = (height + 7) / 8;
  uint64_t tot = 0;
  for (uint32_t lt = 0; lt < ltiles; ++lt) {
    const uint32_t t = shard_index + lt * shard_count;
    for (uint32_t blk = 0; blk < 16; ++blk) {
      const uint32_t bx = (t % tx) * 4 + (blk & 3), by = (t / tx) * 4 + (blk >> 2);
      uint32_t o = 0, n = 0;
      if (bx < nbx && by < nby) {
        o = c.bl_idx[2 * (by * nbx + bx)];
        n = c.bl_idx[2 * (by * nbx + bx) + 1];
      }
      if (idx) { idx[2 * (lt * 16 + blk)] = (uint32_t)tot; idx[2 * (lt * 16 + blk) + 1] = n; }
      for (uint32_t i = 0; ent && i < n; ++i) {
        const uint32_t* e = &c.bl_ent[3 * (o + i)];
        uint32_t* d = ent + 4 * (tot + i);
        d[0] = (uint32_t)kof[e[0]];
        d[1] = (e[1] & 0xffffu) | (e[2] << 16);
        d[2] = (e[1] >> 16) | (e[2] & 0xffff0000u);
        d[3] = c.vis[e[0]].zmin;
      }
      tot += n;
    }
  }
  if (total) *total = tot;
  if (nlb) *nlb = ltiles * 16;
  free(kof);
  rt_release(&c);
  return 0;
}
