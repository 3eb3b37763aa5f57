// rt_setup.hip -- the per-resolution setup of the RT path on the GPU
// (the reference's per-drawcall host pre-pass
// draw3d/main.cpp:179-211 -> graphics::Binning, gfxutil.cpp:103-276).  The
// records and their layouts are described in setup_common.h; each sub-phase
// restates one host routine of app/setup.cpp / app/vis.cpp / app/rt_app.cpp
// operation for operation (fp32 without contraction, IEEE division, x86
// float -> int32 conversion semantics, exact int64 row solving), so the
// device records equal the host path's bit for bit.
#include <hip/hip_runtime.h>

#include "rt_common.h"
#include "setup_common.h"
#include "vx_spawn.h"

namespace {

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// (int32_t)x as the reference's x86 host computes it (cvttss2si: truncation,
// INT32_MIN for NaN and out-of-range values; the GPU's v_cvt_i32_f32
// saturates instead)
__device__ __forceinline__ int32_t cvt_x86(float x) {
  if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT32_MIN;
  return (int32_t)x;
}

// cocogfx TFixed<frac>(float) on the host (app/setup.cpp FixedHost)
__device__ __forceinline__ int32_t fixed_host(float f, int frac) {
  return cvt_x86(f * (float)(1u << frac));
}

// floor(a / b) for b > 0 and |a| < 2^53 (the row solutions: |a| < 2^48,
// 0 < b < 2^31): the IEEE double quotient of two exact integers is within
// one of the exact one, so one integer correction makes it exact -- no
// 64-bit integer divide (a ~100-instruction library sequence per call)
__device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = (int64_t)floor((double)a / (double)b);
  const int64_t r = a - q * b;
  if (r < 0) --q;
  else if (r >= b) ++q;
  return q;
}
__device__ __forceinline__ int64_t ceil_div(int64_t a, int64_t b) { return -floor_div(-a, b); }
// b != 0: whether b divides a (then *q = a / b)
__device__ __forceinline__ bool exact_div(int64_t a, int64_t b, int64_t* q) {
  if (b < 0) { a = -a; b = -b; }
  *q = floor_div(a, b);
  return *q * b == a;
}

__device__ __forceinline__ int32_t edge_at(const int32_t* e, uint32_t x, uint32_t y) {
  return (int32_t)((uint32_t)e[0] * x + (uint32_t)e[1] * y + (uint32_t)e[2]);
}

// app/vis.cpp DepthLowerBound (floor division by 2^24 = arithmetic shift)
__device__ uint32_t depth_lower_bound(const int32_t* z) {
  const int64_t T = (int64_t(1) << 24) + 8;
  const int64_t p0 = (int64_t)z[0] * T, p1 = (int64_t)z[1] * T;
  const int64_t lo = min(int64_t(0), min(p0, p1)), hi = max(int64_t(0), max(p0, p1));
  const int64_t zlo = (int64_t)z[2] + (lo >> 24) - 4;
  const int64_t zhi = (int64_t)z[2] + (hi >> 24) + 4;
  if ((zlo >> 24) != (zhi >> 24)) return 0u;
  return (uint32_t)(zlo & 0xffffff);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, 64));
  return x;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
  return x;
}

struct Setup {
  rt_prim_t prim;
  uint32_t bx, by;   // rt_bbox_t, 0 when not ok
  bool ok;           // setup ok and the screen box is not empty
};

// app/setup.cpp PrimSetup + PrimBBox for primitive g (drawcall dc)
__device__ void prim_setup(const float* v, uint32_t dc, float zn, float zf, uint32_t W,
                           uint32_t H, Setup* s) {
  int32_t* o = reinterpret_cast<int32_t*>(&s->prim);
  for (int k = 0; k < 32; ++k) o[k] = 0;
  s->prim.dc = dc;
  // viewport (0, W, 0, H, near, far): cocogfx ClipToHDC / ClipToScreen
  const float sx = ((float)W - 0.0f) * 0.5f, cx = ((float)W + 0.0f) * 0.5f;
  const float sy = ((float)H - 0.0f) * 0.5f, cy = ((float)H + 0.0f) * 0.5f;
  const float szs = (zf - zn) * 0.5f, szc = (zf + zn) * 0.5f;
  float hx[3], hy[3], hw[3], sz[3];
  for (int i = 0; i < 3; ++i) {
    const float* p = v + 10 * i;
    hx[i] = p[0] * sx + p[3] * cx;
    hy[i] = p[1] * sy + p[3] * cy;
    hw[i] = p[3];
    const float rhw = 1.0f / p[3];
    sz[i] = (p[2] * rhw) * szs + szc;
  }
  float e[3][3];
  for (int i = 0; i < 3; ++i) {
    const int j = (i + 1) % 3, k = (i + 2) % 3;
    e[i][0] = (hy[j] * hw[k]) - (hy[k] * hw[j]);
    e[i][1] = (hx[k] * hw[j]) - (hx[j] * hw[k]);
    e[i][2] = (hx[j] * hy[k]) - (hx[k] * hy[j]);
  }
  const float det = e[0][2] * hw[0] + e[1][2] * hw[1] + e[2][2] * hw[2];
  if (det < 0)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) e[i][j] *= -1.0f;
  bool setup_ok = !(det == 0);
  if (setup_ok) {
    for (int i = 0; i < 3; ++i) e[i][2] += e[i][0] * 0.5f + e[i][1] * 0.5f;
    float m = fabsf(e[0][0]);
    const float c[5] = {fabsf(e[1][0]), fabsf(e[2][0]), fabsf(e[0][1]), fabsf(e[1][1]),
                        fabsf(e[2][1])};
    for (int i = 0; i < 5; ++i) m = (c[i] > m) ? c[i] : m;
    const float scale = 1.0f / m;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) s->prim.edges[i][j] = fixed_host(e[i][j] * scale, 16);
    float a[7][3];
    for (int i = 0; i < 3; ++i) {
      const float* p = v + 10 * i;
      a[0][i] = sz[i];
      for (int k = 0; k < 4; ++k) a[1 + k][i] = p[4 + k];
      a[5][i] = p[8];
      a[6][i] = p[9];
    }
    for (int k = 0; k < 7; ++k) {
      s->prim.attribs[k][0] = fixed_host(a[k][0] - a[k][2], 24);
      s->prim.attribs[k][1] = fixed_host(a[k][1] - a[k][2], 24);
      s->prim.attribs[k][2] = fixed_host(a[k][2], 24);
    }
  }
  // PrimBBox: viewport (0, W, 0, H, 0, 1), x86 fmin / fmax / floor / ceil
  float l = 0, r = 0, t = 0, b = 0;
  for (int i = 0; i < 3; ++i) {
    const float* p = v + 10 * i;
    const float rhw = 1.0f / p[3];
    const float x = (p[0] * rhw) * sx + cx, y = (p[1] * rhw) * sy + cy;
    if (i == 0) {
      l = r = x;
      t = b = y;
    } else {
      l = fminf(l, x); r = fmaxf(r, x);
      t = fminf(t, y); b = fmaxf(b, y);
    }
  }
  int32_t L = cvt_x86(floorf(l)), R = cvt_x86(ceilf(r));
  int32_t T = cvt_x86(floorf(t)), B = cvt_x86(ceilf(b));
  L = L > 0 ? L : 0;
  R = R < (int32_t)W ? R : (int32_t)W;
  T = T > 0 ? T : 0;
  B = B < (int32_t)H ? B : (int32_t)H;
  const bool box_ok = !(R <= L || B <= T);
  s->ok = setup_ok && box_ok;
  s->bx = s->ok ? ((uint32_t)L | ((uint32_t)R << 16)) : 0u;
  s->by = s->ok ? ((uint32_t)T | ((uint32_t)B << 16)) : 0u;
}

// --- sub-phases -------------------------------------------------------------
// Every wide sub-phase is a grid-stride loop over a slice of the launch's
// workgroups: slice_b() = this workgroup's index in the slice, slice_n() = the slice's
// size (run_phases: the sub-phases of one launch run side by side on
// disjoint slices, or all on the whole grid one after the other).
__shared__ uint32_t s_slice[2];
__device__ __forceinline__ uint32_t slice_b() { return s_slice[0]; }
__device__ __forceinline__ uint32_t slice_n() { return s_slice[1]; }

__device__ void phase_fill(const rt_setup_arg_t* a) {
  const uint64_t gid = (uint64_t)slice_b() * RTS_BLOCK + threadIdx.x;
  const uint64_t gstride = (uint64_t)slice_n() * RTS_BLOCK;
  for (uint32_t f = 0; f < a->nfills && f < RTS_MAX_FILLS; ++f) {
    const rts_fill_t fl = a->fills[f];
    uint32_t* dst = vx_ptr<uint32_t>(fl.addr);
    const uint32_t v = fl.value;
    const uint64_t n4 = (fl.addr & 15) ? 0 : fl.count / 4;
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (uint64_t i = gid; i < n4; i += gstride) d4[i] = make_uint4(v, v, v, v);
    for (uint64_t i = 4 * n4 + gid; i < fl.count; i += gstride) dst[i] = v;
  }
}

// workgroup per primitive: every thread computes the setup (uniform
// values), thread 0 stores the records, the 256 threads split the rows of
// the covered-rectangle scan (app/vis.cpp ComputeVisPrim) -- a screen-sized
// layer triangle is 1024 rows at 1024^2, each three exact int64 row
// solutions: 4 rows per thread instead of 16 per lane of one wave (the
// phase's critical path) -- and the rectangle is reduced over the waves in LDS
__device__ void phase_primvis(const rt_setup_arg_t* a) {
  const float* verts = vx_ptr<const float>(a->verts_addr);
  const uint32_t* pdc = vx_ptr<const uint32_t>(a->pdc_addr);
  const float* dcz = vx_ptr<const float>(a->dcz_addr);
  rt_prim_t* prims = vx_ptr<rt_prim_t>(a->prims_addr);
  rt_bbox_t* bbox = vx_ptr<rt_bbox_t>(a->bbox_addr);
  uint4* vis = vx_ptr<uint4>(a->vis_addr);
  const uint32_t W = a->width, H = a->height, l = lane_id(), wv = threadIdx.x >> 6;
  __shared__ uint32_t red[RTS_BLOCK / 64][5];
  for (uint32_t g = slice_b(); g < a->num_prims; g += slice_n()) {
    float v[30];
    const float4* src = reinterpret_cast<const float4*>(verts + 32ull * g);
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      const float4 x = src[q];
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
    {
      const float2 x = reinterpret_cast<const float2*>(src)[14];
      v[28] = x.x; v[29] = x.y;
    }
    const uint32_t dc = pdc[g];
    Setup s;
    prim_setup(v, dc, dcz[2 * dc], dcz[2 * dc + 1], W, H, &s);
    if (threadIdx.x == 0) {
      const uint4* pr = reinterpret_cast<const uint4*>(&s.prim);
      uint4* dst = reinterpret_cast<uint4*>(prims + g);
#pragma unroll
      for (int q = 0; q < 8; ++q) dst[q] = pr[q];
      bbox[g] = rt_bbox_t{s.bx, s.by};
    }
    if (a->raster) continue;
    // covered-pixel rectangle: rows of the binned 32x32 tiles, clipped to the viewport
    uint32_t xmin = 0xffffffffu, xmax = 0, ymin = 0xffffffffu, ymax = 0;
    bool all_zero = false;
    if (s.ok) {
      const uint32_t L = s.bx & 0xffffu, R = s.bx >> 16, T = s.by & 0xffffu, B = s.by >> 16;
      const uint32_t X0 = (L >> RT_TILE_LOG) << RT_TILE_LOG;
      const uint32_t X1 = min(((R + 31u) >> RT_TILE_LOG) << RT_TILE_LOG, W);
      const uint32_t Y0 = (T >> RT_TILE_LOG) << RT_TILE_LOG;
      const uint32_t Y1 = min(((B + 31u) >> RT_TILE_LOG) << RT_TILE_LOG, H);
      const int32_t* e = &s.prim.edges[0][0];
      for (uint32_t y = Y0 + threadIdx.x; y < Y1; y += RTS_BLOCK) {
        int64_t lo = X0, hi = (int64_t)X1 - 1, d[3] = {0, 0, 0};
        bool exact = true;
        for (int i = 0; i < 3 && exact; ++i) {
          const int64_t ea = e[3 * i];
          d[i] = (int64_t)e[3 * i + 1] * y + e[3 * i + 2];
          const int64_t vl = ea * X0 + d[i], vr = ea * ((int64_t)X1 - 1) + d[i];
          if (vl < INT32_MIN || vl > INT32_MAX || vr < INT32_MIN || vr > INT32_MAX) {
            exact = false;
            break;
          }
          if (ea > 0) lo = max(lo, ceil_div(-d[i], ea));
          else if (ea < 0) hi = min(hi, floor_div(d[i], -ea));
          else if (d[i] < 0) hi = lo - 1;
        }
        if (!exact) {  // wrapping edge values: pixel by pixel, as the rasterizer does
          for (uint32_t x = X0; x < X1; ++x) {
            const int32_t e0 = edge_at(e, x, y), e1 = edge_at(e + 3, x, y), e2 = edge_at(e + 6, x, y);
            if (e0 < 0 || e1 < 0 || e2 < 0) continue;
            xmin = min(xmin, x); xmax = max(xmax, x);
            ymin = min(ymin, y); ymax = max(ymax, y);
            all_zero |= (e0 | e1 | e2) == 0;
          }
          continue;
        }
        if (lo > hi) continue;
        xmin = min(xmin, (uint32_t)lo); xmax = max(xmax, (uint32_t)hi);
        ymin = min(ymin, y); ymax = max(ymax, y);
        int k = 0;
        while (k < 3 && e[3 * k] == 0) ++k;
        if (k == 3) {
          all_zero |= d[0] == 0 && d[1] == 0 && d[2] == 0;
        } else {
          int64_t x = 0;
          if (exact_div(-d[k], e[3 * k], &x))
            all_zero |= x >= lo && x <= hi && e[0] * x + d[0] == 0 && e[3] * x + d[1] == 0 &&
                        e[6] * x + d[2] == 0;
        }
      }
    }
    xmin = wave_min_u32(xmin); ymin = wave_min_u32(ymin);
    xmax = wave_max_u32(xmax); ymax = wave_max_u32(ymax);
    all_zero = __ballot(all_zero) != 0;
    if (l == 0) {
      red[wv][0] = xmin; red[wv][1] = xmax; red[wv][2] = ymin; red[wv][3] = ymax; red[wv][4] = all_zero;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (uint32_t k = 1; k < RTS_BLOCK / 64; ++k) {
        xmin = min(xmin, red[k][0]); xmax = max(xmax, red[k][1]);
        ymin = min(ymin, red[k][2]); ymax = max(ymax, red[k][3]);
        all_zero |= red[k][4] != 0;
      }
      const bool any = xmin != 0xffffffffu;
      uint4 rec = make_uint4(RT_VIS_EMPTY_RECT, RT_VIS_EMPTY_RECT, RT_VIS_ZMIN_NONE, 0u);
      if (any)
        rec = make_uint4(xmin | (xmax << 16), ymin | (ymax << 16),
                         all_zero ? 0u : depth_lower_bound(s.prim.attribs[0]), 1u);
      vis[g] = rec;
    }
    __syncthreads();  // red[] is reused by the next primitive
  }
}

// app/vis.cpp MakeVisTri
__device__ __forceinline__ void make_vtri(const rt_prim_t* prims, const uint4* vis, int32_t pid,
                                          rt_vtri_t* out) {
  rt_vtri_t t;
  if (pid < 0) {
    for (int k = 0; k < 9; ++k) t.edges[k] = 0;
    t.rx = t.ry = RT_VIS_EMPTY_RECT;
    t.z[0] = t.z[1] = t.z[2] = 0;
    t.zmin = RT_VIS_ZMIN_NONE;
  } else {
    const rt_prim_t& p = prims[pid];
    const uint4 v = vis[pid];
    for (int k = 0; k < 9; ++k) t.edges[k] = (&p.edges[0][0])[k];
    t.rx = v.x;
    t.ry = v.y;
    for (int k = 0; k < 3; ++k) t.z[k] = p.attribs[0][k];
    t.zmin = v.z;
  }
  t.pid = pid;
  const uint4* s = reinterpret_cast<const uint4*>(&t);
  uint4* d = reinterpret_cast<uint4*>(out);
#pragma unroll
  for (int q = 0; q < 4; ++q) d[q] = s[q];
}

__device__ __forceinline__ int32_t tri_pid(const rt_tri_t* tris, uint32_t k) {
  return __float_as_int(tris[k].v[3]);
}

__device__ void phase_vtris(const rt_setup_arg_t* a) {
  const rt_prim_t* prims = vx_ptr<const rt_prim_t>(a->prims_addr);
  const uint4* vis = vx_ptr<const uint4>(a->vis_addr);
  const rt_tri_t* tris = vx_ptr<const rt_tri_t>(a->tris_addr);
  const int32_t* layers = vx_ptr<const int32_t>(a->layers_addr);
  const int32_t* geometry = vx_ptr<const int32_t>(a->geometry_addr);
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  const uint32_t nt = a->num_tris + 3, nl = a->num_layers, ng = a->num_geom;
  const uint32_t total = nt + nl + ng;
  for (uint32_t i = slice_b() * RTS_BLOCK + threadIdx.x; i < total; i += slice_n() * RTS_BLOCK) {
    int32_t pid;
    rt_vtri_t* out;
    if (i < nt) {
      pid = i < a->num_tris ? tri_pid(tris, i) : -1;
      out = vx_ptr<rt_vtri_t>(a->vtris_addr) + i;
    } else if (i < nt + nl) {
      pid = layers[i - nt];
      out = vx_ptr<rt_vtri_t>(a->vlayers_addr) + (i - nt);
    } else {
      pid = geometry[i - nt - nl];
      out = vx_ptr<rt_vtri_t>(a->vgeom_addr) + (i - nt - nl);
    }
    if (pid >= (int32_t)a->num_prims || (pid < 0 && i < a->num_tris)) {
      atomicOr(&status[0], RTS_ERR_PID);
      pid = -1;
    }
    make_vtri(prims, vis, pid, out);
  }
}

// the 4 child references of node i (BVH4: rt_node4_t slots; BVH2: 2 slots)
__device__ __forceinline__ void node_refs(const rt_setup_arg_t* a, uint32_t i, int32_t r[4]) {
  if (a->bvh4) {
    const int4 c = reinterpret_cast<const int4*>(vx_ptr<const rt_node4_t>(a->nodes_addr) + i)[6];
    r[0] = c.x; r[1] = c.y; r[2] = c.z; r[3] = c.w;
  } else {
    const float4 c = reinterpret_cast<const float4*>(vx_ptr<const rt_node_t>(a->nodes_addr) + i)[3];
    r[0] = __float_as_int(c.x); r[1] = __float_as_int(c.y);
    r[2] = r[3] = RT_EMPTY_REF;
  }
}

// node references: > 0 internal node, < -1 leaf, -1 empty; 0 (the root is
// nobody's child: the zero records of the device BVH4's absorbed nodes) empty
struct Cover {
  uint32_t x0, x1, y0, y1, zmin;
  bool any;
};

__device__ __forceinline__ void cover_add(Cover* c, uint32_t rx, uint32_t ry, uint32_t zmin) {
  c->x0 = min(c->x0, rx & 0xffffu); c->x1 = max(c->x1, rx >> 16);
  c->y0 = min(c->y0, ry & 0xffffu); c->y1 = max(c->y1, ry >> 16);
  c->zmin = min(c->zmin, zmin);
  c->any = true;
}
// a vnode child's rectangle (corners lo = x0 | y0 << 16, hi = x1 | y1 << 16)
__device__ __forceinline__ void cover_add_corners(Cover* c, uint32_t lo, uint32_t hi, uint32_t zmin) {
  cover_add(c, (lo & 0xffffu) | (hi << 16), (lo >> 16) | (hi & 0xffff0000u), zmin);
}
// a leaf's cover: the covered rectangles / depth bounds of its (up to 4)
// triangle records, their loads issued together
__device__ __forceinline__ void leaf_cover(const rt_setup_arg_t* a, uint32_t lr, Cover* c) {
  const rt_tri_t* tris = vx_ptr<const rt_tri_t>(a->tris_addr);
  const uint4* vis = vx_ptr<const uint4>(a->vis_addr);
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  const uint32_t first = (lr >> 4) & 0x07ffffffu, cnt = (lr & 15u) + 1u;
  int32_t pid[16];
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    if (k >= cnt) break;
    pid[k] = first + k < a->num_tris ? tri_pid(tris, first + k) : -1;
  }
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    if (k >= cnt) break;
    if (pid[k] < 0 || (uint32_t)pid[k] >= a->num_prims) {
      atomicOr(&status[0], RTS_ERR_PID);
      continue;
    }
    const uint4 v = vis[pid[k]];
    if (v.w) cover_add(c, v.x, v.y, v.z);
  }
}
__device__ __forceinline__ void put_slot(rt_vnode_t& n, int s, const Cover& c, int32_t ref) {
  n.lo[s] = c.any ? (c.x0 | (c.y0 << 16)) : RT_VIS_EMPTY_RECT;
  n.hi[s] = c.any ? (c.x1 | (c.y1 << 16)) : RT_VIS_EMPTY_RECT;
  n.zmin[s] = c.any ? c.zmin : RT_VIS_ZMIN_NONE;
  n.child[s] = c.any ? ref : RT_EMPTY_REF;
}

// thread per node: the parent slot of each internal child and the node's
// internal-child count (the climb's arrival target), and the node's vnode
// record with its leaf and empty slots final (their covers computed here,
// every node at once, so the climb only unions its children's slots)
__device__ void phase_link(const rt_setup_arg_t* a) {
  int32_t* parent = vx_ptr<int32_t>(a->parent_addr);
  uint32_t* count = vx_ptr<uint32_t>(a->count_addr);
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  rt_vnode_t* vn = vx_ptr<rt_vnode_t>(a->vnodes_addr);
  const uint32_t nn = a->num_nodes;
  for (uint32_t i = slice_b() * RTS_BLOCK + threadIdx.x; i < nn; i += slice_n() * RTS_BLOCK) {
    int32_t r[4];
    node_refs(a, i, r);
    uint32_t nint = 0;
    rt_vnode_t n;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (r[s] > 0 && (uint32_t)r[s] < nn) {  // internal: written by the child's climb
        parent[r[s]] = (int32_t)(4 * i + s);
        ++nint;
        n.lo[s] = n.hi[s] = RT_VIS_EMPTY_RECT;
        n.zmin[s] = RT_VIS_ZMIN_NONE;
        n.child[s] = RT_EMPTY_REF;
        continue;
      }
      if (r[s] > 0) atomicOr(&status[0], RTS_ERR_REF);
      Cover c = {0xffffu, 0u, 0xffffu, 0u, RT_VIS_ZMIN_NONE, false};
      if (r[s] < RT_EMPTY_REF) leaf_cover(a, (uint32_t)r[s], &c);  // leaf: its triangle records
      put_slot(n, s, c, r[s]);
    }
    vn[i] = n;
    count[2 * i] = nint;
    count[2 * i + 1] = 0;
  }
}


// bottom-up vnode records (app/vis.cpp BuildVisNodes): each node's slots get
// the union rectangle / minimum depth bound of the child's subtree; a node's
// climbing thread computes its leaf slots, its internal slots were written by
// the children's climbs, and it writes its own union into its parent's slot
// before the acq_rel arrival count -- the last child to arrive climbs on
// (nobody waits).  WG: the whole tree in one workgroup (trees up to
// RTS_CLIMB_WG_NODES nodes, a one-workgroup phase): the arrivals are
// workgroup-scope atomics, which cost no L2 write-back -- with the grid and
// agent scope every climb step writes back the XCD's L2 (cross-XCD
// visibility), ~55 us for tekkaman's 118-node tree at 1024^2
template <bool WG>
__device__ void phase_climb(const rt_setup_arg_t* a) {
  const int32_t* parent = vx_ptr<const int32_t>(a->parent_addr);
  uint32_t* count = vx_ptr<uint32_t>(a->count_addr);
  const rt_tri_t* tris = vx_ptr<const rt_tri_t>(a->tris_addr);
  const uint4* vis = vx_ptr<const uint4>(a->vis_addr);
  rt_vnode_t* vn = vx_ptr<rt_vnode_t>(a->vnodes_addr);
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  const uint32_t nn = a->num_nodes;
  const uint32_t i0 = WG ? threadIdx.x : slice_b() * RTS_BLOCK + threadIdx.x;
  const uint32_t step = WG ? RTS_BLOCK : slice_n() * RTS_BLOCK;
  for (uint32_t i = i0; i < nn; i += step) {
    if (count[2 * i] != 0) continue;
    uint32_t cur = i;
    for (int guard = 0;; ++guard) {
      if (guard == 64) {
        atomicOr(&status[0], RTS_ERR_CLIMB);
        break;
      }
      // every slot of cur is final: its leaf / empty slots from LINK, its
      // internal slots from the children's climbs -- one record read
      const int32_t p = parent[cur];
      Cover u = {0xffffu, 0u, 0xffffu, 0u, RT_VIS_ZMIN_NONE, false};
      {
        rt_vnode_t n = vn[cur];
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (n.child[s] != RT_EMPTY_REF) cover_add_corners(&u, n.lo[s], n.hi[s], n.zmin[s]);
        // ascending depth bound, stable (vis.cpp SortSlots)
        for (int i = 1; i < 4; ++i)
          for (int j = i; j > 0 && n.zmin[j] < n.zmin[j - 1]; --j) {
            const uint32_t lo = n.lo[j], hi = n.hi[j], zm = n.zmin[j];
            const int32_t ch = n.child[j];
            n.lo[j] = n.lo[j - 1]; n.hi[j] = n.hi[j - 1]; n.zmin[j] = n.zmin[j - 1]; n.child[j] = n.child[j - 1];
            n.lo[j - 1] = lo; n.hi[j - 1] = hi; n.zmin[j - 1] = zm; n.child[j - 1] = ch;
          }
        vn[cur] = n;
      }
      if (p < 0) break;
      const uint32_t pn = (uint32_t)p >> 2, ps = (uint32_t)p & 3u;
      vn[pn].lo[ps] = u.any ? (u.x0 | (u.y0 << 16)) : RT_VIS_EMPTY_RECT;
      vn[pn].hi[ps] = u.any ? (u.x1 | (u.y1 << 16)) : RT_VIS_EMPTY_RECT;
      vn[pn].zmin[ps] = u.any ? u.zmin : RT_VIS_ZMIN_NONE;
      vn[pn].child[ps] = u.any ? (int32_t)cur : RT_EMPTY_REF;
      const uint32_t old =
          WG ? __hip_atomic_fetch_add(&count[2 * pn + 1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP)
             : __hip_atomic_fetch_add(&count[2 * pn + 1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 != count[2 * pn]) break;
      cur = pn;
    }
  }
}

// ---- tile order (app/rt_app.cpp configure): weights = geometry primitives
// whose covered rectangle reaches the tile, as a 2D difference array
__device__ void phase_weight(const rt_setup_arg_t* a) {
  const int32_t* geometry = vx_ptr<const int32_t>(a->geometry_addr);
  const uint4* vis = vx_ptr<const uint4>(a->vis_addr);
  uint32_t* w = vx_ptr<uint32_t>(a->weight_addr);
  const uint32_t W1 = a->tiles_x + 1;
  for (uint32_t j = slice_b() * RTS_BLOCK + threadIdx.x; j < a->num_geom; j += slice_n() * RTS_BLOCK) {
    const uint4 v = vis[geometry[j]];
    if (!v.w) continue;
    const uint32_t tx0 = (v.x & 0xffffu) >> RT_TILE_LOG, tx1 = min((v.x >> 16) >> RT_TILE_LOG, a->tiles_x - 1);
    const uint32_t ty0 = (v.y & 0xffffu) >> RT_TILE_LOG, ty1 = min((v.y >> 16) >> RT_TILE_LOG, a->tiles_y - 1);
    if (tx0 > tx1 || ty0 > ty1) continue;
    atomicAdd(&w[ty0 * W1 + tx0], 1u);
    atomicAdd(&w[ty0 * W1 + tx1 + 1], 0xffffffffu);
    atomicAdd(&w[(ty1 + 1) * W1 + tx0], 0xffffffffu);
    atomicAdd(&w[(ty1 + 1) * W1 + tx1 + 1], 1u);
  }
}

// inclusive prefix sum of v[0], v[s], .., v[(n - 1) s] in place, 16 words
// loaded per round before any is stored: a row / column of the difference
// array is a few dependent memory round trips, not one per word (33 at
// 1024^2, 129 at 4096^2)
__device__ __forceinline__ void prefix_strided(uint32_t* v, uint32_t n, uint32_t s) {
  constexpr uint32_t R = 16;
  uint32_t run = 0;
  for (uint32_t b = 0; b < n; b += R) {
    uint32_t x[R];
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) x[k] = b + k < n ? v[(b + k) * s] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      run += x[k];
      x[k] = run;
    }
#pragma unroll
    for (uint32_t k = 0; k < R; ++k)
      if (b + k < n) v[(b + k) * s] = x[k];
  }
}

__device__ void phase_rowsum(const rt_setup_arg_t* a) {
  uint32_t* w = vx_ptr<uint32_t>(a->weight_addr);
  const uint32_t W1 = a->tiles_x + 1;
  for (uint32_t r = slice_b() * RTS_BLOCK + threadIdx.x; r <= a->tiles_y; r += slice_n() * RTS_BLOCK)
    prefix_strided(w + r * W1, W1, 1u);
}

__device__ void phase_colsum(const rt_setup_arg_t* a) {
  uint32_t* w = vx_ptr<uint32_t>(a->weight_addr);
  const uint32_t W1 = a->tiles_x + 1;
  for (uint32_t c = slice_b() * RTS_BLOCK + threadIdx.x; c < W1; c += slice_n() * RTS_BLOCK)
    prefix_strided(w + c, a->tiles_y + 1, W1);
}

// sort digit of local tile lt: 255 - min(weight, 255) (ascending digit =
// heaviest first; stable, so equal weights keep the tile order)
__device__ __forceinline__ uint32_t tile_digit(const rt_setup_arg_t* a, const uint32_t* w, uint32_t lt) {
  const uint32_t t = a->shard_index + lt * a->shard_count;
  const uint32_t x = w[(t / a->tiles_x) * (a->tiles_x + 1) + t % a->tiles_x];
  return RTS_WEIGHT_CAP - min(x, RTS_WEIGHT_CAP);
}

__device__ void phase_hist(const rt_setup_arg_t* a) {
  const uint32_t* w = vx_ptr<const uint32_t>(a->weight_addr);
  uint32_t* hist = vx_ptr<uint32_t>(a->hist_addr);
  __shared__ uint32_t h[256];
  for (uint32_t b = slice_b(); b < a->nblocks; b += slice_n()) {
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = 0; i < RTS_ITEMS / RTS_BLOCK; ++i) {
      const uint32_t lt = b * RTS_ITEMS + i * RTS_BLOCK + threadIdx.x;
      if (lt < a->local_tiles) atomicAdd(&h[tile_digit(a, w, lt)], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * a->nblocks + b] = h[threadIdx.x];
    if ((a->fold & RTS_FOLD_ORDER) && threadIdx.x == 0) {
      // tiles with weight > 0 (digit < 255): status word 3, SCAN's when not folded
      uint32_t heavy = 0;
      for (uint32_t d = 0; d < 255u; ++d) heavy += h[d];
      if (heavy) atomicAdd(vx_ptr<uint32_t>(a->status_addr) + 3, heavy);
    }
    __syncthreads();
  }
}

// RTS_SCAN: exclusive scan of hist[256][nblocks] (digit-major) by one
// workgroup (run_scans)
__device__ void scan_excl(uint32_t* v, uint32_t n, uint32_t* total);

// stable scatter of the local tile indices (rank = digit offset of the block
// + earlier rounds + earlier waves + lanes below with the same digit)
__device__ void phase_scatter(const rt_setup_arg_t* a) {
  const uint32_t* w = vx_ptr<const uint32_t>(a->weight_addr);
  const uint32_t* hist = vx_ptr<const uint32_t>(a->hist_addr);
  uint32_t* order = vx_ptr<uint32_t>(a->order_addr);
  constexpr uint32_t kW = RTS_BLOCK / 64;
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[kW][256];
  const uint32_t wv = threadIdx.x >> 6, l = lane_id();
  const uint64_t lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
  const bool fold = (a->fold & RTS_FOLD_ORDER) != 0;
  for (uint32_t b = slice_b(); b < a->nblocks; b += slice_n()) {
    if (fold) {
      // SCAN's offset of (digit d = thread, block b) over the raw digit-major
      // histogram: the digits below d in every block + digit d in blocks < b
      uint32_t row = 0, part = 0;
      for (uint32_t j = 0; j < a->nblocks; ++j) {
        const uint32_t c = hist[threadIdx.x * a->nblocks + j];
        row += c;
        part += j < b ? c : 0u;
      }
      wcnt[0][threadIdx.x] = row;
      __syncthreads();
      for (uint32_t o = 1; o < 256u; o <<= 1) {  // inclusive scan of the row totals
        const uint32_t y = threadIdx.x >= o ? wcnt[0][threadIdx.x - o] : 0u;
        __syncthreads();
        wcnt[0][threadIdx.x] += y;
        __syncthreads();
      }
      base[threadIdx.x] = wcnt[0][threadIdx.x] - row + part;
      __syncthreads();
    } else {
      base[threadIdx.x] = hist[threadIdx.x * a->nblocks + b];
    }
    for (uint32_t i = 0; i < kW; ++i) wcnt[i][threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t r = 0; r < RTS_ITEMS / RTS_BLOCK; ++r) {
      const uint32_t lt = b * RTS_ITEMS + r * RTS_BLOCK + threadIdx.x;
      const bool valid = lt < a->local_tiles;
      const uint32_t d = valid ? tile_digit(a, w, lt) : 0u;
      uint64_t peers = __ballot(valid);
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const uint64_t m = __ballot((d >> bit) & 1u);
        peers &= ((d >> bit) & 1u) ? m : ~m;
      }
      const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
      if (valid && below == 0) wcnt[wv][d] = (uint32_t)__popcll(peers);
      __syncthreads();
      uint32_t off = 0;
      if (valid)
        for (uint32_t i = 0; i < wv; ++i) off += wcnt[i][d];
      const uint32_t dst = base[d] + off + below;
      __syncthreads();
      uint32_t sum = 0;
      for (uint32_t i = 0; i < kW; ++i) {
        sum += wcnt[i][threadIdx.x];
        wcnt[i][threadIdx.x] = 0;
      }
      base[threadIdx.x] += sum;
      if (valid) order[dst] = lt;
      __syncthreads();
    }
  }
}

// ---- per-block candidate lists (rt_common.h rt_bentry_t; the host
// restatement is app/rt_app.cpp BuildBlockLists, the oracle's
// oracle/rt.c vis_build_lists).  The reference bins each primitive's screen
// box into 32x32 tiles on the host per drawcall (gfxutil.cpp:237-271); here
// the covered-pixel rectangles are binned into the shard's 8x8 blocks on the
// device: count, scan, fill, per-block sort.

// wave-uniform load through the scalar cache (the data was written by an
// earlier launch)
template <typename T>
__device__ __forceinline__ T sload(const T* p) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return *(const __attribute__((address_space(4))) T*)(((uint64_t)hi << 32) | lo);
}

// the lanes of a wave split the 8x8 blocks of covered rectangle v (vis
// record: rx, ry) that lie in the shard's tiles; f(local block) for each
// (tile t = (by >> 2) * tiles_x + (bx >> 2) belongs to shard t % shard_count,
// local tile t / shard_count)
template <typename F>
__device__ __forceinline__ void for_blocks(const rt_setup_arg_t* a, uint4 v, F f) {
  const uint32_t bx0 = (v.x & 0xffffu) >> 3, bx1 = (v.x >> 16) >> 3;
  const uint32_t by0 = (v.y & 0xffffu) >> 3, by1 = (v.y >> 16) >> 3;
  const uint32_t w = bx1 - bx0 + 1, n = w * (by1 - by0 + 1);
  const uint32_t sc = a->shard_count, si = a->shard_index, tx = a->tiles_x;
  for (uint32_t i = lane_id(); i < n; i += 64) {
    const uint32_t bx = bx0 + i % w, by = by0 + i / w;
    const uint32_t t = (by >> 2) * tx + (bx >> 2);
    if (t % sc != si) continue;
    f(((t / sc) << 4) | ((by & 3u) << 2) | (bx & 3u));
  }
}

// a wave per geometry primitive: +1 in every block its rectangle reaches
__device__ void phase_bcount(const rt_setup_arg_t* a) {
  const int32_t* geometry = vx_ptr<const int32_t>(a->geometry_addr);
  const uint4* vis = vx_ptr<const uint4>(a->vis_addr);
  uint32_t* bcnt = vx_ptr<uint32_t>(a->bcnt_addr);
  const uint32_t waves = slice_n() * (RTS_BLOCK / 64);
  for (uint32_t j = slice_b() * (RTS_BLOCK / 64) + (threadIdx.x >> 6); j < a->num_geom; j += waves) {
    const uint4 v = vis[geometry[j]];
    if (!v.w) continue;
    for_blocks(a, v, [&](uint32_t lb) { atomicAdd(&bcnt[lb], 1u); });
  }
}

// workgroup reduction: the sum of xs and the max of xm over the threads
__device__ __forceinline__ void block_sum_max(uint32_t xs, uint32_t xm, uint32_t* sum, uint32_t* mx) {
  __shared__ uint32_t ss[RTS_BLOCK / 64], sm[RTS_BLOCK / 64];
  uint32_t s = xs, m = xm;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += (uint32_t)__shfl_xor((int)s, o, 64);
    m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  }
  if (lane_id() == 0) { ss[threadIdx.x >> 6] = s; sm[threadIdx.x >> 6] = m; }
  __syncthreads();
  s = 0; m = 0;
  for (int w = 0; w < RTS_BLOCK / 64; ++w) { s += ss[w]; m = max(m, sm[w]); }
  *sum = s;
  *mx = m;
  __syncthreads();
}

// The count -> scan -> offsets steps of a set of lists: the 8x8 blocks'
// candidate lists (status words 1, 2) or the light-space cells' shadow lists
// (status words 4, 5)
struct ListSet {
  uint32_t* cnt;   // entries per list (then the fill cursors)
  uint32_t* part;  // per RTS_BLOCKS_PER_PART lists their sum, then its exclusive scan
  uint2* idx;      // per list (first entry, count)
  uint32_t n, npart;
  uint32_t* longest;  // status word: the longest list
  uint32_t* total;    // status word: entries in total
};
__device__ __forceinline__ ListSet block_set(const rt_setup_arg_t* a) {
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  return ListSet{vx_ptr<uint32_t>(a->bcnt_addr), vx_ptr<uint32_t>(a->bpart_addr), vx_ptr<uint2>(a->bidx_addr),
                 a->nblk, a->nbpart, status + 1, status + 2};
}
__device__ __forceinline__ ListSet cell_set(const rt_setup_arg_t* a) {
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  return ListSet{vx_ptr<uint32_t>(a->scnt_addr), vx_ptr<uint32_t>(a->spart_addr), vx_ptr<uint2>(a->sidx_addr),
                 a->ncells, a->ncpart, status + 4, status + 5};
}

// per RTS_BLOCKS_PER_PART lists: their entry sum -> part, the longest list -> *longest
__device__ void phase_lsum(const ListSet& L) {
  constexpr uint32_t Q = RTS_BLOCKS_PER_PART / RTS_BLOCK;
  for (uint32_t b = slice_b(); b < L.npart; b += slice_n()) {
    uint32_t sum = 0, mx = 0;
    for (uint32_t q = 0; q < Q; ++q) {
      const uint32_t lb = b * RTS_BLOCKS_PER_PART + threadIdx.x * Q + q;
      const uint32_t c = lb < L.n ? L.cnt[lb] : 0u;
      sum += c;
      mx = max(mx, c);
    }
    uint32_t ts, tm;
    block_sum_max(sum, mx, &ts, &tm);
    if (threadIdx.x == 0) {
      L.part[b] = ts;
      atomicMax(L.longest, tm);
    }
  }
}

// exclusive scan of v[0, n) in place by one workgroup; the total -> *total
__device__ void scan_excl(uint32_t* v, uint32_t n, uint32_t* total) {
  __shared__ uint32_t s[RTS_BLOCK];
  const uint32_t chunk = (n + RTS_BLOCK - 1) / RTS_BLOCK;
  const uint32_t b0 = min(threadIdx.x * chunk, n), b1 = min(b0 + chunk, n);
  uint32_t sum = 0;
  for (uint32_t i = b0; i < b1; ++i) sum += v[i];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < RTS_BLOCK; o <<= 1) {
    const uint32_t y = threadIdx.x >= o ? s[threadIdx.x - o] : 0u;
    __syncthreads();
    s[threadIdx.x] += y;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - sum;
  for (uint32_t i = b0; i < b1; ++i) {
    const uint32_t x = v[i];
    v[i] = run;
    run += x;
  }
  if (total && threadIdx.x == RTS_BLOCK - 1) *total = s[RTS_BLOCK - 1];
}

// (one workgroup) exclusive scan of the partial sums, the total -> *total
__device__ void phase_lscan(const ListSet& L) { scan_excl(L.part, L.npart, L.total); }

// per list: (first entry, count) -> idx; the count word zeroed (it becomes
// the list's fill cursor)
__device__ void phase_loff(const ListSet& L, bool fold) {
  __shared__ uint32_t s[RTS_BLOCK];
  constexpr uint32_t Q = RTS_BLOCKS_PER_PART / RTS_BLOCK;
  if (fold && slice_b() == 0) {  // the total (BSCAN / SSCAN's, folded)
    uint32_t x = 0;
    for (uint32_t i = threadIdx.x; i < L.npart; i += RTS_BLOCK) x += L.part[i];
    uint32_t ts, tm;
    block_sum_max(x, 0u, &ts, &tm);
    if (threadIdx.x == 0) *L.total = ts;
  }
  for (uint32_t b = slice_b(); b < L.npart; b += slice_n()) {
    uint32_t pre = 0;  // folded: the exclusive prefix of the raw partial sums
    if (fold) {
      uint32_t x = 0;
      for (uint32_t i = threadIdx.x; i < b; i += RTS_BLOCK) x += L.part[i];
      uint32_t tm;
      block_sum_max(x, 0u, &pre, &tm);
    }
    const uint32_t lb0 = b * RTS_BLOCKS_PER_PART + threadIdx.x * Q;
    uint32_t c[Q], sum = 0;
    for (uint32_t q = 0; q < Q; ++q) {
      c[q] = lb0 + q < L.n ? L.cnt[lb0 + q] : 0u;
      sum += c[q];
    }
    s[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < RTS_BLOCK; o <<= 1) {
      const uint32_t y = threadIdx.x >= o ? s[threadIdx.x - o] : 0u;
      __syncthreads();
      s[threadIdx.x] += y;
      __syncthreads();
    }
    uint32_t run = (fold ? pre : L.part[b]) + s[threadIdx.x] - sum;
    for (uint32_t q = 0; q < Q; ++q) {
      if (lb0 + q < L.n) {
        L.idx[lb0 + q] = make_uint2(run, c[q]);
        L.cnt[lb0 + q] = 0u;
      }
      run += c[q];
    }
    __syncthreads();
  }
}

// a wave per geometry primitive: its (depth bound, index, rectangle) in every
// block it reaches, at the block's next free slot (order fixed by BSORT);
// entries past the capacity bcap are dropped and flagged (status[6])
__device__ void phase_bfill(const rt_setup_arg_t* a) {
  const int32_t* geometry = vx_ptr<const int32_t>(a->geometry_addr);
  const uint4* vis = vx_ptr<const uint4>(a->vis_addr);
  uint32_t* bcnt = vx_ptr<uint32_t>(a->bcnt_addr);
  const uint2* bidx = vx_ptr<const uint2>(a->bidx_addr);
  uint4* btmp = vx_ptr<uint4>(a->btmp_addr);
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  const uint32_t waves = slice_n() * (RTS_BLOCK / 64), cap = a->bcap;
  for (uint32_t j = slice_b() * (RTS_BLOCK / 64) + (threadIdx.x >> 6); j < a->num_geom; j += waves) {
    const uint4 v = vis[geometry[j]];
    if (!v.w) continue;
    for_blocks(a, v, [&](uint32_t lb) {
      const uint32_t pos = bidx[lb].x + atomicAdd(&bcnt[lb], 1u);
      if (pos < cap) btmp[pos] = make_uint4(v.z, j, v.x, v.y);
      else atomicOr(&status[6], 1u);
    });
  }
}

// a wave per local block: every entry's rank in (depth bound, index) order
// (the keys are distinct: one entry per primitive) and the union rectangle
// of the entries at or after it, by one pass over the list per 64 entries
// (wave-uniform scalar loads); the sorted rt_bentry_t -> blist
__device__ void phase_bsort(const rt_setup_arg_t* a) {
  const uint2* bidx = vx_ptr<const uint2>(a->bidx_addr);
  const uint4* btmp = vx_ptr<const uint4>(a->btmp_addr);
  uint4* blist = vx_ptr<uint4>(a->blist_addr);
  const uint32_t waves = slice_n() * (RTS_BLOCK / 64), l = lane_id();
  const uint32_t total = vx_ptr<const uint32_t>(a->status_addr)[2], cap = a->bcap;
  if (slice_b() == 0 && threadIdx.x < RT_BLIST_PAD && total <= cap)  // padding entries (pairs loaded ahead)
    blist[total + threadIdx.x] = make_uint4(0u, RT_BLIST_PAD_LO, RT_BLIST_PAD_HI, RT_VIS_ZMIN_NONE);
  for (uint32_t lb = slice_b() * (RTS_BLOCK / 64) + (threadIdx.x >> 6); lb < a->nblk; lb += waves) {
    const uint2 oc = sload(bidx + lb);
    if (oc.x + oc.y > cap) continue;  // past the capacity (status[6]): the host refills
    for (uint32_t base = 0; base < oc.y; base += 64) {
      const uint32_t i = base + l;
      const uint4 me = btmp[oc.x + (i < oc.y ? i : 0u)];
      uint32_t rank = 0, x0 = 0xffffu, x1 = 0, y0 = 0xffffu, y1 = 0;
      for (uint32_t j = 0; j < oc.y; ++j) {
        const uint4 o = sload(btmp + oc.x + j);
        const bool before = o.x < me.x || (o.x == me.x && o.y < me.y);
        rank += before ? 1u : 0u;
        if (!before) {
          x0 = min(x0, o.z & 0xffffu); x1 = max(x1, o.z >> 16);
          y0 = min(y0, o.w & 0xffffu); y1 = max(y1, o.w >> 16);
        }
      }
      if (i < oc.y) blist[oc.x + rank] = make_uint4(me.y, x0 | (y0 << 16), x1 | (y1 << 16), me.x);
    }
  }
}

// ---- light-space shadow lists (rt_common.h; oracle/rt.c sl_build restates
// them operation for operation: fp32, no contraction, IEEE division)

// The projection of a triangle on a cube face, in registers: polygons as
// 8 static slots per coordinate (a triangle clipped by four planes has at
// most 7 vertices); a vertex written at a dynamic position becomes selects
// over the slots, so nothing goes to scratch memory.  Operation for
// operation oracle/rt.c sl_clip_plane / sl_project (fp32, no contraction).
struct SlPoly {
  float c[3][8];  // c[axis][vertex]
  int n;
};
__device__ __forceinline__ float sl_axis(const SlPoly& P, int q, int k) {
  return k == 0 ? P.c[0][q] : (k == 1 ? P.c[1][q] : P.c[2][q]);
}
// clip `in` to s * x_k * (1 + eps) - sg * x_m >= 0
__device__ __forceinline__ void sl_clip_plane(const SlPoly& in, int k, float s, int m, float sg, SlPoly& out) {
  const float ke = 1.0f + RT_SLIST_EPS;
  int o = 0;
  auto put = [&](float x, float y, float z) {
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (t == o) { out.c[0][t] = x; out.c[1][t] = y; out.c[2][t] = z; }
    ++o;
  };
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (q >= in.n) break;
    const bool wrap = q + 1 >= in.n;
    const int qb = q + 1 < 8 ? q + 1 : 0;
    const float ax = in.c[0][q], ay = in.c[1][q], az = in.c[2][q];
    const float bx = wrap ? in.c[0][0] : in.c[0][qb], by = wrap ? in.c[1][0] : in.c[1][qb],
                bz = wrap ? in.c[2][0] : in.c[2][qb];
    const float ak = k == 0 ? ax : (k == 1 ? ay : az), am = m == 0 ? ax : (m == 1 ? ay : az);
    const float bk = k == 0 ? bx : (k == 1 ? by : bz), bm = m == 0 ? bx : (m == 1 ? by : bz);
    const float da = (s * ak) * ke - sg * am, db = (s * bk) * ke - sg * bm;
    if (da >= 0.0f) put(ax, ay, az);
    if ((da >= 0.0f) != (db >= 0.0f)) {
      const float tq = da / (da - db);
      put(ax + (bx - ax) * tq, ay + (by - ay) * tq, az + (bz - az) * tq);
    }
  }
  out.n = o;
}

struct SlFace {
  float pu[8], pv[8];
  int n;         // polygon vertices (0 with whole = 1)
  int whole;     // the polygon reaches the light: every cell, no separating-axis test
  int x0, x1, y0, y1;
};

// geometry triangle (rt_tri_t record r) on face f; false: nothing on the face
__device__ __forceinline__ bool sl_project(const rt_tri_t& r, const float L[3], int f, int N, SlFace* F) {
  const int k = f >> 1, i = k == 0 ? 1 : 0, j = k == 2 ? 1 : 2;
  const float s = (f & 1) ? -1.0f : 1.0f;
  SlPoly A, B;
  for (int cc = 0; cc < 3; ++cc) {
    A.c[cc][0] = r.v[cc] - L[cc];
    A.c[cc][1] = (r.v[cc] + r.v[4 + cc]) - L[cc];
    A.c[cc][2] = (r.v[cc] + r.v[8 + cc]) - L[cc];
  }
  A.n = 3;
  sl_clip_plane(A, k, s, i, 1.0f, B);
  if (B.n) sl_clip_plane(B, k, s, i, -1.0f, A); else A.n = 0;
  if (A.n) sl_clip_plane(A, k, s, j, 1.0f, B); else B.n = 0;
  if (B.n) sl_clip_plane(B, k, s, j, -1.0f, A); else A.n = 0;
  const int m = A.n;
  if (!m) return false;
  const float hn = (float)N * 0.5f;
  F->whole = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (q < m && !(s * sl_axis(A, q, k) > 0.0f)) F->whole = 1;
  if (F->whole) {
    F->n = 0;
    F->x0 = F->y0 = 0;
    F->x1 = F->y1 = N - 1;
    return true;
  }
  float u0 = 0, u1 = 0, v0 = 0, v1 = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (q >= m) break;
    const float ck = s * sl_axis(A, q, k);
    F->pu[q] = sl_axis(A, q, i) / ck;
    F->pv[q] = sl_axis(A, q, j) / ck;
    if (q == 0 || F->pu[q] < u0) u0 = F->pu[q];
    if (q == 0 || F->pu[q] > u1) u1 = F->pu[q];
    if (q == 0 || F->pv[q] < v0) v0 = F->pv[q];
    if (q == 0 || F->pv[q] > v1) v1 = F->pv[q];
  }
  F->n = m;
  F->x0 = max((int)floorf(((u0 - RT_SLIST_EPS) + 1.0f) * hn), 0);
  F->x1 = min((int)floorf(((u1 + RT_SLIST_EPS) + 1.0f) * hn), N - 1);
  F->y0 = max((int)floorf(((v0 - RT_SLIST_EPS) + 1.0f) * hn), 0);
  F->y1 = min((int)floorf(((v1 + RT_SLIST_EPS) + 1.0f) * hn), N - 1);
  return F->x0 <= F->x1 && F->y0 <= F->y1;
}

// a list entry's sort key: a lower bound of |X - L|^2 over the triangle's
// points X -- the squared distance from the light L to the triangle's
// bounding box (corners v0, v0 + e1, v0 + e2); oracle/rt.c sl_key, the same
// float operations in the same order (no contraction)
__device__ __forceinline__ float sl_key(const rt_tri_t& r, const float L[3]) {
  const float* t = reinterpret_cast<const float*>(&r);
  float s = 0.0f;
  for (int k = 0; k < 3; ++k) {
    const float p = t[k], q = t[k] + t[4 + k], u = t[k] + t[8 + k];
    const float lo = fminf(p, fminf(q, u)), hi = fmaxf(p, fmaxf(q, u));
    const float d = L[k] < lo ? lo - L[k] : (L[k] > hi ? L[k] - hi : 0.0f);
    s = s + d * d;
  }
  return s;
}

// thread per item (geometry triangle j, cube face f), item = 6 j + f: the
// projection of the triangle on the face (sl_project) as an SPROJ record --
// [0] the cell rectangle's corner x0 | y0 << 16, [1] its width, [2] the
// separating axes n (0: every cell of the rectangle -- the polygon reaches
// the light or has fewer than 3 vertices), [3] the face, then per polygon
// edge a its axis (nx, ny) and the polygon's extent [p0, p1] along it, the
// quantities oracle/rt.c sl_cell_meets derives for every cell, computed
// once -- and the rectangle's cell count -> soff[item]; face 0 also stores
// the triangle's sort key
__device__ void phase_sproj(const rt_setup_arg_t* a) {
  const rt_tri_t* geom = vx_ptr<const rt_tri_t>(a->geom_addr);
  uint4* rec = vx_ptr<uint4>(a->sproj_addr);
  uint32_t* soff = vx_ptr<uint32_t>(a->soff_addr);
  uint32_t* skey = vx_ptr<uint32_t>(a->skey_addr);
  const int N = (int)a->slist_n;
  const uint32_t items = 6u * a->num_geom;
  for (uint32_t it = slice_b() * RTS_BLOCK + threadIdx.x; it < items; it += slice_n() * RTS_BLOCK) {
    const uint32_t j = it / 6u, f = it % 6u;
    const rt_tri_t r = geom[j];
    if (f == 0) skey[j] = __float_as_uint(sl_key(r, a->light));
    SlFace F;
    uint32_t cells = 0;
    if (sl_project(r, a->light, (int)f, N, &F)) {
      const uint32_t w = (uint32_t)(F.x1 - F.x0 + 1), h = (uint32_t)(F.y1 - F.y0 + 1);
      const uint32_t n = (F.whole || F.n < 3) ? 0u : (uint32_t)F.n;
      cells = w * h;
      uint4* o = rec + (uint64_t)it * (RTS_SPROJ_WORDS / 4);
      o[0] = make_uint4((uint32_t)F.x0 | ((uint32_t)F.y0 << 16), w, n, f);
#pragma unroll
      for (uint32_t e = 0; e < 7; ++e) {
        if (e >= n) break;
        const bool wrap = e + 1 >= n;
        const float nx = (wrap ? F.pv[0] : F.pv[e + 1]) - F.pv[e];
        const float ny = F.pu[e] - (wrap ? F.pu[0] : F.pu[e + 1]);
        float p0 = 0, p1 = 0;
#pragma unroll
        for (uint32_t q = 0; q < 7; ++q) {
          if (q >= n) break;
          const float d = nx * F.pu[q] + ny * F.pv[q];
          if (q == 0 || d < p0) p0 = d;
          if (q == 0 || d > p1) p1 = d;
        }
        o[1 + e] = make_uint4(__float_as_uint(nx), __float_as_uint(ny), __float_as_uint(p0), __float_as_uint(p1));
      }
    }
    soff[it] = cells;
  }
}

// (one workgroup) exclusive scan of the items' cell counts, the total
// candidates -> soff[items]
__device__ void phase_soscan(const rt_setup_arg_t* a) {
  const uint32_t items = 6u * a->num_geom;
  uint32_t* soff = vx_ptr<uint32_t>(a->soff_addr);
  scan_excl(soff, items, soff + items);
}

// Every candidate (item, cell of its rectangle), one per thread: q -> the
// item whose scanned range holds q (binary search of soff), the cell, and
// the separating-axis test of oracle/rt.c sl_cell_meets against the cell
// widened by RT_SLIST_EPS (the same float operations: its p0 / p1 are the
// record's); f(j, cell) for every cell the polygon meets
__shared__ uint32_t s_soff[RTS_SOFF_LDS + 1];
template <typename Fn>
__device__ __forceinline__ void sl_for_candidates(const rt_setup_arg_t* a, Fn f) {
  const uint4* rec = vx_ptr<const uint4>(a->sproj_addr);
  const uint32_t* soff = vx_ptr<const uint32_t>(a->soff_addr);
  const uint32_t items = 6u * a->num_geom;
  if (a->fold & RTS_FOLD_SOFF) {
    // SOSCAN folded: this workgroup scans the raw counts into LDS
    __shared__ uint32_t sp[RTS_BLOCK];
    const uint32_t chunk = (items + RTS_BLOCK - 1) / RTS_BLOCK;
    const uint32_t b0 = min(threadIdx.x * chunk, items), b1 = min(b0 + chunk, items);
    uint32_t sum = 0;
    for (uint32_t i = b0; i < b1; ++i) sum += soff[i];
    sp[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < RTS_BLOCK; o <<= 1) {
      const uint32_t y = threadIdx.x >= o ? sp[threadIdx.x - o] : 0u;
      __syncthreads();
      sp[threadIdx.x] += y;
      __syncthreads();
    }
    uint32_t run = sp[threadIdx.x] - sum;
    for (uint32_t i = b0; i < b1; ++i) {
      const uint32_t x = soff[i];
      s_soff[i] = run;
      run += x;
    }
    if (threadIdx.x == RTS_BLOCK - 1) s_soff[items] = sp[RTS_BLOCK - 1];
    __syncthreads();
    soff = s_soff;
  }
  const uint32_t total = soff[items];
  const uint32_t N = a->slist_n;
  const float cw = 2.0f / (float)N;
  for (uint32_t q = slice_b() * RTS_BLOCK + threadIdx.x; q < total; q += slice_n() * RTS_BLOCK) {
    uint32_t lo = 0, hi = items;  // the last item with soff <= q
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (soff[mid] <= q) lo = mid; else hi = mid;
    }
    const uint4* o = rec + (uint64_t)lo * (RTS_SPROJ_WORDS / 4);
    const uint4 h = o[0];
    const uint32_t li = q - soff[lo];
    const int cx = (int)(h.x & 0xffffu) + (int)(li % h.y), cy = (int)(h.x >> 16) + (int)(li / h.y);
    bool meets = true;
    if (h.z != 0) {
      const float rx0 = ((float)cx * cw - 1.0f) - RT_SLIST_EPS, rx1 = ((float)(cx + 1) * cw - 1.0f) + RT_SLIST_EPS;
      const float ry0 = ((float)cy * cw - 1.0f) - RT_SLIST_EPS, ry1 = ((float)(cy + 1) * cw - 1.0f) + RT_SLIST_EPS;
      for (uint32_t e = 0; e < h.z && meets; ++e) {
        const uint4 ax = o[1 + e];
        const float nx = __uint_as_float(ax.x), ny = __uint_as_float(ax.y);
        const float p0 = __uint_as_float(ax.z), p1 = __uint_as_float(ax.w);
        const float c0 = nx * rx0 + ny * ry0, c1 = nx * rx1 + ny * ry0;
        const float c2 = nx * rx0 + ny * ry1, c3 = nx * rx1 + ny * ry1;
        const float r0 = fminf(fminf(c0, c1), fminf(c2, c3)), r1 = fmaxf(fmaxf(c0, c1), fmaxf(c2, c3));
        meets = !(p1 < r0 || p0 > r1);
      }
    }
    if (meets) f(lo / 6u, (h.w * N + (uint32_t)cy) * N + (uint32_t)cx);
  }
}

__device__ void phase_scount(const rt_setup_arg_t* a) {
  uint32_t* cnt = vx_ptr<uint32_t>(a->scnt_addr);
  sl_for_candidates(a, [&](uint32_t, uint32_t cell) { atomicAdd(&cnt[cell], 1u); });
}

// the entries at their cells' cursors: geometry index, key, cell (stmp);
// entries past the capacity scap are dropped and flagged (status[7])
__device__ void phase_sfill(const rt_setup_arg_t* a) {
  uint32_t* cur = vx_ptr<uint32_t>(a->scnt_addr);
  const uint2* sidx = vx_ptr<const uint2>(a->sidx_addr);
  const uint32_t* skey = vx_ptr<const uint32_t>(a->skey_addr);
  uint32_t* tj = vx_ptr<uint32_t>(a->stmp_addr);
  uint32_t* status = vx_ptr<uint32_t>(a->status_addr);
  const uint32_t cap = a->scap;
  sl_for_candidates(a, [&](uint32_t j, uint32_t cell) {
    const uint32_t pos = sidx[cell].x + atomicAdd(&cur[cell], 1u);
    if (pos < cap) {
      tj[pos] = j;
      tj[cap + pos] = skey[j];
      tj[2u * cap + pos] = cell;
    } else {
      atomicOr(&status[7], 1u);
    }
  });
}

// thread per entry: its rank in its cell by (sort key, geometry index) --
// the nearest-to-the-light bounding boxes first, ties by index (distinct) --
// and its rt_tri_t copied to that position with the key in the second
// word's w (rt_tri_t e1.w, 0 in the geometry records), where the scan reads
// it; then (block 0) the render arguments' slist_on: the lists are used when
// they all fit (no overflow, the longest within max_list, the total within
// max_entries), else the frame's shadow rays walk the BVH
__device__ void phase_ssort(const rt_setup_arg_t* a) {
  const uint2* sidx = vx_ptr<const uint2>(a->sidx_addr);
  const uint32_t* tj = vx_ptr<const uint32_t>(a->stmp_addr);
  const uint4* geom = vx_ptr<const uint4>(a->geom_addr);
  uint4* out = vx_ptr<uint4>(a->slist_addr);
  const uint32_t* status = vx_ptr<const uint32_t>(a->status_addr);
  const uint32_t cap = a->scap, total = status[5], n = min(total, cap);
  const uint32_t* tk = tj + cap;
  const uint32_t* tc = tj + 2u * cap;
  if (slice_b() == 0 && threadIdx.x < 3 && total <= cap)  // padding record (the kernels load pairs ahead)
    out[3ull * total + threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
  if (slice_b() == 0 && threadIdx.x == 0 && a->rargs_addr) {
    const bool fit = status[7] == 0 && status[4] <= a->max_list && total <= a->max_entries;
    __hip_atomic_store(&vx_ptr<rt_kernel_arg_t>(a->rargs_addr)->slist_on, fit ? 1u : 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  for (uint32_t e = slice_b() * RTS_BLOCK + threadIdx.x; e < n; e += slice_n() * RTS_BLOCK) {
    const uint32_t me = tj[e], mk = tk[e];
    const uint2 oc = sidx[tc[e]];
    if (oc.x + oc.y > cap) continue;  // the cell's list overflowed (status[7]): the host refills
    uint32_t rank = 0;
    for (uint32_t q = oc.x; q < oc.x + oc.y; ++q) {
      const uint32_t j = tj[q], k = tk[q];  // keys >= 0: bits order as floats
      rank += (k < mk || (k == mk && j < me)) ? 1u : 0u;
    }
    const uint64_t d = 3ull * (oc.x + rank);
    out[d] = geom[3ull * me];
    uint4 w1 = geom[3ull * me + 1];
    w1.w = mk;
    out[d + 1] = w1;
    out[d + 2] = geom[3ull * me + 2];
  }
}

// renderer creation (app/rt_app.cpp rt_renderer_create): the clip-space
// triangle of every pid (v0.xyw + pid, e1, e2) and the geometry list's copy
__device__ __forceinline__ void tri_record(const float* verts, uint32_t g, rt_tri_t* out) {
  const float* p = verts + 32ull * g;
  const int src[3] = {0, 1, 3};
  float r[12];
  for (int k = 0; k < 3; ++k) {
    r[k] = p[src[k]];
    r[4 + k] = p[10 + src[k]] - p[src[k]];
    r[8 + k] = p[20 + src[k]] - p[src[k]];
  }
  r[3] = __int_as_float((int32_t)g);
  r[7] = r[11] = 0.0f;
  float4* d = reinterpret_cast<float4*>(out);
  d[0] = make_float4(r[0], r[1], r[2], r[3]);
  d[1] = make_float4(r[4], r[5], r[6], r[7]);
  d[2] = make_float4(r[8], r[9], r[10], r[11]);
}

__device__ void phase_records(const rt_setup_arg_t* a) {
  const float* verts = vx_ptr<const float>(a->verts_addr);
  const int32_t* geometry = vx_ptr<const int32_t>(a->geometry_addr);
  rt_tri_t* ptris = vx_ptr<rt_tri_t>(a->ptris_addr);
  rt_tri_t* geom = vx_ptr<rt_tri_t>(a->geom_addr);
  const uint32_t total = a->num_prims + a->num_geom;
  for (uint32_t i = slice_b() * RTS_BLOCK + threadIdx.x; i < total; i += slice_n() * RTS_BLOCK) {
    if (i < a->num_prims) tri_record(verts, i, ptris + i);
    else tri_record(verts, (uint32_t)geometry[i - a->num_prims], geom + (i - a->num_prims));
  }
}

// one wide sub-phase (on this workgroup's slice, slice_b() / slice_n())
__device__ void run_phase(const rt_setup_arg_t* arg, uint32_t bit) {
  switch (bit) {
    case RTS_FILL: phase_fill(arg); break;
    case RTS_PRIMVIS: phase_primvis(arg); break;
    case RTS_SPROJ: phase_sproj(arg); break;
    case RTS_VTRIS: phase_vtris(arg); break;
    case RTS_WEIGHT: phase_weight(arg); break;
    case RTS_LINK: phase_link(arg); break;
    case RTS_ROWSUM: phase_rowsum(arg); break;
    case RTS_CLIMB: phase_climb<false>(arg); break;
    case RTS_COLSUM: phase_colsum(arg); break;
    case RTS_HIST: phase_hist(arg); break;
    case RTS_SCATTER: phase_scatter(arg); break;
    case RTS_RECORDS: phase_records(arg); break;
    case RTS_BCOUNT: phase_bcount(arg); break;
    case RTS_BSUM: phase_lsum(block_set(arg)); break;
    case RTS_BOFF: phase_loff(block_set(arg), (arg->fold & RTS_FOLD_LISTS) != 0); break;
    case RTS_BFILL: phase_bfill(arg); break;
    case RTS_BSORT: phase_bsort(arg); break;
    case RTS_SCOUNT: phase_scount(arg); break;
    case RTS_SSUM: phase_lsum(cell_set(arg)); break;
    case RTS_SOFF: phase_loff(cell_set(arg), (arg->fold & RTS_FOLD_LISTS) != 0); break;
    case RTS_SFILL: phase_sfill(arg); break;
    case RTS_SSORT: phase_ssort(arg); break;
    default: break;
  }
}
// the wide sub-phases in run order, with their shares of a partitioned
// launch's workgroups (the per-primitive scan of PRIMVIS and the per-entry
// list phases carry the longest per-workgroup chains)
__constant__ const uint32_t kWide[22][2] = {
    {RTS_FILL, 2},   {RTS_PRIMVIS, 16}, {RTS_SPROJ, 3},  {RTS_VTRIS, 1},  {RTS_WEIGHT, 1},  {RTS_LINK, 3},
    {RTS_ROWSUM, 1}, {RTS_CLIMB, 3},   {RTS_COLSUM, 1}, {RTS_HIST, 1},   {RTS_SCATTER, 2}, {RTS_RECORDS, 2},
    {RTS_BCOUNT, 2}, {RTS_BSUM, 1},    {RTS_BOFF, 1},   {RTS_BFILL, 2},  {RTS_BSORT, 4},   {RTS_SCOUNT, 3},
    {RTS_SSUM, 1},   {RTS_SOFF, 2},    {RTS_SFILL, 3},  {RTS_SSORT, 3}};
// the wide sub-phases of `ph` (each independent of the others in the same
// launch).  part: each on its own slice of the grid, in proportion to its
// share, so they run side by side (a launch then takes about its longest
// sub-phase instead of their sum); otherwise each on the whole grid in turn.
__device__ void run_phases(const rt_setup_arg_t* arg, uint32_t ph, bool part) {
  if ((ph & RTS_CLIMB) && arg->num_nodes <= RTS_CLIMB_WG_NODES) ph &= ~RTS_CLIMB;  // one workgroup: run_scans
  uint32_t total = 0;
  for (int i = 0; i < 22; ++i) total += (ph & kWide[i][0]) ? kWide[i][1] : 0u;
  if (total == 0) return;
  const uint32_t G = gridDim.x;
  uint32_t cum = 0;
  for (int i = 0; i < 22; ++i) {
    const uint32_t bit = kWide[i][0];
    if (!(ph & bit)) continue;
    uint32_t b0 = 0, b1 = G;
    if (part) {
      b0 = (uint32_t)((uint64_t)G * cum / total);
      cum += kWide[i][1];
      b1 = (uint32_t)((uint64_t)G * cum / total);
      if (b1 <= b0) b1 = b0 + 1;  // at least one workgroup (G >= the sub-phase count)
      if (blockIdx.x < b0 || blockIdx.x >= b1) continue;
    }
    __syncthreads();  // the previous sub-phase's reads of the slice are done
    if (threadIdx.x == 0) {
      s_slice[0] = blockIdx.x - b0;
      s_slice[1] = b1 - b0;
    }
    __syncthreads();
    run_phase(arg, bit);
  }
}
// the one-workgroup sub-phases of `ph` (scans): the k-th present one by
// workgroup k, so the scans of one launch run side by side
__device__ void run_scans(const rt_setup_arg_t* arg, uint32_t ph) {
  uint32_t k = 0;
  if ((ph & RTS_CLIMB) && arg->num_nodes <= RTS_CLIMB_WG_NODES && blockIdx.x == k++) phase_climb<true>(arg);
  if ((ph & RTS_SOSCAN) && blockIdx.x == k++) phase_soscan(arg);
  if ((ph & RTS_BSCAN) && blockIdx.x == k++) phase_lscan(block_set(arg));
  if ((ph & RTS_SSCAN) && blockIdx.x == k++) phase_lscan(cell_set(arg));
  if ((ph & RTS_SCAN) && blockIdx.x == k++) {
    scan_excl(vx_ptr<uint32_t>(arg->hist_addr), 256u * arg->nblocks, nullptr);
    __syncthreads();
    // local tiles with weight > 0 = items whose digit is below 255 = the
    // exclusive-scan offset of digit 255 in block 0
    if (threadIdx.x == 0)
      vx_ptr<uint32_t>(arg->status_addr)[3] = vx_ptr<const uint32_t>(arg->hist_addr)[255u * arg->nblocks];
  }
}

}  // namespace

// grid: 4 workgroups of 256 threads per CU (1024 on MI355X) -- the phases
// are grid-stride loops, and a sequence's one-workgroup steps (the scans) or
// small steps then pay the dispatch of 1024 workgroups instead of 4096
__device__ __attribute__((used)) uint32_t __vx_grid_per_cu = 4;

// A single launch runs `phases`; launch i of a sequence (nseq > 0, launch
// tag i) runs seq_phases[i] -- the scans, one-workgroup phases, by
// workgroup 0 in either case.  A sequence's dependent steps are launches
// queued back to back on the driver's stream: the launch boundary makes
// each step's stores visible to the next (per-XCD L2s are not coherent
// within a launch), with no host round trip and no device-side counter.
// Registers capped for 4 waves per SIMD (PRIMVIS alone would take 184 VGPRs;
// at 120 nothing spills).
VX_MAIN_OCC(rt_setup_arg_t, arg, RTS_BLOCK, 4) {
  const uint32_t ph = arg->nseq == 0 ? arg->phases
                      : vx_launch_tag < RTS_MAX_SEQ ? arg->seq_phases[vx_launch_tag] : 0u;
  // the last launch of a sequence starts after every earlier one has
  // finished, and its sub-phases write no status word: the status is final
  // (one thread: the words, a system-scope fence, then the nonce the host
  // polls for -- it may return before this launch's own sub-phases finish,
  // which later work follows in stream order anyway)
  if (arg->status_host != 0 && arg->nseq >= 2 && vx_launch_tag + 1 == arg->nseq && blockIdx.x == 0 &&
      threadIdx.x == 0) {
    volatile uint32_t* h = reinterpret_cast<volatile uint32_t*>(arg->status_host);
    const volatile uint32_t* st = vx_ptr<const uint32_t>(arg->status_addr);
    for (int i = 0; i < RTS_STATUS_WORDS; ++i) h[i] = st[i];
    __threadfence_system();
    h[RTS_STATUS_WORDS] = arg->status_nonce;
  }
  run_phases(arg, ph, arg->nseq != 0 && arg->part != 0);
  run_scans(arg, ph);
  return 0;
}
