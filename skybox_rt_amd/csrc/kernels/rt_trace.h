// rt_trace.h -- device pieces shared by the RT kernel programs
// (rt_kernel.hip: primary + shadow rays; pt_kernel.hip: diffuse path trace):
// scene arguments, ray setup, Möller–Trumbore, slab test, the per-lane BVH
// walk (closest hit / any hit, stack in LDS) and the wave-packet walks
// (primary visibility, shadow rays; stack in one VGPR), the per-block
// candidate lists, draw3d-exact shading, pixel addressing.  Numerics are
// bit-identical to the oracle (oracle/rt.c): every fused multiply-add is an
// explicit fmaf, everything else is compiled with -ffp-contract=off,
// divisions and square roots are IEEE (correctly rounded).
//
// Image knobs (Makefile per-image defines; DESIGN.md §4 keeps the record of
// the variants measured and not kept):
//   RT_ONLY_BVH4H   the image walks only the binary16 BVH4 (the regular
//                   images); 0: every layout (the deep images)
//   RT_PUSH_UNCOND  per-lane BVH4 pushes as unconditional rows (path tracer)
//   RT_LAZY_TASK_ARGS  task-map fields re-read from the argument block
//   RT_BVH_WALK     the image walks the BVH for primary and shadow rays (no
//                   block-list / light-space-list code: image rt_bvh)
//   RT_INSTRUMENT   algorithmic counters (node visits, tests, texels)
//   RT_STAMPS / RT_TRACE_CYCLES  diagnostic per-wave stamps
#pragma once

#include <hip/hip_runtime.h>

#include "gfx_device.h"
#include "rt_common.h"
#include "vx_spawn.h"

#ifndef RT_ONLY_BVH4H
#define RT_ONLY_BVH4H 0
#endif
#ifndef RT_BVH_WALK
#define RT_BVH_WALK 0  // 1: image rt_bvh -- primary and shadow rays walk the BVH, no list code
#endif

namespace rtk {


struct Counters {
  uint32_t primary = 0, shadow = 0, hits = 0, occluded = 0, bounce = 0;
// RT_CNT(stmt): a counter update that only the instrumented images
// (RT_INSTRUMENT, the *_stats kernels) compile
#ifdef RT_INSTRUMENT
#define RT_CNT(...) __VA_ARGS__
#else
#define RT_CNT(...)
#endif
#ifdef RT_INSTRUMENT
  uint32_t visits = 0, tests = 0, layer_tests = 0, shaded = 0, texel_bytes = 0;
  uint32_t rect_tests = 0, edge_tests = 0;  // flat image: work executed per wave
#endif
};

// Kernel arguments in scalar registers; buffer addresses become 32-bit
// arena offsets (rt_app checks every buffer lies below 4 GiB).
struct Scene {
  vx_arena A;
  uint32_t nodes, nodes4, tris, prims, dcs, cbuf, ptris, geom, order;
  uint32_t vnodes, vtris, vlayers, vgeom, num_vnodes;  // primary visibility (rt_common.h)
  uint32_t num_nodes, num_nodes4, num_layer, num_geom, flags, width, height;
  uint32_t shard_index, shard_count, tiles_x, clear_color, bounces, seed, split_tiles, split_log;
  uint32_t tiles_x_magic, num_tasks;
  float sx, sy, light[3];
  uint64_t argp;  // the argument block (constant address space), for lazy_args
  uint32_t blist, bidx, blist_blocks;  // per-block candidate lists (rt_bentry_t)
  uint32_t sidx, slist, slist_on, slist_n;  // light-space shadow lists (rt_common.h)
};

// The argument block is read through the scalar cache (constant address
// space, wave-uniform address): the scene's fields then live in SGPRs, and
// the traversal loops form node / triangle addresses in scalar registers
// instead of VGPR + readfirstlane.
//
// The frame's launch words (rt_common.h RT_LW_*), kernel arguments like the
// tag, override the block's light and switch stale lists off.
__device__ __forceinline__ Scene load_scene(const rt_kernel_arg_t* ga, const vx_launch_words_t& lw) {
  const uint64_t p = (uint64_t)ga;
  // (readfirstlane returns int: through uint32_t, or the low word sign-extends)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const uint64_t u = ((uint64_t)hi << 32) | (uint64_t)lo;
  const __attribute__((address_space(4))) rt_kernel_arg_t* a =
      (const __attribute__((address_space(4))) rt_kernel_arg_t*)u;
  Scene s;
  s.argp = (uint64_t)a;
  s.A = vx_arena::get();
  s.nodes = (uint32_t)a->nodes_addr;
  s.nodes4 = (uint32_t)a->nodes4_addr;
  s.tris = (uint32_t)a->tris_addr;
  s.vnodes = (uint32_t)a->vnodes_addr;
  s.vtris = (uint32_t)a->vtris_addr;
  s.vlayers = (uint32_t)a->vlayers_addr;
  s.vgeom = (uint32_t)a->vgeom_addr;
  s.num_vnodes = a->num_vnodes;
  s.prims = (uint32_t)a->prims_addr;
  s.dcs = (uint32_t)a->dcs_addr;
  s.cbuf = (uint32_t)a->cbuf_addr;
  s.ptris = (uint32_t)a->ptris_addr;
  s.geom = (uint32_t)a->geom_addr;
  s.order = (uint32_t)a->order_addr;
  s.num_geom = a->num_geom;
  s.bounces = a->bounces;
  s.seed = a->seed;
  s.split_tiles = a->split_tiles;
  s.split_log = a->split_log;
  s.blist = (uint32_t)a->blist_addr;
  s.bidx = (uint32_t)a->bidx_addr;
  s.blist_blocks = a->blist_blocks;
  s.sidx = (uint32_t)a->sidx_addr;
  s.slist = (uint32_t)a->slist_addr;
  s.slist_on = a->slist_on;
  s.slist_n = a->slist_n;
  s.num_nodes = a->num_nodes;
  s.num_nodes4 = a->num_nodes4;
  s.num_layer = a->num_layer_tris;
  s.flags = a->flags;
  s.width = a->width;
  s.height = a->height;
  s.shard_index = a->shard_index;
  s.shard_count = a->shard_count;
  s.tiles_x = a->tiles_x;
  s.tiles_x_magic = a->tiles_x_magic;
  s.num_tasks = a->num_tasks;  // through the scalar cache (arg->num_tasks would be a flat load)
  s.clear_color = a->clear_color;
  s.sx = a->sx;
  s.sy = a->sy;
  s.light[0] = a->light[0];
  s.light[1] = a->light[1];
  s.light[2] = a->light[2];
  if (lw.w[3] & RT_LW_LIGHT) {
    s.light[0] = __builtin_bit_cast(float, lw.w[0]);
    s.light[1] = __builtin_bit_cast(float, lw.w[1]);
    s.light[2] = __builtin_bit_cast(float, lw.w[2]);
  }
  if (lw.w[3] & RT_LW_NO_SLIST) s.slist_on = 0;
  return s;
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// RT_STAMPS diagnostic image only: count one wave-level execution of the
// enclosing loop body in counter slot `slot` (one lane adds; one-wave
// workgroups, so the slot is this wave's)
#ifdef RT_STAMPS
#define RT_WAVE_ITER(slot)                                                         \
  do {                                                                             \
    if (lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)))                      \
      atomicAdd(&__vx_mpm_lds[slot], 1u);                                         \
  } while (0)
// cycles from issuing a packet walk's record load to its data (rt stamp
// image: slot 0 primary packets, slot 1 shadow packets; s_memtime, explicit
// wait; not in the path tracer's stamp image)
#ifdef RT_TRACE_CYCLES
#define RT_LD_BEGIN() do {} while (0)
#define RT_LD_END(slot) do {} while (0)
#else
#define RT_LD_BEGIN() const uint64_t rt_ld0 = __builtin_amdgcn_s_memtime()
#define RT_LD_END(slot)                                                            \
  do {                                                                             \
    __builtin_amdgcn_s_waitcnt(0xC07F);                                            \
    const uint32_t rt_ldd = (uint32_t)(__builtin_amdgcn_s_memtime() - rt_ld0);     \
    if (lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)))                      \
      atomicAdd(&__vx_mpm_lds[slot], rt_ldd);                                     \
  } while (0)
#endif
#else
#define RT_WAVE_ITER(slot) do {} while (0)
#define RT_LD_BEGIN() do {} while (0)
#define RT_LD_END(slot) do {} while (0)
#endif
// RT_TRACE_CYCLES (path-tracer stamp image only): wave cycles spent in the
// secondary traversal's node loop (slot 11) and leaf rounds (slot 3)
#ifdef RT_TRACE_CYCLES
#define RT_CYC_BEGIN() const uint64_t rt_cyc0 = __builtin_amdgcn_s_memtime()
#define RT_CYC_END(slot)                                                                  \
  do {                                                                                    \
    const uint32_t d = (uint32_t)(__builtin_amdgcn_s_memtime() - rt_cyc0);               \
    if (lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)))                             \
      atomicAdd(&__vx_mpm_lds[slot], d);                                                  \
  } while (0)
#else
#define RT_CYC_BEGIN() do {} while (0)
#define RT_CYC_END(slot) do {} while (0)
#endif

struct Ray {
  float o[3], d[3];
  float inv[3], oi[3];
};

__device__ __forceinline__ float safe_dir(float d) {
  return fabsf(d) < 1e-20f ? (d < 0.0f ? -1e-20f : 1e-20f) : d;
}

__device__ __forceinline__ void ray_setup(Ray& r) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    r.inv[k] = 1.0f / safe_dir(r.d[k]);
    r.oi[k] = r.o[k] * r.inv[k];
  }
}

__device__ __forceinline__ void cross3(float* r, const float* a, const float* b) {
  r[0] = fmaf(a[1], b[2], -(a[2] * b[1]));
  r[1] = fmaf(a[2], b[0], -(a[0] * b[2]));
  r[2] = fmaf(a[0], b[1], -(a[1] * b[0]));
}
__device__ __forceinline__ float dot3(const float* a, const float* b) {
  return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0]));
}

// Möller–Trumbore with the reference's inclusive coverage (oracle/rt.c mt_hit)
__device__ __forceinline__ bool mt_hit(const Ray& r, const float4& a, const float4& b,
                                       const float4& c, float tmin, float* t_out) {
  const float v0[3] = {a.x, a.y, a.z}, e1[3] = {b.x, b.y, b.z}, e2[3] = {c.x, c.y, c.z};
  float pvec[3], tvec[3], qvec[3];
  cross3(pvec, r.d, e2);
  const float det = dot3(e1, pvec);
  tvec[0] = r.o[0] - v0[0];
  tvec[1] = r.o[1] - v0[1];
  tvec[2] = r.o[2] - v0[2];
  float u = dot3(tvec, pvec);
  cross3(qvec, tvec, e1);
  float v = dot3(r.d, qvec);
  float adet = det;
  if (det < 0.0f) { adet = -det; u = -u; v = -v; }
  if (!(adet > 0.0f) || u < 0.0f || v < 0.0f || u + v > adet) return false;
  const float t = dot3(e2, qvec) / det;
  if (!(t > tmin)) return false;
  *t_out = t;
  return true;
}

// mt_hit without branches: the same operations in the same order, every
// value computed, the verdict one predicate (a leaf's tests run without
// exec-mask branching; *t_out is meaningful only when it returns true)
__device__ __forceinline__ bool mt_hit_bf(const Ray& r, const float4& a, const float4& b,
                                          const float4& c, float tmin, float* t_out) {
  const float v0[3] = {a.x, a.y, a.z}, e1[3] = {b.x, b.y, b.z}, e2[3] = {c.x, c.y, c.z};
  float pvec[3], tvec[3], qvec[3];
  cross3(pvec, r.d, e2);
  const float det = dot3(e1, pvec);
  tvec[0] = r.o[0] - v0[0];
  tvec[1] = r.o[1] - v0[1];
  tvec[2] = r.o[2] - v0[2];
  float u = dot3(tvec, pvec);
  cross3(qvec, tvec, e1);
  float v = dot3(r.d, qvec);
  const bool neg = det < 0.0f;
  const float adet = neg ? -det : det;
  u = neg ? -u : u;
  v = neg ? -v : v;
  const float t = dot3(e2, qvec) / det;
  *t_out = t;
  return (adet > 0.0f) & !(u < 0.0f) & !(v < 0.0f) & !(u + v > adet) & (t > tmin);
}

// slab test of one child; box planes interleaved as in rt_node_t
__device__ __forceinline__ bool slab(float lox, float hix, float loy, float hiy, float loz,
                                     float hiz, const Ray& r, float tmin, float tmax,
                                     float* tnear) {
  const float ax = fmaf(lox, r.inv[0], -r.oi[0]), bx = fmaf(hix, r.inv[0], -r.oi[0]);
  const float ay = fmaf(loy, r.inv[1], -r.oi[1]), by = fmaf(hiy, r.inv[1], -r.oi[1]);
  const float az = fmaf(loz, r.inv[2], -r.oi[2]), bz = fmaf(hiz, r.inv[2], -r.oi[2]);
  const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), tmin));
  const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
  *tnear = tn;
  return tn <= tf;
}
// the same test, also returning the far value (for a lane-mask compare)
__device__ __forceinline__ bool slab_nf(float lox, float hix, float loy, float hiy, float loz,
                                        float hiz, const Ray& r, float tmin, float tmax,
                                        float* tnear, float* tfar) {
  const float ax = fmaf(lox, r.inv[0], -r.oi[0]), bx = fmaf(hix, r.inv[0], -r.oi[0]);
  const float ay = fmaf(loy, r.inv[1], -r.oi[1]), by = fmaf(hiy, r.inv[1], -r.oi[1]);
  const float az = fmaf(loz, r.inv[2], -r.oi[2]), bz = fmaf(hiz, r.inv[2], -r.oi[2]);
  const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), tmin));
  const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
  *tnear = tn;
  *tfar = tf;
  return tn <= tf;
}
// lane masks straight from one v_cmp (inactive lanes 0), instead of a
// ballot of a combined bool (which the compiler re-materialises with a
// v_cndmask + v_cmp pair): ordered a <= b, unsigned a == b, unsigned a <= b
// (fcmpf: the float form; __builtin_amdgcn_fcmp takes doubles and compares in f64)
__device__ __forceinline__ uint64_t mask_fle(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, 5); }
__device__ __forceinline__ uint64_t mask_ueq(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 32); }
__device__ __forceinline__ uint64_t mask_ule(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 37); }

// closest-hit order: t, then pid by the drawcall's depth-compare tie rule
__device__ __forceinline__ bool closer(float t, int32_t pid, float bt, int32_t bpid, bool tie_high) {
  return (t < bt) || (t == bt && (tie_high ? pid > bpid : pid < bpid));
}

// BVH2 node step (deep images only: RT_RENDER_BVH2 and the LBVH's BVH2):
// both slabs of an rt_node_t
struct NodeStep {
  int32_t c0, c1;
  float tn0, tn1;
  bool h0, h1;
};

__device__ __forceinline__ NodeStep node_step(const float4& n0, const float4& n1, const float4& n2,
                                              const float4& n3, const Ray& r, float tmin,
                                              float lim) {
  NodeStep o;
  o.c0 = __float_as_int(n3.x);
  o.c1 = __float_as_int(n3.y);
  o.tn0 = 0.0f;
  o.tn1 = 0.0f;
  o.h0 = (o.c0 != RT_EMPTY_REF) && slab(n0.x, n0.y, n1.x, n1.y, n2.x, n2.y, r, tmin, lim, &o.tn0);
  o.h1 = (o.c1 != RT_EMPTY_REF) && slab(n0.z, n0.w, n1.z, n1.w, n2.z, n2.w, r, tmin, lim, &o.tn1);
  return o;
}

// Per-lane traversal stack: LDS column stack[entry][lane] (conflict-free);
// a push onto a full stack is dropped -- the oracle's overflow rule
// (oracle/rt.c bvh_trace)
struct LaneStack {
  int32_t* mem;
  int sp = 0;
  __device__ __forceinline__ explicit LaneStack(int32_t* m) : mem(m) {}
  __device__ __forceinline__ void push(int32_t x) {
    if (sp < RT_MAX_STACK) mem[64 * sp++] = x;
  }
  // push the hit children c[1..n-1] of a sorted node step (c[n-1] first, so
  // c[1] ends on top) -- push()'s order and overflow rule, as predicated
  // stores instead of a branch per push
  __device__ __forceinline__ void push_sorted(const int32_t c[4], int n) {
#if RT_PUSH_UNCOND
    // the same rows get the same entries (row sp + i holds c[n-1-i]); the
    // three stores run unconditionally -- rows from the new top up hold
    // garbage never read, and a full stack's stores land in the slack rows
    int32_t c1 = c[1], c2 = c[2], c3 = c[3];
    // opaque register values: keeps the selects below from being folded
    // into a dynamically indexed (scratch) load of c[]
    asm("" : "+v"(c1), "+v"(c2), "+v"(c3));
    int32_t* m = mem + 64 * sp;
    m[0] = n == 2 ? c1 : (n == 3 ? c2 : c3);
    m[64] = n == 3 ? c1 : c2;
    m[128] = c1;
#else
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const int pos = sp + n - 1 - j;
      if (j < n && pos < RT_MAX_STACK) mem[64 * pos] = c[j];
    }
#endif
    const int top = sp + n - 1;
    sp = top < RT_MAX_STACK ? top : RT_MAX_STACK;
  }
  __device__ __forceinline__ bool pop(int32_t& x) {
    if (sp == 0) return false;
    x = mem[64 * --sp];
    return true;
  }
};

// BVH4 node step (RT_FLAG_BVH4; oracle/rt.c bvh4_step restates it): 7
// per-lane 16-B loads (boxes SoA over the 4 children + child refs), 4 slab
// tests, the hits ordered by tnear with a 5-exchange sorting network (strict
// <, misses keyed +inf, hit keys clamped to FLT_MAX so they sort first); the
// nearest is returned, the other hits are pushed farthest first.  Any-hit
// walks (`any`) key the hits by slot instead: children in fixed slot order,
// the order a wave's shadow packet (occluded_packet) walks them, so a lane's
// visits are the same either way.  Halves the dependent load -> test ->
// branch steps of a root-to-leaf walk vs BVH2.
template <bool SCALAR, bool F16>
__device__ __forceinline__ int32_t node4_step(const Scene& S, uint32_t ref, const Ray& r,
                                              float tmin, float lim, bool any, LaneStack& st) {
  // SCALAR: every active lane is at this node -- one scalar-cache load per
  // record for the wave instead of 64 lanes of vector data return
  auto ld = [&](uint32_t o) { return SCALAR ? S.A.sld_f4(o) : S.A.ld_f4(o); };
  float4 lx, hx, ly, hy, lz, hz, cf;
  if (F16) {
    // binary16 planes: 3 + 1 loads of 16 B; the conversions are exact, so the
    // planes equal rt_node4_t's (the host rounded those to binary16 values),
    // and each folds into its slab FMA (v_fma_mix_f32: f16 operand, f32 math)
    // -- the layout is a template parameter so no phi separates them
    const uint32_t no = S.nodes4 + 128u * S.num_nodes4 + 64u * ref;
    const float4 px = ld(no), py = ld(no + 16), pz = ld(no + 32);
    cf = ld(no + 48);
    auto h2 = [](float w, float& a, float& b) {
      const uint32_t u = __float_as_uint(w);
      a = (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu));
      b = (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16));
    };
    h2(px.x, lx.x, lx.y); h2(px.y, lx.z, lx.w); h2(px.z, hx.x, hx.y); h2(px.w, hx.z, hx.w);
    h2(py.x, ly.x, ly.y); h2(py.y, ly.z, ly.w); h2(py.z, hy.x, hy.y); h2(py.w, hy.z, hy.w);
    h2(pz.x, lz.x, lz.y); h2(pz.y, lz.z, lz.w); h2(pz.z, hz.x, hz.y); h2(pz.w, hz.z, hz.w);
  } else {
    const uint32_t no = S.nodes4 + 128u * ref;
    lx = ld(no); hx = ld(no + 16); ly = ld(no + 32);
    hy = ld(no + 48); lz = ld(no + 64); hz = ld(no + 80);
    cf = ld(no + 96);
  }
  const float alx[4] = {lx.x, lx.y, lx.z, lx.w}, ahx[4] = {hx.x, hx.y, hx.z, hx.w};
  const float aly[4] = {ly.x, ly.y, ly.z, ly.w}, ahy[4] = {hy.x, hy.y, hy.z, hy.w};
  const float alz[4] = {lz.x, lz.y, lz.z, lz.w}, ahz[4] = {hz.x, hz.y, hz.z, hz.w};
  int32_t c[4] = {__float_as_int(cf.x), __float_as_int(cf.y), __float_as_int(cf.z),
                  __float_as_int(cf.w)};
  float k[4];
  int n = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float tn = 0.0f;
    // every lane evaluates all four slabs (no exec-mask branch per child)
    const bool hs = slab(alx[i], ahx[i], aly[i], ahy[i], alz[i], ahz[i], r, tmin, lim, &tn);
    const bool h = hs & (c[i] != RT_EMPTY_REF);
    k[i] = h ? (any ? (float)i : fminf(tn, 3.402823466e38f)) : __builtin_inff();
    n += h ? 1 : 0;
  }
  auto cx = [&](int a, int b) {
    const bool s = k[b] < k[a];
    const float ka = k[a], kb = k[b];
    const int32_t ca = c[a], cb = c[b];
    k[a] = s ? kb : ka;
    k[b] = s ? ka : kb;
    c[a] = s ? cb : ca;
    c[b] = s ? ca : cb;
  };
  cx(0, 1);
  cx(2, 3);
  cx(0, 2);
  cx(1, 3);
  cx(1, 2);
  if (n == 0) return RT_EMPTY_REF;
  st.push_sorted(c, n);
  return c[0];
}

// MODE 0: closest hit, 1: any hit (first occluder below tmax), 2: chosen
// per lane by `any_rt` -- lanes of one wave tracing different ray kinds in
// the same traversal loop (the path tracer's paired shadow + bounce rays).
// Per ray, every mode visits the same nodes and returns the same result.
template <int MODE>
__device__ __forceinline__ int32_t trace_impl(const Scene& S, const Ray& r, float tmin, float tmax,
                                              int32_t skip, bool tie_high, float* t_out,
                                              int32_t* stack, Counters& cnt, bool any_rt) {
  const bool ANY = MODE == 1 || (MODE == 2 && any_rt);
  if (S.num_nodes == 0) return -1;
  LaneStack lst(stack);
  int32_t ref = 0;
  float bt = tmax;
  int32_t bpid = -1;
  // one node step: the next node to visit (nearest hit child), the other hit
  // children pushed farthest first; RT_EMPTY_REF when no child is hit
  auto node_next = [&](bool uni, int32_t r0) -> int32_t {
    RT_CNT(++cnt.visits;)
    const float lim = ANY ? tmax : bt;
    if (RT_ONLY_BVH4H || (S.flags & RT_FLAG_BVH4H))
      return uni ? node4_step<true, true>(S, (uint32_t)r0, r, tmin, lim, ANY, lst)
                 : node4_step<false, true>(S, (uint32_t)ref, r, tmin, lim, ANY, lst);
#if !RT_ONLY_BVH4H
    if (S.flags & RT_FLAG_BVH4)
      return uni ? node4_step<true, false>(S, (uint32_t)r0, r, tmin, lim, ANY, lst)
                 : node4_step<false, false>(S, (uint32_t)ref, r, tmin, lim, ANY, lst);
    NodeStep st;
    if (uni) {
      const uint32_t no = S.nodes + 64u * (uint32_t)r0;
      st = node_step(S.A.sld_f4(no), S.A.sld_f4(no + 16), S.A.sld_f4(no + 32),
                     S.A.sld_f4(no + 48), r, tmin, lim);
    } else {
      const uint32_t no = S.nodes + 64u * (uint32_t)ref;
      st = node_step(S.A.ld_f4(no), S.A.ld_f4(no + 16), S.A.ld_f4(no + 32),
                     S.A.ld_f4(no + 48), r, tmin, lim);
    }
    if (st.h0 && st.h1) {
      const bool swap = !ANY && st.tn1 < st.tn0;  // any-hit: fixed slot order
      lst.push(swap ? st.c0 : st.c1);
      return swap ? st.c1 : st.c0;
    }
    if (st.h0) return st.c0;
    if (st.h1) return st.c1;
    return RT_EMPTY_REF;
#endif
  };
  {
    // every lane starts at the root: one wave-uniform (scalar) step; a walk
    // whose root step hits no child has pushed nothing and is over
    const int32_t nx = node_next(true, 0);
    if (nx == RT_EMPTY_REF) return -1;
    ref = nx;
  }
  for (;;) {
    // while-while (Aila & Laine 2009): a lane steps through inner nodes until
    // it reaches a leaf or its stack runs dry, and the wave tests leaves only
    // once no lane is still in the node loop -- the per-lane sequence of node
    // visits and leaf tests (hence every counter and result) is unchanged
    bool dry = false;
    {
      RT_CYC_BEGIN();
      while (ref >= 0) {
        RT_WAVE_ITER(9);
        const int32_t nx = node_next(false, 0);
        if (nx != RT_EMPTY_REF) { ref = nx; continue; }
        if (!lst.pop(ref)) { dry = true; break; }
      }
      RT_CYC_END(11);
    }
    if (dry) break;
    {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      RT_WAVE_ITER(9);
      // a leaf's (up to 4) triangles: all 4 slots loaded at once (the tris
      // array carries 3 padding records), so their loads overlap
      const uint32_t to = S.tris + 48u * first;
      float4 ta[4], tb[4], tc[4];
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        ta[k] = S.A.ld_f4(to + 48u * k);
        tb[k] = S.A.ld_f4(to + 48u * k + 16);
        tc[k] = S.A.ld_f4(to + 48u * k + 32);
      }
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        if (k < count) {
          const int32_t pid = __float_as_int(ta[k].w);
          RT_CNT(++cnt.tests;)
          float t;
          if (pid != skip && mt_hit(r, ta[k], tb[k], tc[k], tmin, &t)) {
            if (ANY) {
              if (t < tmax) { *t_out = t; return pid; }
            } else if (closer(t, pid, bt, bpid, tie_high)) {
              bt = t;
              bpid = pid;
            }
          }
        }
      }
    }
    if (!lst.pop(ref)) break;
  }
  if (bpid >= 0) *t_out = bt;
  return bpid;
}

// Any-hit packet walk for the shadow segments of a wave (binary16 BVH4):
// the wave's rays walk the tree together -- node and leaf records
// wave-uniform through the scalar cache, children in fixed slot order, a
// child entered when some unfinished lane's ray hits its box and all its
// ancestors', the triangles of a leaf tested by every such lane, a lane
// finished at its first occluder, the walk over when every lane is
// finished.  Restricted to one lane, that is the per-lane any-hit walk
// (trace<true>: same fixed order, same first occluder), so each lane's
// verdict and its visit / test counts are the per-lane walk's: a lane counts
// a node or triangle only while it is on the path (it hit the node's box and
// its ancestors') and unfinished.  Measured (A/B, tekkaman 1024^2 primary +
// shadow): -9 % kernel time vs per-lane walks (0.0565 -> 0.0514 ms, r02):
// the heavy tiles' shadow rays are coherent.  Every active lane calls it
// (any EXEC mask).  The walk's per-lane state is wave masks in SGPRs (r06):
// `live` (on the path and unfinished), `done`, and per stack entry the mask
// of the lanes on it -- a child's lanes are one v_cmp of the slab's near /
// far values ANDed with `live`, no per-lane booleans materialised and
// balloted again, no per-lane bit stack; BVH-walk frame 0.03436 -> 0.0324
// ms, the heaviest tile alone 0.02919 -> 0.02756 (r06c).  A node step has
// no branch (r06f): every slot's box tested, empty slots dropped by a scalar
// select, the pushes written unconditionally at the top with the top
// advanced by need & (need - 1) -- a lone wave issues one instruction per
// cycle slot, and a taken branch per slot cost more than the slot's work
// (with the same for the primary packet walk: BVH-walk frame 0.03133 ->
// 0.03087 ms, the heaviest tile alone 0.02644 -> 0.02526).  The stack is
// three VGPRs, entry i in lane i (v_writelane / v_readlane: no LDS round
// trip on the pop -> node-load chain): the ref and the lane mask's halves.
// A node (64 B) and a leaf's records, two at a time, arrive through one
// pointer each as wide s_loads; the leaf triangles are tested branch-free
// (mt_hit_bf: mt_hit's operations, one predicate).
// Packet leaves load this many records before testing any (A/B,
// profiles/r02/ab_packet_leaf_hoist.json: 1 0.0450 ms, 2 0.0426, 4 0.0436)
constexpr uint32_t kLeafHoist = 2;
// v_writelane_b32: lane `lane` of v := val (wave-uniform val and lane; EXEC
// is ignored, so it works under any mask)
__device__ __forceinline__ int32_t vwritelane(int32_t v, int32_t val, int32_t lane) {
  const int32_t x = __builtin_amdgcn_readfirstlane(val), l = __builtin_amdgcn_readfirstlane(lane);
  // lane select in M0 (one constant-bus read per VALU op on gfx9; the
  // compiler loads M0 for the operand and knows it is read)
  asm("v_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(x), "{m0}"(l));
  return v;
}
__device__ __forceinline__ float4 u4f(const uint4 u) {
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                     __uint_as_float(u.w));
}
__device__ __forceinline__ bool occluded_packet(const Scene& S, const Ray& r, bool act, int32_t skip,
                                                float tmax, Counters& cnt) {
  const uint64_t act_m = __ballot(act);
  if (S.num_nodes4 == 0 || act_m == 0) return false;
  uint64_t done_m = 0, live_m = act_m;  // live: on the current node's path and unfinished
  int32_t vstk = 0, vmlo = 0, vmhi = 0;  // stack entry i in lane i: ref, lanes on it (lo, hi)
  int sp = 0;
  int32_t ref = 0;
#ifdef RT_INSTRUMENT
  const uint32_t lane = lane_id();
#endif
  for (;;) {
    if (ref >= 0) {
      RT_CNT(cnt.visits += (uint32_t)(live_m >> lane) & 1u;)
      RT_WAVE_ITER(9);
      const uint32_t no = S.nodes4 + 128u * S.num_nodes4 + 64u * (uint32_t)ref;
      uint4 nw[4];
      RT_LD_BEGIN();
      S.A.sld_u4n<4>(no, nw);  // one s_load_dwordx16
      RT_LD_END(1);
      const uint4 px = nw[0], py = nw[1], pz = nw[2], cf = nw[3];
      float lx[4], hx[4], ly[4], hy[4], lz[4], hz[4];
      auto h2 = [](uint32_t u, float& a, float& b) {
        a = (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu));
        b = (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16));
      };
      h2(px.x, lx[0], lx[1]); h2(px.y, lx[2], lx[3]); h2(px.z, hx[0], hx[1]); h2(px.w, hx[2], hx[3]);
      h2(py.x, ly[0], ly[1]); h2(py.y, ly[2], ly[3]); h2(py.z, hy[0], hy[1]); h2(py.w, hy[2], hy[3]);
      h2(pz.x, lz[0], lz[1]); h2(pz.y, lz[2], lz[3]); h2(pz.z, hz[0], hz[1]); h2(pz.w, hz[2], hz[3]);
      const int32_t c[4] = {(int32_t)cf.x, (int32_t)cf.y, (int32_t)cf.z, (int32_t)cf.w};
      uint64_t hm[4];
      uint32_t need = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float tn, tf;
        slab_nf(lx[i], hx[i], ly[i], hy[i], lz[i], hz[i], r, 0.0f, tmax, &tn, &tf);
        // every slot's box tested, the empty slot's mask dropped by a scalar
        // select afterwards: the volatile use pins the mask before the
        // select, so no branch skips the VALU work of an empty slot
        // (readfirstlane: an asm result counts as divergent, the mask is not);
        // the slot's bit of `need` as integer arithmetic, min(popcount, 1):
        // a bool here becomes a lane mask and a v_cndmask + readfirstlane
        uint64_t m = mask_fle(tn, tf);
        asm volatile("" : "+s"(m));
        m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(m >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)m);
        hm[i] = m & live_m & (c[i] == RT_EMPTY_REF ? 0ull : ~0ull);
        const uint32_t pc = (uint32_t)__builtin_popcountll(hm[i]);
        need |= (pc < 1u ? pc : 1u) << i;
      }
      if (need) {
        // branch-free pushes: the slots after the first hit one, last slot
        // first, each written at the top (the lanes at and above it are
        // free) and kept by advancing the top -- no branch per slot
        // (the pushed slots: need's bits but its lowest; the stack bound as
        // a clamp -- at the bound the write lands on lane RT_MAX_STACK and
        // the top stays, which is the bounded push's skip)
        const uint32_t pm = need & (need - 1u);
#pragma unroll
        for (int i = 3; i >= 1; --i) {
          vstk = vwritelane(vstk, c[i], sp);
          vmlo = vwritelane(vmlo, (int32_t)(uint32_t)hm[i], sp);
          vmhi = vwritelane(vmhi, (int32_t)(uint32_t)(hm[i] >> 32), sp);
          const uint32_t nsp = (uint32_t)sp + ((pm >> i) & 1u);
          sp = (int)(nsp < (uint32_t)RT_MAX_STACK ? nsp : (uint32_t)RT_MAX_STACK);
        }
        // the first hit slot by scalar selects
        ref = (need & 1u) ? c[0] : (need & 2u) ? c[1] : (need & 4u) ? c[2] : c[3];
        live_m = (need & 1u) ? hm[0] : (need & 2u) ? hm[1] : (need & 4u) ? hm[2] : hm[3];
        continue;
      }
    } else {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      RT_WAVE_ITER(9);
      constexpr uint32_t H = kLeafHoist;
#pragma unroll
      for (uint32_t q0 = 0; q0 < 4; q0 += H) {
        if (q0 >= count) break;
        float4 ta[H], tb[H], tc[H];
        {
          uint4 tw[3 * H];
          RT_LD_BEGIN();
          S.A.sld_u4n<3 * H>(S.tris + 48u * (first + q0), tw);
          RT_LD_END(1);
#pragma unroll
          for (uint32_t j = 0; j < H; ++j) {
            ta[j] = u4f(tw[3 * j]); tb[j] = u4f(tw[3 * j + 1]); tc[j] = u4f(tw[3 * j + 2]);
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < H; ++j) {
          if (q0 + j < count) {
            RT_CNT(cnt.tests += (uint32_t)(live_m >> lane) & 1u;)
            float t;
            const bool hit = mt_hit_bf(r, ta[j], tb[j], tc[j], 0.0f, &t) && t < tmax &&
                             __float_as_int(ta[j].w) != skip;
            const uint64_t m = __ballot(hit) & live_m;
            done_m |= m;
            live_m &= ~m;
          }
        }
      }
      if ((act_m & ~done_m) == 0) break;
    }
    if (sp == 0) break;
    --sp;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(vmlo, sp);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(vmhi, sp);
    live_m = (((uint64_t)hi << 32) | lo) & ~done_m;
    ref = __builtin_amdgcn_readlane(vstk, sp);
  }
  return act && ((done_m >> lane_id()) & 1u);
}

// A shadow segment's any-hit over its light-space cell list (rt_common.h;
// oracle/rt.c sl_occluded): the cell of its direction from the light, then
// the cell's triangles in the list's (key, geometry index) order -- nearest
// to the light first, key = squared distance from the light to the
// triangle's bounding box (in e1.w) -- until the first occluder (t in
// (0, 1), the primary winner `skip` excluded) or the first record whose key
// exceeds the segment's squared length (x 1.001: no later record can reach
// the segment either).  Per lane: a lane's chain is its own list, not the
// wave's union of BVH paths; the records are copies in list order, two per
// load round.  Tests count per lane.
__device__ __forceinline__ uint32_t slist_cell(const Ray& s, uint32_t N) {
  const float u0 = -s.d[0], u1 = -s.d[1], u2 = -s.d[2];
  int k = 0;
  float m = fabsf(u0);
  if (fabsf(u1) > m) { k = 1; m = fabsf(u1); }
  if (fabsf(u2) > m) { k = 2; m = fabsf(u2); }
  if (!(m > 0.0f)) return 0u;
  const float uk = k == 0 ? u0 : (k == 1 ? u1 : u2);
  const float ui = k == 0 ? u1 : u0, uj = k == 2 ? u1 : u2;
  const int f = 2 * k + (uk < 0.0f ? 1 : 0);
  const float hn = (float)N * 0.5f;
  const int cx = min(max((int)floorf((ui / m + 1.0f) * hn), 0), (int)N - 1);
  const int cy = min(max((int)floorf((uj / m + 1.0f) * hn), 0), (int)N - 1);
  return ((uint32_t)f * N + (uint32_t)cy) * N + (uint32_t)cx;
}
// The scan bound: a cell's records come nearest-to-the-light first (sort
// key = squared distance from the light to the triangle's bounding box, in
// the record's e1.w; rt_setup.hip SSORT); a triangle whose key exceeds
// |light - origin|^2 (with a 0.1 % margin) has no point on the segment, nor
// has any record after it, so the scan ends there, untested.
__device__ __forceinline__ float slist_limit(const Ray& s) {
  return (s.d[0] * s.d[0] + s.d[1] * s.d[1] + s.d[2] * s.d[2]) * 1.001f;
}
__device__ __forceinline__ bool occluded_list(const Scene& S, const Ray& s, bool act, int32_t skip,
                                              Counters& cnt) {
  if (!act) return false;
  const uint32_t cell = slist_cell(s, S.slist_n);
  const uint32_t off = S.A.ld_u32(S.sidx + 8u * cell), n = S.A.ld_u32(S.sidx + 8u * cell + 4u);
  const float lim = slist_limit(s);
  uint32_t o = S.slist + 48u * off;
  for (uint32_t q = 0; q < n; q += 2, o += 96u) {
    float4 t[6];
#pragma unroll
    for (int w = 0; w < 6; ++w) t[w] = S.A.ld_f4(o + 16u * w);  // 2 records (a padding one at the end)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (q + e >= n) break;
      if (t[3 * e + 1].w > lim) return false;
      RT_CNT(++cnt.tests;)
      float th;
      if (__float_as_int(t[3 * e].w) != skip && mt_hit(s, t[3 * e], t[3 * e + 1], t[3 * e + 2], 0.0f, &th) &&
          th < 1.0f)
        return true;
    }
  }
  return false;
}

// Cooperative walks for the path tracer's 32-pixel waves (pt_kernel
// PT_COOP): the wave's upper 32 lanes hold no pixel, so lane l and its
// partner l ^ 32 trace the same ray together -- the lower lane takes a BVH4
// node's children 0-1 and a leaf's triangles 0-1, the upper lane children
// 2-3 and triangles 2-3 (node4_step's four slab tests and four triangle
// tests split two and two), a light-space list two records each per round.
// The pair exchanges values with v_permlane32_swap (no LDS); both lanes hold
// the same stack pointer, node and best hit throughout, so per ray the node
// visits, the order of the stack and the result are the per-lane walk's
// (trace_impl / occluded_list), and so are the counters (visits counted by
// the lower lane, tests by the lane that made them).  The pair is lanes 2p,
// 2p + 1: one DPP quad_perm move per exchange, fused into its consumer (r04;
// the pair l, l ^ 32 exchanged by permlane32_swap was slower).  In the
// images with the stack's slack rows (RT_PUSH_UNCOND) node4_coop exchanges
// once and sorts the four children in both lanes; the others split the
// network over the pair in three exchange rounds.  Measured and not kept
// (r04-r05): branch-free leaf tests and list rounds, the
// leaf's triangles dealt 0, 1 | 2, 3 instead of 0, 2 | 1, 3, the whole node
// loaded by both lanes, the stack's top entry in a register.
// the partner's value (lane l <-> l ^ 1)
__device__ __forceinline__ uint32_t xpart(uint32_t v, bool hi) {
  (void)hi;
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ float xpartf(float v, bool hi) {
  return __uint_as_float(xpart(__float_as_uint(v), hi));
}
// the lower lane's value in both lanes of the pair
__device__ __forceinline__ uint32_t xlow(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
}
__device__ __forceinline__ float xlowf(float v) { return __uint_as_float(xlow(__float_as_uint(v))); }

// node4_step<SCALAR, true> (closest hit) over a lane pair: the four hits in
// the same sorting network (cx(0,1) | cx(2,3) within each lane, cx(0,2) and
// cx(1,3) slot against slot across the pair, cx(1,2) the lower lane's slot 1
// against the upper's slot 0), the hit children c[1..n-1] pushed at the rows
// push_sorted gives them (the lower lane writes c[1], the upper c[2], c[3]),
// the nearest returned to both lanes.  `mem` / `sp`: the pair's stack (the
// lower lane's LDS column).
// A lane's half of a binary16 BVH4 node as loaded (6 dword + 1 dword-pair
// loads instead of all 64 B and a select per word): the planes of children
// 0-1 (lower lane) or 2-3 (upper) -- every other dword -- and the child
// refs, a pair
struct CoopHalf {
  uint32_t w[6];
  uint2 cc;
};
__device__ __forceinline__ CoopHalf coop_half_load(const Scene& S, uint32_t ref, bool hi) {
  const uint32_t no = S.nodes4 + 128u * S.num_nodes4 + 64u * ref;
  const uint32_t hb = no + (hi ? 4u : 0u);
  CoopHalf h;
#pragma unroll
  for (int i = 0; i < 6; ++i) h.w[i] = S.A.ld_u32(hb + 8u * i);
  h.cc = S.A.ld_u2(no + 48u + (hi ? 8u : 0u));
  return h;
}
template <bool SCALAR>
__device__ __forceinline__ int32_t node4_coop(const Scene& S, uint32_t ref, const Ray& r, float lim,
                                              bool hi, int32_t* mem, int& sp,
                                              const CoopHalf* pre = nullptr) {
  auto ld = [&](uint32_t o) { return SCALAR ? S.A.sld_f4(o) : S.A.ld_f4(o); };
  const uint32_t no = S.nodes4 + 128u * S.num_nodes4 + 64u * ref;
  auto h2 = [](float w, float& a, float& b) {
    const uint32_t u = __float_as_uint(w);
    a = (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu));
    b = (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16));
  };
  float lx[2], hx[2], ly[2], hy[2], lz[2], hz[2];
  int32_t c[2];
  if (!SCALAR) {
    // each lane loads only its half (or has it already: `pre`, loaded while
    // the pair tested a leaf -- trace_coop)
    const CoopHalf hh = pre ? *pre : coop_half_load(S, ref, hi);
    const auto f = [&](int i) { return __uint_as_float(hh.w[i]); };
    h2(f(0), lx[0], lx[1]); h2(f(1), hx[0], hx[1]);
    h2(f(2), ly[0], ly[1]); h2(f(3), hy[0], hy[1]);
    h2(f(4), lz[0], lz[1]); h2(f(5), hz[0], hz[1]);
    c[0] = (int32_t)hh.cc.x; c[1] = (int32_t)hh.cc.y;
  } else {
    const float4 px = ld(no), py = ld(no + 16), pz = ld(no + 32), cf = ld(no + 48);
    h2(hi ? px.y : px.x, lx[0], lx[1]); h2(hi ? px.w : px.z, hx[0], hx[1]);
    h2(hi ? py.y : py.x, ly[0], ly[1]); h2(hi ? py.w : py.z, hy[0], hy[1]);
    h2(hi ? pz.y : pz.x, lz[0], lz[1]); h2(hi ? pz.w : pz.z, hz[0], hz[1]);
    c[0] = __float_as_int(hi ? cf.z : cf.x); c[1] = __float_as_int(hi ? cf.w : cf.y);
  }
  float k[2];
  uint32_t nh = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float tn = 0.0f;
    const bool h = slab(lx[i], hx[i], ly[i], hy[i], lz[i], hz[i], r, 0.0f, lim, &tn) &
                   (c[i] != RT_EMPTY_REF);
    k[i] = h ? fminf(tn, 3.402823466e38f) : __builtin_inff();
    nh += h ? 1u : 0u;
  }
#if RT_PUSH_UNCOND
  // One exchange round: both lanes take the partner's two keys and children
  // (four independent swaps), then run the whole network of node4_step
  // locally in slot order -- the same comparisons, so the same order, ties
  // included -- and push without branches: each lane writes two rows, an
  // entry past the hit count to the slack row RT_MAX_STACK (RT_PUSH_UNCOND).
  {
    const float pk0 = xpartf(k[0], hi), pk1 = xpartf(k[1], hi);
    const int32_t pc0 = (int32_t)xpart((uint32_t)c[0], hi), pc1 = (int32_t)xpart((uint32_t)c[1], hi);
    float K[4] = {hi ? pk0 : k[0], hi ? pk1 : k[1], hi ? k[0] : pk0, hi ? k[1] : pk1};
    int32_t C[4] = {hi ? pc0 : c[0], hi ? pc1 : c[1], hi ? c[0] : pc0, hi ? c[1] : pc1};
    auto cx = [&](int a, int b) {  // node4_step's compare-exchange: swap iff K[b] < K[a]
      const bool s = K[b] < K[a];
      const float ka = K[a], kb = K[b];
      const int32_t ca = C[a], cb = C[b];
      K[a] = s ? kb : ka; K[b] = s ? ka : kb;
      C[a] = s ? cb : ca; C[b] = s ? ca : cb;
    };
    cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
    const int n = (int)(nh + xpart(nh, hi));
    if (n == 0) return RT_EMPTY_REF;
    // entry C[j] at row sp + n - 1 - j (0 < j < n, below RT_MAX_STACK): the
    // lower lane writes C[1], the upper C[2] and C[3]
    auto row = [&](int j) {
      const int rr = sp + n - 1 - j;
      return (j < n && rr < RT_MAX_STACK) ? rr : RT_MAX_STACK;
    };
    const int ra = row(hi ? 2 : 1), rb = hi ? row(3) : RT_MAX_STACK;
    mem[64 * ra] = hi ? C[2] : C[1];
    mem[64 * rb] = C[3];
    const int nt = sp + n - 1;
    sp = nt < RT_MAX_STACK ? nt : RT_MAX_STACK;
    return C[0];
  }
#endif
  {  // cx(0,1) | cx(2,3)
    const bool s = k[1] < k[0];
    const float k0 = k[0], k1 = k[1];
    const int32_t c0 = c[0], c1 = c[1];
    k[0] = s ? k1 : k0; k[1] = s ? k0 : k1;
    c[0] = s ? c1 : c0; c[1] = s ? c0 : c1;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {  // cx(0,2), cx(1,3)
    const float pk = xpartf(k[j], hi);
    const int32_t pc = (int32_t)xpart((uint32_t)c[j], hi);
    const bool s = hi ? k[j] < pk : pk < k[j];
    k[j] = s ? pk : k[j];
    c[j] = s ? pc : c[j];
  }
  {  // cx(1,2)
    const float kx = hi ? k[0] : k[1];
    const int32_t cv = hi ? c[0] : c[1];
    const float pk = xpartf(kx, hi);
    const int32_t pc = (int32_t)xpart((uint32_t)cv, hi);
    const bool s = hi ? kx < pk : pk < kx;
    if (hi) { c[0] = s ? pc : c[0]; }
    else { c[1] = s ? pc : c[1]; }
  }
  const int n = (int)(nh + xpart(nh, hi));
  if (n == 0) return RT_EMPTY_REF;
  // entry c[j] at row sp + n - 1 - j (j < n, below RT_MAX_STACK)
  const int r0 = sp + n - (hi ? 3 : 2), r1 = sp + n - 4;
  if (r0 >= sp && r0 < RT_MAX_STACK) mem[64 * r0] = hi ? c[0] : c[1];
  if (hi && r1 >= sp && r1 < RT_MAX_STACK) mem[64 * r1] = c[1];
  const int nt = sp + n - 1;
  sp = nt < RT_MAX_STACK ? nt : RT_MAX_STACK;
  return (int32_t)xlow((uint32_t)c[0]);
}

// With the slack rows (RT_PUSH_UNCOND), after a leaf round's triangle loads
// are issued the pair pops the next stack entry and, when it is a node, issues that node's loads
// too, before the triangle tests; the node's step then runs on those
// registers (its slab tests still use the best hit after the leaf).  The
// same visits in the same order: only the load latency overlaps the tests.
// A/B r05n (config 4, median kernel ms): 0.11599 vs 0.11786.  (Reading the
// stack's top before every node step, so an empty step pops without an LDS
// round trip, measured neutral: r05o 0.11613 vs 0.11603, not kept; the same
// leaf-round prefetch in the wave-packet walks of the BVH-walk image cost 44
// SGPR spills and measured slower: r05p 0.0350 vs 0.03325, not kept; so did
// a branch-free push of the packet walks' children -- every slot written,
// sp advanced by the push bit: r05s 0.03414 vs 0.03326, not kept; and two
// cursors per ray -- each lane of the pair a whole node or leaf from one
// shared stack, the pair's best merged every iteration (same frames, more
// visits): r05v 0.12505 vs 0.11556, not kept; nor the BVH4 staged in LDS
// by every pair-walking wave, the halves read from there: r05af 0.12778 vs
// 0.11769 -- the copy and the lower occupancy cost more than L1 hits save.)

// trace<false> (closest hit from 0 below +inf, binary16 BVH4) by a lane pair;
// both lanes return the hit and *t_out
__device__ __forceinline__ int32_t trace_coop(const Scene& S, const Ray& r, int32_t skip, bool tie_high,
                                              float* t_out, int32_t* mem, bool hi, Counters& cnt) {
  if (S.num_nodes == 0) return -1;
  int sp = 0;
  float bt = INFINITY;
  int32_t bpid = -1;
  RT_CNT(cnt.visits += hi ? 0u : 1u;)
  int32_t ref = node4_coop<true>(S, 0u, r, bt, hi, mem, sp);
  if (ref == RT_EMPTY_REF) return -1;
  auto pop = [&](int32_t& x) {
    if (sp == 0) return false;
    x = mem[64 * --sp];
    return true;
  };
  int32_t nref = RT_EMPTY_REF;  // the entry popped during a leaf round (RT_PUSH_UNCOND)
  bool pf = false;              // ... a node, whose loads are in `pre`
  CoopHalf pre;
  (void)nref; (void)pf; (void)pre;
  for (;;) {
    bool dry = false;
    {
      RT_CYC_BEGIN();
      while (ref >= 0) {  // while-while, as trace_impl
        RT_WAVE_ITER(9);
        RT_CNT(cnt.visits += hi ? 0u : 1u;)
        const int32_t nx = node4_coop<false>(S, (uint32_t)ref, r, bt, hi, mem, sp);
        if (nx != RT_EMPTY_REF) { ref = nx; continue; }
        if (!pop(ref)) { dry = true; break; }
      }
      RT_CYC_END(11);
    }
    if (dry) break;
    {
      RT_WAVE_ITER(9);  // this lane's two of the leaf's (up to 4) triangles (padding records past the end)
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      // the lower lane triangles 0 and 2, the upper 1 and 3: a two-triangle
      // leaf is one test per lane
      const uint32_t k0 = hi ? 1u : 0u, ks = 2u;
      const uint32_t to = S.tris + 48u * (first + k0);
      float4 ta[2], tb[2], tc[2];
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        ta[k] = S.A.ld_f4(to + 48u * ks * k);
        tb[k] = S.A.ld_f4(to + 48u * ks * k + 16);
        tc[k] = S.A.ld_f4(to + 48u * ks * k + 32);
      }
#if RT_PUSH_UNCOND
      // the next entry and, for a node, its loads -- in flight during the tests
      const bool more = sp > 0;
      nref = more ? mem[64 * (sp - 1)] : RT_EMPTY_REF;
      sp = more ? sp - 1 : sp;
      pf = more && nref >= 0;
      if (pf) pre = coop_half_load(S, (uint32_t)nref, hi);
#endif
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        if (k0 + ks * k < count) {
          const int32_t pid = __float_as_int(ta[k].w);
          RT_CNT(++cnt.tests;)
          float t;
          if (pid != skip && mt_hit(r, ta[k], tb[k], tc[k], 0.0f, &t) && closer(t, pid, bt, bpid, tie_high)) {
            bt = t;
            bpid = pid;
          }
        }
      }
      // the pair's best: closer() is a strict total order, so both lanes
      // agree and it is the four tests' sequential result
      const float pbt = xpartf(bt, hi);
      const int32_t pb = (int32_t)xpart((uint32_t)bpid, hi);
      if (pb >= 0 && closer(pbt, pb, bt, bpid, tie_high)) {
        bt = pbt;
        bpid = pb;
      }
    }
#if RT_PUSH_UNCOND
    if (nref == RT_EMPTY_REF) break;  // the stack was empty
    ref = nref;
    if (pf) {
      // the popped node's step on the registers loaded during the tests
      // (node4_coop's own step: the same visit, the same pushes)
      RT_CNT(cnt.visits += hi ? 0u : 1u;)
      const int32_t nx = node4_coop<false>(S, (uint32_t)ref, r, bt, hi, mem, sp, &pre);
      if (nx != RT_EMPTY_REF) ref = nx;
      else if (!pop(ref)) break;
    }
#else
    if (!pop(ref)) break;
#endif
  }
  if (bpid >= 0) *t_out = bt;
  return bpid;
}

// occluded_list by a lane pair: rounds of four records, the lower lane
// testing the first two, the upper the other two; the verdict is whether any
// record occludes (order-free), the tests counted are the sequential scan's
// (the upper lane's only when the lower lane's two did not occlude)
__device__ __forceinline__ bool occluded_list_coop(const Scene& S, const Ray& s, bool act, int32_t skip,
                                                   bool hi, Counters& cnt) {
  if (!act) return false;
  const uint32_t cell = slist_cell(s, S.slist_n);
  const uint32_t off = S.A.ld_u32(S.sidx + 8u * cell), n = S.A.ld_u32(S.sidx + 8u * cell + 4u);
  const uint32_t e0 = hi ? 2u : 0u;
  const float lim = slist_limit(s);
  uint32_t o = S.slist + 48u * (off + e0);
  for (uint32_t q = 0; q < n; q += 4, o += 192u) {
    bool hit = false, end = false;  // end: a record past the bound (occluded_list)
    RT_CNT(uint32_t tests = 0;)
    if (q + e0 < n) {  // 2 records (a padding one at the list's end)
      float4 t[6];
#pragma unroll
      for (int w = 0; w < 6; ++w) t[w] = S.A.ld_f4(o + 16u * w);
#pragma unroll
      for (uint32_t e = 0; e < 2; ++e) {
        if (!hit && !end && q + e0 + e < n) {
          end = t[3 * e + 1].w > lim;
          if (!end) {
            RT_CNT(++tests;)
            float th;
            hit = __float_as_int(t[3 * e].w) != skip &&
                  mt_hit(s, t[3 * e], t[3 * e + 1], t[3 * e + 2], 0.0f, &th) && th < 1.0f;
          }
        }
      }
    }
    // the records are sorted: past the lower lane's bound the upper lane's
    // are too, so the first event in list order decides
    const uint32_t ev = (hit ? 1u : 0u) | (end ? 2u : 0u), pev = xpart(ev, hi);
    RT_CNT(cnt.tests += (hi && pev != 0u) ? 0u : tests;)
    if (((ev | pev) & 1u) != 0u) return true;
    if (((ev | pev) & 2u) != 0u) return false;
  }
  return false;
}

template <bool ANY>
__device__ __forceinline__ int32_t trace(const Scene& S, const Ray& r, float tmin, float tmax,
                                         int32_t skip, bool tie_high, float* t_out,
                                         int32_t* stack, Counters& cnt) {
  return trace_impl<ANY ? 1 : 0>(S, r, tmin, tmax, skip, tie_high, t_out, stack, cnt, ANY);
}

__device__ __forceinline__ int32_t trace_mixed(const Scene& S, const Ray& r, float tmin, float tmax,
                                               int32_t skip, bool tie_high, float* t_out,
                                               int32_t* stack, Counters& cnt, bool any) {
  return trace_impl<2>(S, r, tmin, tmax, skip, tie_high, t_out, stack, cnt, any);
}

// Flat triangle list, no BVH (BASELINE config 2; the oracle's brute_trace):
// one wave's share [k0, k1) of the geometry list in ascending pid order (the
// flat image splits every ray's list across the waves of its workgroup), the
// same record in all lanes at once through the scalar cache.  Closest hit
// (ANY = false) or the first hit in list order (ANY = true: *first = its
// index, else UINT32_MAX).  Counts nothing: the caller accounts the
// algorithmic tests.
template <bool ANY>
__device__ __forceinline__ int32_t trace_flat_range(const Scene& S, const Ray& r, uint32_t k0,
                                                    uint32_t k1, float tmin, float tmax,
                                                    int32_t skip, bool tie_high, float* t_out,
                                                    uint32_t* first) {
  float bt = tmax;
  int32_t bpid = -1;
  *first = 0xffffffffu;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t o = S.geom + 48u * k;
    const float4 ta = S.A.sld_f4(o), tb = S.A.sld_f4(o + 16), tc = S.A.sld_f4(o + 32);
    const int32_t pid = __float_as_int(ta.w);
    if (pid == skip) continue;
    float t;
    if (mt_hit(r, ta, tb, tc, tmin, &t)) {
      if (ANY) {
        if (t < tmax) { *t_out = t; *first = k; return pid; }
      } else if (closer(t, pid, bt, bpid, tie_high)) {
        bt = t;
        bpid = pid;
      }
    }
  }
  *t_out = bt;
  return bpid;
}

// shade primitive `pid` at (x, y) from per-lane (vector) record loads
__device__ __forceinline__ uint32_t shade_lane(const Scene& S, int32_t pid, uint32_t x,
                                               uint32_t y, Counters& cnt) {
  gfx::Prim p;
  gfx::load_prim(S.A, S.prims + 128u * (uint32_t)pid, p);
  const gfx::DcState s = gfx::load_dcstate(S.A, S.dcs + 64u * p.dc());
#ifdef RT_INSTRUMENT
  ++cnt.shaded;
  if (s.flags & RT_DC_TEX) cnt.texel_bytes += (s.filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * s.stride;
#endif
  return gfx::shade(S.A, p, s, x, y);
}

// Shade every lane with spid >= 0 from per-lane record loads (wave-uniform
// records through the scalar cache for the wave's most common primitives
// measured neutral)
// A wave whose shaded pixels all show one primitive (a background wave on
// one screen-layer triangle) loads the primitive and drawcall records once
// through the scalar cache (s_load into SGPRs: two dependent scalar round
// trips) instead of per lane (11 dependent 16-B vector loads of the same 192
// bytes in every lane); other waves per lane.  Same records, same
// arithmetic.  Config 3 A/B (r03r, with the counter gate of vx_spawn.h):
// 0.02256 -> 0.01982 ms.
__device__ __forceinline__ uint32_t shade_wave(const Scene& S, int32_t spid, uint32_t x,
                                               uint32_t y, uint32_t color, Counters& cnt) {
  const uint64_t need = __ballot(spid >= 0);
  if (need == 0) return color;
  const bool mine = (need & (1ull << lane_id())) != 0;
  const int32_t p0 = __builtin_amdgcn_readlane(spid, (int)__builtin_ctzll(need));
  if (__ballot(mine && spid == p0) == need) {
    if (mine) {
      gfx::Prim p;
      gfx::load_prim<true>(S.A, S.prims + 128u * (uint32_t)p0, p);
      const gfx::DcState s = gfx::load_dcstate<true>(S.A, S.dcs + 64u * p.dc());
#ifdef RT_INSTRUMENT
      ++cnt.shaded;
      if (s.flags & RT_DC_TEX) cnt.texel_bytes += (s.filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * s.stride;
#endif
      color = gfx::shade(S.A, p, s, x, y);
    }
    return color;
  }
  // mixed primitives: each lane's primitive record per lane (vector loads,
  // all in flight together), the drawcall state per distinct drawcall of the
  // wave through the scalar cache (usually one or two: the model and the
  // backdrop), so the sampler's format / filter / wrap switches are
  // wave-uniform branches instead of exec-mask branches per lane
  gfx::Prim p;
  gfx::load_prim(S.A, S.prims + 128u * (uint32_t)(mine ? spid : p0), p);
  const uint32_t dc = p.dc();
  uint64_t pend = need;
  while (pend != 0) {
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)dc, (int)__builtin_ctzll(pend));
    const bool take = mine && dc == d0;
    pend &= ~__ballot(take);
    const gfx::DcState s = gfx::load_dcstate<true>(S.A, S.dcs + 64u * d0);
    if (take) {
#ifdef RT_INSTRUMENT
      ++cnt.shaded;
      if (s.flags & RT_DC_TEX) cnt.texel_bytes += (s.filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * s.stride;
#endif
      color = gfx::shade(S.A, p, s, x, y);
    }
  }
  return color;
}

// ---- primary visibility (rt_common.h "primary visibility"; app/vis.cpp) ----
// A primary ray through pixel (px, py) is resolved the way draw3d's raster
// resolves that pixel: coverage by the Q15.16 edge functions inside the
// primitive's binned tiles, closest hit = the depth test's winner on the
// 24-bit depth word.  Exact, so the RT frame equals the reference's raster
// frame; the BVH only narrows the candidates (2D point-in-rect per child,
// culled by the children's depth lower bounds).
__device__ __forceinline__ bool rect_in(uint32_t r, uint32_t p) {
  return p >= (r & 0xffffu) && p <= (r >> 16);
}
// pixel p = x | y << 16 inside the rectangle with corners lo, hi (packed the
// same way, lo <= hi per half): two packed 16-bit clamps (v_pk_max_u16,
// v_pk_min_u16) and one compare for both axes
typedef uint16_t rt_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t rect2_clamp(uint32_t lo, uint32_t hi, uint32_t p) {
  const rt_u16x2 v = __builtin_bit_cast(rt_u16x2, p);
  const rt_u16x2 c = __builtin_elementwise_min(
      __builtin_elementwise_max(v, __builtin_bit_cast(rt_u16x2, lo)), __builtin_bit_cast(rt_u16x2, hi));
  return __builtin_bit_cast(uint32_t, c);
}
__device__ __forceinline__ bool rect2_in(uint32_t lo, uint32_t hi, uint32_t p) {
  return rect2_clamp(lo, hi, p) == p;
}

// the depth word draw3d's shader computes from the three edge values
// (GRADIENTS + INTERPOLATE z, draw3d/kernel.cpp:37-59; gfx::shade_edges)
__device__ __forceinline__ uint32_t vis_depth(int32_t E0, int32_t E1, int32_t E2, const int32_t z[3]) {
  const float f0 = gfx::fx_to_float(E0, 24), f1 = gfx::fx_to_float(E1, 24),
              f2 = gfx::fx_to_float(E2, 24);
  const float r = 1.0f / (f0 + f1 + f2);
  const int32_t dx = gfx::fx_from_float_dev(r * f0, 24), dy = gfx::fx_from_float_dev(r * f1, 24);
  return (uint32_t)gfx::interp(z, dx, dy) & VX_OM_DEPTH_MASK;
}

// DepthTencil::test against the winner so far (graphics.cpp:564-596; per-tile
// ascending pid order gpu_sw.h:46-60): LESS keeps the first drawn of equal
// words and never beats the cleared word 0xffffff; LEQUAL takes the last
// drawn.  (bz, bpid) start at (0xffffff, -1), the cleared depth buffer.
__device__ __forceinline__ bool vis_better(uint32_t z, int32_t pid, uint32_t bz, int32_t bpid,
                                           bool tie_high) {
  return z < bz || (z == bz && (tie_high ? pid > bpid : (bpid >= 0 && pid < bpid)));
}

// one rt_vtri_t candidate whose rectangle test is already known (`inr`);
// updates (bz, bpid)
__device__ __forceinline__ void vis_test_in(const uint4& A, const uint4& B, const uint4& C,
                                            const uint4& D, bool inr, uint32_t px, uint32_t py,
                                            bool tie_high, uint32_t& bz, int32_t& bpid) {
  if (!inr || D.w > bz) return;
  const int32_t e0[3] = {(int32_t)A.x, (int32_t)A.y, (int32_t)A.z};
  const int32_t e1[3] = {(int32_t)A.w, (int32_t)B.x, (int32_t)B.y};
  const int32_t e2[3] = {(int32_t)B.z, (int32_t)B.w, (int32_t)C.x};
  const int32_t E0 = gfx::edge_eval(e0, px, py), E1 = gfx::edge_eval(e1, px, py),
                E2 = gfx::edge_eval(e2, px, py);
  if (E0 < 0 || E1 < 0 || E2 < 0) return;
  const int32_t z3[3] = {(int32_t)D.x, (int32_t)D.y, (int32_t)D.z};
  const uint32_t z = vis_depth(E0, E1, E2, z3);
  const int32_t pid = (int32_t)C.w;
  if (vis_better(z, pid, bz, bpid, tie_high)) {
    bz = z;
    bpid = pid;
  }
}
// (vis_test_in without branches -- every lane evaluating the edges and the
// depth word, one predicate deciding, so the compiler keeps the record's
// loads in one scalar round trip instead of sinking them into the branches
// -- measured slower: r06d, config 3 0.01646 vs 0.01621 ms, BVH walk
// 0.03385 vs 0.03181; the division for every lane costs more)
__device__ __forceinline__ void vis_test(const uint4& A, const uint4& B, const uint4& C, const uint4& D,
                                         uint32_t px, uint32_t py, bool tie_high, uint32_t& bz,
                                         int32_t& bpid) {
  vis_test_in(A, B, C, D, rect_in(C.y, px) && rect_in(C.z, py), px, py, tie_high, bz, bpid);
}

// The primary ray's hit: the draw3d depth-test winner among the geometry
// primitives covering (px, py), or -1.  The wave's pixels walk the tree
// together (oracle/rt.c vis_trace_packet).
// A child is entered when, for some lane, the pixel lies in the child's
// rectangle and the child's depth bound can still beat that lane's best
// (ballot); the entered children are taken in slot order (= ascending
// bound, vis.cpp SortSlots: no sorting network per step) and the others
// pushed farthest first on the wave's VGPR stack.  Node
// and leaf records are wave-uniform: scalar loads, one per record for the
// wave instead of 64 lanes' gathers.  Each lane runs the exact coverage and
// depth test on every leaf primitive of the walk, so the result is the
// per-lane walk's (order independent); node visits and leaf tests count once
// per wave (oracle/rt.c vis_trace_packet restates the walk, counters
// included).  Every lane of the wave must call it; `act` = this lane holds
// a pixel.
__device__ __forceinline__ int32_t trace_primary_packet(const Scene& S, uint32_t px, uint32_t py,
                                                        bool act, bool tie_high, Counters& cnt) {
  // a wave with no pixel in the image (edge tiles overhang it) walks nothing
  // (oracle/rt.c vis_tile_row skips it too)
  if (S.num_vnodes == 0 || __ballot(act) == 0) return -1;
  if (!act) px = 0xffffffffu;  // in no rectangle
  const uint32_t pp = px > 0xffffu ? 0xffffffffu : px | (py << 16);  // packed pixel (rect2_in)
  int32_t vstk = 0;  // stack entry i in lane i of this VGPR
  const bool l0 = lane_id() == 0;
  uint32_t bz = VX_OM_DEPTH_MASK;
  int32_t bpid = -1;
  int sp = 0;  // wave-uniform
  int32_t ref = 0;
  for (;;) {
    if (ref >= 0) {
      RT_CNT(cnt.visits += l0;)
      RT_WAVE_ITER(7);
      const uint32_t o = S.vnodes + 64u * (uint32_t)ref;
      uint4 vw[4];
      RT_LD_BEGIN();
      S.A.sld_u4n<4>(o, vw);  // one s_load_dwordx16
      RT_LD_END(0);
      const uint4 rl = vw[0], rh = vw[1], zm = vw[2], cf = vw[3];
      const uint32_t alo[4] = {rl.x, rl.y, rl.z, rl.w}, ahi[4] = {rh.x, rh.y, rh.z, rh.w};
      const uint32_t azm[4] = {zm.x, zm.y, zm.z, zm.w};
      int32_t c[4] = {(int32_t)cf.x, (int32_t)cf.y, (int32_t)cf.z, (int32_t)cf.w};
      uint32_t need = 0u;  // wave-uniform: children some lane must enter
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // lanes whose pixel is in the child's rectangle and whose best depth
        // word can still lose to the child's bound: two lane masks, one AND
        const rt_u16x2 cl = __builtin_elementwise_min(
            __builtin_elementwise_max(__builtin_bit_cast(rt_u16x2, pp), __builtin_bit_cast(rt_u16x2, alo[i])),
            __builtin_bit_cast(rt_u16x2, ahi[i]));
        // (no short-circuit: a branch per child made the compiler sink the
        // node's loads into three dependent scalar round trips; BVH walk
        // 0.03181 -> 0.03132 ms, r06d)
        const uint64_t m = mask_ueq(__builtin_bit_cast(uint32_t, cl), pp) & mask_ule(azm[i], bz);
        need |= ((m != 0) & (c[i] != RT_EMPTY_REF)) ? 1u << i : 0u;
      }
      if (need != 0u) {
        // branch-free pushes as in occluded_packet: every slot after the
        // first needed one written at the top, the top advanced by its bit of
        // need & (need - 1), clamped at the bound (the bounded push's skip)
        const uint32_t pm = need & (need - 1u);
#pragma unroll
        for (int i = 3; i >= 1; --i) {
          vstk = vwritelane(vstk, c[i], sp);
          const uint32_t nsp = (uint32_t)sp + ((pm >> i) & 1u);
          sp = (int)(nsp < (uint32_t)RT_MAX_STACK ? nsp : (uint32_t)RT_MAX_STACK);
        }
        ref = (need & 1u) ? c[0] : (need & 2u) ? c[1] : (need & 4u) ? c[2] : c[3];
        continue;
      }
    } else {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      RT_WAVE_ITER(8);
      // kLeafHoist slots' records in flight at once (the vtris array
      // carries 3 padding records), then their tests: fewer scalar-load
      // round trips on the walk's dependent chain
      constexpr uint32_t H = kLeafHoist;
#pragma unroll
      for (uint32_t k0 = 0; k0 < 4; k0 += H) {
        if (k0 >= count) break;
        uint4 A[H], B[H], C[H], D[H];
        {  // the H consecutive records from one address (wide s_loads)
          uint4 tw[4 * H];
          RT_LD_BEGIN();
          S.A.sld_u4n<4 * H>(S.vtris + 64u * (first + k0), tw);
          RT_LD_END(0);
#pragma unroll
          for (uint32_t j = 0; j < H; ++j) {
            A[j] = tw[4 * j]; B[j] = tw[4 * j + 1]; C[j] = tw[4 * j + 2]; D[j] = tw[4 * j + 3];
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < H; ++j) {
          if (k0 + j < count) {
            RT_CNT(cnt.tests += l0;)
            vis_test(A[j], B[j], C[j], D[j], px, py, tie_high, bz, bpid);
          }
        }
      }
    }
    if (sp == 0) break;
    --sp;
    ref = __builtin_amdgcn_readlane(vstk, sp);
  }
  return bpid;
}

// The wave's 8x8 block resolved from its candidate list (rt_common.h
// rt_bentry_t; oracle/rt.c vis_scan_block): entries in ascending (depth
// bound, geometry index), two per round; every lane runs the exact test on
// both records; the scan stops once no lane can change its winner -- its
// pixel is outside the union rectangle of the remaining entries, or their
// smallest bound exceeds its best depth word.  Same winners as the tree walk
// (vis_better is a strict order).  The next round's entries are loaded with
// this round's records, so a round is one scalar-load round trip.  Tests
// count once per wave per record tested, as the packet walk's do.  Every
// lane of the wave calls it with the wave's local block `lb` (uniform);
// lanes with !act get -1.
__device__ __forceinline__ int32_t block_primary(const Scene& S, uint32_t lb, uint32_t px, uint32_t py,
                                                 bool act, bool tie_high, Counters& cnt) {
  (void)cnt;
  if (!act) px = 0xffffffffu;
  const uint32_t pp = px > 0xffffu ? 0xffffffffu : px | (py << 16);
  const uint2 oc = S.A.sld<uint2>(S.bidx + 8u * lb);
  uint32_t bz = VX_OM_DEPTH_MASK;
  int32_t bpid = -1;
  // (skipping the list load of a block no candidate reaches measured no
  // gain, r04zj: the wave's next scalar load waits on it either way)
  uint4 e[2];
  S.A.sld_u4n<2>(S.blist + 16u * oc.x, e);  // the list array carries RT_BLIST_PAD padding entries
  for (uint32_t k = 0; k < oc.y; k += 2) {
    if (__ballot(rect2_in(e[0].y, e[0].z, pp) && e[0].w <= bz) == 0) break;
    uint4 r0[4], r1[4], en[2];
    S.A.sld_u4n<4>(S.vgeom + 64u * e[0].x, r0);
    S.A.sld_u4n<4>(S.vgeom + 64u * e[1].x, r1);
    S.A.sld_u4n<2>(S.blist + 16u * (oc.x + k + 2), en);
#ifdef RT_INSTRUMENT
    cnt.tests += lane_id() == 0 ? (k + 1 < oc.y ? 2u : 1u) : 0u;  // once per wave per record
#endif
    vis_test(r0[0], r0[1], r0[2], r0[3], px, py, tie_high, bz, bpid);
    if (k + 1 < oc.y) vis_test(r1[0], r1[1], r1[2], r1[3], px, py, tie_high, bz, bpid);
    e[0] = en[0];
    e[1] = en[1];
  }
  return act ? bpid : -1;
}

// primary visibility of the wave's pixels: the block's candidate list when
// the host built lists (blist_blocks), else the packet walk of the tree
__device__ __forceinline__ int32_t trace_primary(const Scene& S, uint32_t lb, uint32_t px, uint32_t py,
                                                 bool act, bool tie_high, Counters& cnt) {
  if (!RT_BVH_WALK && S.blist_blocks) return block_primary(S, lb, px, py, act, tie_high, cnt);
  const int32_t h = trace_primary_packet(S, px, py, act, tie_high, cnt);
  return act ? h : -1;
}

// ray parameter of the primary ray's intersection with the plane of
// triangle `pid` (rt_tri_t by pid in ptris): MT's t without the coverage
// test (mt_hit's operations); the origin of the shadow ray / path.  Not
// finite or <= 0 (a plane edge-on to the ray): no secondary rays.
__device__ __forceinline__ float plane_t(const Scene& S, const Ray& r, int32_t pid) {
  const uint32_t o = S.ptris + 48u * (uint32_t)pid;
  const float4 a = S.A.ld_f4(o), b = S.A.ld_f4(o + 16), c = S.A.ld_f4(o + 32);
  const float e1[3] = {b.x, b.y, b.z}, e2[3] = {c.x, c.y, c.z};
  float pvec[3], tvec[3], qvec[3];
  cross3(pvec, r.d, e2);
  const float det = dot3(e1, pvec);
  tvec[0] = r.o[0] - a.x;
  tvec[1] = r.o[1] - a.y;
  tvec[2] = r.o[2] - a.z;
  cross3(qvec, tvec, e1);
  return dot3(e2, qvec) / det;
}
__device__ __forceinline__ bool secondary_ok(float t) { return t > 0.0f && t < INFINITY; }

// Screen layers (depth test off) for lanes with `need` (no geometry
// winner): painter order, the highest covering pid wins (layers drawn in
// order, each overwriting; draw3d/main.cpp:179 + gpu_sw.h:38-61); one
// wave-uniform rt_vtri_t per step through the scalar cache.  Returns the pid
// to shade (layer pid, or `spid` unchanged).
// `tests` (the RT_INSTRUMENT count): the layer records the wave fetched,
// counted once per wave by its first active lane -- a record is one scalar
// load for the whole wave, the rule block_primary's and the packet walks'
// record tests follow (oracle/rt.c layer_waves: max over the wave's lanes)
// (loading the first layer record at wave start, its latency under the
// primary pass, measured no gain: r04zj)
__device__ __forceinline__ int32_t resolve_layers_n(const Scene& S, uint32_t px, uint32_t py, bool need,
                                                    int32_t spid, uint32_t* tests) {
  uint64_t pend = __ballot(need);
  const uint32_t lead = lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)) ? 1u : 0u;
  for (uint32_t k = 0; pend != 0 && k < S.num_layer; ++k) {
    uint4 lw[3];
    S.A.sld_u4n<3>(S.vlayers + 64u * k, lw);  // one pointer: merged wide s_loads
    const uint4 A = lw[0], B = lw[1], C = lw[2];
    const bool mine = (pend & (1ull << lane_id())) != 0;
    *tests += lead;
    bool f = false;
    if (mine && rect_in(C.y, px) && rect_in(C.z, py)) {
      const int32_t e0[3] = {(int32_t)A.x, (int32_t)A.y, (int32_t)A.z};
      const int32_t e1[3] = {(int32_t)A.w, (int32_t)B.x, (int32_t)B.y};
      const int32_t e2[3] = {(int32_t)B.z, (int32_t)B.w, (int32_t)C.x};
      f = gfx::edge_eval(e0, px, py) >= 0 && gfx::edge_eval(e1, px, py) >= 0 &&
          gfx::edge_eval(e2, px, py) >= 0;
    }
    if (f) spid = (int32_t)C.w;
    pend &= ~__ballot(f);
  }
  return spid;
}
__device__ __forceinline__ int32_t resolve_layers(const Scene& S, uint32_t px, uint32_t py, bool need,
                                                  int32_t spid, Counters& cnt) {
  uint32_t tests = 0;
  spid = resolve_layers_n(S, px, py, need, spid, &tests);
#ifdef RT_INSTRUMENT
  cnt.layer_tests += tests;
#else
  (void)cnt;
#endif
  return spid;
}

// task -> (shard-local 32x32 tile, pixel of the tile) -> pixel
// Tasks are worked in the host's tile order (heaviest 32x32 tiles first, so
// the long waves start at once instead of trailing the frame).  A tile is
// 16 chunks of 64 tasks, one 8x8 pixel block each -- except the first
// `split_tiles` tiles of the order (the ones geometry touches), which take
// 32 chunks of 64 tasks with only lanes 0-31 live, one 8x4 half-block each:
// half as many divergent rays per wave where the per-wave union of BVH
// paths is widest, which shortens the frame's critical path.
// global tile gt -> (column, row) with no integer division: the row is
// mulhi(gt, magic), magic = rt_tiles_x_magic(tiles_x) (rt_common.h), then at
// most one correction either way (exact for every gt < 2^32 / tiles_x)
__device__ __forceinline__ void tile_xy(uint32_t gt, uint32_t tiles_x, uint32_t magic, uint32_t* tx,
                                        uint32_t* ty) {
  uint32_t q = __umulhi(gt, magic);
  int32_t r = (int32_t)(gt - q * tiles_x);
  if (r < 0) {
    --q;
    r += (int32_t)tiles_x;
  } else if (r >= (int32_t)tiles_x) {
    ++q;
    r -= (int32_t)tiles_x;
  }
  *tx = (uint32_t)r;
  *ty = q;
}
struct TaskPix {
  uint32_t lt;   // shard-local tile
  uint32_t idx;  // pixel of the tile in block order: (8x8 block) * 64 + lane of the block
  bool live;
};
// 1: the task-map fields (split, order, shard) are read from the argument
// block where they are used, through an opaque pointer, instead of living in
// SGPRs across the walks (the chunk loop keeps loop-invariant values live)
#ifndef RT_LAZY_TASK_ARGS
#define RT_LAZY_TASK_ARGS 1
#endif
struct TaskArgs {
  uint32_t split_tiles, split_log, order, shard_index, shard_count, tiles_x, quad_tiles, tiles_x_magic;
};
__device__ __forceinline__ TaskArgs task_args(const Scene& S) {
  TaskArgs t;
#if RT_LAZY_TASK_ARGS
  uint64_t p = S.argp;
  asm volatile("" : "+s"(p));  // opaque: re-issued here, not hoisted or CSE'd
  const __attribute__((address_space(4))) rt_kernel_arg_t* a =
      (const __attribute__((address_space(4))) rt_kernel_arg_t*)p;
  t.split_tiles = a->split_tiles; t.split_log = a->split_log; t.order = (uint32_t)a->order_addr;
  t.shard_index = a->shard_index; t.shard_count = a->shard_count; t.tiles_x = a->tiles_x;
  t.quad_tiles = a->quad_tiles; t.tiles_x_magic = a->tiles_x_magic;
#else
  t.split_tiles = S.split_tiles; t.split_log = S.split_log; t.order = S.order;
  t.shard_index = S.shard_index; t.shard_count = S.shard_count; t.tiles_x = S.tiles_x;
  t.quad_tiles = 0; t.tiles_x_magic = S.tiles_x_magic;
#endif
  return t;
}
// Tiers: the first quad_tiles tiles of the order at 16 pixels per wave
// (4096 tasks each), the rest of the split tiles at 2^split_log, then the
// whole-block tiles.
__device__ __forceinline__ TaskPix task_map(const Scene& S, const TaskArgs& T, uint32_t t) {
  TaskPix m;
  uint32_t pl = T.split_log;         // split tiles: 2^pl pixels per wave (pl <= 6)
  uint32_t base = 0, ns = T.split_tiles;
  if (T.quad_tiles) {
    const uint32_t hq = T.quad_tiles << 12;
    if (t < hq) {
      pl = 4u;
      ns = T.quad_tiles;
    } else {
      t -= hq;
      base = T.quad_tiles;
      ns -= T.quad_tiles;
    }
  }
  const uint32_t cl = 16u - pl;      // log2 tasks per split tile (1024 >> pl chunks of 64)
  const uint32_t hs = ns << cl;
  uint32_t pos;
  if (t < hs) {
    const uint32_t sub = 6u - pl;    // log2 chunks per 8x8 block
    const uint32_t c = (t >> 6) & ((1024u >> pl) - 1u), ln = t & 63u;
    pos = base + (t >> cl);
    m.idx = ((c >> sub) << 6) + ((c & ((1u << sub) - 1u)) << pl) + (ln & ((1u << pl) - 1u));
    m.live = ln < (1u << pl);
  } else {
    pos = base + ns + ((t - hs) >> 10);
    m.idx = t & 1023u;
    m.live = true;
  }
  m.lt = T.order ? S.A.ld_u32(T.order + 4u * pos) : pos;
  return m;
}
__device__ __forceinline__ TaskPix task_map(const Scene& S, uint32_t t) {
  return task_map(S, task_args(S), t);
}

// pixel of task t (dead lanes of split tiles: x = 0xffffffff, off-image)
// and, optionally, its local 8x8 block lt * 16 + block of the tile (the same
// for every lane of a wave: wave-uniform)
__device__ __forceinline__ void task_pixel(const Scene& S, uint32_t t, uint32_t* x, uint32_t* y,
                                           uint32_t* lb = nullptr) {
  const TaskArgs T = task_args(S);
  const TaskPix m = task_map(S, T, t);
  if (lb) *lb = (uint32_t)__builtin_amdgcn_readfirstlane((m.lt << 4) | (m.idx >> 6));
  const uint32_t blk = m.idx >> 6, ln = m.idx & 63u;
  uint32_t tx, ty;
  tile_xy(T.shard_index + m.lt * T.shard_count, T.tiles_x, T.tiles_x_magic, &tx, &ty);
  *x = m.live ? (tx << RT_TILE_LOG) + ((blk & 3u) << 3) + (ln & 7u) : 0xffffffffu;  // dead lane:
  *y = (ty << RT_TILE_LOG) + ((blk >> 2) << 3) + (ln >> 3);                          // off-image
}

// The task map of one 64-task chunk, wave-uniform (every lane of a wave runs
// the same chunk: vx_spawn deals whole chunks), all in scalar registers: the
// chunk's tier (quad / split / whole-block tiles, task_map's rule), its
// local tile (one scalar load of the work order), the tile's position
// (tile_xy) and its 8x8 block; a lane's pixel is then a few VALU operations
// (chunk_pixel).  Equals task_map / task_pixel for every task of the chunk.
struct ChunkMap {
  uint32_t lt, blk, part, pl, tx, ty;
};
__device__ __forceinline__ ChunkMap chunk_map(const Scene& S, const TaskArgs& T, uint32_t c) {
  ChunkMap m;
  uint32_t pl = T.split_log, base = 0, ns = T.split_tiles;
  if (T.quad_tiles) {
    const uint32_t hq = T.quad_tiles << 6;  // 4096 tasks = 64 chunks per quad tile
    if (c < hq) {
      pl = 4u;
      ns = T.quad_tiles;
    } else {
      c -= hq;
      base = T.quad_tiles;
      ns -= T.quad_tiles;
    }
  }
  const uint32_t ccl = 10u - pl;     // log2 chunks per split tile (1024 >> pl)
  const uint32_t hs = ns << ccl;
  uint32_t pos;
  if (c < hs) {
    const uint32_t sub = 6u - pl;    // log2 chunks per 8x8 block
    const uint32_t ci = c & ((1u << ccl) - 1u);
    pos = base + (c >> ccl);
    m.blk = ci >> sub;
    m.part = ci & ((1u << sub) - 1u);
    m.pl = pl;
  } else {
    pos = base + ns + ((c - hs) >> 4);
    m.blk = c & 15u;
    m.part = 0;
    m.pl = 6u;
  }
  m.lt = T.order ? S.A.sld<uint32_t>(T.order + 4u * pos) : pos;
  tile_xy(T.shard_index + m.lt * T.shard_count, T.tiles_x, T.tiles_x_magic, &m.tx, &m.ty);
  return m;
}
// lane `ln` of the chunk: its pixel (dead lanes of split chunks: x =
// 0xffffffff, off-image) and its framebuffer word (store_out)
__device__ __forceinline__ void chunk_pixel(const Scene& S, const ChunkMap& m, uint32_t ln, uint32_t* x,
                                            uint32_t* y, uint32_t* out) {
  const uint32_t ib = (m.part << m.pl) + (ln & ((1u << m.pl) - 1u));  // pixel of the 8x8 block
  const bool live = ln < (1u << m.pl);
  const uint32_t px = (m.tx << RT_TILE_LOG) + ((m.blk & 3u) << 3) + (ib & 7u);
  *x = live ? px : 0xffffffffu;
  *y = (m.ty << RT_TILE_LOG) + ((m.blk >> 2) << 3) + (ib >> 3);
  // compact shard buffers: local-tile order, each tile row-major (store_pixel)
  *out = (S.flags & RT_FLAG_COMPACT) ? (m.lt << 10) | ((*y & 31u) << 5) | (px & 31u) : *y * S.width + px;
}
__device__ __forceinline__ void store_out(const Scene& S, uint32_t out, uint32_t color) {
  S.A.st_u32(S.cbuf + 4u * out, color);
}

__device__ __forceinline__ void primary_dir(const Scene& S, uint32_t x, uint32_t y, Ray& r) {
  r.o[0] = 0.0f; r.o[1] = 0.0f; r.o[2] = 0.0f;
  r.d[0] = fmaf((float)x + 0.5f, S.sx, -1.0f);
  r.d[1] = fmaf((float)y + 0.5f, S.sy, -1.0f);
  r.d[2] = 1.0f;
}

// shadow segment from the (eye-ward nudged) hit point to the light
__device__ __forceinline__ void shadow_ray(const Scene& S, const Ray& p, float th, Ray& s) {
  const float tt = th * 0.999755859375f;  // origin pulled toward the eye by 2^-12 of t
  s.o[0] = p.d[0] * tt; s.o[1] = p.d[1] * tt; s.o[2] = p.d[2] * tt;
  s.d[0] = S.light[0] - s.o[0];
  s.d[1] = S.light[1] - s.o[1];
  s.d[2] = S.light[2] - s.o[2];
  ray_setup(s);
}

// Path tracing in two kernels (BASELINE config 4's wave64 active-ray
// compaction): the first pass (pt_primary, rt_kernel.hip built
// with RT_PATHQ) appends every pixel that starts a path to the frame's path
// queue -- one atomic per wave, the wave's paths at ballot / mbcnt slots --
// and pt_queue (pt_kernel.hip PT_MODE 2) runs the queued paths on full
// waves.  The queue fields are read from the argument block where used.
struct PathQ {
  uint32_t q, ctr, lanes, cap;
};
__device__ __forceinline__ PathQ pathq_args(const Scene& S) {
  uint64_t p = S.argp;
  asm volatile("" : "+s"(p));
  const __attribute__((address_space(4))) rt_kernel_arg_t* a =
      (const __attribute__((address_space(4))) rt_kernel_arg_t*)p;
  PathQ o;
  o.q = (uint32_t)a->pathq_addr;
  o.ctr = (uint32_t)a->pathq_ctr_addr;
  o.lanes = a->pathq_lanes ? a->pathq_lanes : 64u;
  o.cap = a->pathq_seg_cap;
  return o;
}
// every lane of the wave calls it; lanes with `want` append (task, t, pid, colour)
__device__ __forceinline__ void pathq_append(const Scene& S, bool want, uint32_t task, float t,
                                             int32_t pid, uint32_t color) {
  const uint64_t m = __ballot(want);
  if (m == 0) return;
  const PathQ Q = pathq_args(S);
  const uint32_t seg = __builtin_amdgcn_readfirstlane(task >> 6) % RT_PQ_SEGS;  // the wave's chunk
  const int first = __builtin_ctzll(m);
  uint32_t base = 0;
  if ((int)lane_id() == first)
    base = atomicAdd(vx_ptr<uint32_t>(Q.ctr + 128u * seg), (uint32_t)__popcll(m));
  base = __builtin_amdgcn_readlane(base, first);
  if (!want) return;
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  S.A.st_u4(Q.q + 16u * (seg * Q.cap + base + rank),
            make_uint4(task, __float_as_uint(t), (uint32_t)pid, color));
}

__device__ __forceinline__ uint32_t shadowed(uint32_t c) {
  return (c & 0xff000000u) | ((c >> 1) & 0x007f7f7fu);
}

__device__ __forceinline__ void store_pixel(const Scene& S, uint32_t t, uint32_t x, uint32_t y,
                                            uint32_t color) {
  // compact shard buffers stay in local-tile order whatever the work order,
  // each tile row-major (32 rows of 128 B), so the frame assembly on rank 0
  // moves whole 128-B tile rows (runtime/frame_assemble.hip)
  uint32_t idx = y * S.width + x;
  if (S.flags & RT_FLAG_COMPACT) {
    const TaskPix m = task_map(S, t);
    idx = (m.lt << 10) | ((y & 31u) << 5) | (x & 31u);
  }
  S.A.st_u32(S.cbuf + 4u * idx, color);
}


}  // namespace rtk
