// rt_kernel.hip -- the north-star hot path as a Vortex kernel program for
// gfx950: per-pixel ray generation, BVH2 traversal, Möller–Trumbore closest
// hit, screen layers, draw3d-exact shading of the hit and an any-hit shadow
// ray per geometry hit, with the shadow rays compacted into full waves
// (ballot + mbcnt into an LDS queue).
//
// Launched by libvortex-hip.so (vx_start) as `vx_main`; the body reads its
// rt_kernel_arg_t from the STARTUP_ARG DCRs and calls vx_spawn_tasks_ex()
// with one task per pixel (64 consecutive tasks = one wave = an 8x8 pixel
// block, 16 waves = one 32x32 raster tile, the reference's tile unit).
//
// Traversal: each lane walks the BVH alone (near child first) with its
// stack in LDS, stack[depth][lane] (conflict-free, no VGPR cost); a leaf's
// triangles come in as one batch of 16-B loads.  The node-visit /
// triangle-test counts of the RT_INSTRUMENT image are exactly the per-ray
// traversal work the oracle (oracle/rt.c bvh_trace) restates, the basis of
// the algorithmic byte count of SURVEY.md 8(d).  (A wave-packet form --
// scalar-cache node loads, ballot-steered shared stack -- measured 20-25 %
// slower on tekkaman and was dropped.)
//
// Scene reads are buffer loads through one arena descriptor
// (vx_arena): 32-bit offsets, no FLAT loads.  Numerics are bit-identical to
// the oracle (oracle/rt.c): every fused multiply-add is an explicit fmaf,
// everything else is compiled with -ffp-contract=off, divisions are IEEE.
//
#include <hip/hip_runtime.h>

#include "gfx_device.h"
#include "rt_common.h"
#include "vx_spawn.h"

#ifndef RT_SHADOW_QUEUE
#define RT_SHADOW_QUEUE 1
#endif
// 1: wave-uniform node / leaf records through the scalar cache (trace());
// measured 3-4 % slower than per-lane loads on tekkaman, so off by default
#ifndef RT_SCALAR
#define RT_SCALAR 0
#endif
// distinct primitives per wave shaded from SGPR records (shade_wave());
// measured neutral, off by default
#ifndef RT_SHADE_UNIFORM
#define RT_SHADE_UNIFORM 0
#endif

namespace {

constexpr int kWaves = RT_BLOCK_THREADS / 64;

struct Counters {
  uint32_t primary = 0, shadow = 0, hits = 0, occluded = 0;
#ifdef RT_INSTRUMENT
  uint32_t visits = 0, tests = 0, layer_tests = 0, shaded = 0, texel_bytes = 0;
#endif
};

// Kernel arguments in scalar registers; buffer addresses become 32-bit
// arena offsets (rt_app checks every buffer lies below 4 GiB).
struct Scene {
  vx_arena A;
  uint32_t nodes, tris, layers, prims, dcs, cbuf;
  uint32_t num_nodes, num_layer, flags, width, height;
  uint32_t shard_index, shard_count, tiles_x, clear_color;
  float sx, sy, light[3];
};

__device__ __forceinline__ Scene load_scene(const rt_kernel_arg_t* a) {
  Scene s;
  s.A = vx_arena::get();
  s.nodes = (uint32_t)a->nodes_addr;
  s.tris = (uint32_t)a->tris_addr;
  s.layers = (uint32_t)a->layers_addr;
  s.prims = (uint32_t)a->prims_addr;
  s.dcs = (uint32_t)a->dcs_addr;
  s.cbuf = (uint32_t)a->cbuf_addr;
  s.num_nodes = a->num_nodes;
  s.num_layer = a->num_layer_tris;
  s.flags = a->flags;
  s.width = a->width;
  s.height = a->height;
  s.shard_index = a->shard_index;
  s.shard_count = a->shard_count;
  s.tiles_x = a->tiles_x;
  s.clear_color = a->clear_color;
  s.sx = a->sx;
  s.sy = a->sy;
  s.light[0] = a->light[0];
  s.light[1] = a->light[1];
  s.light[2] = a->light[2];
  return s;
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

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

// closest-hit order: t, then pid by the drawcall's depth-compare tie rule
__device__ __forceinline__ bool closer(float t, int32_t pid, float bt, int32_t bpid, bool tie_high) {
  return (t < bt) || (t == bt && (tie_high ? pid > bpid : pid < bpid));
}

// Per-ray traversal with the LDS stack (oracle/rt.c bvh_trace restates it
// exactly, counters included).  Each step first checks whether every active
// lane is at the same node / leaf -- the common case for the coherent rays of
// an 8x8 pixel wave -- and then reads the record ONCE for the wave through
// the scalar cache into SGPRs (s_load) instead of 64 lanes x 16 B of
// vector-memory data return per load (the L1 -> VGPR return path, 64 B/clk
// per CU, was the busiest unit of the all-vector form).  Divergent steps use
// per-lane buffer loads.  Both forms compute identical values.
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

template <bool ANY>
__device__ __forceinline__ int32_t trace(const Scene& S, const Ray& r, float tmin, float tmax,
                                         int32_t skip, bool tie_high, float* t_out,
                                         int32_t* stack, Counters& cnt) {
  if (S.num_nodes == 0) return -1;
  int sp = 0;
  int32_t ref = 0;
  float bt = tmax;
  int32_t bpid = -1;
  for (;;) {
    const int32_t r0 = __builtin_amdgcn_readfirstlane(ref);
    const bool uni = RT_SCALAR && __ballot(ref != r0) == 0;  // wave-uniform branch
    if (ref >= 0) {
#ifdef RT_INSTRUMENT
      ++cnt.visits;
#endif
      const float lim = ANY ? tmax : bt;
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
        const bool swap = st.tn1 < st.tn0;
        const int32_t near_ref = swap ? st.c1 : st.c0, far_ref = swap ? st.c0 : st.c1;
        if (sp < RT_MAX_STACK) stack[64 * sp++] = far_ref;
        ref = near_ref;
        continue;
      }
      if (st.h0) { ref = st.c0; continue; }
      if (st.h1) { ref = st.c1; continue; }
    } else {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      if (uni) {
        // one leaf for the whole wave: triangle records in SGPRs, one by one
        const uint32_t to = S.tris + 48u * first;
        bool done = false;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
          if (k < count && !done) {
            const float4 ta = S.A.sld_f4(to + 48u * k), tb = S.A.sld_f4(to + 48u * k + 16);
            const float4 tc = S.A.sld_f4(to + 48u * k + 32);
            const int32_t pid = __float_as_int(ta.w);
#ifdef RT_INSTRUMENT
            ++cnt.tests;
#endif
            float t;
            if (pid != skip && mt_hit(r, ta, tb, tc, tmin, &t)) {
              if (ANY) {
                if (t < tmax) { bt = t; bpid = pid; done = true; }
              } else if (closer(t, pid, bt, bpid, tie_high)) {
                bt = t;
                bpid = pid;
              }
            }
          }
        }
        if (ANY && done) { *t_out = bt; return bpid; }
      } else {
        // A leaf's (up to 4) triangles are fetched in one batch -- the tris
        // array carries 3 padding records.
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
#ifdef RT_INSTRUMENT
            ++cnt.tests;
#endif
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
    }
    if (sp == 0) break;
    ref = stack[64 * --sp];
  }
  if (bpid >= 0) *t_out = bt;
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

// Shade every lane with spid >= 0: the wave's most common primitives first
// from SGPR records (s_load, one record read per wave -- the background
// layer's two triangles cover most waves), then whatever is left from
// per-lane record loads.
__device__ __forceinline__ uint32_t shade_wave(const Scene& S, int32_t spid, uint32_t x,
                                               uint32_t y, uint32_t color, Counters& cnt) {
  uint64_t need = __ballot(spid >= 0);
#pragma unroll 1
  for (int it = 0; need != 0 && it < RT_SHADE_UNIFORM; ++it) {
    const int32_t u = __builtin_amdgcn_readlane(spid, (int)__builtin_ctzll(need));
    gfx::Prim p;
    gfx::load_prim<true>(S.A, S.prims + 128u * (uint32_t)u, p);
    const gfx::DcState s = gfx::load_dcstate<true>(S.A, S.dcs + 64u * p.dc());
    if (spid == u) {
      color = gfx::shade(S.A, p, s, x, y);
#ifdef RT_INSTRUMENT
      ++cnt.shaded;
      if (s.flags & RT_DC_TEX) cnt.texel_bytes += (s.filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * s.stride;
#endif
    }
    need &= ~__ballot(spid == u);
  }
  if (need != 0 && (need & (1ull << lane_id())) != 0) color = shade_lane(S, spid, x, y, cnt);
  return color;
}

// task -> (shard-local 32x32 tile, 8x8 block, lane) -> pixel
__device__ __forceinline__ void task_pixel(const Scene& S, uint32_t t, uint32_t* x, uint32_t* y) {
  const uint32_t lt = t >> 10, blk = (t >> 6) & 15u, ln = t & 63u;
  const uint32_t gt = S.shard_index + lt * S.shard_count;
  const uint32_t tx = gt % S.tiles_x, ty = gt / S.tiles_x;
  *x = (tx << RT_TILE_LOG) + ((blk & 3u) << 3) + (ln & 7u);
  *y = (ty << RT_TILE_LOG) + ((blk >> 2) << 3) + (ln >> 3);
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

__device__ __forceinline__ uint32_t shadowed(uint32_t c) {
  return (c & 0xff000000u) | ((c >> 1) & 0x007f7f7fu);
}

__device__ __forceinline__ void store_pixel(const Scene& S, uint32_t t, uint32_t x, uint32_t y,
                                            uint32_t color) {
  const uint32_t idx = (S.flags & RT_FLAG_COMPACT) ? t : y * S.width + x;
  S.A.st_u32(S.cbuf + 4u * idx, color);
}

// Wave-private LDS: the per-ray traversal stack (stack[depth][lane]) and the
// compaction queue of deferred shadow rays.
#define RT_QUEUE 128
struct WaveLds {
  int32_t stack[RT_MAX_STACK][64];
#if RT_SHADOW_QUEUE
  uint32_t q_task[RT_QUEUE];
  float q_t[RT_QUEUE];
  int32_t q_pid[RT_QUEUE];
  uint32_t q_color[RT_QUEUE];
  uint32_t q_count;
#endif
};

// closest / any hit for lanes with `active` (all 64 lanes call these)
__device__ __forceinline__ int32_t trace_closest(const Scene& S, const Ray& r, bool tie_high,
                                                 bool active, float* th, WaveLds& w,
                                                 Counters& cnt) {
  if (!active) return -1;
  return trace<false>(S, r, 0.0f, INFINITY, -1, tie_high, th, &w.stack[0][lane_id()], cnt);
}
__device__ __forceinline__ bool occluded(const Scene& S, const Ray& s, int32_t skip, bool tie_high,
                                         bool active, WaveLds& w, Counters& cnt) {
  float ts;
  if (!active) return false;
  return trace<true>(S, s, 0.0f, 1.0f, skip, tie_high, &ts, &w.stack[0][lane_id()], cnt) >= 0;
}

__device__ __forceinline__ void kernel_body(const vx_task_t& task, const Scene& S, WaveLds& w,
                                            Counters& cnt) {
  const uint32_t t = task.blockIdx.x;
  uint32_t x, y;
  task_pixel(S, t, &x, &y);
  const bool in = x < S.width && y < S.height;  // edge tiles overhang the image
  Ray r;
  primary_dir(S, x, y, r);
  ray_setup(r);
  cnt.primary += in;
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  float th = 0.0f;
  const int32_t hit = trace_closest(S, r, tie_high, in, &th, w, cnt);
  cnt.hits += hit >= 0;
  // screen layers where no geometry was hit: highest pid first, first
  // covering triangle wins (one wave-uniform triangle per step)
  int32_t spid = hit;
  uint64_t pend = __ballot(in && hit < 0);
#ifdef RT_ABLATE_LAYERS  // timing-only ablation (scripts/ab_variants.py)
  pend = 0;
#endif
  for (uint32_t k = 0; pend != 0 && k < S.num_layer; ++k) {
    const uint32_t lo = S.layers + 48u * k;
    const float4 ta = S.A.sld_f4(lo), tb = S.A.sld_f4(lo + 16), tc = S.A.sld_f4(lo + 32);
    const bool mine = (pend & (1ull << lane_id())) != 0;
#ifdef RT_INSTRUMENT
    cnt.layer_tests += mine;
#endif
    float tl;
    const bool f = mine && mt_hit(r, ta, tb, tc, 0.0f, &tl);
    if (f) spid = __float_as_int(ta.w);
    pend &= ~__ballot(f);
  }
#ifdef RT_ABLATE_SHADE  // timing-only ablation (scripts/ab_variants.py)
  uint32_t color = 0xff000000u | (uint32_t)spid;
#else
  uint32_t color = shade_wave(S, spid, x, y, S.clear_color, cnt);
#endif
  const bool shadow = hit >= 0 && (S.flags & RT_FLAG_SHADOWS) != 0;
#if RT_SHADOW_QUEUE
  // wave64 compaction: lanes with a pending shadow ray append it to the
  // wave's LDS queue at ballot/mbcnt-assigned slots
  const uint64_t m = __ballot(shadow);
  if (m) {
    const uint32_t base = w.q_count;
    if (shadow) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const uint32_t slot = base + rank;
      w.q_task[slot] = t;
      w.q_t[slot] = th;
      w.q_pid[slot] = hit;
      w.q_color[slot] = color;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane_id() == 0) w.q_count = base + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  if (in && !shadow) store_pixel(S, t, x, y, color);
#else
  Ray s;
  shadow_ray(S, r, th, s);
  cnt.shadow += shadow;
  if (occluded(S, s, hit, tie_high, shadow, w, cnt)) {
    ++cnt.occluded;
    color = shadowed(color);
  }
  if (in) store_pixel(S, t, x, y, color);
#endif
}

#if RT_SHADOW_QUEUE
// Called by all 64 lanes after every chunk: trace full waves of 64 shadow
// rays while the queue holds >= 64 (or whatever is left at the end).
__device__ __forceinline__ void shadow_drain(bool final, const Scene& S, WaveLds& w,
                                             Counters& cnt) {
  if (!(S.flags & RT_FLAG_SHADOWS)) return;
  const uint32_t lane = lane_id();
  uint32_t n = w.q_count;
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  while (n >= 64 || (final && n > 0)) {
    const uint32_t take = n < 64 ? n : 64;
    const uint32_t base = n - take;
    const bool active = lane < take;
    const uint32_t slot = base + lane;  // < RT_QUEUE for every lane
    const uint32_t t = w.q_task[slot];
    uint32_t x, y;
    task_pixel(S, t, &x, &y);
    Ray p, s;
    primary_dir(S, x, y, p);
    shadow_ray(S, p, w.q_t[slot], s);
    cnt.shadow += active;
    uint32_t color = w.q_color[slot];
    if (occluded(S, s, w.q_pid[slot], tie_high, active, w, cnt)) {
      ++cnt.occluded;
      color = shadowed(color);
    }
    if (active) store_pixel(S, t, x, y, color);
    n = base;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) w.q_count = n;
  __builtin_amdgcn_wave_barrier();
}
#endif

// RT statistics go to the user MPM counters (VX_CSR_MPM_USER = 0xB03 + slot),
// which the driver zeroes before every launch and vx_mpm_query() reads back.
__device__ __forceinline__ void flush(int slot, uint32_t v) { vx_mpm_add(RT_MPM_USER + slot, v); }

}  // namespace

#ifdef RT_WAVES_PER_EU
VX_MAIN_OCC(rt_kernel_arg_t, arg, RT_BLOCK_THREADS, RT_WAVES_PER_EU) {
#else
VX_MAIN(rt_kernel_arg_t, arg, RT_BLOCK_THREADS) {
#endif
  __shared__ WaveLds s_wave[kWaves];
  WaveLds& w = s_wave[threadIdx.x >> 6];
  Counters cnt;
  const Scene S = load_scene(arg);
#if RT_SHADOW_QUEUE
  if ((threadIdx.x & 63u) == 0) w.q_count = 0;
  __builtin_amdgcn_wave_barrier();
  const int rc = vx_spawn_tasks_ex(
      arg->num_tasks,
      [&](const vx_task_t& task, const Scene* s) { kernel_body(task, *s, w, cnt); },
      [&](bool final, const Scene* s) { shadow_drain(final, *s, w, cnt); }, &S);
#else
  const int rc = vx_spawn_tasks(
      arg->num_tasks,
      [&](const vx_task_t& task, const Scene* s) { kernel_body(task, *s, w, cnt); }, &S);
#endif
  flush(RT_STAT_PRIMARY, cnt.primary);
  flush(RT_STAT_SHADOW, cnt.shadow);
  flush(RT_STAT_HITS, cnt.hits);
  flush(RT_STAT_OCCLUDED, cnt.occluded);
#ifdef RT_INSTRUMENT
  flush(RT_STAT_NODE_VISITS, cnt.visits);
  flush(RT_STAT_TRI_TESTS, cnt.tests);
  flush(RT_STAT_LAYER_TESTS, cnt.layer_tests);
  flush(RT_STAT_SHADED, cnt.shaded);
  flush(RT_STAT_TEXEL_BYTES, cnt.texel_bytes);
#endif
  return rc;
}
