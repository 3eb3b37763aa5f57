// rt_kernel.hip -- the north-star hot path as a Vortex kernel program for
// gfx950: per-pixel ray generation, BVH2 traversal with an LDS-resident
// per-wave stack, Möller–Trumbore closest hit, screen layers, draw3d-exact
// shading of the hit and an any-hit shadow ray per geometry hit.
//
// Launched by libvortex-hip.so (vx_start) as `vx_main`; the body reads its
// rt_kernel_arg_t from the STARTUP_ARG DCRs and calls vx_spawn_tasks() with
// one task per pixel (64 consecutive tasks = one wave = an 8x8 pixel block,
// 16 waves = one 32x32 raster tile, the reference's tile unit).
//
// Numerics are bit-identical to the oracle (oracle/rt.c): every fused
// multiply-add is an explicit fmaf, everything else is compiled with
// -ffp-contract=off, divisions are IEEE (correctly rounded).
// Build with -DRT_INSTRUMENT for the counting variant (node visits, triangle
// tests, shading bytes) used to derive the algorithmic byte count.
#include <hip/hip_runtime.h>

#include "gfx_device.h"
#include "rt_common.h"
#include "vx_spawn.h"

namespace {

constexpr int kWaves = RT_BLOCK_THREADS / 64;

#ifndef RT_SHADOW_QUEUE
#define RT_SHADOW_QUEUE 1
#endif

struct Counters {
  uint32_t primary = 0, shadow = 0, hits = 0, occluded = 0;
#ifdef RT_INSTRUMENT
  uint32_t visits = 0, tests = 0, layer_tests = 0, shaded = 0, texel_bytes = 0;
#endif
};

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

// Closest hit (ANY = false) or any hit excluding `skip` (ANY = true).
// Traversal order and culling are restated exactly by oracle/rt.c bvh_trace.
template <bool ANY>
__device__ __forceinline__ int32_t trace(const rt_kernel_arg_t* a, const Ray& r, float tmin,
                                         float tmax, int32_t skip, bool tie_high, float* t_out,
                                         int32_t* stack, Counters& cnt) {
  if (a->num_nodes == 0) return -1;
  const float4* nodes = vx_ptr<const float4>(a->nodes_addr);
  const float4* tris = vx_ptr<const float4>(a->tris_addr);
  int sp = 0;
  int32_t ref = 0;
  float bt = tmax;
  int32_t bpid = -1;
  for (;;) {
    if (ref >= 0) {
      const float4 n0 = nodes[4 * ref + 0], n1 = nodes[4 * ref + 1];
      const float4 n2 = nodes[4 * ref + 2], n3 = nodes[4 * ref + 3];
#ifdef RT_INSTRUMENT
      ++cnt.visits;
#endif
      const int32_t c0 = __float_as_int(n3.x), c1 = __float_as_int(n3.y);
      const float lim = ANY ? tmax : bt;
      float tn0 = 0.0f, tn1 = 0.0f;
      const bool h0 = (c0 != RT_EMPTY_REF) && slab(n0.x, n0.y, n1.x, n1.y, n2.x, n2.y, r, tmin, lim, &tn0);
      const bool h1 = (c1 != RT_EMPTY_REF) && slab(n0.z, n0.w, n1.z, n1.w, n2.z, n2.w, r, tmin, lim, &tn1);
      if (h0 && h1) {
        const bool swap = tn1 < tn0;
        const int32_t near_ref = swap ? c1 : c0, far_ref = swap ? c0 : c1;
        if (sp < RT_MAX_STACK) stack[64 * sp++] = far_ref;
        ref = near_ref;
        continue;
      }
      if (h0) { ref = c0; continue; }
      if (h1) { ref = c1; continue; }
    } else {
      const uint32_t lr = (uint32_t)ref;
      const uint32_t first = (lr >> 4) & 0x07ffffffu, count = (lr & 15u) + 1u;
      for (uint32_t k = 0; k < count; ++k) {
        const float4 ta = tris[3 * (first + k) + 0];
        const int32_t pid = __float_as_int(ta.w);
#ifdef RT_INSTRUMENT
        ++cnt.tests;
#endif
        if (pid == skip) continue;
        const float4 tb = tris[3 * (first + k) + 1], tc = tris[3 * (first + k) + 2];
        float t;
        if (!mt_hit(r, ta, tb, tc, tmin, &t)) continue;
        if (ANY) {
          if (t < tmax) { *t_out = t; return pid; }
          continue;
        }
        const bool better = (t < bt) || (t == bt && (tie_high ? pid > bpid : pid < bpid));
        if (better) { bt = t; bpid = pid; }
      }
    }
    if (sp == 0) break;
    ref = stack[64 * --sp];
  }
  if (bpid >= 0) *t_out = bt;
  return bpid;
}

__device__ __forceinline__ uint32_t shade_prim(const rt_kernel_arg_t* a, int32_t pid, uint32_t x,
                                               uint32_t y, Counters& cnt) {
  const rt_prim_t& p = vx_ptr<const rt_prim_t>(a->prims_addr)[pid];
  const rt_dcstate_t& s = vx_ptr<const rt_dcstate_t>(a->dcs_addr)[p.dc];
#ifdef RT_INSTRUMENT
  ++cnt.shaded;
  if (s.flags & RT_DC_TEX) cnt.texel_bytes += (s.tex_filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * s.tex_stride;
#endif
  return gfx::shade(p, s, x, y);
}

// task -> (shard-local 32x32 tile, 8x8 block, lane) -> pixel
__device__ __forceinline__ void task_pixel(const rt_kernel_arg_t* a, uint32_t t, uint32_t* x,
                                           uint32_t* y) {
  const uint32_t lt = t >> 10, blk = (t >> 6) & 15u, ln = t & 63u;
  const uint32_t gt = a->shard_index + lt * a->shard_count;
  const uint32_t tx = gt % a->tiles_x, ty = gt / a->tiles_x;
  *x = (tx << RT_TILE_LOG) + ((blk & 3u) << 3) + (ln & 7u);
  *y = (ty << RT_TILE_LOG) + ((blk >> 2) << 3) + (ln >> 3);
}

__device__ __forceinline__ void primary_dir(const rt_kernel_arg_t* a, uint32_t x, uint32_t y, Ray& r) {
  r.o[0] = 0.0f; r.o[1] = 0.0f; r.o[2] = 0.0f;
  r.d[0] = fmaf((float)x + 0.5f, a->sx, -1.0f);
  r.d[1] = fmaf((float)y + 0.5f, a->sy, -1.0f);
  r.d[2] = 1.0f;
}

// shadow segment from the (eye-ward nudged) hit point to the light
__device__ __forceinline__ void shadow_ray(const rt_kernel_arg_t* a, const Ray& p, float th, Ray& s) {
  const float tt = th * 0.999755859375f;  // origin pulled toward the eye by 2^-12 of t
  s.o[0] = p.d[0] * tt; s.o[1] = p.d[1] * tt; s.o[2] = p.d[2] * tt;
  s.d[0] = a->light[0] - s.o[0];
  s.d[1] = a->light[1] - s.o[1];
  s.d[2] = a->light[2] - s.o[2];
  ray_setup(s);
}

__device__ __forceinline__ uint32_t shadowed(uint32_t c) {
  return (c & 0xff000000u) | ((c >> 1) & 0x007f7f7fu);
}

__device__ __forceinline__ void store_pixel(const rt_kernel_arg_t* a, uint32_t t, uint32_t x,
                                            uint32_t y, uint32_t color) {
  if (a->flags & RT_FLAG_COMPACT)
    vx_ptr<uint32_t>(a->cbuf_addr)[t] = color;
  else
    vx_ptr<uint32_t>(a->cbuf_addr)[(uint64_t)y * a->width + x] = color;
}

// Wave-private LDS: traversal stack (stack[depth][lane]: conflict-free
// ds_read/write_b32) and the compaction queue of deferred shadow rays.
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

__device__ __forceinline__ void kernel_body(const vx_task_t& task, const rt_kernel_arg_t* a,
                                            WaveLds& w, Counters& cnt) {
  const uint32_t t = task.blockIdx.x;
  uint32_t x, y;
  task_pixel(a, t, &x, &y);
  if (x >= a->width || y >= a->height) return;
  int32_t* stack = &w.stack[0][threadIdx.x & 63u];
  Ray r;
  primary_dir(a, x, y, r);
  ray_setup(r);
  ++cnt.primary;
  const bool tie_high = (a->flags & RT_FLAG_TIE_HIGH) != 0;
  float th = 0.0f;
  const int32_t hit = trace<false>(a, r, 0.0f, INFINITY, -1, tie_high, &th, stack, cnt);
  uint32_t color = a->clear_color;
  bool defer = false;
  if (hit >= 0) {
    ++cnt.hits;
    color = shade_prim(a, hit, x, y, cnt);
    if (a->flags & RT_FLAG_SHADOWS) {
#if RT_SHADOW_QUEUE
      defer = true;
#else
      Ray s;
      shadow_ray(a, r, th, s);
      ++cnt.shadow;
      float ts;
      if (trace<true>(a, s, 0.0f, 1.0f, hit, tie_high, &ts, stack, cnt) >= 0) {
        ++cnt.occluded;
        color = shadowed(color);
      }
#endif
    }
  } else if (a->num_layer_tris) {
    // screen layers: highest pid first, first covering triangle wins
    const float4* lt4 = vx_ptr<const float4>(a->layers_addr);
    for (uint32_t k = 0; k < a->num_layer_tris; ++k) {
      const float4 ta = lt4[3 * k], tb = lt4[3 * k + 1], tc = lt4[3 * k + 2];
#ifdef RT_INSTRUMENT
      ++cnt.layer_tests;
#endif
      float tl;
      if (mt_hit(r, ta, tb, tc, 0.0f, &tl)) {
        color = shade_prim(a, __float_as_int(ta.w), x, y, cnt);
        break;
      }
    }
  }
#if RT_SHADOW_QUEUE
  // wave64 compaction: lanes with a pending shadow ray append it to the
  // wave's LDS queue at ballot/mbcnt-assigned slots
  const uint64_t m = __ballot(defer);
  if (m) {
    const uint32_t base = w.q_count;
    if (defer) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const uint32_t slot = base + rank;
      w.q_task[slot] = t;
      w.q_t[slot] = th;
      w.q_pid[slot] = hit;
      w.q_color[slot] = color;
    }
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x == (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x))
      w.q_count = base + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  if (!defer) store_pixel(a, t, x, y, color);
#else
  (void)defer;
  store_pixel(a, t, x, y, color);
#endif
}

#if RT_SHADOW_QUEUE
// Called by all 64 lanes after every chunk: trace full waves of 64 shadow
// rays while the queue holds >= 64 (or whatever is left at the end).
__device__ __forceinline__ void shadow_drain(bool final, const rt_kernel_arg_t* a, WaveLds& w,
                                             Counters& cnt) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t n = w.q_count;
  if (!(a->flags & RT_FLAG_SHADOWS)) return;
  const bool tie_high = (a->flags & RT_FLAG_TIE_HIGH) != 0;
  int32_t* stack = &w.stack[0][lane];
  while (n >= 64 || (final && n > 0)) {
    const uint32_t take = n < 64 ? n : 64;
    const uint32_t base = n - take;
    if (lane < take) {
      const uint32_t slot = base + lane;
      const uint32_t t = w.q_task[slot];
      uint32_t x, y;
      task_pixel(a, t, &x, &y);
      Ray p, s;
      primary_dir(a, x, y, p);
      shadow_ray(a, p, w.q_t[slot], s);
      ++cnt.shadow;
      uint32_t color = w.q_color[slot];
      float ts;
      if (trace<true>(a, s, 0.0f, 1.0f, w.q_pid[slot], tie_high, &ts, stack, cnt) >= 0) {
        ++cnt.occluded;
        color = shadowed(color);
      }
      store_pixel(a, t, x, y, color);
    }
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
#if RT_SHADOW_QUEUE
  if ((threadIdx.x & 63u) == 0) w.q_count = 0;
  __builtin_amdgcn_wave_barrier();
  const int rc = vx_spawn_tasks_ex(
      arg->num_tasks,
      [&](const vx_task_t& task, const rt_kernel_arg_t* a) { kernel_body(task, a, w, cnt); },
      [&](bool final, const rt_kernel_arg_t* a) { shadow_drain(final, a, w, cnt); },
      (const rt_kernel_arg_t*)arg);
#else
  const int rc = vx_spawn_tasks(
      arg->num_tasks,
      [&](const vx_task_t& task, const rt_kernel_arg_t* a) { kernel_body(task, a, w, cnt); },
      (const rt_kernel_arg_t*)arg);
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
