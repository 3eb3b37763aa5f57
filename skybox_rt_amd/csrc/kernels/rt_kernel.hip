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

__device__ __forceinline__ void kernel_body(const vx_task_t& task, const rt_kernel_arg_t* a,
                                            int32_t* stack, Counters& cnt) {
  // task -> (shard-local 32x32 tile, 8x8 block, lane) -> pixel
  const uint32_t t = task.blockIdx.x;
  const uint32_t lt = t >> 10, blk = (t >> 6) & 15u, ln = t & 63u;
  const uint32_t gt = a->shard_index + lt * a->shard_count;
  const uint32_t tx = gt % a->tiles_x, ty = gt / a->tiles_x;
  const uint32_t x = (tx << RT_TILE_LOG) + ((blk & 3u) << 3) + (ln & 7u);
  const uint32_t y = (ty << RT_TILE_LOG) + ((blk >> 2) << 3) + (ln >> 3);
  if (x >= a->width || y >= a->height) return;

  Ray r;
  r.o[0] = 0.0f; r.o[1] = 0.0f; r.o[2] = 0.0f;
  r.d[0] = fmaf((float)x + 0.5f, a->sx, -1.0f);
  r.d[1] = fmaf((float)y + 0.5f, a->sy, -1.0f);
  r.d[2] = 1.0f;
  ray_setup(r);
  ++cnt.primary;
  const bool tie_high = (a->flags & RT_FLAG_TIE_HIGH) != 0;
  float th = 0.0f;
  const int32_t hit = trace<false>(a, r, 0.0f, INFINITY, -1, tie_high, &th, stack, cnt);
  uint32_t color = a->clear_color;
  if (hit >= 0) {
    ++cnt.hits;
    color = shade_prim(a, hit, x, y, cnt);
    if (a->flags & RT_FLAG_SHADOWS) {
      // origin pulled toward the eye by 2^-12 of t; segment to the light
      const float tt = th * 0.999755859375f;
      Ray s;
      s.o[0] = r.d[0] * tt; s.o[1] = r.d[1] * tt; s.o[2] = r.d[2] * tt;
      s.d[0] = a->light[0] - s.o[0];
      s.d[1] = a->light[1] - s.o[1];
      s.d[2] = a->light[2] - s.o[2];
      ray_setup(s);
      ++cnt.shadow;
      float ts;
      if (trace<true>(a, s, 0.0f, 1.0f, hit, tie_high, &ts, stack, cnt) >= 0) {
        ++cnt.occluded;
        color = (color & 0xff000000u) | ((color >> 1) & 0x007f7f7fu);
      }
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
  if (a->flags & RT_FLAG_COMPACT)
    vx_ptr<uint32_t>(a->cbuf_addr)[t] = color;
  else
    vx_ptr<uint32_t>(a->cbuf_addr)[(uint64_t)y * a->width + x] = color;
}

// RT statistics go to the user MPM counters (VX_CSR_MPM_USER = 0xB03 + slot),
// which the driver zeroes before every launch and vx_mpm_query() reads back.
__device__ __forceinline__ void flush(int slot, uint32_t v) {
  const uint32_t s = __vx_wave_sum(v);
  if ((threadIdx.x & 63u) == 0 && s) atomicAdd(&__vx_mpm[RT_MPM_USER + slot], (unsigned long long)s);
}

}  // namespace

VX_MAIN(rt_kernel_arg_t, arg, RT_BLOCK_THREADS) {
  __shared__ int32_t s_stack[kWaves][RT_MAX_STACK][64];
  int32_t* stack = &s_stack[threadIdx.x >> 6][0][threadIdx.x & 63];
  Counters cnt;
  const int rc = vx_spawn_tasks(
      arg->num_tasks,
      [&](const vx_task_t& task, const rt_kernel_arg_t* a) { kernel_body(task, a, stack, cnt); },
      (const rt_kernel_arg_t*)arg);
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
