// pt_kernel.hip -- diffuse path tracing on the RT hot path (SURVEY.md 8(a)
// row A7, BASELINE config 4: 1024^2, 4-bounce diffuse, wave64 active-ray
// compaction).  NO REFERENCE EXISTS for this row; the estimator is the build's
// own documented choice (DESIGN.md "Path tracing"), restated op for op by the
// oracle (oracle/rt.c path_trace), against which the output is bit-exact.
//
// Per pixel: the primary ray (raster-exact, trace_primary), screen layers and
// draw3d shading exactly as in rt_kernel.hip.  A pixel whose primary ray
// hits geometry starts a path at the hit's plane intersection:
// throughput T = its shaded colour, radiance L = 0.  At every path vertex:
// one any-hit shadow ray to the point light (direct term T * max(0, cos)),
// then -- for `bounces` segments -- a cosine-weighted bounce about the
// geometric normal (PCG-hash RNG keyed by pixel, vertex and seed; disk
// rejection sampling, no transcendentals); a miss adds T * sky and ends the
// path, a hit multiplies T by the draw3d shader's colour at the hit's
// barycentrics.  The pixel gets clamp(L) (alpha of the primary colour).
//
// Two images: pt_kernel (PT_MODE 1, the default) runs each path on its own
// lane, the 32-pixel waves of geometry tiles with paired shadow / bounce
// lanes; pt_compact (PT_MODE 0) keeps a 256-thread workgroup's live paths in
// an LDS queue and after each vertex appends the survivors to the other
// queue at ballot + mbcnt slots (wave64 compaction).
#include <hip/hip_runtime.h>

#ifndef PT_MODE
#define PT_MODE 1
#endif
#if PT_MODE == 0
#define PT_BLOCK 256
#else
#define PT_BLOCK 64
#endif
#define VX_BLOCK_THREADS PT_BLOCK  // vx_spawn.h: the workgroup size as a constant
#include "rt_trace.h"

// PT_MODE 1 (default image pt_kernel): every lane runs its own path to the
// end in registers (one-wave workgroups, no queue): divergent, but waves
// never wait on each other and the oversubscribed grid keeps the CUs fed.
// PT_MODE 0 (image pt_compact): block-level wave64 compaction of live paths
// through LDS queues (256-thread workgroups, barrier-separated vertex
// phases).  Measured on tekkaman 1024^2, 4 bounces: 0.39 ms (mode 1) vs
// 0.47 ms (mode 0) -- the time is the per-vertex latency chain of the
// deepest paths (each extra bounce level adds ~0.08 ms whatever the number
// of live paths), which compaction does not shorten and its barriers
// lengthen.  Both images are parity-tested.
// PT_MODE 2 (image pt_queue, with pt_primary): the second kernel of a
// two-kernel frame -- the compacted path queue the first kernel filled, one
// path per lane on full waves (rt_trace.h pathq_append).
#ifndef PT_PAIR
#define PT_PAIR 1        // 0: no paired-vertex code (the shadow lists never pair)
#endif
#define PT_SKY 0.25f     // radiance of an escaped bounce ray (oracle ORC_PT_SKY)
#define PT_TRIES 8u      // disk rejection-sampling attempts (ORC_PT_TRIES)

namespace {

using namespace rtk;

constexpr int kWaves = PT_BLOCK / 64;

__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
  const uint32_t state = v * 747796405u + 2891336453u;
  const uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
  return (word >> 22u) ^ word;
}
__device__ __forceinline__ uint32_t pt_key(uint32_t seed, uint32_t px, uint32_t v) {
  return pcg_hash(px ^ pcg_hash(seed ^ (0x9E3779B9u * (v + 1u))));
}
__device__ __forceinline__ float pt_u11(uint32_t h) {
  return (float)(h >> 8) * 0x1p-23f - 1.0f;
}

// cosine-weighted direction about unit normal n (oracle pt_bounce_dir)
__device__ __forceinline__ void bounce_dir(const float n[3], uint32_t key, float dir[3]) {
  float x = 0.0f, y = 0.0f;
  for (uint32_t i = 0; i < PT_TRIES; ++i) {
    const float a = pt_u11(pcg_hash(key + 2u * i)), b = pt_u11(pcg_hash(key + 2u * i + 1u));
    if (fmaf(a, a, b * b) < 1.0f) { x = a; y = b; break; }
  }
  const float z = sqrtf(1.0f - fmaf(x, x, y * y));
  const float sgn = n[2] >= 0.0f ? 1.0f : -1.0f;
  const float a = -1.0f / (sgn + n[2]);
  const float b = (n[0] * n[1]) * a;
  const float t1[3] = {fmaf(sgn * (n[0] * n[0]), a, 1.0f), sgn * b, -(sgn * n[0])};
  const float t2[3] = {b, fmaf(n[1] * n[1], a, sgn), -n[1]};
#pragma unroll
  for (int k = 0; k < 3; ++k) dir[k] = fmaf(x, t1[k], fmaf(y, t2[k], z * n[k]));
}

__device__ __forceinline__ void load_tri(const Scene& S, int32_t pid, float v0[3], float e1[3],
                                         float e2[3]) {
  const uint32_t o = S.ptris + 48u * (uint32_t)pid;
  const float4 a = S.A.ld_f4(o), b = S.A.ld_f4(o + 16), c = S.A.ld_f4(o + 32);
  v0[0] = a.x; v0[1] = a.y; v0[2] = a.z;
  e1[0] = b.x; e1[1] = b.y; e1[2] = b.z;
  e2[0] = c.x; e2[1] = c.y; e2[2] = c.z;
}

// unit geometric normal facing against din (oracle pt_normal)
__device__ __forceinline__ void tri_normal(const float e1[3], const float e2[3], const float din[3],
                                           float n[3]) {
  cross3(n, e1, e2);
  const float len = sqrtf(dot3(n, n));
  n[0] = n[0] / len; n[1] = n[1] / len; n[2] = n[2] / len;
  if (dot3(n, din) > 0.0f) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
}

// MT barycentrics of vertex 1 and 2 (oracle mt_bary)
__device__ __forceinline__ void mt_bary(const float o[3], const float d[3], const float v0[3],
                                        const float e1[3], const float e2[3], float* b1,
                                        float* b2) {
  float pvec[3], tvec[3], qvec[3];
  cross3(pvec, d, e2);
  const float det = dot3(e1, pvec);
  tvec[0] = o[0] - v0[0]; tvec[1] = o[1] - v0[1]; tvec[2] = o[2] - v0[2];
  float u = dot3(tvec, pvec);
  cross3(qvec, tvec, e1);
  float v = dot3(d, qvec);
  float adet = det;
  if (det < 0.0f) { adet = -det; u = -u; v = -v; }
  *b1 = u / adet;
  *b2 = v / adet;
}

__device__ __forceinline__ uint32_t to8(float x) {
  return x >= 1.0f ? 255u : (x > 0.0f ? (uint32_t)fmaf(x, 255.0f, 0.5f) : 0u);
}

// A live path at a vertex: the ray that reached it (o, d, hit t, hit pid),
// its throughput T and radiance L so far, its pixel task and vertex index
// (implicit: the bounce loop's), the primary colour's alpha.  SoA in LDS.
struct PathQueue {
  uint32_t task[PT_BLOCK], alpha[PT_BLOCK];
  int32_t pid[PT_BLOCK];
  float t[PT_BLOCK];
  float o[3][PT_BLOCK], d[3][PT_BLOCK], T[3][PT_BLOCK], L[3][PT_BLOCK];
};

struct PtLds {
  int32_t stack[kWaves][RT_STACK_ROWS][64];
#if PT_MODE == 0
  PathQueue q[2];
  uint32_t n[2];
#endif
};

#if PT_MODE == 0
// append this lane's path (if `want`) to queue q at a ballot/mbcnt slot
__device__ __forceinline__ void enqueue(PtLds& L, int qi, bool want, uint32_t task, uint32_t alpha,
                                        int32_t pid, float t, const float o[3], const float d[3],
                                        const float T[3], const float Lr[3]) {
  const uint64_t m = __ballot(want);
  if (m == 0) return;
  uint32_t base = 0;
  if (lane_id() == (uint32_t)__builtin_ctzll(m)) base = atomicAdd(&L.n[qi], (uint32_t)__popcll(m));
  base = __builtin_amdgcn_readlane(base, (int)__builtin_ctzll(m));
  if (!want) return;
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const uint32_t s = base + rank;
  PathQueue& q = L.q[qi];
  q.task[s] = task;
  q.alpha[s] = alpha;
  q.pid[s] = pid;
  q.t[s] = t;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    q.o[k][s] = o[k];
    q.d[k][s] = d[k];
    q.T[k][s] = T[k];
    q.L[k][s] = Lr[k];
  }
}

// primary phase of one task (every thread of the block calls it)
__device__ __forceinline__ void primary(const vx_task_t& task, bool valid, const Scene& S,
                                        PtLds& L, Counters& cnt) {
  const uint32_t t = task.blockIdx.x;
  uint32_t x = 0, y = 0, lb = 0;
  if (valid) task_pixel(S, t, &x, &y, &lb);
  const bool in = valid && x < S.width && y < S.height;
  cnt.primary += in;
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  // primary visibility: the raster's winner at this pixel (trace_primary)
  const int32_t hit = trace_primary(S, lb, x, y, in, tie_high, cnt);
  cnt.hits += hit >= 0;
  const int32_t spid = resolve_layers(S, x, y, in && hit < 0, hit, cnt);
  const uint32_t color = shade_wave(S, spid, x, y, S.clear_color, cnt);
  Ray r;
  primary_dir(S, x, y, r);
  const float th = hit >= 0 ? plane_t(S, r, hit) : 0.0f;
  const bool path = hit >= 0 && secondary_ok(th);
  const float k255 = 1.0f / 255.0f;
  const float T[3] = {(float)((color >> 16) & 0xffu) * k255, (float)((color >> 8) & 0xffu) * k255,
                      (float)(color & 0xffu) * k255};
  const float Lr[3] = {0.0f, 0.0f, 0.0f};
  enqueue(L, 0, path, t, color & 0xff000000u, hit, th, r.o, r.d, T, Lr);
  if (in && !path) store_pixel(S, t, x, y, color);
}

#endif

// A path at a vertex: the ray that reached it (o, d, hit t, hit pid), its
// throughput T and radiance L so far, its pixel task, the primary alpha.
struct PathState {
  uint32_t task, alpha;
  uint32_t xy, out;  // the pixel (x | y << 16: the bounce RNG key) and its framebuffer word, set once
  int32_t pid;
  float t;
  float o[3], d[3], T[3], L[3];
};
// (the pair form carrying the vertex normal from the hit instead of loading
// the triangle again at the next vertex measured no gain, r05)

// The next vertex of a path whose bounce ray b from P hit triangle np at t:
// albedo = the draw3d shader at the hit's MT barycentrics, T *= albedo
__device__ __forceinline__ void path_hit(const Scene& S, PathState& st, const float P[3], const Ray& b,
                                         int32_t np, float nt, Counters& cnt, bool counted = true) {
  float w0[3], f1[3], f2[3], b1, b2;
  load_tri(S, np, w0, f1, f2);
  mt_bary(b.o, b.d, w0, f1, f2, &b1, &b2);
  gfx::Prim p;
  gfx::load_prim(S.A, S.prims + 128u * (uint32_t)np, p);
  const gfx::DcState dst = gfx::load_dcstate(S.A, S.dcs + 64u * p.dc());
#ifdef RT_INSTRUMENT
  if (counted) {
    ++cnt.shaded;
    if (dst.flags & RT_DC_TEX)
      cnt.texel_bytes += (dst.filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * dst.stride;
  }
#endif
  const uint32_t a = gfx::shade_weights(S.A, p, dst, gfx::fx_from_float_dev((1.0f - b1) - b2, 24),
                                        gfx::fx_from_float_dev(b1, 24));
  const float k255 = 1.0f / 255.0f;
  st.T[0] = st.T[0] * ((float)((a >> 16) & 0xffu) * k255);
  st.T[1] = st.T[1] * ((float)((a >> 8) & 0xffu) * k255);
  st.T[2] = st.T[2] * ((float)(a & 0xffu) * k255);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    st.o[k] = P[k];
    st.d[k] = b.d[k];
  }
  st.pid = np;
  st.t = nt;
}

#ifdef RT_STAMPS  // diagnostic image: per-wave cycle accumulators (scripts/wave_timeline.py)
#define PT_CYC() __builtin_amdgcn_s_memtime()
#define PT_ACC(slot, v)                                                            \
  do {                                                                             \
    if (lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)))                      \
      ((volatile uint32_t*)__vx_mpm_lds)[slot] += (uint32_t)(v);                  \
  } while (0)
#else
#define PT_CYC() 0ull
#define PT_ACC(slot, v) do {} while (0)
#endif

// One path vertex for an active lane: direct light through a shadow ray,
// then (v < bounces) the bounce; returns whether the path continues (st then
// describes the next vertex), else the pixel is final.  Every lane of the
// wave calls it; `act` masks the work.  CO 1: the lane pairs of a 32-pixel
// wave (lanes 2p and 2p + 1 hold the same path, role 1 = the upper lane)
// trace the shadow ray on its list and the bounce ray together (trace_coop,
// occluded_list_coop).  Every lane of the pair computes the rest, role 0
// counts.  (Quads of four lanes per path in 16-pixel waves measured slower,
// r04-r05, and were removed in r06.)
template <int CO>
__device__ __forceinline__ bool path_step(const Scene& S, int32_t* stack, PathState& st, uint32_t v,
                                          bool act, Counters& cnt, uint32_t role = 0u) {
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  const bool hi = role != 0u;
  const uint32_t one = hi ? 0u : 1u;  // per-path counters: the group's first lane
  float nrm[3], P[3];
  {
    float v0[3], e1[3], e2[3];
    load_tri(S, act ? st.pid : 0, v0, e1, e2);
    tri_normal(e1, e2, st.d, nrm);
  }
  const float tt = st.t * 0.999755859375f;
#pragma unroll
  for (int k = 0; k < 3; ++k) P[k] = fmaf(st.d[k], tt, st.o[k]);
  // direct light: shadow segment P -> light
  Ray s;
  s.o[0] = P[0]; s.o[1] = P[1]; s.o[2] = P[2];
  s.d[0] = S.light[0] - P[0];
  s.d[1] = S.light[1] - P[1];
  s.d[2] = S.light[2] - P[2];
  ray_setup(s);
  cnt.shadow += act ? one : 0u;
  float ts;
  const uint64_t c0 = PT_CYC();
  // the light-space lists when built (occluded_list), else the BVH
  const bool occ = CO == 1 ? occluded_list_coop(S, s, act, st.pid, hi, cnt)
                 : S.slist_on ? occluded_list(S, s, act, st.pid, cnt)
                              : act && trace<true>(S, s, 0.0f, 1.0f, st.pid, tie_high, &ts, stack, cnt) >= 0;
  cnt.occluded += occ ? one : 0u;
  const uint64_t c1 = PT_CYC();
  if (CO) {
    PT_ACC(4, c1 - c0);  // cycles in the shadow-list scan
    PT_ACC(5, 1);        // vertex steps
  }
  if (act && !occ) {
    const float cosl = dot3(nrm, s.d) / sqrtf(dot3(s.d, s.d));
    if (cosl > 0.0f) {
#pragma unroll
      for (int k = 0; k < 3; ++k) st.L[k] = fmaf(st.T[k], cosl, st.L[k]);
    }
  }
  bool alive = act && v < S.bounces;
  int32_t np = -1;
  float nt = 0.0f;
  Ray b;
  if (alive) {
    b.o[0] = P[0]; b.o[1] = P[1]; b.o[2] = P[2];
    bounce_dir(nrm, pt_key(S.seed, (st.xy >> 16) * S.width + (st.xy & 0xffffu), v), b.d);  // keyed by pixel
    ray_setup(b);
    cnt.bounce += one;
    np = CO == 1 ? trace_coop(S, b, st.pid, tie_high, &nt, stack, hi, cnt)
                 : trace<false>(S, b, 0.0f, INFINITY, st.pid, tie_high, &nt, stack, cnt);
    if (np < 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) st.L[k] = fmaf(st.T[k], PT_SKY, st.L[k]);
      alive = false;
    }
  }
  const uint64_t c2 = PT_CYC();
  if (alive) path_hit(S, st, P, b, np, nt, cnt, !hi);
  if (CO) {
    PT_ACC(2, c2 - c1);           // cycles in the bounce walk (and its setup)
    PT_ACC(6, PT_CYC() - c2);     // cycles shading the bounce hit
  }
  return alive;
}

// Paired form of path_step for a wave whose upper 32 lanes hold no pixel
// (the 32-pixel waves of geometry tiles, task_map): lane l < 32 owns a path,
// lane l + 32 traces that path's shadow ray while lane l traces its bounce
// ray -- one traversal loop for both (trace_mixed), so a vertex costs the
// longer of the two traversals instead of their sum.  Same rays, same
// arithmetic, same order of the radiance updates as path_step: the output
// and every counter are identical.  All 64 lanes call it.
// (Shadow rays as wave packets, occluded_packet, then the bounce rays per
// lane: 0.31 ms vs 0.22 ms, measured -- a path's later shadow rays are
// incoherent and the two traversals no longer overlap.)
__device__ __forceinline__ bool path_step_pair(const Scene& S, int32_t* stack, PathState& st,
                                               uint32_t v, bool act, Counters& cnt) {
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  const int32_t ln = (int32_t)lane_id();
  const bool owner = ln < 32;
  float v0[3], e1[3], e2[3], nrm[3], P[3];
  load_tri(S, act ? st.pid : 0, v0, e1, e2);
  tri_normal(e1, e2, st.d, nrm);
  const float tt = st.t * 0.999755859375f;
#pragma unroll
  for (int k = 0; k < 3; ++k) P[k] = fmaf(st.d[k], tt, st.o[k]);
  float sd[3] = {S.light[0] - P[0], S.light[1] - P[1], S.light[2] - P[2]};
  bool alive = act && v < S.bounces;
  Ray b;
  b.o[0] = P[0]; b.o[1] = P[1]; b.o[2] = P[2];
  if (alive) {
    bounce_dir(nrm, pt_key(S.seed, (st.xy >> 16) * S.width + (st.xy & 0xffffu), v), b.d);  // keyed by pixel
  } else {
    b.d[0] = 1.0f; b.d[1] = 1.0f; b.d[2] = 1.0f;
  }
  // the helper lane receives its owner's vertex and shadow direction (the
  // cross-lane reads run with all 64 lanes active: a bpermute from an
  // inactive lane returns 0)
  const int src = ln ^ 32;
  const bool h_act = __shfl((int)act, src) != 0;
  const int32_t h_pid = __shfl(st.pid, src);
  Ray r;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float ho = __shfl(P[k], src), hd = __shfl(sd[k], src);
    r.o[k] = owner ? b.o[k] : ho;
    r.d[k] = owner ? b.d[k] : hd;
  }
  ray_setup(r);
  float tr = 0.0f;
  const bool tracing = owner ? alive : h_act;
  const uint64_t c0 = PT_CYC();
  const int32_t res = tracing ? trace_mixed(S, r, 0.0f, owner ? INFINITY : 1.0f,
                                            owner ? st.pid : h_pid, tie_high, &tr, stack, cnt,
                                            !owner)
                              : -1;
  const bool h_occ = __shfl((int)(res >= 0), src) != 0;  // the helper's verdict (all lanes)
  const uint64_t c1 = PT_CYC();
  PT_ACC(4, c1 - c0);  // cycles in the paired traversal
  PT_ACC(5, 1);        // vertex steps
  const bool occ = act && h_occ;
  cnt.shadow += act;
  cnt.occluded += occ;
  if (act && !occ) {
    const float cosl = dot3(nrm, sd) / sqrtf(dot3(sd, sd));
    if (cosl > 0.0f) {
#pragma unroll
      for (int k = 0; k < 3; ++k) st.L[k] = fmaf(st.T[k], cosl, st.L[k]);
    }
  }
  const int32_t np = res;
  const float nt = tr;
  if (alive) {
    cnt.bounce += 1;
    if (np < 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) st.L[k] = fmaf(st.T[k], PT_SKY, st.L[k]);
      alive = false;
    }
  }
  if (alive) {
    float w0[3], f1[3], f2[3], b1, b2;
    load_tri(S, np, w0, f1, f2);
    mt_bary(b.o, b.d, w0, f1, f2, &b1, &b2);
    gfx::Prim p;
    gfx::load_prim(S.A, S.prims + 128u * (uint32_t)np, p);
    const gfx::DcState dst = gfx::load_dcstate(S.A, S.dcs + 64u * p.dc());
#ifdef RT_INSTRUMENT
    ++cnt.shaded;
    if (dst.flags & RT_DC_TEX)
      cnt.texel_bytes += (dst.filter == VX_TEX_FILTER_BILINEAR ? 4u : 1u) * dst.stride;
#endif
    const uint32_t a = gfx::shade_weights(S.A, p, dst, gfx::fx_from_float_dev((1.0f - b1) - b2, 24),
                                          gfx::fx_from_float_dev(b1, 24));
    const float k255 = 1.0f / 255.0f;
    st.T[0] = st.T[0] * ((float)((a >> 16) & 0xffu) * k255);
    st.T[1] = st.T[1] * ((float)((a >> 8) & 0xffu) * k255);
    st.T[2] = st.T[2] * ((float)(a & 0xffu) * k255);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      st.o[k] = P[k];
      st.d[k] = b.d[k];
    }
    st.pid = np;
    st.t = nt;
  }
  PT_ACC(6, PT_CYC() - c1);  // cycles after the traversal (shading the bounce hit)
  return alive;
}

__device__ __forceinline__ void store_path_pixel(const Scene& S, const PathState& st) {
  store_out(S, st.out, st.alpha | (to8(st.L[0]) << 16) | (to8(st.L[1]) << 8) | to8(st.L[2]));
}
// st.xy / st.out from st.task (the queued forms: a path's pixel once, not per vertex)
__device__ __forceinline__ void path_pixel(const Scene& S, PathState& st) {
  uint32_t x, y;
  task_pixel(S, st.task, &x, &y);
  st.xy = x | (y << 16);
  st.out = y * S.width + x;
  if (S.flags & RT_FLAG_COMPACT) {
    const TaskPix m = task_map(S, st.task);
    st.out = (m.lt << 10) | ((y & 31u) << 5) | (x & 31u);
  }
}

#if PT_MODE == 0
// one path vertex for queue entry i (lanes with i < n; whole waves past n skip)
__device__ __forceinline__ void vertex(const Scene& S, PtLds& L, int qi, uint32_t v, uint32_t n,
                                       Counters& cnt) {
  const uint32_t i = threadIdx.x;
  const bool act = i < n;
  const PathQueue& q = L.q[qi];
  const uint32_t j = act ? i : 0u;
  PathState st;
  st.task = q.task[j];
  path_pixel(S, st);
  st.alpha = q.alpha[j];
  st.pid = q.pid[j];
  st.t = q.t[j];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    st.o[k] = q.o[k][j];
    st.d[k] = q.d[k][j];
    st.T[k] = q.T[k][j];
    st.L[k] = q.L[k][j];
  }
  int32_t* stack = &L.stack[threadIdx.x >> 6][0][lane_id()];
  const bool alive = path_step<0>(S, stack, st, v, act, cnt);
  enqueue(L, qi ^ 1, alive, st.task, st.alpha, st.pid, st.t, st.o, st.d, st.T, st.L);
  if (act && !alive) store_path_pixel(S, st);
}

// after each block step: run the path vertices of the queued paths, bounce
// by bounce, on compacted waves
__device__ __forceinline__ void bounces(const Scene& S, PtLds& L, Counters& cnt) {
  __syncthreads();  // primary enqueues complete
  int qi = 0;
  for (uint32_t v = 0;; ++v) {
    const uint32_t n = L.n[qi];
    __syncthreads();  // every thread has read n before anyone resets it
    if (threadIdx.x == 0) L.n[qi ^ 1] = 0;
    __syncthreads();
    if (n == 0) break;
    if ((threadIdx.x & ~63u) < n) vertex(S, L, qi, v, n, cnt);  // wave-uniform skip
    __syncthreads();  // next queue complete
    qi ^= 1;
  }
  if (threadIdx.x == 0) { L.n[0] = 0; L.n[1] = 0; }
  __syncthreads();
}

#elif PT_MODE == 2

// one queued path (pt_primary appended it: task, plane t, hit pid, primary
// colour) on its own lane to the end; the other lanes of the wave hold the
// paths queued next to it
// Work item g = task / 64 takes paths [j * lanes, (j + 1) * lanes) of
// segment s = g % RT_PQ_SEGS, j = g / RT_PQ_SEGS (Q.lanes paths per wave,
// the rest of the wave idles); nseg = this lane's segment count (lane s
// holds segment s's)
__device__ __forceinline__ void queued_path(const vx_task_t& task, const Scene& S, const PathQ& Q,
                                            uint32_t nseg, int32_t* stack, Counters& cnt) {
  const uint32_t g = task.task_id >> 6, s = g % RT_PQ_SEGS, j = g / RT_PQ_SEGS;
  const uint32_t n = __builtin_amdgcn_readlane(nseg, (int)s);
  const uint32_t i = j * Q.lanes + (task.task_id & 63u);
  if ((task.task_id & 63u) >= Q.lanes || i >= n) return;
  const uint4 e = S.A.ld_u4(Q.q + 16u * (s * Q.cap + i));
  uint32_t x, y;
  task_pixel(S, e.x, &x, &y);
  Ray r;
  primary_dir(S, x, y, r);
  const uint32_t color = e.w;
  const float k255 = 1.0f / 255.0f;
  PathState st;
  st.task = e.x;
  st.xy = x | (y << 16);
  st.out = y * S.width + x;
  if (S.flags & RT_FLAG_COMPACT) {
    const TaskPix m = task_map(S, e.x);
    st.out = (m.lt << 10) | ((y & 31u) << 5) | (x & 31u);
  }
  st.alpha = color & 0xff000000u;
  st.pid = (int32_t)e.z;
  st.t = __uint_as_float(e.y);
  st.T[0] = (float)((color >> 16) & 0xffu) * k255;
  st.T[1] = (float)((color >> 8) & 0xffu) * k255;
  st.T[2] = (float)(color & 0xffu) * k255;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    st.o[k] = r.o[k];
    st.d[k] = r.d[k];
    st.L[k] = 0.0f;
  }
  for (uint32_t v = 0; path_step<0>(S, stack, st, v, true, cnt); ++v) {
  }
  store_path_pixel(S, st);
}

#else  // PT_MODE == 1

// one pixel's whole path on its own lane (no compaction)
__device__ __forceinline__ void lane_path(const vx_task_t& task, const Scene& S, int32_t* stack,
                                          Counters& cnt) {
  const uint32_t t = task.blockIdx.x;
  // the chunk's task map in scalar registers (every lane runs the same chunk)
  const ChunkMap cm = chunk_map(S, task_args(S), (uint32_t)__builtin_amdgcn_readfirstlane(t) >> 6);
  uint32_t x, y, out;
  chunk_pixel(S, cm, t & 63u, &x, &y, &out);
  const uint32_t lb = (cm.lt << 4) | cm.blk;
  const bool in = x < S.width && y < S.height;
  // the whole wave is here and its upper 32 lanes hold no pixel (a 32-pixel
  // wave of a geometry tile) -- wave-uniform: with the light-space shadow
  // lists and the binary16 BVH4, lane pairs per path (path_step<true>);
  // without the lists, paired vertices (path_step_pair: a list scan and a BVH
  // walk cannot share one loop)
  const bool split = __ballot(1) == ~0ull && (__ballot(in) >> 32) == 0;
  const bool pair = PT_PAIR && !S.slist_on && split;
  const bool coop = S.slist_on && split && (RT_ONLY_BVH4H || (S.flags & RT_FLAG_BVH4H));
  cnt.primary += in;
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  // primary visibility: the raster's winner at this pixel (trace_primary)
  const int32_t hit = trace_primary(S, lb, x, y, in, tie_high, cnt);
  cnt.hits += hit >= 0;
  const int32_t spid = resolve_layers(S, x, y, in && hit < 0, hit, cnt);
  const uint32_t color = shade_wave(S, spid, x, y, S.clear_color, cnt);
  Ray r;
  primary_dir(S, x, y, r);
  const float th = hit >= 0 ? plane_t(S, r, hit) : 0.0f;
  const bool path = hit >= 0 && secondary_ok(th);  // a path starts at the winner's plane
  if (!path && in) store_out(S, out, color);
  if (!path && !pair && !coop) return;
  const float k255 = 1.0f / 255.0f;
  PathState st;
  st.task = t;
  st.xy = x | (y << 16);
  st.out = out;
  st.alpha = color & 0xff000000u;
  st.pid = hit;
  st.t = th;
  st.T[0] = (float)((color >> 16) & 0xffu) * k255;
  st.T[1] = (float)((color >> 8) & 0xffu) * k255;
  st.T[2] = (float)(color & 0xffu) * k255;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    st.o[k] = r.o[k];
    st.d[k] = r.d[k];
    st.L[k] = 0.0f;
  }
  if (pair) {
    // every lane stays in the loop (helpers trace their owner's shadow ray)
    bool act = path;
    const bool own = act;
    for (uint32_t v = 0; __ballot(act) != 0; ++v) act = path_step_pair(S, stack, st, v, act, cnt);
    if (own) store_path_pixel(S, st);
    return;
  }
  if (coop) {
    // lanes 2p, 2p + 1 take pixel p's path (lane p); both trace it, lane 2p
    // stores it
    const bool hi = (lane_id() & 1u) != 0u;
    const int src = (int)(lane_id() >> 1);
    bool act = __shfl((int)path, src) != 0;
    const bool own = act && !hi;
    st.task = (uint32_t)__shfl((int)st.task, src);
    st.xy = (uint32_t)__shfl((int)st.xy, src);
    st.out = (uint32_t)__shfl((int)st.out, src);
    st.alpha = (uint32_t)__shfl((int)st.alpha, src);
    st.pid = __shfl(st.pid, src);
    st.t = __shfl(st.t, src);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      st.o[k] = __shfl(st.o[k], src);
      st.d[k] = __shfl(st.d[k], src);
      st.T[k] = __shfl(st.T[k], src);
    }
    int32_t* pstack = hi ? stack - 1 : stack;  // the pair's stack: lane 2p's column
    for (uint32_t v = 0; act; ++v) act = path_step<1>(S, pstack, st, v, act, cnt, hi ? 1u : 0u);
    if (own) store_path_pixel(S, st);
    return;
  }
  for (uint32_t v = 0; path_step<0>(S, stack, st, v, true, cnt); ++v) {
  }
  store_path_pixel(S, st);
}
#endif

__device__ __forceinline__ void flush(int slot, uint32_t v) { vx_mpm_add(RT_MPM_USER + slot, v); }

}  // namespace

// grid for the driver: 128 64-thread blocks per CU (32768), one 64-task chunk
// per wave for the split heavy tiles too (r01: 96/CU, 0.2262 -> 0.2222 ms;
// r02 after the scalar argument block: 128/CU 0.1765 vs 96/CU 0.1801 ms,
// profiles/r02/ab_pt_grid.json; 64/CU is best for rt_kernel)
#if PT_MODE == 2
// pt_queue: the waves that run queued paths are all resident at once (16
// one-wave blocks per CU = 4 per SIMD at <= 128 VGPRs); a wave takes chunks
// w, w + W, ... of the queue
#define PT_GRID_PER_CU 16
__device__ __attribute__((used)) uint32_t __vx_grid_per_cu = PT_GRID_PER_CU;
#elif PT_BLOCK == 64
#define PT_GRID_PER_CU 128
__device__ __attribute__((used)) uint32_t __vx_grid_per_cu = PT_GRID_PER_CU;
#endif

VX_MAIN(rt_kernel_arg_t, arg, PT_BLOCK) {
  __shared__ PtLds s_pt;
#ifdef RT_STAMPS  // diagnostic image: per-wave start/end timestamps (scripts/wave_timeline.py)
  const uint64_t t_stamp0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t t_cyc0 = __builtin_amdgcn_s_memtime();
#endif
  Counters cnt;
  Scene S = load_scene(arg, vx_launch_words);
#if PT_MODE == 0
  if (threadIdx.x == 0) { s_pt.n[0] = 0; s_pt.n[1] = 0; }
  __syncthreads();
  const int rc = vx_spawn_tasks_block(
      S.num_tasks,
      [&](const vx_task_t& task, bool valid, const Scene* s) { primary(task, valid, *s, s_pt, cnt); },
      [&](uint32_t, const Scene* s) { bounces(*s, s_pt, cnt); }, &S);
#elif PT_MODE == 2
  int32_t* stack = &s_pt.stack[threadIdx.x >> 6][0][lane_id()];
  const PathQ Q = pathq_args(S);
  // the paths the first kernel queued (a vector load: written by the
  // previous launch, after this launch's cache invalidation)
  // every segment's count, lane s holding segment s's (RT_PQ_SEGS = 64), and
  // the most waves of Q.lanes paths any segment needs
  static_assert(RT_PQ_SEGS == 64, "one segment per lane");
  const uint32_t nseg = S.A.ld_u32(Q.ctr + 128u * lane_id());
  uint32_t jmax = (nseg + Q.lanes - 1) / Q.lanes;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) jmax = max(jmax, (uint32_t)__shfl_xor((int)jmax, off, 64));
  const int rc = vx_spawn_tasks(
      RT_PQ_SEGS * jmax * VX_CHUNK,
      [&](const vx_task_t& task, const Scene* s) { queued_path(task, *s, Q, nseg, stack, cnt); }, &S);
  // every wave counts itself done once, on its group's counter (wave id
  // mod 64: the atomics spread over 64 lines); the wave completing a group
  // counts the group, and the one completing the last group zeroes every
  // counter for the next frame -- by then every wave has read them.  Nobody
  // waits.
  const uint32_t nwaves = gridDim.x * (PT_BLOCK >> 6);
  const uint32_t wid = blockIdx.x * (PT_BLOCK >> 6) + (threadIdx.x >> 6);
  const uint32_t grp = wid % RT_PQ_SEGS;
  const uint32_t in_grp = nwaves / RT_PQ_SEGS + (grp < nwaves % RT_PQ_SEGS ? 1u : 0u);
  const uint32_t ngrp = nwaves < RT_PQ_SEGS ? nwaves : RT_PQ_SEGS;
  uint32_t last = 0;
  if (lane_id() == 0) {
    uint32_t* ctr = vx_ptr<uint32_t>(Q.ctr);
    __threadfence();
    if (atomicAdd(&ctr[32u * (RT_PQ_SEGS + grp)], 1u) == in_grp - 1u &&
        atomicAdd(&ctr[32u * 2u * RT_PQ_SEGS], 1u) == ngrp - 1u)
      last = 1;
  }
  if (__builtin_amdgcn_readfirstlane(last)) {  // lanes zero segment / group counter l
    S.A.st_u32(Q.ctr + 128u * lane_id(), 0u);
    S.A.st_u32(Q.ctr + 128u * (RT_PQ_SEGS + lane_id()), 0u);
    if (lane_id() == 0) S.A.st_u32(Q.ctr + 128u * 2u * RT_PQ_SEGS, 0u);
  }
#else
  int32_t* stack = &s_pt.stack[threadIdx.x >> 6][0][lane_id()];
  const int rc = vx_spawn_tasks(
      S.num_tasks,
      [&](const vx_task_t& task, const Scene* s) { lane_path(task, *s, stack, cnt); }, &S);
#endif
#ifndef RT_STAMPS  // the stamp image keeps slots 4-6 for its cycle accumulators
  flush(RT_STAT_PRIMARY, cnt.primary);
  flush(RT_STAT_SHADOW, cnt.shadow);
  flush(RT_STAT_HITS, cnt.hits);
  flush(RT_STAT_OCCLUDED, cnt.occluded);
  flush(RT_STAT_BOUNCE, cnt.bounce);
#endif
#ifdef RT_STAMPS
  if (threadIdx.x == 0) {
    __vx_mpm_lds[12] = (uint32_t)t_stamp0;
    __vx_mpm_lds[13] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    __vx_mpm_lds[14] = (uint32_t)t_stamp0;
    __vx_mpm_lds[15] = 0;
    __vx_mpm_lds[10] = (uint32_t)(__builtin_amdgcn_s_memtime() - t_cyc0);  // wave cycles
  }
#endif
#ifdef RT_INSTRUMENT
  flush(RT_STAT_NODE_VISITS, cnt.visits);
  flush(RT_STAT_TRI_TESTS, cnt.tests);
  flush(RT_STAT_LAYER_TESTS, cnt.layer_tests);
  flush(RT_STAT_SHADED, cnt.shaded);
  flush(RT_STAT_TEXEL_BYTES, cnt.texel_bytes);
#endif
  return rc;
}
