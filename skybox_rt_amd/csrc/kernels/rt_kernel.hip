// rt_kernel.hip -- the north-star hot path as a Vortex kernel program for
// gfx950: per-pixel primary rays resolved raster-exactly (trace_primary: the
// wave's 8x8 block scans its candidate list, or walks the tree as a packet;
// the draw3d fixed-point coverage + 24-bit depth test decide), screen layers,
// draw3d-exact shading of the winner, and an any-hit Möller–Trumbore shadow
// ray per geometry hit, with the shadow rays compacted into full waves
// (ballot + mbcnt into an LDS queue).  A full queue of shadow rays is traced
// per lane over each ray's light-space cell list (occluded_list) when the
// lists are built -- the default -- or as one packet walking the binary16
// BVH4 (occluded_packet).  Image rt_bvh (RT_BVH_WALK) keeps only the BVH
// walks: the packet walk of the tree for primary visibility and the shadow
// packet (BASELINE config 3's "full BVH traversal").
//
// Launched by libvortex-hip.so (vx_start) as its entry (VX_ENTRY); the body
// reads its rt_kernel_arg_t from the STARTUP_ARG DCRs and calls
// vx_spawn_tasks_ex() with one task per pixel (64 consecutive tasks = one
// wave = an 8x8 pixel block, 16 waves = one 32x32 raster tile, the
// reference's tile unit).  The node-visit / triangle-test counts of the
// RT_INSTRUMENT image are exactly the traversal work the oracle (oracle/rt.c)
// restates, the basis of the algorithmic byte count of SURVEY.md 8(d).
//
// Scene reads are buffer loads through one arena descriptor (vx_arena):
// 32-bit offsets, no FLAT loads.  Numerics are bit-identical to the oracle:
// every fused multiply-add is an explicit fmaf, everything else is compiled
// with -ffp-contract=off, divisions are IEEE.
//
// Images (Makefile): rt_kernel (binary16 BVH4 only), rt_bvh (the same
// without the list code paths), rt_kernel_deep (every
// BVH layout: per-lane walks with a 32-entry LDS stack for the layouts the
// packet walk does not read), rt_flat (RT_FLAT: BASELINE config 2, the flat
// geometry list, no BVH).
#include <hip/hip_runtime.h>

#ifndef RT_BLOCK_THREADS
#define RT_BLOCK_THREADS 64
#endif
#define VX_BLOCK_THREADS RT_BLOCK_THREADS  // vx_spawn.h: the workgroup size as a constant
#include "rt_trace.h"

#ifndef RT_FLAT
#define RT_FLAT 0
#endif
#ifndef RT_PATHQ
#define RT_PATHQ 0  // 1: image pt_primary, the path tracer's first kernel (rt_trace.h pathq_append)
#endif

namespace {

using namespace rtk;

constexpr int kWaves = RT_BLOCK_THREADS / 64;

// Wave-private LDS: the compaction queue of deferred shadow rays, and the
// per-lane walks' stack[depth][lane] (deep images: layouts other than the
// binary16 BVH4 walk per lane)
#define RT_QUEUE 128
// (queued shadow rays walking the BVH per lane instead of as one packet:
// BVH-walk frame 0.0411 vs 0.0333 ms, r05n -- 102 VGPRs, 4 waves per SIMD)
#define RT_LANE_STACK (!RT_FLAT && !RT_ONLY_BVH4H)
struct WaveLds {
#if RT_LANE_STACK
  int32_t stack[RT_STACK_ROWS][64];
#define RT_WSTACK(w, lane) (&(w).stack[0][(lane)])
#else
#define RT_WSTACK(w, lane) ((int32_t*)nullptr)
#endif
#if !RT_FLAT
  uint32_t q_out[RT_QUEUE];  // framebuffer word (chunk_pixel)
  uint32_t q_xy[RT_QUEUE];   // pixel x | y << 16
  float q_t[RT_QUEUE];
  int32_t q_pid[RT_QUEUE];
  uint32_t q_color[RT_QUEUE];
  uint32_t q_count;
#endif
};

// Config 2 reads the geometry list straight from L2: the block test reads
// 64 rectangle words per instruction with vector loads, so a workgroup
// starts on its chunk at once (r05j, 256^2, median ms: the rectangle words
// staged in LDS 0.0101, unstaged 0.0096, unstaged with 512-thread workgroups
// at 8 waves per SIMD 0.0090; r02: whole 64-B records in LDS 0.0479).  The
// shadow rays read the MT records (rt_tri_t) of S.geom.

#if !RT_FLAT
__device__ __forceinline__ void kernel_body(const vx_task_t& task, const Scene& S, WaveLds& w,
                                            Counters& cnt) {
  const uint32_t t = task.blockIdx.x;
  // the chunk's task map in scalar registers (every lane runs the same chunk)
  const ChunkMap cm = chunk_map(S, task_args(S), (uint32_t)__builtin_amdgcn_readfirstlane(t) >> 6);
  uint32_t x, y, out;
  chunk_pixel(S, cm, t & 63u, &x, &y, &out);
  const uint32_t lb = (cm.lt << 4) | cm.blk;
  const bool in = x < S.width && y < S.height;  // edge tiles overhang the image
  cnt.primary += in;
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
#ifdef RT_STAMPS
  if (lane_id() == 0) __vx_mpm_lds[3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  // primary visibility: the raster's winner at this pixel
  const int32_t hit = trace_primary(S, lb, x, y, in, tie_high, cnt);
#ifdef RT_STAMPS
  if (lane_id() == 0) __vx_mpm_lds[14] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  cnt.hits += hit >= 0;
  const int32_t spid = resolve_layers(S, x, y, in && hit < 0, hit, cnt);
#ifdef RT_STAMPS
  if (lane_id() == 0) __vx_mpm_lds[4] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  uint32_t color = shade_wave(S, spid, x, y, S.clear_color, cnt);
#ifdef RT_STAMPS
  if (lane_id() == 0) __vx_mpm_lds[11] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  Ray r;
  primary_dir(S, x, y, r);
  const float th = hit >= 0 ? plane_t(S, r, hit) : 0.0f;
#if RT_PATHQ
  // path tracing, first kernel: a path starts at the winner's plane; its
  // pixel is written by pt_queue when the path ends
  const bool path = hit >= 0 && secondary_ok(th);
  pathq_append(S, path, t, th, hit, color);
  if (in && !path) store_out(S, out, color);
  (void)w;
  return;
#endif
  const bool shadow = hit >= 0 && secondary_ok(th) && (S.flags & RT_FLAG_SHADOWS) != 0;
  // wave64 compaction: lanes with a pending shadow ray append it to the
  // wave's LDS queue at ballot/mbcnt-assigned slots
  const uint64_t m = __ballot(shadow);
  if (m) {
    const uint32_t base = w.q_count;
    if (shadow) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const uint32_t slot = base + rank;
      w.q_out[slot] = out;
      w.q_xy[slot] = x | (y << 16);
      w.q_t[slot] = th;
      w.q_pid[slot] = hit;
      w.q_color[slot] = color;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane_id() == 0) w.q_count = base + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  if (in && !shadow) store_out(S, out, color);
#ifdef RT_STAMPS
  if (lane_id() == 0) __vx_mpm_lds[5] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
}
#endif

#if !RT_FLAT
// Called by all 64 lanes after every chunk: trace full waves of 64 shadow
// rays while the queue holds >= 64 (or whatever is left at the end).
__device__ __forceinline__ void shadow_drain(bool final, const Scene& S, WaveLds& w,
                                             Counters& cnt) {
#ifdef RT_STAMPS
  if (final && lane_id() == 0) __vx_mpm_lds[15] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  if (final && lane_id() == 0) __vx_mpm_lds[8] = w.q_count;  // the final drain's shadow rays
  if (!final && w.q_count >= 64 && lane_id() == 0)
    __vx_mpm_lds[6] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  if (!(S.flags & RT_FLAG_SHADOWS)) return;
  const uint32_t lane = lane_id();
  uint32_t n = w.q_count;
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  while (n >= 64 || (final && n > 0)) {
    const uint32_t take = n < 64 ? n : 64;
    const uint32_t base = n - take;
    const bool active = lane < take;
    const uint32_t slot = base + lane;  // < RT_QUEUE for every lane
    const uint32_t xy = w.q_xy[slot];
    Ray p, s;
    primary_dir(S, xy & 0xffffu, xy >> 16, p);
    shadow_ray(S, p, w.q_t[slot], s);
    cnt.shadow += active;
    uint32_t color = w.q_color[slot];
    float ts;
    // the light-space lists when built (occluded_list), else the BVH: the
    // binary16 BVH4 as one packet, other layouts per lane (deep images)
    const bool occ = !RT_BVH_WALK && S.slist_on ? occluded_list(S, s, active, w.q_pid[slot], cnt)
                     : (RT_ONLY_BVH4H || (S.flags & RT_FLAG_BVH4H))
                         ? occluded_packet(S, s, active, w.q_pid[slot], 1.0f, cnt)
                         : active && trace<true>(S, s, 0.0f, 1.0f, w.q_pid[slot], tie_high, &ts,
                                                 RT_WSTACK(w, lane), cnt) >= 0;
    if (occ) {
      ++cnt.occluded;
      color = shadowed(color);
    }
    if (active) store_out(S, w.q_out[slot], color);
    n = base;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) w.q_count = n;
  __builtin_amdgcn_wave_barrier();
}
#endif

#if RT_FLAT
// Config 2 with every ray's primitive list split across the workgroup's
// waves: a workgroup step takes one 64-task chunk (vx_spawn_chunks_block),
// wave w tests the list entries w, w + kWaves, ... for the chunk's 64
// pixels (flat_chunk), the per-wave winners meet in LDS (vis_better is a
// strict order on (depth word, pid), so the reduction order is immaterial)
// and wave 0 shades and stores; shadow rays split the list in ranges, the
// first occluder in list order found by a min over the waves' first hits
// (which is also brute_trace's test count).
// Without shadow rays waves 1.. leave the chunk once their winners are in
// LDS and wave 0 shades and stores with no second barrier -- the winners
// double-buffered by chunk parity, so a wave's next chunk never overwrites
// words wave 0 is still reducing (it must pass the next chunk's barrier,
// which wave 0 reaches only after its reduction)
struct FlatLds {
  uint32_t z[2][kWaves][64];
  int32_t pid[2][kWaves][64];
  uint32_t first[kWaves][64];
};

// a record's rectangle word with its rectangle as packed corners (lo = x0 |
// y0 << 16, hi = x1 | y1 << 16 in .y / .z; an empty rectangle becomes
// lo = 0xffffffff, hi = 0xfffefffe, which no pixel matches), so a wave's
// rectangle test is two packed 16-bit clamps and one compare (rect2_in)
__device__ __forceinline__ uint4 rect_corners(uint4 c) {
  const uint32_t rx = c.y, ry = c.z;
  const bool empty = (rx & 0xffffu) > (rx >> 16) || (ry & 0xffffu) > (ry >> 16);
  c.y = empty ? 0xffffffffu : (rx & 0xffffu) | (ry << 16);
  c.z = empty ? 0xfffefffeu : (rx >> 16) | (ry & 0xffff0000u);
  return c;
}
__device__ __forceinline__ void flat_chunk(const vx_task_t& task, bool valid, const Scene& S,
                                           FlatLds& L, uint32_t& par, Counters& cnt) {
  const uint32_t w = threadIdx.x >> 6, lane = lane_id();
  const uint32_t pb = par;  // this chunk's winner buffer
  par ^= 1u;
  const uint32_t t = task.blockIdx.x;
  uint32_t x = 0, y = 0, out = 0;
  if (valid) {
    // the chunk's task map in scalar registers (block-uniform chunk)
    const ChunkMap cm = chunk_map(S, task_args(S), (uint32_t)__builtin_amdgcn_readfirstlane(t) >> 6);
    chunk_pixel(S, cm, t & 63u, &x, &y, &out);
  }
  const bool in = valid && x < S.width && y < S.height;
  const uint32_t px = in ? x : 0xffffffffu;  // outside every pixel rectangle
  const uint32_t pp = in ? x | (y << 16) : 0xffffffffu;  // packed pixel (rect_corners)
  const bool tie_high = (S.flags & RT_FLAG_TIE_HIGH) != 0;
  const uint32_t n = S.num_geom, per = (n + kWaves - 1) / kWaves;
  const uint32_t k0 = w * per < n ? w * per : n, k1 = k0 + per < n ? k0 + per : n;
  uint32_t bz = VX_OM_DEPTH_MASK;
  int32_t bp = -1;
  // Two levels: the wave's lanes take 64 of its entries at once and test
  // each one's rectangle against the chunk's 8x8 block (packed corners:
  // lo <= block hi and hi >= block lo, halfwise); then, for the entries that
  // reach the block only, the per-pixel rectangle test and, where a lane
  // lies in it, the edges and depth -- the records two at a time (one
  // 64-B scalar load each, the second in flight while the first is tested).
  // The same entries get the same tests as a one-level scan of every entry
  // per pixel (the block test only skips entries no pixel of the block lies
  // in): identical winners and counts, with 1/64 of the rectangle-test
  // instructions (r04).  Wave w takes entries w, w + kWaves, ...: a region's
  // triangles, often consecutive in the list, spread over the waves.
  {
    const uint32_t bx = (uint32_t)__builtin_amdgcn_readfirstlane(x) & ~7u;  // lane 0: the block's corner
    const uint32_t by = (uint32_t)__builtin_amdgcn_readfirstlane(y) & ~7u;
    const uint32_t blo = bx | (by << 16), bhi = (bx + 7u) | ((by + 7u) << 16);
    const uint32_t mine = w < n ? (n - w + kWaves - 1) / kWaves : 0u;  // this wave's entries
    for (uint32_t i = 0; i < mine; i += 64u) {
      const uint32_t il = i + lane;
      bool ov = false;
      if (il < mine) {
        const uint32_t kl = il * kWaves + w;
        const uint4 C = rect_corners(S.A.ld_u4(S.vgeom + 64u * kl + 32u));
        // max(lo, block hi) == block hi and min(hi, block lo) == block lo
        ov = rect2_clamp(C.y, 0xffffffffu, bhi) == bhi && rect2_clamp(0u, C.z, blo) == blo;
      }
      uint64_t m = __ballot(ov);
#ifdef RT_INSTRUMENT
      cnt.rect_tests += lane == 0 ? (mine - i < 64u ? mine - i : 64u) : 0u;
#endif
      while (m != 0) {
        const uint32_t j0 = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const bool two = m != 0;
        const uint32_t j1 = two ? (uint32_t)__builtin_ctzll(m) : j0;
        if (two) m &= m - 1;
        const uint32_t ka = (i + j0) * kWaves + w, kb = (i + j1) * kWaves + w;
        uint4 ra[4], rb[4];
        S.A.sld_u4n<4>(S.vgeom + 64u * ka, ra);
        S.A.sld_u4n<4>(S.vgeom + 64u * kb, rb);
        const uint4 Ca = rect_corners(ra[2]), Cb = rect_corners(rb[2]);
        const bool ina = rect2_in(Ca.y, Ca.z, pp);
        if (__ballot(ina) != 0) {  // wave-uniform
#ifdef RT_INSTRUMENT
          cnt.edge_tests += lane == 0 ? 1u : 0u;
#endif
          vis_test_in(ra[0], ra[1], ra[2], ra[3], ina, px, y, tie_high, bz, bp);
        }
        const bool inb = two && rect2_in(Cb.y, Cb.z, pp);
        if (__ballot(inb) != 0) {
#ifdef RT_INSTRUMENT
          cnt.edge_tests += lane == 0 ? 1u : 0u;
#endif
          vis_test_in(rb[0], rb[1], rb[2], rb[3], inb, px, y, tie_high, bz, bp);
        }
      }
    }
#ifdef RT_INSTRUMENT
    cnt.tests += in ? mine : 0u;  // the whole list per ray, summed over the waves
#endif
  }
#ifdef RT_STAMPS  // 3: wave 0's list scan done, 4: the slowest wave's (after the barrier)
  if (threadIdx.x == 0) __vx_mpm_lds[3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  L.z[pb][w][lane] = bz;
  L.pid[pb][w][lane] = bp;
  __syncthreads();
#ifdef RT_STAMPS
  if (threadIdx.x == 0) __vx_mpm_lds[4] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  const bool early = (S.flags & RT_FLAG_SHADOWS) == 0;  // block-uniform
  if (early && w != 0) return;
  int32_t hit = -1;
  uint32_t hz = VX_OM_DEPTH_MASK;
  for (uint32_t i = 0; i < kWaves; ++i) {
    const int32_t p = L.pid[pb][i][lane];
    if (p >= 0 && vis_better(L.z[pb][i][lane], p, hz, hit, tie_high)) {
      hz = L.z[pb][i][lane];
      hit = p;
    }
  }
  uint32_t color = 0;
  if (w == 0) {
    cnt.primary += in;
    cnt.hits += hit >= 0;
    const int32_t spid = resolve_layers(S, x, y, in && hit < 0, hit, cnt);
    color = shade_wave(S, spid, x, y, S.clear_color, cnt);
#ifdef RT_STAMPS  // 5: shaded (wave 0)
    asm volatile("" : : "v"(color));  // the colour is complete before the stamp
    if (threadIdx.x == 0) __vx_mpm_lds[5] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  }
  if (early) {  // wave 0 only: no shadow rays, no second barrier
    if (in) store_out(S, out, color);
    return;
  }
  Ray r;
  primary_dir(S, x, y, r);
  const float th = hit >= 0 ? plane_t(S, r, hit) : 0.0f;
  const bool shadow = in && hit >= 0 && secondary_ok(th) && (S.flags & RT_FLAG_SHADOWS) != 0;
  if (__ballot(shadow)) {  // block-uniform: every wave holds the same 64 rays
    Ray sr;
    shadow_ray(S, r, th, sr);
    float ts;
    uint32_t first = 0xffffffffu;
    if (shadow) trace_flat_range<true>(S, sr, k0, k1, 0.0f, 1.0f, hit, tie_high, &ts, &first);
    L.first[w][lane] = first;
  }
  __syncthreads();
  if (w == 0) {
    if (shadow) {
      uint32_t first = 0xffffffffu;
      for (uint32_t i = 0; i < kWaves; ++i) first = L.first[i][lane] < first ? L.first[i][lane] : first;
      cnt.shadow += 1;
#ifdef RT_INSTRUMENT
      cnt.tests += first != 0xffffffffu ? first + 1 : n;  // brute_trace stops at the first occluder
#endif
      if (first != 0xffffffffu) {
        ++cnt.occluded;
        color = shadowed(color);
      }
    }
    if (in) store_out(S, out, color);
  }
}
#endif

// RT statistics go to the user MPM counters (VX_CSR_MPM_USER = 0xB03 + slot),
// which the driver zeroes before every launch and vx_mpm_query() reads back.
__device__ __forceinline__ void flush(int slot, uint32_t v) { vx_mpm_add(RT_MPM_USER + slot, v); }

}  // namespace

// primary + shadow images: registers for 7 waves per SIMD (<= 72 VGPRs: 67,
// 22 SGPR spills) -- A/B on the light-space-list image (r03g, same frames):
// 5 (71 VGPRs, 6-7 resident) 0.02574 ms, 7 0.02470, 8 (64 VGPRs, 39 SGPR
// spills) 0.02532: the frame is latency-bound with the chip full of waves
// (DESIGN 4.1), so more resident waves win until the spills cost more.
// (r02: capping occupancy lower with LDS padding cost +27 / +80 %.)  The
// deep images (every layout, 32-entry stack) keep the compiler's choice.
// The BVH-walk image (rt_bvh: packet walks, no lists) is better at 5
// (A/B r04f: 5 0.03644 ms, 6 0.03676, 7 0.03768, 8 0.03752).
#if !defined(RT_WAVES_PER_EU) && !RT_FLAT && RT_ONLY_BVH4H
#if RT_BVH_WALK
#define RT_WAVES_PER_EU 5
#else
#define RT_WAVES_PER_EU 7
#endif
#endif
#if RT_FLAT
// config 2: 4 workgroups per CU (1 024: one per 256^2 chunk) -- A/B r04i:
// 0.01084 ms vs 0.01108 at 16/CU; registers for 8 waves per SIMD, so all
// 1 024 workgroups of 512 threads are resident at once (r05j)
__device__ __attribute__((used)) uint32_t __vx_grid_per_cu = 4;
#define RT_WAVES_PER_EU 8
#endif
#ifdef RT_WAVES_PER_EU
VX_MAIN_OCC(rt_kernel_arg_t, arg, RT_BLOCK_THREADS, RT_WAVES_PER_EU) {
#else
VX_MAIN(rt_kernel_arg_t, arg, RT_BLOCK_THREADS) {
#endif
  __shared__ WaveLds s_wave[kWaves];
  WaveLds& w = s_wave[threadIdx.x >> 6];
#ifdef RT_STAMPS
  const uint64_t t_stamp0 = __builtin_amdgcn_s_memrealtime();
#endif
  Counters cnt;
  Scene S = load_scene(arg, vx_launch_words);
#ifdef RT_STAMPS
  if (threadIdx.x == 0) __vx_mpm_lds[10] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
#if RT_FLAT
  // the workgroup's waves start their first chunk together
  __syncthreads();
#ifdef RT_STAMPS  // 11: past the start barrier
  if (threadIdx.x == 0) __vx_mpm_lds[11] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  __shared__ FlatLds s_flat;
  (void)w;
  uint32_t par = 0;
  const int rc = vx_spawn_chunks_block(
      S.num_tasks,
      [&](const vx_task_t& task, bool valid, const Scene* s) { flat_chunk(task, valid, *s, s_flat, par, cnt); },
      &S);
#else
  if ((threadIdx.x & 63u) == 0) w.q_count = 0;
  __builtin_amdgcn_wave_barrier();
  const int rc = vx_spawn_tasks_ex(
      S.num_tasks,
      [&](const vx_task_t& task, const Scene* s) { kernel_body(task, *s, w, cnt); },
      [&](bool final, const Scene* s) { shadow_drain(final, *s, w, cnt); }, &S);
#endif
#ifdef RT_STAMPS  // diagnostic image: per-wave phase timestamps
  if (threadIdx.x == 0) {
    // 12: start, 13: end, 14: primary traced, 15: shadow drain begins
    // (low 32 bits of s_memrealtime, 100 MHz)
    __vx_mpm_lds[12] = (uint32_t)t_stamp0;
    __vx_mpm_lds[13] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  }
#endif
#ifndef RT_STAMPS  // the stamp image keeps slots 3-9 for phase stamps / iteration counts
  flush(RT_STAT_PRIMARY, cnt.primary);
  flush(RT_STAT_SHADOW, cnt.shadow);
  flush(RT_STAT_HITS, cnt.hits);
  flush(RT_STAT_OCCLUDED, cnt.occluded);
#endif
#ifdef RT_INSTRUMENT
  flush(RT_STAT_NODE_VISITS, cnt.visits);
  flush(RT_STAT_TRI_TESTS, cnt.tests);
  flush(RT_STAT_LAYER_TESTS, cnt.layer_tests);
  flush(RT_STAT_SHADED, cnt.shaded);
  flush(RT_STAT_TEXEL_BYTES, cnt.texel_bytes);
#if RT_FLAT
  flush(RT_STAT_RECT_TESTS, cnt.rect_tests);
  flush(RT_STAT_EDGE_TESTS, cnt.edge_tests);
#endif
#endif
  return rc;
}

