// bvh_build.hip -- GPU BVH build, one launch per
// phase of bvh_common.h: centroid bounds, Morton codes, a stable 4-pass LSD
// radix sort (8-bit digits: per-block histograms, one scan, a stable
// scatter ranked with wave ballots), the binary radix tree of Karras 2012
// over the sorted 62-bit keys (code << 32 | index: unique, so the tree is
// well defined with duplicate codes), boxes bottom-up (the second child to
// arrive at a node builds its box and climbs -- in LDS inside a workgroup's
// window of leaves, through agent-scope acq_rel counters above it; nobody
// waits), and the rt_node_t / rt_tri_t records the traversal
// reads, subtrees of <= 4 triangles emitted as leaves.  Deterministic: the
// oracle (oracle/lbvh.c) restates every phase and the tests compare the
// emitted arrays bit for bit.
#include <hip/hip_runtime.h>

#include "bvh_common.h"
#include "half4.h"
#include "rt_common.h"
#include "vx_spawn.h"

namespace {

constexpr uint32_t kWaves = BVHB_BLOCK / 64;

__device__ __forceinline__ uint32_t lane() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// float <-> uint with the float order (atomicMin / atomicMax on floats)
__device__ __forceinline__ uint32_t ord(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ void tri_box(const float4* v, uint32_t t, float* lo, float* hi) {
  const float4 a = v[3 * t], b = v[3 * t + 1], c = v[3 * t + 2];
  lo[0] = fminf(fminf(a.x, b.x), c.x);
  lo[1] = fminf(fminf(a.y, b.y), c.y);
  lo[2] = fminf(fminf(a.z, b.z), c.z);
  hi[0] = fmaxf(fmaxf(a.x, b.x), c.x);
  hi[1] = fmaxf(fmaxf(a.y, b.y), c.y);
  hi[2] = fmaxf(fmaxf(a.z, b.z), c.z);
}

__device__ __forceinline__ float wave_min(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fminf(x, __shfl_xor(x, o, 64));
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
  return x;
}

__device__ __forceinline__ uint32_t expand10(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__device__ __forceinline__ uint32_t quant(float c, float lo, float hi) {
  const float e = hi - lo;
  const float t = e > 0.0f ? (c - lo) / e : 0.0f;
  const uint32_t q = (uint32_t)(t * 1024.0f);
  return q < 1023u ? q : 1023u;
}

// --- phases ---------------------------------------------------------------

__device__ void phase_bounds(const bvh_build_arg_t* a) {
  const float4* v = vx_ptr<const float4>(a->verts_addr);
  float4* cen = vx_ptr<float4>(a->cen_addr);
  uint32_t* bounds = vx_ptr<uint32_t>(a->bounds_addr);
  __shared__ float red[kWaves][7];
  if (blockIdx.x * BVHB_BLOCK >= a->n) return;  // no triangles: no atomics (uniform exit)
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  float am = 0.0f;
  for (uint32_t t = blockIdx.x * BVHB_BLOCK + threadIdx.x; t < a->n; t += gridDim.x * BVHB_BLOCK) {
    float lo[3], hi[3];
    tri_box(v, t, lo, hi);
    float c[3];
    for (int k = 0; k < 3; ++k) {
      c[k] = (lo[k] + hi[k]) * 0.5f;
      mn[k] = fminf(mn[k], c[k]);
      mx[k] = fmaxf(mx[k], c[k]);
      am = fmaxf(am, fmaxf(fabsf(lo[k]), fabsf(hi[k])));
    }
    cen[t] = make_float4(c[0], c[1], c[2], 0.0f);
  }
  const uint32_t w = threadIdx.x >> 6;
  float r[7] = {mn[0], mn[1], mn[2], mx[0], mx[1], mx[2], am};
  for (int k = 0; k < 3; ++k) r[k] = wave_min(r[k]);
  for (int k = 3; k < 7; ++k) r[k] = wave_max(r[k]);
  if (lane() == 0)
    for (int k = 0; k < 7; ++k) red[w][k] = r[k];
  __syncthreads();
  if (threadIdx.x < 7) {
    const int k = threadIdx.x;
    float x = red[0][k];
    for (uint32_t i = 1; i < kWaves; ++i) x = k < 3 ? fminf(x, red[i][k]) : fmaxf(x, red[i][k]);
    if (k < 3) atomicMin(&bounds[k], ord(x));
    else atomicMax(&bounds[k], ord(x));
  }
}

__device__ __forceinline__ float unord(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ void phase_morton(const bvh_build_arg_t* a) {
  const float4* cen = vx_ptr<const float4>(a->cen_addr);
  const uint32_t* bounds = vx_ptr<const uint32_t>(a->bounds_addr);
  uint32_t* keys = vx_ptr<uint32_t>(a->keys_addr[0]);
  uint32_t* vals = vx_ptr<uint32_t>(a->vals_addr[0]);
  float lo[3], hi[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = unord(bounds[k]);
    hi[k] = unord(bounds[3 + k]);
  }
  for (uint32_t t = blockIdx.x * BVHB_BLOCK + threadIdx.x; t < a->n; t += gridDim.x * BVHB_BLOCK) {
    const float4 c = cen[t];
    keys[t] = (expand10(quant(c.x, lo[0], hi[0])) << 2) | (expand10(quant(c.y, lo[1], hi[1])) << 1) |
              expand10(quant(c.z, lo[2], hi[2]));
    vals[t] = t;
  }
}

__device__ void phase_hist(const bvh_build_arg_t* a) {
  const uint32_t* keys = vx_ptr<const uint32_t>(a->keys_addr[a->pass & 1]);
  uint32_t* hist = vx_ptr<uint32_t>(a->hist_addr);
  __shared__ uint32_t h[256];
  const uint32_t shift = 8u * a->pass;
  for (uint32_t b = blockIdx.x; b < a->nblocks; b += gridDim.x) {
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = 0; i < BVHB_ITEMS / BVHB_BLOCK; ++i) {
      const uint32_t t = b * BVHB_ITEMS + i * BVHB_BLOCK + threadIdx.x;
      if (t < a->n) atomicAdd(&h[(keys[t] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * a->nblocks + b] = h[threadIdx.x];
    __syncthreads();
  }
}

// exclusive scan of hist[256][nblocks] (digit-major) by workgroup 0: each
// thread sums a contiguous chunk (independent loads), one workgroup scan of
// the 256 chunk sums, then each thread rewrites its chunk
__device__ void phase_scan(const bvh_build_arg_t* a) {
  if (blockIdx.x != 0) return;
  uint32_t* hist = vx_ptr<uint32_t>(a->hist_addr);
  __shared__ uint32_t s[BVHB_BLOCK];
  const uint32_t total = 256u * a->nblocks;
  const uint32_t chunk = (total + BVHB_BLOCK - 1) / BVHB_BLOCK;
  const uint32_t b0 = threadIdx.x * chunk;
  const uint32_t b1 = b0 + chunk < total ? b0 + chunk : total;
  uint32_t sum = 0;
#pragma unroll 8
  for (uint32_t i = b0; i < b1; ++i) sum += hist[i];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < BVHB_BLOCK; o <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t y = threadIdx.x >= o ? s[threadIdx.x - o] : 0u;
    __syncthreads();
    s[threadIdx.x] += y;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - sum;
  for (uint32_t i = b0; i < b1; ++i) {
    const uint32_t x = hist[i];
    hist[i] = run;
    run += x;
  }
}

// stable scatter: the items of a block in 4 rounds of 256 (in index order);
// rank = digit offset of the block + earlier rounds + earlier waves + lanes
// of this wave with the same digit below this lane (8 ballots)
__device__ void phase_scatter(const bvh_build_arg_t* a) {
  const uint32_t src = a->pass & 1;
  const uint32_t* keys = vx_ptr<const uint32_t>(a->keys_addr[src]);
  const uint32_t* vals = vx_ptr<const uint32_t>(a->vals_addr[src]);
  uint32_t* okeys = vx_ptr<uint32_t>(a->keys_addr[src ^ 1]);
  uint32_t* ovals = vx_ptr<uint32_t>(a->vals_addr[src ^ 1]);
  const uint32_t* hist = vx_ptr<const uint32_t>(a->hist_addr);
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[kWaves][256];
  const uint32_t shift = 8u * a->pass, w = threadIdx.x >> 6, l = lane();
  const uint64_t lt = (l == 0) ? 0ull : (~0ull >> (64 - l));
  for (uint32_t b = blockIdx.x; b < a->nblocks; b += gridDim.x) {
    base[threadIdx.x] = hist[threadIdx.x * a->nblocks + b];
    for (uint32_t i = 0; i < kWaves; ++i) wcnt[i][threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t r = 0; r < BVHB_ITEMS / BVHB_BLOCK; ++r) {
      const uint32_t t = b * BVHB_ITEMS + r * BVHB_BLOCK + threadIdx.x;
      const bool valid = t < a->n;
      const uint32_t key = valid ? keys[t] : 0u, val = valid ? vals[t] : 0u;
      const uint32_t d = (key >> shift) & 255u;
      uint64_t peers = __ballot(valid);
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const uint64_t m = __ballot((d >> bit) & 1u);
        peers &= ((d >> bit) & 1u) ? m : ~m;
      }
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      if (valid && below == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
      __syncthreads();
      uint32_t off = 0;
      if (valid)
        for (uint32_t i = 0; i < w; ++i) off += wcnt[i][d];
      const uint32_t dst = base[d] + off + below;
      __syncthreads();
      // advance the per-digit base past this round, clear the wave counts
      uint32_t sum = 0;
      for (uint32_t i = 0; i < kWaves; ++i) {
        sum += wcnt[i][threadIdx.x];
        wcnt[i][threadIdx.x] = 0;
      }
      base[threadIdx.x] += sum;
      if (valid) {
        okeys[dst] = key;
        ovals[dst] = val;
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ int delta(const uint32_t* keys, const uint32_t* vals, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint64_t ki = ((uint64_t)keys[i] << 32) | vals[i];
  const uint64_t kj = ((uint64_t)keys[j] << 32) | vals[j];
  return __clzll((long long)(ki ^ kj));
}

__device__ void phase_tree(const bvh_build_arg_t* a) {
  const uint32_t* keys = vx_ptr<const uint32_t>(a->keys_addr[0]);
  const uint32_t* vals = vx_ptr<const uint32_t>(a->vals_addr[0]);
  int32_t* parent = vx_ptr<int32_t>(a->parent_addr);
  uint32_t* range = vx_ptr<uint32_t>(a->range_addr);
  int32_t* child = vx_ptr<int32_t>(a->child_addr);
  uint32_t* flags = vx_ptr<uint32_t>(a->flags_addr);
  const int n = (int)a->n;
  for (int i = blockIdx.x * BVHB_BLOCK + threadIdx.x; i < n - 1; i += gridDim.x * BVHB_BLOCK) {
    const int d = (delta(keys, vals, n, i, i + 1) - delta(keys, vals, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, vals, n, i, i - d);
    int lmax = 2;
    while (delta(keys, vals, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
      if (delta(keys, vals, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, vals, n, i, j);
    int s = 0, t = l;
    do {
      t = (t + 1) / 2;
      if (delta(keys, vals, n, i, i + (s + t) * d) > dnode) s += t;
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
    flags[i] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) parent[0] = -1;
}

// Boxes bottom-up.  Workgroup b owns the sorted leaves [256b, 256b + 256):
// internal nodes whose leaf range lies inside that window ("local" -- their
// index is one of their range's ends, so also inside it) are completed in
// LDS with workgroup-scope counters; a thread that climbs out of the window
// carries its subtree's box on through global memory with agent-scope
// acq_rel counters (the second child to arrive builds the node; nobody waits).
__device__ __forceinline__ float4 fmin4(float4 a, float4 b) {
  return make_float4(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), 0.0f);
}
__device__ __forceinline__ float4 fmax4(float4 a, float4 b) {
  return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), 0.0f);
}

__device__ void phase_boxes(const bvh_build_arg_t* a) {
  const float4* v = vx_ptr<const float4>(a->verts_addr);
  const uint32_t* vals = vx_ptr<const uint32_t>(a->vals_addr[0]);
  const int32_t* parent = vx_ptr<const int32_t>(a->parent_addr);
  const int32_t* child = vx_ptr<const int32_t>(a->child_addr);
  const uint32_t* range = vx_ptr<const uint32_t>(a->range_addr);
  uint32_t* flags = vx_ptr<uint32_t>(a->flags_addr);
  float4* boxes = vx_ptr<float4>(a->boxes_addr);
  __shared__ float4 llo[2 * BVHB_BLOCK], lhi[2 * BVHB_BLOCK];  // [leaf slot | internal slot]
  __shared__ uint32_t lcnt[BVHB_BLOCK];
  const int n = (int)a->n;
  const int nwin = (n + BVHB_BLOCK - 1) / BVHB_BLOCK;
  for (int b = blockIdx.x; b < nwin; b += gridDim.x) {
    const int L0 = b * BVHB_BLOCK, L1 = L0 + BVHB_BLOCK < n ? L0 + BVHB_BLOCK : n;
    const int k = L0 + (int)threadIdx.x;
    const bool valid = k < L1;
    lcnt[threadIdx.x] = 0;
    float4 lo = make_float4(0, 0, 0, 0), hi = lo;
    if (valid) {
      float l[3], h[3];
      tri_box(v, vals[k], l, h);
      lo = make_float4(l[0], l[1], l[2], 0.0f);
      hi = make_float4(h[0], h[1], h[2], 0.0f);
      boxes[2 * (n + k)] = lo;
      boxes[2 * (n + k) + 1] = hi;
      llo[threadIdx.x] = lo;
      lhi[threadIdx.x] = hi;
    }
    __syncthreads();
    int p = (valid && n >= 2) ? parent[n + k] : -1;
    bool alive = p >= 0;
    // local climb: LDS boxes, workgroup-scope counters
    while (alive && (int)range[2 * p] >= L0 && (int)range[2 * p + 1] < L1) {
      const uint32_t old = __hip_atomic_fetch_add(&lcnt[p - L0], 1u, __ATOMIC_ACQ_REL,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
      if (old == 0) {
        alive = false;
        break;
      }
      const int c0 = child[2 * p], c1 = child[2 * p + 1];
      const int s0 = c0 >= 0 ? BVHB_BLOCK + c0 - L0 : ~c0 - L0;
      const int s1 = c1 >= 0 ? BVHB_BLOCK + c1 - L0 : ~c1 - L0;
      lo = fmin4(llo[s0], llo[s1]);
      hi = fmax4(lhi[s0], lhi[s1]);
      llo[BVHB_BLOCK + p - L0] = lo;
      lhi[BVHB_BLOCK + p - L0] = hi;
      boxes[2 * p] = lo;
      boxes[2 * p + 1] = hi;
      p = parent[p];
      alive = p >= 0;
    }
    // global climb from the first node outside the window
    for (int guard = 0; alive && guard < 4096; ++guard) {
      const uint32_t old = __hip_atomic_fetch_add(&flags[p], 1u, __ATOMIC_ACQ_REL,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      if (old == 0) break;
      const int c0 = child[2 * p], c1 = child[2 * p + 1];
      const int i0 = c0 >= 0 ? c0 : n + ~c0, i1 = c1 >= 0 ? c1 : n + ~c1;
      boxes[2 * p] = fmin4(boxes[2 * i0], boxes[2 * i1]);
      boxes[2 * p + 1] = fmax4(boxes[2 * i0 + 1], boxes[2 * i1 + 1]);
      p = parent[p];
      alive = p >= 0;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ void set_child(float* node, int ch, float4 lo, float4 hi, float pad,
                                          int32_t ref) {
  const bool empty = ref == RT_EMPTY_REF;
  const float l[3] = {lo.x, lo.y, lo.z}, h[3] = {hi.x, hi.y, hi.z};
  for (int k = 0; k < 3; ++k) {
    node[4 * k + 2 * ch + 0] = empty ? 0.0f : l[k] - pad;
    node[4 * k + 2 * ch + 1] = empty ? 0.0f : h[k] + pad;
  }
  node[12 + ch] = __int_as_float(ref);
}

__device__ void phase_emit(const bvh_build_arg_t* a) {
  const uint32_t* vals = vx_ptr<const uint32_t>(a->vals_addr[0]);
  const int32_t* parent = vx_ptr<const int32_t>(a->parent_addr);
  const int32_t* child = vx_ptr<const int32_t>(a->child_addr);
  const uint32_t* range = vx_ptr<const uint32_t>(a->range_addr);
  const float4* boxes = vx_ptr<const float4>(a->boxes_addr);
  const rt_tri_t* geom = vx_ptr<const rt_tri_t>(a->geom_addr);
  uint32_t* bounds = vx_ptr<uint32_t>(a->bounds_addr);
  rt_node_t* nodes = vx_ptr<rt_node_t>(a->nodes_addr);
  rt_tri_t* tris = vx_ptr<rt_tri_t>(a->tris_addr);
  const int n = (int)a->n;
  const float pad = fmaxf(unord(bounds[6]) * (1.0f / 65536.0f), 1e-6f);
  const int gid = blockIdx.x * BVHB_BLOCK + threadIdx.x, gstride = gridDim.x * BVHB_BLOCK;
  for (int k = gid; k < n + 3; k += gstride) {
    if (k < n) {
      tris[k] = geom[vals[k]];
    } else {
      for (int q = 0; q < 12; ++q) tris[k].v[q] = 0.0f;
    }
  }
  if (n <= BVHB_LEAF_MAX) {  // one node: a leaf of every triangle + an empty child
    if (gid == 0 && n > 0) {
      float4 lo = boxes[2 * n], hi = boxes[2 * n + 1];
      for (int k = 1; k < n; ++k) {
        const float4 l = boxes[2 * (n + k)], h = boxes[2 * (n + k) + 1];
        lo = make_float4(fminf(lo.x, l.x), fminf(lo.y, l.y), fminf(lo.z, l.z), 0.0f);
        hi = make_float4(fmaxf(hi.x, h.x), fmaxf(hi.y, h.y), fmaxf(hi.z, h.z), 0.0f);
      }
      float* nd = nodes[0].v;
      for (int q = 0; q < 16; ++q) nd[q] = 0.0f;
      set_child(nd, 0, lo, hi, pad, (int32_t)(RT_LEAF_FLAG | (uint32_t)(n - 1)));
      set_child(nd, 1, lo, hi, pad, RT_EMPTY_REF);
      atomicMax(&bounds[7], 1u);
    }
    return;
  }
  uint32_t maxdepth = 0;
  for (int i = gid; i < n - 1; i += gstride) {
    float* nd = nodes[i].v;
    for (int q = 0; q < 16; ++q) nd[q] = 0.0f;
    const uint32_t size = range[2 * i + 1] - range[2 * i] + 1;
    if (i != 0 && size <= BVHB_LEAF_MAX) continue;  // inside a leaf: unreachable
    for (int ch = 0; ch < 2; ++ch) {
      const int c = child[2 * i + ch];
      int32_t ref;
      int bi;
      if (c < 0) {
        ref = (int32_t)(RT_LEAF_FLAG | ((uint32_t)~c << 4));
        bi = n + ~c;
      } else {
        const uint32_t cs = range[2 * c + 1] - range[2 * c] + 1;
        ref = cs <= BVHB_LEAF_MAX ? (int32_t)(RT_LEAF_FLAG | (range[2 * c] << 4) | (cs - 1)) : c;
        bi = c;
      }
      set_child(nd, ch, boxes[2 * bi], boxes[2 * bi + 1], pad, ref);
    }
    uint32_t depth = 1;
    for (int p = i; p != 0; p = parent[p]) ++depth;
    maxdepth = depth > maxdepth ? depth : maxdepth;
  }
  // one atomic per wave (100k same-address atomics cost ~0.4 ms)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)maxdepth, o, 64);
    maxdepth = y > maxdepth ? y : maxdepth;
  }
  if (lane() == 0 && maxdepth) atomicMax(&bounds[7], maxdepth);
}

// BVH4 collapse of the emitted BVH2 (bvh_build.hip's own rule, restated by
// oracle/lbvh.c orc_lbvh_collapse4): every reachable internal node at even
// depth (root = 0) becomes a BVH4 node at its own index, its children being
// its BVH2 children with each internal child (odd depth) replaced by that
// child's two children -- slots in order, leaves and even-depth nodes kept as
// refs, boxes copied from the emitted rt_node_t records (already padded).
// No allocation or ordering pass: every node decides alone.  Also the
// worst-case traversal stack (near-first BVH4 pushes slots - 1 per node):
// the max over nodes of the sum of (slots - 1) over its BVH4 ancestors and
// itself, into bounds[8].
struct Slots4 {
  int count;
  int32_t ref[4];
  float lo[4][3], hi[4][3];
};

__device__ __forceinline__ Slots4 slots4_of(const rt_node_t* nodes, int i) {
  Slots4 s;
  s.count = 0;
  const float* nd = nodes[i].v;
  for (int ch = 0; ch < 2; ++ch) {
    const int32_t r = __float_as_int(nd[12 + ch]);
    if (r == RT_EMPTY_REF) continue;
    if (r < 0) {
      for (int k = 0; k < 3; ++k) {
        s.lo[s.count][k] = nd[4 * k + 2 * ch];
        s.hi[s.count][k] = nd[4 * k + 2 * ch + 1];
      }
      s.ref[s.count++] = r;
      continue;
    }
    const float* cd = nodes[r].v;
    for (int g = 0; g < 2; ++g) {
      const int32_t r2 = __float_as_int(cd[12 + g]);
      if (r2 == RT_EMPTY_REF) continue;
      for (int k = 0; k < 3; ++k) {
        s.lo[s.count][k] = cd[4 * k + 2 * g];
        s.hi[s.count][k] = cd[4 * k + 2 * g + 1];
      }
      s.ref[s.count++] = r2;
    }
  }
  return s;
}

__device__ void phase_collapse(const bvh_build_arg_t* a) {
  const int32_t* parent = vx_ptr<const int32_t>(a->parent_addr);
  const uint32_t* range = vx_ptr<const uint32_t>(a->range_addr);
  const rt_node_t* nodes = vx_ptr<const rt_node_t>(a->nodes_addr);
  rt_node4_t* nodes4 = vx_ptr<rt_node4_t>(a->nodes4_addr);
  uint32_t* bounds = vx_ptr<uint32_t>(a->bounds_addr);
  const int n = (int)a->n, nn = n > 1 ? n - 1 : 1;
  const int gid = blockIdx.x * BVHB_BLOCK + threadIdx.x, gstride = gridDim.x * BVHB_BLOCK;
  uint32_t maxstack = 0;
  for (int i = gid; i < nn; i += gstride) {
    float* o = nodes4[i].v;
    for (int q = 0; q < 32; ++q) o[q] = 0.0f;
    const bool reach = i == 0 || (n > BVHB_LEAF_MAX && range[2 * i + 1] - range[2 * i] + 1 > BVHB_LEAF_MAX);
    if (!reach) continue;
    int depth = 0;
    if (n > BVHB_LEAF_MAX)
      for (int p = i; p != 0; p = parent[p]) ++depth;
    if (depth & 1) continue;
    const Slots4 s = slots4_of(nodes, i);
    for (int q = 0; q < 4; ++q) {
      const bool used = q < s.count;
      for (int k = 0; k < 3; ++k) {
        o[8 * k + q] = used ? s.lo[q][k] : 0.0f;
        o[8 * k + 4 + q] = used ? s.hi[q][k] : 0.0f;
      }
      o[24 + q] = __int_as_float(used ? s.ref[q] : RT_EMPTY_REF);
    }
    uint32_t st = (uint32_t)(s.count > 0 ? s.count - 1 : 0);
    if (n > BVHB_LEAF_MAX)
      for (int p = i; p != 0;) {
        p = parent[parent[p]];  // the BVH4 parent (two BVH2 levels up)
        const int c = slots4_of(nodes, p).count;
        st += (uint32_t)(c > 0 ? c - 1 : 0);
      }
    maxstack = st > maxstack ? st : maxstack;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)maxstack, o, 64);
    maxstack = y > maxstack ? y : maxstack;
  }
  if (lane() == 0 && maxstack) atomicMax(&bounds[8], maxstack);
}

__device__ void phase_half(const bvh_build_arg_t* a) {
  const int n = (int)a->n, nn = n > 1 ? n - 1 : 1;
  rt_node4_t* nodes4 = vx_ptr<rt_node4_t>(a->nodes4_addr);
  uint32_t* half = vx_ptr<uint32_t>(a->nodes4_addr + 128ull * (uint64_t)nn);
  const int gid = blockIdx.x * BVHB_BLOCK + threadIdx.x, gstride = gridDim.x * BVHB_BLOCK;
  for (int i = gid; i < nn; i += gstride) {
    half4_node(nodes4[i].v, half + 16 * i);
  }
}

}  // namespace

VX_MAIN(bvh_build_arg_t, arg, BVHB_BLOCK) {
  switch (arg->phase) {
    case BVHB_BOUNDS: phase_bounds(arg); break;
    case BVHB_MORTON: phase_morton(arg); break;
    case BVHB_HIST: phase_hist(arg); break;
    case BVHB_SCAN: phase_scan(arg); break;
    case BVHB_SCATTER: phase_scatter(arg); break;
    case BVHB_TREE: phase_tree(arg); break;
    case BVHB_BOXES: phase_boxes(arg); break;
    case BVHB_COLLAPSE: phase_collapse(arg); break;
    case BVHB_HALF: phase_half(arg); break;
    default: phase_emit(arg); break;
  }
  return 0;
}
