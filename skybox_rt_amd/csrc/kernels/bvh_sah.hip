// bvh_sah.hip -- GPU binned-SAH BVH build that reproduces the host builder
// (app/bvh.cpp Builder + Collapser + binary16 planes) bit for bit; the
// phases and the argument block are described in sah_common.h.  Float
// arithmetic follows the host operation for operation (fp32 without
// contraction, the SAH cost in double, x86 float -> int conversion), and
// every reduction is a min / max / count, so no result depends on the
// order the GPU performs it in.
#include <hip/hip_runtime.h>

#include "half4.h"
#include "rt_common.h"
#include "sah_common.h"
#include "vx_spawn.h"

namespace {

constexpr uint32_t kWaves = SAH_BLOCK / 64;
// triangles per thread per pass of a workgroup segment's loops (their loads
// in flight together; a partition round is SAH_ITEMS * SAH_BLOCK triangles,
// whose counts fit the 16-bit halves of one word)
#define SAH_ITEMS 4
static_assert(SAH_ITEMS * SAH_BLOCK < 65536, "partition round counts in 16 bits");

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// float <-> uint preserving the float order (min / max as integer atomics)
__device__ __forceinline__ uint32_t ord(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// (int)x as the host's x86 build computes it (cvttss2si)
__device__ __forceinline__ int cvt_x86(float x) {
  if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT32_MIN;
  return (int)x;
}

__device__ __forceinline__ float comp(const float4& v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

struct Box {  // app/bvh.cpp Box
  float lo[3], hi[3];
  __device__ void empty() {
    for (int k = 0; k < 3; ++k) {
      lo[k] = INFINITY;
      hi[k] = -INFINITY;
    }
  }
  __device__ void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = fminf(lo[k], b.lo[k]);
      hi[k] = fmaxf(hi[k], b.hi[k]);
    }
  }
  __device__ double area() const {  // g_wside = 1 (the default; 1.0 * x == x)
    if (lo[0] > hi[0]) return 0.0;
    const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    return 2.0 * (dx * dy + (dy * dz + dz * dx));
  }
};

__device__ __forceinline__ float scene_pad(const uint32_t* ctl) {
  const float ext = __uint_as_float(ctl[SAH_CTL_EXT]);
  return fmaxf(ext * (1.0f / 65536.0f), 1e-6f);
}

// ---- SAH_INIT --------------------------------------------------------------
__device__ void phase_init(const sah_arg_t* a) {
  const float4* v = vx_ptr<const float4>(a->verts_addr);
  float4* tbox = vx_ptr<float4>(a->tbox_addr);
  float4* cen = vx_ptr<float4>(a->cen_addr);
  uint32_t* idx = vx_ptr<uint32_t>(a->idx_addr[0]);
  uint32_t* cnt = vx_ptr<uint32_t>(a->cnt_addr);
  uint32_t* d0 = vx_ptr<uint32_t>(a->d0_addr);
  uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
  const uint32_t n = a->n;
  float ext = 0.0f;
  for (uint32_t i = blockIdx.x * SAH_BLOCK + threadIdx.x; i <= n; i += gridDim.x * SAH_BLOCK) {
    cnt[i] = 0;
    if (i == n) break;
    d0[i] = 0xffffffffu;
    idx[i] = i;
    const float4 p0 = v[3 * i], p1 = v[3 * i + 1], p2 = v[3 * i + 2];
    const float4 lo = make_float4(fminf(fminf(p0.x, p1.x), p2.x), fminf(fminf(p0.y, p1.y), p2.y),
                                  fminf(fminf(p0.z, p1.z), p2.z), 0.0f);
    const float4 hi = make_float4(fmaxf(fmaxf(p0.x, p1.x), p2.x), fmaxf(fmaxf(p0.y, p1.y), p2.y),
                                  fmaxf(fmaxf(p0.z, p1.z), p2.z), 0.0f);
    tbox[2 * i] = lo;
    tbox[2 * i + 1] = hi;
    cen[i] = make_float4((lo.x + hi.x) * 0.5f, (lo.y + hi.y) * 0.5f, (lo.z + hi.z) * 0.5f, 0.0f);
    ext = fmaxf(ext, fmaxf(fmaxf(fabsf(p0.x), fabsf(p0.y)), fabsf(p0.z)));
    ext = fmaxf(ext, fmaxf(fmaxf(fabsf(p1.x), fabsf(p1.y)), fabsf(p1.z)));
    ext = fmaxf(ext, fmaxf(fmaxf(fabsf(p2.x), fabsf(p2.y)), fabsf(p2.z)));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ext = fmaxf(ext, __shfl_xor(ext, o, 64));
  if (lane_id() == 0 && ext > 0.0f) atomicMax(&ctl[SAH_CTL_EXT], __float_as_uint(ext));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    sah_seg_t* s0 = vx_ptr<sah_seg_t>(a->segs_addr[0]);
    s0[0] = sah_seg_t{0, n, 0, 1};
    ctl[SAH_CTL_SEG + 0] = 1;
    ctl[SAH_CTL_NODES] = 1;
    ctl[SAH_CTL_DEPTH] = 1;
  }
}

// ---- SAH_SPLIT: one workgroup per segment of level `level` -----------------
struct Decision {  // the SAH split of a segment (axis -1: none, the median)
  int axis;
  uint32_t s, nl;
  float box[2][6];                      // child boxes (lo xyz, hi xyz)
};
struct SplitLds {  // a workgroup's segment
  uint32_t cb[6];                       // centroid bounds (ordered uints)
  uint32_t bin[3][SAH_BINS][7];         // lo xyz, hi xyz (ordered), count
  uint32_t side[2][6];                  // child boxes by reduction (median / root)
  Decision dec;
  uint32_t wsum[kWaves], lbase, rbase;  // partition round: per-wave (left | right << 16) counts
};
struct SmallLds {  // a wave's segment (<= SAH_SMALL triangles)
  uint32_t bin[3][SAH_BINS][7];
  Decision dec;
};
union SplitShared {  // the two loops of a SAH_SPLIT launch run one after the other
  SplitLds big;
  SmallLds small[kWaves];
};

__device__ __forceinline__ int bin_of(float c, float cl, float ext) {
  const int bi = cvt_x86((c - cl) * ((float)SAH_BINS / ext));
  return min(max(bi, 0), SAH_BINS - 1);
}

// The SAH decision over a segment's bins (all 64 lanes of one wave): lane i
// prices candidate i = axis * 15 + (split - 1) -- its prefix / suffix boxes
// and counts over the bins, the cost in the host's double arithmetic -- and
// the wave takes the minimum, ties to the lowest index: the host's sequential
// scan keeps the first strict minimum in (axis, split) order (NaN / inf costs
// never win there, so they are +inf here).  The winning lane writes *d; with
// no winner *d is left as the caller set it (axis -1).
__device__ void sah_price(const uint32_t (*bin)[SAH_BINS][7], const float* cl, const float* ch,
                          uint32_t l, Decision* d) {
  const int ax = (int)l / (SAH_BINS - 1), q = (int)l % (SAH_BINS - 1) + 1;
  double c = INFINITY;
  Box lb, rb;
  lb.empty();
  rb.empty();
  uint32_t nl = 0;
  if (l < 3u * (SAH_BINS - 1) && ch[ax] - cl[ax] > 0.0f) {
    uint32_t rc = 0;
    for (int k = 0; k < SAH_BINS; ++k) {
      Box bb;
      for (int e = 0; e < 3; ++e) {
        bb.lo[e] = unord(bin[ax][k][e]);
        bb.hi[e] = unord(bin[ax][k][3 + e]);
      }
      const uint32_t cnt = bin[ax][k][6];
      if (k < q) { lb.grow(bb); nl += cnt; }
      else { rb.grow(bb); rc += cnt; }
    }
    if (nl != 0 && rc != 0) {
      c = (double)nl * lb.area() + (double)rc * rb.area();
      if (!(c < INFINITY)) c = INFINITY;  // NaN / overflow: never chosen
    }
  }
  double cm = c;
  uint32_t im = l;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double oc = __shfl_xor(cm, o, 64);
    const uint32_t oi = (uint32_t)__shfl_xor((int)im, o, 64);
    if (oc < cm || (oc == cm && oi < im)) {
      cm = oc;
      im = oi;
    }
  }
  if (cm < INFINITY && l == im) {
    d->axis = ax;
    d->s = (uint32_t)q;
    d->nl = nl;
    for (int k = 0; k < 3; ++k) {
      d->box[0][k] = lb.lo[k]; d->box[0][3 + k] = lb.hi[k];
      d->box[1][k] = rb.lo[k]; d->box[1][3 + k] = rb.hi[k];
    }
  }
}

// The node record of segment sg (split at b + nl; child boxes bx) and its
// children: <= SAH_LEAF triangles a leaf, <= SAH_SMALL a segment of the
// next level's wave list, else of its workgroup list (one thread).  Node ids
// and next-level slots come in blocks: `need` counts a node's internal
// children (and the small ones among them), `emit_node_at` places them from
// the bases the caller allocated -- every segment of a level bumps the same
// few counter words, so they are bumped once per node (emit_node) or once
// per workgroup round (split_small), and the tree depth once per level
// (phase_split)
__device__ __forceinline__ void node_needs(const sah_seg_t& sg, uint32_t nl, uint32_t* nin, uint32_t* nsmall) {
  const uint32_t m[2] = {nl, sg.e - sg.b - nl};
  *nin = *nsmall = 0;
  for (int q = 0; q < 2; ++q)
    if (m[q] > SAH_LEAF) {
      ++*nin;
      *nsmall += m[q] <= SAH_SMALL ? 1u : 0u;
    }
}
__device__ void emit_node_at(const sah_arg_t* a, uint32_t L, const sah_seg_t& sg, uint32_t nl,
                             const float (*bx)[6], uint32_t id0, uint32_t s_small, uint32_t s_big) {
  uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
  sah_seg_t* next = vx_ptr<sah_seg_t>(a->segs_addr[(L + 1) & 1]);
  sah_seg_t* next_small = vx_ptr<sah_seg_t>(a->small_addr[(L + 1) & 1]);
  int32_t ref[2];
  const uint32_t b = sg.b, e = sg.e;
  const uint32_t cb[2] = {b, b + nl}, ce[2] = {b + nl, e};
  for (int q = 0; q < 2; ++q) {
    const uint32_t m = ce[q] - cb[q];
    if (m == 0) {
      ref[q] = RT_EMPTY_REF;  // only the small root's second child
    } else if (m <= SAH_LEAF) {
      ref[q] = (int32_t)(RT_LEAF_FLAG | (cb[q] << 4) | (m - 1));
    } else {
      const bool small = m <= SAH_SMALL;
      const uint32_t id = id0++;
      const uint32_t slot = small ? s_small++ : s_big++;
      if (id >= a->n || slot >= a->n || L + 2 >= SAH_MAX_LEVELS) {
        atomicOr(&ctl[SAH_CTL_ERR], 1u);
        ref[q] = RT_EMPTY_REF;
        continue;
      }
      (small ? next_small : next)[slot] = sah_seg_t{cb[q], ce[q], id, sg.depth + 1};
      ref[q] = (int32_t)id;
    }
  }
  vx_ptr<uint4>(a->nrec_addr)[sg.node] = make_uint4(b, sg.depth, (uint32_t)ref[0], (uint32_t)ref[1]);
  float4* nb = vx_ptr<float4>(a->nbox_addr) + 4 * sg.node;
  nb[0] = make_float4(bx[0][0], bx[0][1], bx[0][2], 0.0f);
  nb[1] = make_float4(bx[0][3], bx[0][4], bx[0][5], 0.0f);
  nb[2] = make_float4(bx[1][0], bx[1][1], bx[1][2], 0.0f);
  nb[3] = make_float4(bx[1][3], bx[1][4], bx[1][5], 0.0f);
}
__device__ void emit_node(const sah_arg_t* a, uint32_t L, const sah_seg_t& sg, uint32_t nl,
                          const float (*bx)[6]) {
  uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
  uint32_t nin, nsmall;
  node_needs(sg, nl, &nin, &nsmall);
  uint32_t id0 = 0, s_small = 0, s_big = 0;
  if (nin) id0 = atomicAdd(&ctl[SAH_CTL_NODES], nin);
  if (nsmall) s_small = atomicAdd(&ctl[SAH_CTL_SMALL + L + 1], nsmall);
  if (nin > nsmall) s_big = atomicAdd(&ctl[SAH_CTL_SEG + L + 1], nin - nsmall);
  emit_node_at(a, L, sg, nl, bx, id0, s_small, s_big);
}

__device__ __forceinline__ float wmin(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fminf(x, __shfl_xor(x, o, 64));
  return x;
}
__device__ __forceinline__ float wmax(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
  return x;
}

// one thread: the round's node ids and next-level slots for the workgroup's
// waves (their needs in s_need), one atomic per counter
__device__ __forceinline__ void small_alloc(uint32_t* ctl, uint32_t L, const uint32_t (*need)[2],
                                            uint32_t (*base)[3]) {
  uint32_t tin = 0, tsmall = 0;
  for (uint32_t k = 0; k < kWaves; ++k) {
    tin += need[k][0];
    tsmall += need[k][1];
  }
  uint32_t id = tin ? atomicAdd(&ctl[SAH_CTL_NODES], tin) : 0u;
  uint32_t ss = tsmall ? atomicAdd(&ctl[SAH_CTL_SMALL + L + 1], tsmall) : 0u;
  uint32_t sb = tin > tsmall ? atomicAdd(&ctl[SAH_CTL_SEG + L + 1], tin - tsmall) : 0u;
  for (uint32_t k = 0; k < kWaves; ++k) {
    base[k][0] = id;
    base[k][1] = ss;
    base[k][2] = sb;
    id += need[k][0];
    ss += need[k][1];
    sb += need[k][0] - need[k][1];
  }
}

// Segments of <= SAH_SMALL (64) triangles, one per wave (the deep levels'
// thousands of small nodes): a triangle per lane, wave reductions instead of
// workgroup barriers, the bins in the wave's own LDS; the same decisions,
// order and records as the workgroup path.
__device__ void split_small(const sah_arg_t* a, uint32_t L, SmallLds& W, uint32_t w, uint32_t l, uint64_t lt) {
  const uint32_t nseg = vx_ptr<const uint32_t>(a->ctl_addr)[SAH_CTL_SMALL + L];
  const sah_seg_t* segs = vx_ptr<const sah_seg_t>(a->small_addr[L & 1]);
  const uint32_t* idx = vx_ptr<const uint32_t>(a->idx_addr[L & 1]);
  uint32_t* out = vx_ptr<uint32_t>(a->idx_addr[(L + 1) & 1]);
  uint32_t* fin = vx_ptr<uint32_t>(a->final_addr);
  const float4* cen = vx_ptr<const float4>(a->cen_addr);
  const float4* tbox = vx_ptr<const float4>(a->tbox_addr);
  // rounds of one segment per wave, the round's bound workgroup-uniform:
  // the waves' node ids and next-level slots are allocated together
  __shared__ uint32_t s_need[kWaves][2], s_base[kWaves][3];
  uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
  for (uint32_t r0 = blockIdx.x * kWaves; r0 < nseg; r0 += gridDim.x * kWaves) {
    const uint32_t si = r0 + w;
    const bool have = si < nseg;  // wave-uniform: this wave has a segment this round
    sah_seg_t sg{0, 0, 0, 0};
    uint32_t nl = 0;
    float bx[2][6];
    if (have) {
      sg = segs[si];
      const uint32_t b = sg.b, n = sg.e - sg.b;  // 5 .. SAH_SMALL
      const bool valid = l < n;
      const uint32_t i = b + l;
      const uint32_t t = valid ? idx[i] : 0u;
      const float4 c = cen[t], lo = tbox[2 * t], hi = tbox[2 * t + 1];
      float cl[3], ch[3];
      for (int k = 0; k < 3; ++k) {
        cl[k] = wmin(valid ? comp(c, k) : INFINITY);
        ch[k] = wmax(valid ? comp(c, k) : -INFINITY);
      }
      uint32_t* bins = &W.bin[0][0][0];
      for (uint32_t k = l; k < 3 * SAH_BINS * 7; k += 64) {
        const uint32_t f = k % 7;
        bins[k] = f < 3 ? ord(INFINITY) : (f < 6 ? ord(-INFINITY) : 0u);
      }
      if (l == 0) W.dec.axis = -1;
      __builtin_amdgcn_wave_barrier();  // (one wave: its LDS operations complete in order)
      if (valid)
        for (int ax = 0; ax < 3; ++ax) {
          const float ext = ch[ax] - cl[ax];
          if (!(ext > 0.0f)) continue;
          uint32_t* bn = W.bin[ax][bin_of(comp(c, ax), cl[ax], ext)];
          atomicMin(&bn[0], ord(lo.x)); atomicMin(&bn[1], ord(lo.y)); atomicMin(&bn[2], ord(lo.z));
          atomicMax(&bn[3], ord(hi.x)); atomicMax(&bn[4], ord(hi.y)); atomicMax(&bn[5], ord(hi.z));
          atomicAdd(&bn[6], 1u);
        }
      __builtin_amdgcn_wave_barrier();
      sah_price(W.bin, cl, ch, l, &W.dec);
      __builtin_amdgcn_wave_barrier();
      const int axis = W.dec.axis;
      nl = axis >= 0 ? W.dec.nl : n / 2;
      const bool leaf0 = nl <= SAH_LEAF, leaf1 = n - nl <= SAH_LEAF;
      if (axis >= 0) {
        for (int q = 0; q < 2; ++q)
          for (int k = 0; k < 6; ++k) bx[q][k] = W.dec.box[q][k];
        const float ext = ch[axis] - cl[axis];
        const bool f = valid && (uint32_t)bin_of(comp(c, axis), cl[axis], ext) < W.dec.s;
        const bool g = valid && !f;
        const uint64_t mL = __ballot(f), mR = __ballot(g);
        if (valid) {
          const uint32_t dst = f ? b + (uint32_t)__popcll(mL & lt) : b + nl + (uint32_t)__popcll(mR & lt);
          out[dst] = t;
          if (f ? leaf0 : leaf1) fin[dst] = t;
        }
      } else {  // the median: order unchanged, boxes of the two halves
        const bool left = l < nl;
        for (int q = 0; q < 2; ++q) {
          const bool in = valid && (q == 0) == left;
          for (int k = 0; k < 3; ++k) {
            bx[q][k] = wmin(in ? comp(lo, k) : INFINITY);
            bx[q][3 + k] = wmax(in ? comp(hi, k) : -INFINITY);
          }
        }
        if (valid) {
          out[i] = t;
          if (left ? leaf0 : leaf1) fin[i] = t;
        }
      }
    }
    if (l == 0) {
      if (have) {
        node_needs(sg, nl, &s_need[w][0], &s_need[w][1]);
      } else {
        s_need[w][0] = s_need[w][1] = 0;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) small_alloc(ctl, L, s_need, s_base);
    __syncthreads();
    if (have && l == 0) emit_node_at(a, L, sg, nl, bx, s_base[w][0], s_base[w][1], s_base[w][2]);
    __builtin_amdgcn_wave_barrier();  // W is reused by the wave's next segment
  }
}

__device__ void phase_split(const sah_arg_t* a, uint32_t L) {
  uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
  const uint32_t nseg = ctl[SAH_CTL_SEG + L];
  const sah_seg_t* segs = vx_ptr<const sah_seg_t>(a->segs_addr[L & 1]);
  const uint32_t* idx = vx_ptr<const uint32_t>(a->idx_addr[L & 1]);
  uint32_t* out = vx_ptr<uint32_t>(a->idx_addr[(L + 1) & 1]);
  uint32_t* fin = vx_ptr<uint32_t>(a->final_addr);
  const float4* cen = vx_ptr<const float4>(a->cen_addr);
  const float4* tbox = vx_ptr<const float4>(a->tbox_addr);
  __shared__ SplitShared U;
  SplitLds& S = U.big;
  const uint32_t tid = threadIdx.x, w = tid >> 6, l = lane_id();
  // a level-L segment is a node of depth L + 1 (the root: level 0, depth 1)
  if (blockIdx.x == 0 && tid == 0 && nseg + ctl[SAH_CTL_SMALL + L] > 0) atomicMax(&ctl[SAH_CTL_DEPTH], L + 1);
  const uint64_t lt = (l == 0) ? 0ull : (~0ull >> (64 - l));
  for (uint32_t si = blockIdx.x; si < nseg; si += gridDim.x) {
    const sah_seg_t sg = segs[si];
    const uint32_t b = sg.b, e = sg.e, n = e - b;
    // 1. centroid bounds
    if (tid < 6) S.cb[tid] = tid < 3 ? ord(INFINITY) : ord(-INFINITY);
    for (uint32_t k = tid; k < 3 * SAH_BINS * 7; k += SAH_BLOCK) {
      const uint32_t f = k % 7;
      (&S.bin[0][0][0])[k] = f < 3 ? ord(INFINITY) : (f < 6 ? ord(-INFINITY) : 0u);
    }
    if (tid < 12) (&S.side[0][0])[tid] = (tid % 6) < 3 ? ord(INFINITY) : ord(-INFINITY);
    if (tid == 0) {
      S.lbase = S.rbase = 0;
      S.dec.axis = -1;
    }
    __syncthreads();
    float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
    // SAH_ITEMS triangles per thread per pass: their loads in flight together
    for (uint32_t i0 = b + tid; i0 < e; i0 += SAH_ITEMS * SAH_BLOCK) {
      uint32_t t[SAH_ITEMS];
      float4 c[SAH_ITEMS];
#pragma unroll
      for (int j = 0; j < SAH_ITEMS; ++j) t[j] = idx[min(i0 + j * SAH_BLOCK, e - 1)];
#pragma unroll
      for (int j = 0; j < SAH_ITEMS; ++j) c[j] = cen[t[j]];
#pragma unroll
      for (int j = 0; j < SAH_ITEMS; ++j) {  // a clamped duplicate changes no min / max
        cl[0] = fminf(cl[0], c[j].x); cl[1] = fminf(cl[1], c[j].y); cl[2] = fminf(cl[2], c[j].z);
        ch[0] = fmaxf(ch[0], c[j].x); ch[1] = fmaxf(ch[1], c[j].y); ch[2] = fmaxf(ch[2], c[j].z);
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        cl[k] = fminf(cl[k], __shfl_xor(cl[k], o, 64));
        ch[k] = fmaxf(ch[k], __shfl_xor(ch[k], o, 64));
      }
    }
    if (l == 0)
      for (int k = 0; k < 3; ++k) {
        atomicMin(&S.cb[k], ord(cl[k]));
        atomicMax(&S.cb[3 + k], ord(ch[k]));
      }
    __syncthreads();
    for (int k = 0; k < 3; ++k) {
      cl[k] = unord(S.cb[k]);
      ch[k] = unord(S.cb[3 + k]);
    }
    const bool split_node = n > SAH_LEAF;
    // 2. bins over every axis with extent (app/bvh.cpp split)
    if (split_node)
      for (uint32_t i0 = b + tid; i0 < e; i0 += SAH_ITEMS * SAH_BLOCK) {
        uint32_t t[SAH_ITEMS];
        float4 c[SAH_ITEMS], lo[SAH_ITEMS], hi[SAH_ITEMS];
#pragma unroll
        for (int j = 0; j < SAH_ITEMS; ++j) t[j] = idx[min(i0 + j * SAH_BLOCK, e - 1)];
#pragma unroll
        for (int j = 0; j < SAH_ITEMS; ++j) {
          c[j] = cen[t[j]];
          lo[j] = tbox[2 * t[j]];
          hi[j] = tbox[2 * t[j] + 1];
        }
#pragma unroll
        for (int j = 0; j < SAH_ITEMS; ++j) {
          if (i0 + j * SAH_BLOCK >= e) break;  // (the count must not see the clamped duplicates)
          for (int ax = 0; ax < 3; ++ax) {
            const float ext = ch[ax] - cl[ax];
            if (!(ext > 0.0f)) continue;
            uint32_t* bn = S.bin[ax][bin_of(comp(c[j], ax), cl[ax], ext)];
            atomicMin(&bn[0], ord(lo[j].x)); atomicMin(&bn[1], ord(lo[j].y)); atomicMin(&bn[2], ord(lo[j].z));
            atomicMax(&bn[3], ord(hi[j].x)); atomicMax(&bn[4], ord(hi[j].y)); atomicMax(&bn[5], ord(hi[j].z));
            atomicAdd(&bn[6], 1u);
          }
        }
      }
    __syncthreads();
    // 3. the SAH decision (wave 0)
    if (w == 0 && split_node) sah_price(S.bin, cl, ch, l, &S.dec);
    __syncthreads();
    const int axis = S.dec.axis;
    // the root of <= 4 triangles: one leaf child and an empty one; no SAH
    // split: the median, order unchanged
    const uint32_t nl = !split_node ? n : (axis >= 0 ? S.dec.nl : n / 2);
    if (axis < 0) {  // child boxes by reduction over the two halves
      float bl[2][6];
      for (int q = 0; q < 2; ++q)
        for (int k = 0; k < 3; ++k) {
          bl[q][k] = INFINITY;
          bl[q][3 + k] = -INFINITY;
        }
      for (uint32_t i = b + tid; i < e; i += SAH_BLOCK) {
        const uint32_t t = idx[i];
        const int q = i < b + nl ? 0 : 1;
        const float4 lo = tbox[2 * t], hi = tbox[2 * t + 1];
        for (int k = 0; k < 3; ++k) {
          bl[q][k] = fminf(bl[q][k], comp(lo, k));
          bl[q][3 + k] = fmaxf(bl[q][3 + k], comp(hi, k));
        }
      }
      for (int q = 0; q < 2; ++q)
        for (int k = 0; k < 6; ++k) {
          float x = bl[q][k];
#pragma unroll
          for (int o = 32; o > 0; o >>= 1)
            x = k < 3 ? fminf(x, __shfl_xor(x, o, 64)) : fmaxf(x, __shfl_xor(x, o, 64));
          if (l == 0) {
            if (k < 3) atomicMin(&S.side[q][k], ord(x));
            else atomicMax(&S.side[q][k], ord(x));
          }
        }
      __syncthreads();
      if (tid < 12) (&S.dec.box[0][0])[tid] = unord((&S.side[0][0])[tid]);
    }
    __syncthreads();
    const bool leaf0 = nl <= SAH_LEAF, leaf1 = n - nl <= SAH_LEAF;
    // 4. the children's triangle order: a stable partition by the split bin
    //    (ballot ranks, rounds of SAH_BLOCK in order), else a copy; leaf
    //    ranges also go to the final order
    if (axis >= 0) {
      // rounds of SAH_ITEMS * SAH_BLOCK triangles, thread tid holding the
      // round's items SAH_ITEMS * tid .. + SAH_ITEMS - 1 (so thread order is
      // triangle order): each thread's (left | right << 16) count, their
      // exclusive prefix over the workgroup (a wave scan, then the waves'
      // sums), the items placed in order from there
      const float ext = ch[axis] - cl[axis];
      for (uint32_t r0 = b; r0 < e; r0 += SAH_ITEMS * SAH_BLOCK) {
        const uint32_t i0 = r0 + SAH_ITEMS * tid;
        uint32_t t[SAH_ITEMS];
        float4 c[SAH_ITEMS];
#pragma unroll
        for (int j = 0; j < SAH_ITEMS; ++j) t[j] = idx[min(i0 + j, e - 1)];
#pragma unroll
        for (int j = 0; j < SAH_ITEMS; ++j) c[j] = cen[t[j]];
        uint32_t fl = 0, cnt = 0;  // left bits; (left | right << 16)
#pragma unroll
        for (int j = 0; j < SAH_ITEMS; ++j) {
          if (i0 + j >= e) break;
          const bool f = (uint32_t)bin_of(comp(c[j], axis), cl[axis], ext) < S.dec.s;
          fl |= f ? 1u << j : 0u;
          cnt += f ? 1u : 0x10000u;
        }
        uint32_t inc = cnt;  // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
          if (l >= (uint32_t)o) inc += y;
        }
        if (l == 63) S.wsum[w] = inc;
        __syncthreads();
        uint32_t pre = inc - cnt, tot = 0;
        for (uint32_t k = 0; k < kWaves; ++k) {
          const uint32_t ws = S.wsum[k];
          pre += k < w ? ws : 0u;
          tot += ws;
        }
        uint32_t offL = b + S.lbase + (pre & 0xffffu), offR = b + nl + S.rbase + (pre >> 16);
#pragma unroll
        for (int j = 0; j < SAH_ITEMS; ++j) {
          if (i0 + j >= e) break;
          const bool f = (fl >> j) & 1u;
          const uint32_t dst = f ? offL++ : offR++;
          out[dst] = t[j];
          if (f ? leaf0 : leaf1) fin[dst] = t[j];
        }
        __syncthreads();
        if (tid == 0) {
          S.lbase += tot & 0xffffu;
          S.rbase += tot >> 16;
        }
        __syncthreads();
      }
    } else {
      for (uint32_t i = b + tid; i < e; i += SAH_BLOCK) {
        const uint32_t t = idx[i];
        out[i] = t;
        if (i < b + nl ? leaf0 : leaf1) fin[i] = t;
      }
    }
    // 5. the node record and the next level's segments
    if (tid == 0) emit_node(a, L, sg, nl, S.dec.box);
    __syncthreads();
  }
  __syncthreads();  // the union's other member from here on
  split_small(a, L, U.small[w], w, l, lt);
}

// ---- preorder numbering ------------------------------------------------------
__device__ void phase_number(const sah_arg_t* a) {
  const uint4* nrec = vx_ptr<const uint4>(a->nrec_addr);
  uint32_t* cnt = vx_ptr<uint32_t>(a->cnt_addr);
  uint32_t* d0 = vx_ptr<uint32_t>(a->d0_addr);
  const uint32_t nodes = vx_ptr<const uint32_t>(a->ctl_addr)[SAH_CTL_NODES];
  for (uint32_t x = blockIdx.x * SAH_BLOCK + threadIdx.x; x < nodes; x += gridDim.x * SAH_BLOCK) {
    const uint4 r = nrec[x];
    atomicAdd(&cnt[r.x], 1u);
    atomicMin(&d0[r.x], r.y);
  }
}

// exclusive scan of u32 [total] in place, total at [total] (workgroup 0:
// contiguous chunks per thread, a workgroup scan of the chunk sums)
__device__ void phase_scan(uint32_t* x, uint32_t total) {
  if (blockIdx.x != 0) return;
  __shared__ uint32_t s[SAH_BLOCK];
  const uint32_t chunk = (total + SAH_BLOCK - 1) / SAH_BLOCK;
  const uint32_t b0 = min(threadIdx.x * chunk, total), b1 = min(b0 + chunk, total);
  uint32_t sum = 0;
  uint32_t i = b0;
  for (; i + 8 <= b1; i += 8) {  // eight loads in flight
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[i + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += v[j];
  }
  for (; i < b1; ++i) sum += x[i];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < SAH_BLOCK; o <<= 1) {
    const uint32_t y = threadIdx.x >= o ? s[threadIdx.x - o] : 0u;
    __syncthreads();
    s[threadIdx.x] += y;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - sum;
  for (i = b0; i + 8 <= b1; i += 8) {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[i + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x[i + j] = run;
      run += v[j];
    }
  }
  for (; i < b1; ++i) {
    const uint32_t v = x[i];
    x[i] = run;
    run += v;
  }
  if (threadIdx.x == SAH_BLOCK - 1) x[total] = s[SAH_BLOCK - 1];
}

// preorder index of BFS node x: its rank in (first position, depth) order
__device__ __forceinline__ uint32_t pre_of(const uint4* nrec, const uint32_t* P, const uint32_t* d0,
                                           uint32_t x) {
  const uint4 r = nrec[x];
  return P[r.x] + r.y - d0[r.x];
}

__device__ void phase_emit(const sah_arg_t* a) {
  const uint4* nrec = vx_ptr<const uint4>(a->nrec_addr);
  const float4* nbox = vx_ptr<const float4>(a->nbox_addr);
  const uint32_t* P = vx_ptr<const uint32_t>(a->cnt_addr);
  const uint32_t* d0 = vx_ptr<const uint32_t>(a->d0_addr);
  const uint32_t* ctl = vx_ptr<const uint32_t>(a->ctl_addr);
  int32_t* parent = vx_ptr<int32_t>(a->parent_addr);
  float4* nodes = vx_ptr<float4>(a->nodes_addr);
  const uint32_t nodes_n = ctl[SAH_CTL_NODES];
  const float pad = scene_pad(ctl);
  const uint32_t gid = blockIdx.x * SAH_BLOCK + threadIdx.x, gs = gridDim.x * SAH_BLOCK;
  for (uint32_t x = gid; x < nodes_n; x += gs) {
    const uint4 r = nrec[x];
    const uint32_t px = pre_of(nrec, P, d0, x);
    if (x == 0) parent[px] = -1;
    int32_t ref[2] = {(int32_t)r.z, (int32_t)r.w};
    float v[16];
    for (int q = 0; q < 2; ++q) {
      const bool empty = ref[q] == RT_EMPTY_REF;
      const float4 lo = nbox[4 * x + 2 * q], hi = nbox[4 * x + 2 * q + 1];
      for (int k = 0; k < 3; ++k) {
        v[4 * k + 2 * q + 0] = empty ? 0.0f : comp(lo, k) - pad;
        v[4 * k + 2 * q + 1] = empty ? 0.0f : comp(hi, k) + pad;
      }
      if (ref[q] >= 0) {
        const uint32_t py = pre_of(nrec, P, d0, (uint32_t)ref[q]);
        parent[py] = (int32_t)px;
        ref[q] = (int32_t)py;
      }
      v[12 + q] = __int_as_float(ref[q]);
    }
    v[14] = v[15] = 0.0f;
    float4* o = nodes + 4 * px;
    for (int q = 0; q < 4; ++q) o[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  // triangle records in leaf order (+3 zero padding records)
  const uint32_t* fin = vx_ptr<const uint32_t>(a->final_addr);
  const float4* geom = vx_ptr<const float4>(a->geom_addr);
  float4* tris = vx_ptr<float4>(a->tris_addr);
  for (uint32_t i = gid; i < a->n + 3; i += gs) {
    const bool pad_rec = i >= a->n;
    const uint32_t t = pad_rec ? 0u : fin[i];
    for (int q = 0; q < 3; ++q) tris[3 * i + q] = pad_rec ? make_float4(0, 0, 0, 0) : geom[3 * t + q];
  }
}

// ---- BVH4 collapse (app/bvh.cpp Collapser) ---------------------------------
struct Child {
  float lo[3], hi[3];
  int32_t ref, src;  // src = BVH2 node << 1 | slot holding the box
};

__device__ __forceinline__ Child child_of(const float* nodes, uint32_t p, int ch) {
  const float* v = nodes + 16ull * p;
  Child c;
  for (int k = 0; k < 3; ++k) {
    c.lo[k] = v[4 * k + 2 * ch];
    c.hi[k] = v[4 * k + 2 * ch + 1];
  }
  c.ref = __float_as_int(v[12 + ch]);
  c.src = (int32_t)(2 * p + ch);
  return c;
}

__device__ __forceinline__ double child_area(const Child& c) {
  const double dx = (double)c.hi[0] - c.lo[0], dy = (double)c.hi[1] - c.lo[1],
               dz = (double)c.hi[2] - c.lo[2];
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}

// the expansion of every BVH2 node for a W-wide collapse (W = 4: cs): W
// refs, then W sources (node << 1 | slot)
template <int W>
__device__ void phase_cs(const sah_arg_t* a) {
  const float* nodes = vx_ptr<const float>(a->nodes_addr);
  int32_t* cs = vx_ptr<int32_t>(a->cs_addr);
  const uint32_t nn = vx_ptr<const uint32_t>(a->ctl_addr)[SAH_CTL_NODES];
  for (uint32_t p = blockIdx.x * SAH_BLOCK + threadIdx.x; p < nn; p += gridDim.x * SAH_BLOCK) {
    Child c[W];
    int m = 0;
    for (int ch = 0; ch < 2; ++ch) {
      const Child x = child_of(nodes, p, ch);
      if (x.ref != RT_EMPTY_REF) c[m++] = x;
    }
    while (m < W) {
      int best = -1;
      double ba = -1.0;
      for (int i = 0; i < m; ++i)
        if (c[i].ref >= 0 && child_area(c[i]) > ba) {
          ba = child_area(c[i]);
          best = i;
        }
      if (best < 0) break;
      const uint32_t q = (uint32_t)c[best].ref;
      Child sub[2];
      int ns = 0;
      for (int ch = 0; ch < 2; ++ch) {
        const Child x = child_of(nodes, q, ch);
        if (x.ref != RT_EMPTY_REF) sub[ns++] = x;
      }
      // erase c[best], insert sub there (m - 1 + ns <= W)
      Child t[W];
      int k = 0;
      for (int i = 0; i < best; ++i) t[k++] = c[i];
      for (int i = 0; i < ns; ++i) t[k++] = sub[i];
      for (int i = best + 1; i < m; ++i) t[k++] = c[i];
      for (int i = 0; i < k; ++i) c[i] = t[i];
      m = k;
    }
    int32_t* o = cs + 2ull * W * p;
    for (int i = 0; i < W; ++i) {
      o[i] = i < m ? c[i].ref : RT_EMPTY_REF;
      o[W + i] = i < m ? c[i].src : -1;
    }
  }
}

// BVH4 membership: walk the node's root path down, following the BVH4 node
// whose expansion the path is in; depth and the worst-case stack (the sum of
// (children - 1) over the BVH4 nodes of the path) of every BVH4 node.  The
// path is kept as one bit per step (no per-thread array, which would live in
// scratch memory): in preorder a node's first internal child is the node
// right after it, so the way up records whether each step came from that
// child (bit 0) or from the other one (bit 1, its id read from the parent's
// record on the way down).
template <int W>
__device__ void phase_mark(const sah_arg_t* a) {
  const int32_t* parent = vx_ptr<const int32_t>(a->parent_addr);
  const int32_t* cs = vx_ptr<const int32_t>(a->cs_addr);
  const int32_t* nodes = vx_ptr<const int32_t>(a->nodes_addr);  // rt_node_t: refs at words 12, 13
  uint32_t* is4 = vx_ptr<uint32_t>(a->is4_addr);
  uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
  const uint32_t nn = ctl[SAH_CTL_NODES];
  // the BVH4 depth and stack maxima: per lane over its nodes, then one
  // atomic per wave (one per member node serialised on the two words)
  uint32_t dmax = 0, smax = 0;
  for (uint32_t m = blockIdx.x * SAH_BLOCK + threadIdx.x; m < nn; m += gridDim.x * SAH_BLOCK) {
    uint64_t bits = 0;
    int len = 0;
    int32_t x = (int32_t)m;
    while (x > 0 && len < SAH_MAX_LEVELS - 1) {
      const int32_t p = parent[x];
      if (x != p + 1) bits |= 1ull << len;
      ++len;
      x = p;
    }
    if (x != 0) {  // no root within the level table
      atomicOr(&ctl[SAH_CTL_ERR], 2u);
      is4[m] = 0;
      continue;
    }
    // a BVH4 (BVH8) node's children: the expansion's refs (one (two) 16-B
    // loads); their count = the refs before the first empty one
    const int4* cs4 = reinterpret_cast<const int4*>(cs);
    auto nch4 = [](const int4& r) {
      return r.x == RT_EMPTY_REF ? 0u : r.y == RT_EMPTY_REF ? 1u : r.z == RT_EMPTY_REF ? 2u : r.w == RT_EMPTY_REF ? 3u : 4u;
    };
    constexpr int Q = W / 4;  // int4 words of refs per expansion
    struct Refs {
      int4 r[Q];
    };
    auto load = [&](int32_t node) {
      Refs x;
      for (int q = 0; q < Q; ++q) x.r[q] = cs4[(2 * W / 4) * node + q];
      return x;
    };
    auto nch = [&](const Refs& x) {
      uint32_t n = 0;
      for (int q = 0; q < Q; ++q) {
        const uint32_t k = nch4(x.r[q]);
        n += (n == 4u * q) ? k : 0u;  // counts stop at the first empty ref
      }
      return n;
    };
    auto has = [&](const Refs& x, int32_t c) {
      bool in = false;
      for (int q = 0; q < Q; ++q) in = in || x.r[q].x == c || x.r[q].y == c || x.r[q].z == c || x.r[q].w == c;
      return in;
    };
    Refs cc = load(0);  // the root's expansion
    int32_t p = 0;
    uint32_t depth4 = 1, stack = nch(cc) > 0 ? nch(cc) - 1 : 0;
    bool member = len == 0;
    for (int k = len - 1; k >= 0; --k) {
      const int32_t c = ((bits >> k) & 1ull) ? nodes[16 * p + 13] : p + 1;
      const bool in = has(cc, c);
      if (in) {
        cc = load(c);
        ++depth4;
        const uint32_t n4 = nch(cc);
        stack += n4 > 0 ? n4 - 1 : 0;
      }
      if (k == 0) member = in;
      p = c;
    }
    is4[m] = member ? 1u : 0u;
    if (member) {
      dmax = max(dmax, depth4);
      smax = max(smax, stack);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    dmax = max(dmax, (uint32_t)__shfl_xor((int)dmax, o, 64));
    smax = max(smax, (uint32_t)__shfl_xor((int)smax, o, 64));
  }
  if (lane_id() == 0 && dmax != 0) {
    atomicMax(&ctl[SAH_CTL_DEPTH4], dmax);
    atomicMax(&ctl[SAH_CTL_STACK4], smax);
  }
}

__device__ void phase_emit4(const sah_arg_t* a) {
  const float* nodes = vx_ptr<const float>(a->nodes_addr);
  const int32_t* cs = vx_ptr<const int32_t>(a->cs_addr);
  const uint32_t* pre4 = vx_ptr<const uint32_t>(a->is4_addr);
  rt_node4_t* nodes4 = vx_ptr<rt_node4_t>(a->nodes4_addr);
  uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
  const uint32_t nn = ctl[SAH_CTL_NODES];
  // the binary16 records (rt_node4h_t) follow the nn4 rt_node4_t records
  const uint32_t nn4 = pre4[nn];  // the membership scan's total
  uint32_t* half = vx_ptr<uint32_t>(a->nodes4_addr + 128ull * (uint64_t)nn4);
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[SAH_CTL_NODES4] = nn4;
  for (uint32_t m = blockIdx.x * SAH_BLOCK + threadIdx.x; m < nn; m += gridDim.x * SAH_BLOCK) {
    if (pre4[m + 1] == pre4[m]) continue;  // not a BVH4 node
    float v[32];
    for (int i = 0; i < 32; ++i) v[i] = 0.0f;
    for (int i = 0; i < 4; ++i) {
      int32_t ref = cs[8 * m + i];
      const int32_t src = cs[8 * m + 4 + i];
      if (ref != RT_EMPTY_REF) {
        const float* s = nodes + 16ull * (uint32_t)(src >> 1);
        const int ch = src & 1;
        for (int k = 0; k < 3; ++k) {
          v[8 * k + i] = s[4 * k + 2 * ch];
          v[8 * k + 4 + i] = s[4 * k + 2 * ch + 1];
        }
        if (ref >= 0) ref = (int32_t)pre4[ref];
      }
      v[24 + i] = __int_as_float(ref);
    }
    // the planes rounded outward to binary16 (in v: the fp32 record keeps
    // the rounded planes too) and the half record
    half4_node(v, half + 16ull * pre4[m]);
    float4* o = reinterpret_cast<float4*>(nodes4 + pre4[m]);
    for (int q = 0; q < 8; ++q) o[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
}

// the numbering's counters as SAH_INIT leaves them, and the collapse's
// maxima (a sequence that ran its finishing phases before its last level)
__device__ void phase_reset(const sah_arg_t* a) {
  uint32_t* cnt = vx_ptr<uint32_t>(a->cnt_addr);
  uint32_t* d0 = vx_ptr<uint32_t>(a->d0_addr);
  for (uint32_t i = blockIdx.x * SAH_BLOCK + threadIdx.x; i <= a->n; i += gridDim.x * SAH_BLOCK) {
    cnt[i] = 0;
    if (i < a->n) d0[i] = 0xffffffffu;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t* ctl = vx_ptr<uint32_t>(a->ctl_addr);
    ctl[SAH_CTL_DEPTH4] = 0;
    ctl[SAH_CTL_STACK4] = 0;
    ctl[SAH_CTL_ERR] &= ~2u;
  }
}

}  // namespace

// Launch i of the host's sequence runs seq[i] (its launch tag).  The
// sequence's steps are launches queued back to back on the driver's stream:
// each launch boundary makes one step's stores visible to the next (per-XCD
// L2s are not coherent within a launch); counts a step needs (segments of a
// level, nodes, BVH4 nodes) are read from device memory, never from the host.
VX_MAIN(sah_arg_t, arg, SAH_BLOCK) {
  if (vx_launch_tag >= arg->nseq || vx_launch_tag >= SAH_MAX_SEQ) return 0;
  const uint32_t e = arg->seq[vx_launch_tag];
  const uint32_t L = e >> 8;
  const uint32_t ph = e & 0xffu;
  // the finishing phases carry the level after the sequence's last split
  // level: while that level still holds segments the tree is partial (deeper
  // than the host's level budget) -- node ids of the last split level have no
  // records yet -- so they do nothing; the host continues with SAH_RESET, the
  // next levels and the finishing phases again
  if (ph != SAH_INIT && ph != SAH_SPLIT && ph != SAH_RESET && L < SAH_MAX_LEVELS) {
    const uint32_t* ctl = vx_ptr<const uint32_t>(arg->ctl_addr);
    if (ctl[SAH_CTL_SEG + L] != 0 || ctl[SAH_CTL_SMALL + L] != 0) return 0;
  }
  switch (ph) {
    case SAH_INIT: phase_init(arg); break;
    case SAH_SPLIT: phase_split(arg, L); break;
    case SAH_NUMBER: phase_number(arg); break;
    case SAH_SCAN: phase_scan(vx_ptr<uint32_t>(arg->cnt_addr), arg->n); break;
    case SAH_EMIT: phase_emit(arg); break;
    case SAH_CS: phase_cs<4>(arg); break;
    case SAH_MARK: phase_mark<4>(arg); break;
    case SAH_EMIT4: phase_emit4(arg); break;
    case SAH_RESET: phase_reset(arg); break;
    case SAH_SCAN4:
      phase_scan(vx_ptr<uint32_t>(arg->is4_addr), vx_ptr<const uint32_t>(arg->ctl_addr)[SAH_CTL_NODES]);
      break;
    default: break;
  }
  return 0;
}
