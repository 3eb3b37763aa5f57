// half4.h -- binary16 box planes of a BVH4 node on the device, shared by the
// two device builders (bvh_build.hip LBVH, bvh_sah.hip binned SAH).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Binary16 box planes for the device tree (app/bvh.cpp HalfRound /
// HalfBits, restated by oracle/lbvh.c orc_half4): each plane rounded
// outward to a binary16 value by exact scaling with its binade's quantum,
// floor (lower planes) or ceil (upper planes), saturating outward past
// +-65504 -- so a rounded box contains the original and the slab test
// accepts every ray the original accepted; the fp32 node keeps the rounded
// values (both layouts describe one tree) and the 64-B half record goes
// behind the rt_node4_t array, where the kernels' F16 node step reads it.
__device__ inline float half_round(float x, int dir) {
  if (__builtin_isnan(x) || __builtin_isinf(x) || x == 0.0f) return x;
  const float kmax = 65504.0f;
  if (x > kmax) return dir < 0 ? kmax : INFINITY;
  if (x < -kmax) return dir < 0 ? -INFINITY : -kmax;
  int e;
  frexpf(fabsf(x), &e);
  const int q = (e - 1 > -14 ? e - 1 : -14) - 10;
  const float m = ldexpf(x, -q);
  const float r = dir < 0 ? floorf(m) : ceilf(m);
  const float v = ldexpf(r, q);
  return v > kmax ? INFINITY : (v < -kmax ? -INFINITY : v);
}

__device__ inline uint32_t half_bits(float v) {
  const uint32_t u = __float_as_uint(v);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const float a = fabsf(v);
  if (a == 0.0f) return sign;
  if (__builtin_isinf(a)) return sign | 0x7c00u;
  int e;
  const float m = frexpf(a, &e);
  if (e - 1 >= -14) return sign | ((uint32_t)(e - 1 + 15) << 10) | (uint32_t)ldexpf(2.0f * m - 1.0f, 10);
  return sign | (uint32_t)ldexpf(a, 24);
}

// one node: planes of rt_node4_t (v, 32 floats) rounded outward in place,
// the 64-B rt_node4h_t record (24 halves + 4 child refs) to h (16 words)
__device__ inline void half4_node(float* v, uint32_t* h) {
#pragma unroll
  for (int k = 0; k < 24; k += 2) {
    const float r0 = half_round(v[k], (k & 4) ? 1 : -1);
    const float r1 = half_round(v[k + 1], ((k + 1) & 4) ? 1 : -1);
    v[k] = r0;
    v[k + 1] = r1;
    h[k / 2] = half_bits(r0) | (half_bits(r1) << 16);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) h[12 + q] = __float_as_uint(v[24 + q]);
}
