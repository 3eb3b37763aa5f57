// bvh.h -- deterministic binned-SAH BVH2 builder (host).
//
// NO REFERENCE: the reference has no ray tracer; its
// acceleration structure for the same scenes is the screen-tile binning of
// gfxutil.cpp:237-250.  The BVH is built once per scene in clip (x, y, w)
// space, so it is independent of the render resolution.  Boxes are padded by
// 2^-16 of the scene extent so that fp32 slab tests are conservative for every
// hit the (inclusive) Möller–Trumbore test can report.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../kernels/rt_common.h"

namespace rt {

struct BuildTri {
  float v[3][3];  // clip-space (x, y, w) of the three corners
  int32_t pid;    // global primitive id
};

struct Bvh {
  std::vector<rt_node_t> nodes;  // root = 0 (empty if no triangles)
  std::vector<rt_tri_t> tris;    // leaf order
  uint32_t depth = 0;            // internal levels on the deepest path
  uint32_t leaves = 0;
  // BVH4 collapsed from `nodes` (same leaves; the padded boxes rounded outward
  // to binary16-representable values, see f16_boxes); root = 0
  std::vector<rt_node4_t> nodes4;
  std::vector<rt_node4h_t> nodes4h;  // the same nodes, binary16 boxes (the kernel's form)
  uint32_t depth4 = 0;
  uint32_t stack4 = 0;           // worst-case traversal stack entries (near-first, BVH4)
};

constexpr uint32_t kBvhLeafSize = 4;   // the kernel fetches at most 4 triangles per leaf
constexpr uint32_t kBvhBins = 16;
constexpr uint32_t kBvhMaxBins = 64;

struct BvhParams {
  uint32_t leaf_size = kBvhLeafSize;   // max triangles per leaf (1..4)
  uint32_t bins = kBvhBins;            // SAH bins per axis (2..64)
  bool all_axes = true;                // SAH over x, y and w, not only the widest axis
  bool f16_boxes = true;               // BVH4 boxes rounded outward to binary16 values
};

int BuildBvh(const std::vector<BuildTri>& tris, Bvh* out, std::string* error);
// the same with explicit parameters (no environment knobs)
int BuildBvhWith(const std::vector<BuildTri>& tris, const BvhParams& bp, Bvh* out, std::string* error);

}  // namespace rt
