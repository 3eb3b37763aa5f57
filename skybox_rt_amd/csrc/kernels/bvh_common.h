// bvh_common.h -- argument block of the GPU BVH builder (bvh_build.hip),
// shared with the host (app/rt_app.cpp rt_renderer_build_bvh).
//
// NO REFERENCE (the reference has no BVH; SURVEY.md 8(f) rank 2 "GPU-side
// ingestion + BVH build").  A linear BVH (Karras 2012): Morton codes of the
// triangle centroids, a stable LSD radix sort, the binary radix tree over
// the sorted codes, bottom-up boxes; subtrees of <= 4 triangles become
// leaves.  Output = the rt_node_t / rt_tri_t layout the traversal reads.
#pragma once

#include <stdint.h>

#define BVHB_BLOCK 256
#define BVHB_ITEMS 1024          // sort items per block (4 per thread)
#define BVHB_LEAF_MAX 4          // subtrees of up to 4 triangles become one leaf

enum {
  BVHB_BOUNDS = 0,   // centroid bounds + max |coordinate| (float atomics as ordered uints)
  BVHB_MORTON = 1,   // 30-bit Morton codes, values = triangle index
  BVHB_HIST = 2,     // radix pass `pass`: per-block digit histogram
  BVHB_SCAN = 3,     //   exclusive scan of the histograms (digit-major)
  BVHB_SCATTER = 4,  //   stable scatter
  BVHB_TREE = 5,     // binary radix tree (internal nodes: ranges, children, parents)
  BVHB_BOXES = 6,    // bottom-up boxes (agent-scope counters, no spinning)
  BVHB_EMIT = 7,     // rt_node_t / rt_tri_t records, depth
  BVHB_COLLAPSE = 8, // rt_node4_t: every even-depth node absorbs its internal children
  BVHB_HALF = 9,     // binary16 planes: rt_node4_t rounded outward in place + rt_node4h_t
                     //   records right behind the rt_node4_t array
};

typedef struct {
  uint64_t verts_addr;    // float4 [n][3]: clip (x, y, w, 0) per corner
  uint64_t geom_addr;     // rt_tri_t [n]: the same triangles as records (v0, e1, e2, pid)
  uint64_t cen_addr;      // float4 [n]: centroid
  uint64_t keys_addr[2];  // u32 [n] Morton codes (ping-pong)
  uint64_t vals_addr[2];  // u32 [n] triangle indices
  uint64_t hist_addr;     // u32 [256][nblocks]
  uint64_t bounds_addr;   // u32 [10]: ordered-uint min xyz, max xyz, max |coord|, depth,
                          //   BVH4 worst-case traversal stack, pad
  uint64_t parent_addr;   // i32 [2n]: parent of internal node i at [i], of leaf k at [n + k]
  uint64_t flags_addr;    // u32 [n]: arrival counters of the bottom-up pass
  uint64_t boxes_addr;    // float4 [2n][2]: lo, hi of internal node i at [i], of leaf k at [n + k]
  uint64_t range_addr;    // u32 [n][2]: first, last sorted triangle under internal node i
  uint64_t child_addr;    // i32 [n][2]: children (>= 0 internal, else ~leaf)
  uint64_t nodes_addr;    // rt_node_t [max(n - 1, 1)]
  uint64_t tris_addr;     // rt_tri_t [n + 3]
  uint64_t nodes4_addr;   // rt_node4_t [max(n - 1, 1)]: BVH4 node at the BVH2 index of
                          //   every even-depth internal node, zeros elsewhere; then
                          //   rt_node4h_t [max(n - 1, 1)] (BVHB_HALF)
  uint32_t n, phase, pass, nblocks;
} bvh_build_arg_t;
