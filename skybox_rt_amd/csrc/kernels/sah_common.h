// sah_common.h -- argument block of the GPU binned-SAH BVH builder
// (bvh_sah.hip), shared with the host (app/rt_app.cpp rt_renderer_build_bvh_ex).
//
// NO REFERENCE.  The device restatement of the host
// builder app/bvh.cpp (binned SAH over all three clip axes, 16 bins, leaves
// of <= 4 triangles, stable partitions, boxes padded by 2^-16 of the scene
// extent; the BVH4 collapse that repeatedly opens the largest-area internal
// child; binary16 planes) that produces the host's arrays bit for bit:
//   * one stream-ordered launch sequence (launch i runs seq[i]: its launch
//     tag, vx_spawn.h), the host reading the control words once at the end;
//   * top-down, one launch per tree level: a workgroup per node (segment of
//     the triangle order; a wave per node of <= 64 triangles) computes the
//     centroid bounds, the 3 x 16 bins in LDS, the SAH decision (45
//     candidates priced by 45 lanes in the host's double arithmetic, the
//     first minimum in the host's order) and the stable partition (ballot
//     ranks) into the other triangle-order buffer;
//   * the host numbers nodes in depth-first preorder; an internal node's
//     preorder index is its rank in (first triangle position, depth) order --
//     the nodes starting at one position form a chain of left children -- so
//     it is a prefix sum over positions plus the depth within the chain;
//   * the BVH4 collapse per BVH2 node (its expansion), membership by a walk
//     down the node's root path, BVH4 preorder = the BVH2 preorder
//     restricted to BVH4 nodes (a prefix sum).
#pragma once

#include <stdint.h>

#ifndef SAH_BLOCK
#define SAH_BLOCK 256
#endif
#define SAH_BINS 16
#define SAH_LEAF 4
#define SAH_SMALL 64             // segments up to this many triangles: one wave each
#define SAH_MAX_LEVELS 64
#define SAH_MAX_SEQ 96           // launches of one sequence

enum {
  SAH_INIT = 0,    // triangle boxes, centroids, extent; root segment; counters
  SAH_SPLIT = 1,   // level `level`: every segment of the level split by a workgroup
  SAH_NUMBER = 2,  // per internal node: count / min depth at its first position
  SAH_SCAN = 3,    // exclusive scan of u32 [count] at scan_addr (workgroup 0)
  SAH_EMIT = 4,    // rt_node_t at preorder indices, parents, rt_tri_t in leaf order
  SAH_CS = 5,      // BVH4 expansion of every BVH2 node
  SAH_MARK = 6,    // BVH4 membership, depth, worst-case stack (root-path walks)
  SAH_EMIT4 = 7,   // rt_node4_t at BVH4 preorder indices, planes rounded outward to binary16,
                   // and the rt_node4h_t records behind the rt_node4_t array
                   // (8: the binary16 pass, folded into SAH_EMIT4 in r04)
  SAH_RESET = 9,   // the numbering's counters again (a sequence continued past its level budget)
  SAH_SCAN4 = 10,  // exclusive scan of the BVH4 membership (is4, one word per BVH2 node)
};
// a sequence entry: the phase, and the tree level of a SAH_SPLIT
#define SAH_SEQ(phase, level) ((uint32_t)(phase) | ((uint32_t)(level) << 8))

// ctl words (u32)
#define SAH_CTL_NODES 0    // BFS node ids allocated
#define SAH_CTL_DEPTH 1    // max internal depth (root 1)
#define SAH_CTL_EXT 2      // max |coordinate| (float bits, non-negative)
#define SAH_CTL_DEPTH4 3   // BVH4 depth
#define SAH_CTL_STACK4 4   // BVH4 worst-case traversal stack
#define SAH_CTL_ERR 5      // != 0: capacity / depth overflow
#define SAH_CTL_NODES4 6   // BVH4 nodes (SAH_EMIT4: the membership scan's total)
#define SAH_CTL_SEG 8      // [SAH_CTL_SEG + L]: workgroup segments of level L
#define SAH_CTL_SMALL (SAH_CTL_SEG + SAH_MAX_LEVELS + 1)  // [.. + L]: wave segments of level L
#define SAH_CTL_WORDS (SAH_CTL_SMALL + SAH_MAX_LEVELS + 1)

typedef struct {
  uint32_t b, e, node, depth;
} sah_seg_t;

typedef struct {
  uint64_t verts_addr;    // float4 [n][3]: clip (x, y, w, 0) per corner (BuildTri order)
  uint64_t geom_addr;     // rt_tri_t [n]: the same triangles as records (v0, e1, e2, pid)
  uint64_t tbox_addr;     // float4 [n][2]: triangle box lo, hi
  uint64_t cen_addr;      // float4 [n]: centroid
  uint64_t idx_addr[2];   // u32 [n]: triangle order, ping-pong per level
  uint64_t final_addr;    // u32 [n]: the final order (leaf ranges written when created)
  uint64_t segs_addr[2];  // sah_seg_t [n]: workgroup segments of the current / next level
  uint64_t small_addr[2]; // sah_seg_t [n]: wave segments (<= SAH_SMALL triangles)
  uint64_t nrec_addr;     // u32 [n][4]: BFS node: b, depth, ref0, ref1 (ref: > 0 BFS id,
                          //   < -1 leaf, -1 empty)
  uint64_t nbox_addr;     // float4 [n][4]: child 0 lo, hi, child 1 lo, hi (unpadded)
  uint64_t cnt_addr;      // u32 [n + 1]: internal nodes per first position -> scan
  uint64_t d0_addr;       // u32 [n]: min depth of the nodes at a first position
  uint64_t parent_addr;   // i32 [n]: BVH2 preorder parent (-1 root)
  uint64_t cs_addr;       // i32 [n][8]: BVH4 expansion: 4 refs, 4 sources (node << 1 | slot)
  uint64_t is4_addr;      // u32 [n + 1]: BVH4 membership -> scan -> BVH4 preorder
  uint64_t ctl_addr;      // u32 [SAH_CTL_WORDS]
  uint64_t nodes_addr;    // rt_node_t [max(n, 1)] (nn = ctl[SAH_CTL_NODES] used)
  uint64_t tris_addr;     // rt_tri_t [n + 3]
  uint64_t nodes4_addr;   // rt_node4_t [nn4], then rt_node4h_t [nn4] (nn4 = is4[nn]; room for n each)
  uint32_t n, nseq;
  uint32_t seq[SAH_MAX_SEQ];  // SAH_SEQ entries, launch i runs seq[i]
} sah_arg_t;
