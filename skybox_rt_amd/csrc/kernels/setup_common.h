// setup_common.h -- argument block of the device-side per-resolution setup
// (rt_setup.hip), shared with the host (app/rt_app.cpp device_setup).
//
// The reference's host pre-pass per drawcall is draw3d/main.cpp:179-211 ->
// graphics::Binning (sim/common/gfxutil.cpp:103-276): per primitive the
// clip -> device transform, edge equations, Q15.16 / Q7.24 fixed-point
// record (rast_prim_t) and the 32x32 tiles its screen box reaches.  Here the
// same work runs on the GPU, one launch per row below, in the records the RT
// kernels read:
//   prims   rt_prim_t per primitive              (app/setup.cpp PrimSetup)
//   bbox    rt_bbox_t per primitive              (app/setup.cpp PrimBBox)
//   vis     uint4 per primitive: covered-pixel rectangle, depth bound, any
//                                                (app/vis.cpp ComputeVisPrim)
//   vtris / vlayers / vgeom  rt_vtri_t records   (app/vis.cpp MakeVisTri)
//   vnodes  rt_vnode_t per tree node, bottom-up  (app/vis.cpp BuildVisNodes)
//   order   the shard's tiles, heaviest first    (app/rt_app.cpp tile order)
//   bidx / blist  per local 8x8 block its candidate list (rt_bentry_t,
//           rt_common.h): count, scan, fill, sort    (app/rt_app.cpp BuildBlockLists)
// and the resolution-independent triangle records at renderer creation
// (ptris by pid, geom).  Every record equals the host path's bit for bit
// (tests/test_gpu_setup.py; the host path stays selectable: RT_SETUP=host).
#pragma once

#include <stdint.h>

#define RTS_BLOCK 256
#define RTS_ITEMS 1024            // tile-order sort items per block (4 per thread)
#define RTS_MAX_FILLS 6
#define RTS_WEIGHT_CAP 255u       // tile-order key: min(weight, 255), one 8-bit digit

// sub-phases, OR-ed into `phases`: a launch runs every selected sub-phase
// (each independent of the others in the same launch)
#define RTS_FILL     0x001u  // fills[0..nfills): u32 words = value
#define RTS_PRIMVIS  0x002u  // wave per primitive: rt_prim_t + rt_bbox_t (+ vis unless raster)
#define RTS_VTRIS    0x004u  // thread per record: leaf vtris (+3 pads), vlayers, vgeom
#define RTS_WEIGHT   0x008u  // per geometry primitive: the 4 corners of its tile rectangle
                             //   in a 2D difference array (tiles_x + 1) x (tiles_y + 1)
#define RTS_LINK     0x010u  // thread per tree node: parent slot of each internal child,
                             //   internal-child count, arrival counter 0
#define RTS_ROWSUM   0x020u  // thread per tile row: prefix sums along x
#define RTS_CLIMB    0x040u  // thread per node without internal children: vnode rectangles
                             //   bottom-up (the last child to arrive climbs on)
#define RTS_COLSUM   0x080u  // thread per tile column: prefix sums along y -> tile weights
#define RTS_HIST     0x100u  // tile order: per-block histograms of 255 - min(weight, 255)
#define RTS_SCAN     0x200u  //   exclusive scan (workgroup 0)
#define RTS_SCATTER  0x400u  //   stable scatter of the local tile indices -> order
#define RTS_RECORDS  0x800u  // renderer creation: rt_tri_t per pid (ptris), geometry list (geom)
// per-block candidate lists (rt_bentry_t): a wave per geometry primitive
// visits the shard's 8x8 blocks its covered rectangle reaches
#define RTS_BCOUNT   0x1000u // atomic count per local block
#define RTS_BSUM     0x2000u // per 1024 blocks: sum (-> bpart) and the longest list (status[1])
#define RTS_BSCAN    0x4000u // exclusive scan of bpart (workgroup 0), total -> status[2]
#define RTS_BOFF     0x8000u // per local block (first entry, count) -> bidx; counts zeroed
#define RTS_BFILL    0x10000u // unsorted (zmin, k, rx, ry) per (block, primitive) -> btmp
#define RTS_BSORT    0x20000u // wave per block: rank + suffix union -> blist (+2 pads)
#define RTS_BLOCKS_PER_PART 1024u  // blocks summed per bpart word (4 per thread)
// light-space shadow lists (rt_common.h): SPROJ projects every (geometry
// triangle, cube face) pair once -- the clipped polygon's cell rectangle and
// its separating axes, precomputed -- and counts the rectangle's cells; the
// candidates (item, cell of its rectangle) are then dealt one per thread
// (binary search of the scanned counts), so a large projection is spread
// over many waves instead of one.  SSUM / SSCAN / SOFF are BSUM / BSCAN /
// BOFF over the cells.
#define RTS_SCOUNT   0x40000u // thread per candidate: separating-axis test, atomic count per cell
#define RTS_SFILL    0x80000u // thread per candidate: (geometry index, key, cell) at the cell's cursor
#define RTS_SSORT    0x100000u // thread per entry: rank in its cell by (key, geometry index) -> slist
                               // (rt_tri_t copies, the key -- squared light-to-bounding-box distance --
                               // in e1.w; +1 pad); then the render arguments' slist fields
#define RTS_SPROJ    0x200000u // thread per (triangle, face): projection record, cell count, key
#define RTS_SOSCAN   0x400000u // exclusive scan of the per-item cell counts (one workgroup)
#define RTS_SSUM     0x800000u // BSUM over the cells
#define RTS_SSCAN    0x1000000u // BSCAN over the cells
#define RTS_SOFF     0x2000000u // BOFF over the cells -> sidx

// status words (u32 [RTS_STATUS_WORDS]): [0] malformed-input flags
// (RTS_ERR_*), [1] the longest block list, [2] block-list entries in total,
// [3] local tiles with weight > 0 (the scan of the tile order), [4] the
// longest cell list, [5] cell-list entries in total, [6] block-list entries
// beyond bcap (nonzero: the host refills at the exact size), [7] cell-list
// entries beyond scap
#define RTS_STATUS_WORDS 8
#define RTS_FOLD_LISTS 0x1u   // BOFF / SOFF sum the raw partial sums they need (no BSCAN / SSCAN)
#define RTS_FOLD_ORDER 0x2u   // SCATTER scans the digit histogram itself, HIST counts the heavy tiles (no SCAN)
#define RTS_FOLD_SOFF  0x4u   // SCOUNT / SFILL scan the candidate counts into LDS (no SOSCAN)
#define RTS_SOFF_LDS 6144u    // candidate-count items (6 per geometry triangle) RTS_FOLD_SOFF holds
#define RTS_SPROJ_WORDS 32u  // u32 per SPROJ record: header uint4 + 7 separating axes (nx, ny, p0, p1)
#define RTS_MAX_SEQ 32
#define RTS_CLIMB_WG_NODES 4096u  // trees this small climb in one workgroup (rt_setup.hip phase_climb)
#define RTS_ERR_REF   0x1u   // a tree reference out of range
#define RTS_ERR_PID   0x2u   // a leaf record's pid out of range
#define RTS_ERR_CLIMB 0x4u   // a climb longer than 64 levels

typedef struct {
  uint64_t addr;     // u32 words
  uint64_t count;
  uint32_t value, pad;
} rts_fill_t;

typedef struct {
  uint64_t verts_addr;     // float [P][32]: 3 x (x, y, z, w, r, g, b, a, u, v), 2 pad
  uint64_t pdc_addr;       // u32 [P]: drawcall of each primitive
  uint64_t dcz_addr;       // float [num_dc][2]: viewport near, far
  uint64_t prims_addr;     // rt_prim_t [P]
  uint64_t bbox_addr;      // rt_bbox_t [P] (empty: degenerate or outside the viewport)
  uint64_t vis_addr;       // uint4 [P]: rx, ry, zmin, any
  uint64_t tris_addr;      // rt_tri_t [num_tris]: leaf records (pid bits in v[3])
  uint64_t nodes_addr;     // the traversed tree: rt_node4_t [num_nodes] (bvh4) or rt_node_t
  uint64_t vnodes_addr;    // rt_vnode_t [num_nodes]
  uint64_t vtris_addr;     // rt_vtri_t [num_tris + 3]
  uint64_t vlayers_addr;   // rt_vtri_t [num_layers]
  uint64_t vgeom_addr;     // rt_vtri_t [num_geom]
  uint64_t layers_addr;    // i32 [num_layers]: screen-layer pids, last drawn first
  uint64_t geometry_addr;  // i32 [num_geom]: depth-tested pids, ascending
  uint64_t parent_addr;    // i32 [num_nodes]: parent * 4 + slot, -1 for the root / unreached
  uint64_t count_addr;     // u32 [num_nodes][2]: internal children, arrivals
  uint64_t weight_addr;    // u32 [(tiles_y + 1) * (tiles_x + 1)]
  uint64_t hist_addr;      // u32 [256][nblocks]
  uint64_t order_addr;     // u32 [local_tiles]
  uint64_t status_addr;    // u32 [4]
  uint64_t ptris_addr;     // rt_tri_t [P]
  uint64_t geom_addr;      // rt_tri_t [num_geom]
  uint64_t bcnt_addr;      // u32 [nblk]: entries per local block (then the fill cursors)
  uint64_t bpart_addr;     // u32 [nbpart]: per RTS_BLOCKS_PER_PART blocks their sum, then its scan
  uint64_t bidx_addr;      // uint32[2] [nblk]: first entry, count
  uint64_t btmp_addr;      // uint4 [entries]: unsorted (zmin, k, rx, ry)
  uint64_t blist_addr;     // rt_bentry_t [entries + 2]
  rts_fill_t fills[RTS_MAX_FILLS];
  uint32_t phases, nfills;
  uint32_t num_prims, width, height, raster;
  uint32_t num_tris, num_nodes, bvh4, num_layers, num_geom;
  uint32_t tiles_x, tiles_y, shard_index, shard_count, local_tiles, nblocks;
  uint32_t nblk, nbpart, blist_entries;  // local 8x8 blocks, bpart words, list entries (BSORT)
  float light[3];          // shadow lists: the point light (clip x, y, w)
  uint32_t slist_n;        // shadow lists: cells per cube-face side
  uint64_t slist_addr;     // shadow lists: rt_tri_t [scap + 1]
  // shadow lists (the cell-level arrays, apart from the block lists' so one
  // launch can build both)
  uint64_t scnt_addr;      // u32 [ncells]: entries per cell (then the fill cursors)
  uint64_t spart_addr;     // u32 [ncpart]: per RTS_BLOCKS_PER_PART cells their sum, then its scan
  uint64_t sidx_addr;      // uint32[2] [ncells]: first entry, count
  uint64_t sproj_addr;     // u32 [num_geom * 6][RTS_SPROJ_WORDS]: SPROJ records
  uint64_t soff_addr;      // u32 [num_geom * 6 + 1]: cells per item, then their exclusive scan + total
  uint64_t skey_addr;      // u32 [num_geom]: sl_key of each triangle (float bits)
  uint64_t stmp_addr;      // u32 [3][scap]: unsorted entries -- geometry index, key, cell
  uint64_t rargs_addr;     // the render arguments (rt_kernel_arg_t): SSORT writes their slist fields
  uint32_t ncells, ncpart, scap, bcap;  // cells (6 N^2), spart words, entry capacities
  uint32_t max_list;       // lists longer than this are not used (RT_BLIST_MAX_LIST)
  uint32_t max_entries;    // nor more entries in total than this
  // launch sequences: the host enqueues nseq launches of this one argument
  // block back to back (no host wait between them), launch i with launch
  // tag i (vx_hip_set_launch_tag: the entry's kernel argument); launch i
  // runs seq_phases[i] -- its one-workgroup phases (the scans) by workgroups
  // 0, 1, ..; part: a launch's wide sub-phases on disjoint slices of the grid
  // (rt_setup.hip run_phases)
  uint32_t nseq, part;
  uint32_t seq_phases[RTS_MAX_SEQ];
  // the sequence's last launch copies the status words, then status_nonce,
  // to this pinned host buffer (a raw device pointer; 0 = none): the host
  // reads them there after waiting for the sequence
  uint64_t status_host;
  uint32_t status_nonce;
  // RTS_FOLD_*: the scans done inside the launches that need them (each
  // workgroup scans what it reads; no one-workgroup scan launch)
  uint32_t fold;

} rt_setup_arg_t;
