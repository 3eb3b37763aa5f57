// rt_common.h -- data layout shared by the RT host app and the HIP kernel.
//
// Everything the kernel reads lives in the driver's HBM arena and is addressed
// by the device addresses the app got from vx_mem_alloc (see DESIGN.md
// "Data layout in HBM"):
//   nodes   [num_nodes]  rt_node_t   64 B  BVH2 node = both children's boxes
//   tris    [num_tris]   rt_tri_t    48 B  clip-space v0,e1,e2 + pid (leaf order)
//   vnodes  [num nodes]  rt_vnode_t  64 B  primary visibility per traversed node
//   vtris   [num_tris]   rt_vtri_t   64 B  primary visibility per leaf record
//   vlayers [num_layer]  rt_vtri_t   64 B  screen layers, highest pid first
//   vgeom   [num_geom]   rt_vtri_t   64 B  geometry, ascending pid (flat mode)
//   prims   [num_prims]  rt_prim_t  128 B  fixed-point shading record
//   dcs     [num_dc]     rt_dcstate_t 64 B per-drawcall shading state
//   ptris   [num_prims]  rt_tri_t    48 B  clip-space triangle by pid
//   geom    [num_geom]   rt_tri_t    48 B  geometry triangles, ascending pid (flat)
//   cbuf    W*H*4 (linear, row 0 = NDC y=-1) or tiles*1024*4 (compact shard)
#pragma once

#include <stdint.h>

// one wave per workgroup: the dispatcher places (and retires) single waves,
// so a long wave never holds three finished partners' slots (64 vs 256
// threads: -7 % kernel time on tekkaman 1024^2)
#ifndef RT_BLOCK_THREADS
#define RT_BLOCK_THREADS 64
#endif
// per-wave LDS traversal stack depth: the regular image holds 24 entries
// (6 KB per wave: LDS still fits more waves than the VGPR budget allows),
// the deep image 32; the host picks the image from the built BVH's
// worst-case stack (BVH2: its depth; BVH4: stack4, e.g. 16-17 for the
// reference scenes)
#define RT_STACK_SHALLOW 24
#define RT_STACK_DEEP 32
#ifndef RT_MAX_STACK
#define RT_MAX_STACK RT_STACK_SHALLOW
#endif
// 1: a per-lane BVH4 step writes all three push rows unconditionally (rows at
// or above the new top hold garbage that is never read); the stack then
// carries 3 slack rows past its capacity for the writes of a full stack
#ifndef RT_PUSH_UNCOND
#define RT_PUSH_UNCOND 0
#endif
#define RT_STACK_ROWS (RT_MAX_STACK + (RT_PUSH_UNCOND ? 3 : 0))
#define RT_TILE_LOG 5            // RASTER_TILE_LOGSIZE (VX_config.vh:477-479)
#define RT_TILE_PIXELS 1024
#define RT_RASTER_TILE_LOG 4     // raster workgroup tile: 16x16 pixels, one per thread

#define RT_FLAG_SHADOWS  0x1u
#define RT_FLAG_TIE_HIGH 0x2u    // LEQUAL geometry: equal t -> highest pid
#define RT_FLAG_COMPACT  0x4u    // shard output: compact tile buffer
#define RT_FLAG_PATH     0x8u    // diffuse path trace (pt_kernel.hip)
#define RT_FLAG_FLAT     0x10u   // flat triangle list, no BVH (BASELINE config 2)
#define RT_FLAG_RASTER   0x20u   // draw3d raster pipeline (raster_kernel.hip)
#define RT_FLAG_BVH4     0x40u   // traverse the 4-wide BVH (nodes4) instead of the BVH2
#define RT_FLAG_BVH4H    0x80u   // BVH4 node steps read the binary16 rt_node4h_t form
#define RT_FLAG_COVERAGE 0x100u  // raster mode: covered pixels white, no shading / OM

// a render launch's words (vortex_hip.h vx_hip_set_launch_words, vx_spawn.h
// vx_launch_words; rt_render_start sets them on every frame): w[0..2] the
// frame's light (float bits), w[3] flags -- a moved light reaches the frame
// in its dispatch packet, not through a copy into the argument block
#define RT_LW_LIGHT    0x1u  // w[0..2] is the light (over arg.light)
#define RT_LW_NO_SLIST 0x2u  // the light-space lists are stale: shadow rays walk the BVH

#define RT_DC_DEPTH   0x1u
#define RT_DC_COLOR   0x2u
#define RT_DC_TEX     0x4u
#define RT_DC_MODULATE 0x8u

#define RT_LEAF_FLAG 0x80000000u
#define RT_EMPTY_REF (-1)

// statistics: user MPM counters, vx_mpm_query(VX_CSR_MPM_BASE + RT_MPM_USER + slot)
#define RT_MPM_USER 3
enum {
  RT_STAT_PRIMARY = 0, RT_STAT_SHADOW, RT_STAT_HITS, RT_STAT_OCCLUDED,
  RT_STAT_NODE_VISITS, RT_STAT_TRI_TESTS, RT_STAT_LAYER_TESTS, RT_STAT_SHADED,
  RT_STAT_TEXEL_BYTES, RT_STAT_BOUNCE, RT_STAT_RECT_TESTS, RT_STAT_EDGE_TESTS, RT_STAT_COUNT = 16
};

// rt_node_t: 4 x float4 =
//   (b0lo.x, b0hi.x, b1lo.x, b1hi.x), (.. y ..), (.. z ..), (c0, c1, 0, 0)
// child ref c: >= 0 internal node index; -1 empty; otherwise a leaf:
//   (c & 0x7fffffff) >> 4 = first triangle, (c & 15) + 1 = triangle count.
typedef struct { float v[16]; } rt_node_t;

// rt_node4_t (BVH4, 128 B): SoA over the 4 children --
//   lo.x[4], hi.x[4], lo.y[4], hi.y[4], lo.z[4], hi.z[4], child[4], pad[4];
// child refs as in rt_node_t (unused slots -1).  Collapsed from the BVH2
// (bvh.cpp): same leaves, same padded boxes, half the levels.
typedef struct { float v[32]; } rt_node4_t;

// rt_node4h_t (BVH4, 64 B): the same node with its 24 box planes as IEEE
// binary16 in rt_node4_t's order (lo.x[4], hi.x[4], lo.y[4], ...), then the
// 4 child refs.  The host rounds every BVH4 box outward to binary16-
// representable values (bvh.cpp RoundBoxes4), so rt_node4_t holds exactly the
// values this form decodes to and both describe one tree.  The kernel reads
// this form (4 loads of 16 B per node step instead of 7); it is uploaded right
// behind the rt_node4_t array (nodes4_addr + 128 * num_nodes4).
typedef struct { uint16_t b[24]; int32_t child[4]; } rt_node4h_t;


// rt_tri_t: (v0.x, v0.y, v0.w, pid), (e1.xyw, 0), (e2.xyw, 0) -- clip (x,y,w)
typedef struct { float v[12]; } rt_tri_t;

// ---- primary visibility (raster-exact primary rays, app/vis.cpp) ----------
// A primary ray through pixel (x, y) hits primitive p exactly where draw3d's
// rasterizer covers (x, y) with p: all three Q15.16 edge values >= 0
// (graphics.cpp:813-825, int32 wrap) inside a 32x32 tile p was binned to
// (gfxutil.cpp:237-271), and the closest hit is the draw3d depth test's
// winner: the smallest 24-bit depth word (graphics.cpp:564-596), ties to the
// first drawn (LESS) or last drawn (LEQUAL) primitive.  Per resolution the
// host computes every primitive's covered-pixel rectangle (exact, integer)
// and a lower bound of its depth word, and the BVH's nodes get the union /
// minimum over their subtrees: primary traversal is a 2D point-in-rect walk
// with depth culling, then the exact fixed-point test at the leaves.
// Pixel rectangles: x0 | x1 << 16 and y0 | y1 << 16, inclusive; an empty
// rectangle is x0 = 0xffff, x1 = 0.
#define RT_VIS_EMPTY_RECT 0x0000ffffu
#define RT_VIS_ZMIN_NONE 0xffffffffu
// rt_vnode_t (64 B), index-aligned with the traversed tree's nodes (BVH4, or
// BVH2 in slots 0-1): per child its covered-pixel rectangle as its corners
// lo = x0 | y0 << 16 and hi = x1 | y1 << 16 (inclusive: a pixel packed as
// x | y << 16 is inside iff two packed 16-bit clamps leave it unchanged),
// depth lower bound and reference (RT_EMPTY_REF when the child covers no
// pixel; its lo = hi = RT_VIS_EMPTY_RECT)
typedef struct {
  uint32_t lo[4], hi[4], zmin[4];
  int32_t child[4];
} rt_vnode_t;
// rt_vtri_t (64 B), index-aligned with the leaf triangle records (tris):
// edges[3][3] Q15.16, covered rectangle, pid, the z attribute (Q7.24
// a0-a2, a1-a2, a2) and the depth lower bound
typedef struct {
  int32_t edges[9];
  uint32_t rx, ry;
  int32_t pid;
  int32_t z[3];
  uint32_t zmin;
} rt_vtri_t;

typedef struct {
  int32_t edges[3][3];     // Q15.16 (graphics.h:61-64)
  int32_t attribs[7][3];   // Q7.24  z,r,g,b,a,u,v x (a0-a2, a1-a2, a2)
  uint32_t dc;             // drawcall index
  uint32_t pad;
} rt_prim_t;

typedef struct {
  uint32_t flags;          // RT_DC_*
  uint32_t tex_logw, tex_logh, tex_format, tex_filter, tex_wrapu, tex_wrapv, tex_stride;
  uint64_t tex_addr;
  uint32_t pad[6];
} rt_dcstate_t;

// Output-merger state of a drawcall for the raster pipeline (raster_kernel):
// DepthTencil / Blender / OutputMerger configuration derived from the
// draw3d DCR writes (draw3d/main.cpp:223-284 -> graphics.cpp:534-620,
// gpu_sw.h:78-98), quirks included.  32 words.
typedef struct {
  uint32_t depth_func, depth_writemask, depth_test_on;
  uint32_t stencil_func, stencil_zpass, stencil_zfail, stencil_fail;
  uint32_t stencil_ref, stencil_mask, stencil_writemask, stencil_on;
  uint32_t blend_mode_rgb, blend_mode_a, blend_src_rgb, blend_src_a, blend_dst_rgb, blend_dst_a;
  uint32_t blend_const, logic_op, blend_on;
  uint32_t cbuf_writemask, color_read, color_write;
  uint32_t prim_offset, prim_count;   // the drawcall's primitives (global pids)
  uint32_t pad[7];
} rt_omstate_t;

// screen bounding box of a primitive in pixels (gfxutil.cpp:168-192, clamped
// to the viewport): x in [lo & 0xffff, lo >> 16), y in [hi & 0xffff, hi >> 16);
// empty (x0 == x1) for degenerate or culled primitives
typedef struct {
  uint32_t x, y;
} rt_bbox_t;

typedef struct {
  uint64_t cbuf_addr, nodes_addr, tris_addr, vlayers_addr, prims_addr, dcs_addr;
  uint64_t ptris_addr;     // rt_tri_t per pid (path trace: bounce-hit barycentrics)
  uint64_t geom_addr;      // rt_tri_t of the geometry prims, ascending pid (flat mode)
  uint32_t width, height, tiles_x, tiles_y;
  uint32_t num_tasks, num_nodes, num_layer_tris, flags;
  uint32_t clear_color, shard_index, shard_count, bounces;
  float sx, sy;            // 2/W, 2/H
  float light[3];
  uint32_t seed;           // path-trace RNG seed
  uint32_t num_geom;       // geometry triangles (flat mode)
  uint32_t num_drawcalls;  // raster mode
  uint32_t raster_tile_log;  // raster mode: tile side 2^log (4: 16x16 px, 1 px/thread; 5: 32x32, 2x2/thread)
  uint32_t num_vnodes;     // rt_vnode_t records (0: no primitive covers a pixel)
  uint64_t zbuf_addr;      // raster mode: depth/stencil buffer, W*H u32
  uint64_t oms_addr;       // raster mode: rt_omstate_t per drawcall
  uint64_t bbox_addr;      // raster mode: rt_bbox_t per pid
  uint64_t nodes4_addr;    // rt_node4_t BVH4 (images built with RT_BVH4)
  uint32_t num_nodes4;
  uint32_t split_tiles;    // the first split_tiles tiles of the work order run 32 pixels per wave
  uint64_t order_addr;     // RT modes: u32 per local tile, the order tiles are worked in
                           // (heaviest first; 0 = identity), see rt_app.cpp TileOrder
  uint64_t vnodes_addr;    // rt_vnode_t per node of the traversed tree (primary visibility)
  uint64_t vtris_addr;     // rt_vtri_t per leaf triangle record (+3 padding records)
  uint64_t vgeom_addr;     // rt_vtri_t per geometry primitive, ascending pid (flat mode)
  uint32_t split_log;      // split tiles run 2^split_log pixels per wave (5: 32, an 8x4 half block)
  uint32_t blist_blocks;   // per-block candidate lists: local 8x8 blocks (local_tiles * 16), 0 = walk the tree
  uint64_t blist_addr;     // rt_bentry_t [entries + 2]: every local block's list, concatenated
  uint64_t bidx_addr;      // uint32[2] per local block lt * 16 + (by & 3) * 4 + (bx & 3): first entry, count
  uint32_t slist_on;       // light-space shadow lists built for `light` (0: shadow rays walk the BVH)
  uint32_t slist_n;        // their cells per cube-face side (RT_SLIST_N unless env RT_SLIST_N)
  uint64_t sidx_addr;      // uint32[2] per light-space cell: first entry, count
  uint64_t slist_addr;     // rt_tri_t per entry (+1 padding record): every cell's triangles, ascending pid
  uint32_t raster_bin_log; // raster mode: binning tile side 2^log (RASTER_TILE_LOGSIZE; draw3d -k)
  uint32_t pathq_lanes;    // pt_queue: paths per wave (64, 32 or 16; 0 = 64)
  uint64_t pathq_addr;     // path tracing in two kernels (pt_primary + pt_queue): uint4 per path
                           // start (task, plane t, hit pid, primary colour), compacted in
                           // RT_PQ_SEGS segments of pathq_seg_cap entries
  uint64_t pathq_ctr_addr; // counters, one 128-B line each (u32 word 32 * i): i < RT_PQ_SEGS
                           // paths queued in segment i; RT_PQ_SEGS + g pt_queue waves done of
                           // group g; 2 * RT_PQ_SEGS groups done (the last zeroes them all)
  uint32_t pathq_seg_cap;  // entries per segment
  uint32_t quad_tiles;     // the first quad_tiles of the split tiles run 16 pixels per wave
                           // (env RT_QUAD_TILES, a task-map probe; 0 by default)
  uint32_t tiles_x_magic;  // min(ceil(2^32 / tiles_x), 2^32 - 1): a tile's row is
                           // mulhi(tile, magic) plus at most one correction (rt_trace.h
                           // tile_row) -- no integer division in the kernels' task map
} rt_kernel_arg_t;
// the reciprocal rt_kernel_arg_t::tiles_x_magic holds for `tiles_x` tiles per row
static inline uint32_t rt_tiles_x_magic(uint32_t tiles_x) {
  if (tiles_x <= 1) return 0xffffffffu;
  return (uint32_t)((0x100000000ull + tiles_x - 1) / tiles_x);
}
// the path queue is split into segments (a primary chunk c appends to segment
// c % RT_PQ_SEGS) so its atomics spread over that many counters: one
// device-scope counter for the whole frame serialised ~1 600 atomics
#define RT_PQ_SEGS 64

// ---- light-space shadow lists (shadow rays to the point light) ------------
// A shadow segment P -> L is identified by its direction from the light,
// u = P - L, binned on the 6 faces of a cube around the light: face 2k +
// (u_k < 0) for the dominant axis k (ties to the lower axis), face
// coordinates (u_i, u_j) / |u_k| in [-1, 1] with (i, j) the other two axes in
// order, RT_SLIST_N x RT_SLIST_N cells, cell = (face * N + cy) * N + cx.  A
// cell's list holds every geometry triangle whose projection from the light
// reaches it (clipped to the face frustum widened by RT_SLIST_EPS, polygon
// box and separating-axis test against the cell widened by RT_SLIST_EPS):
// conservative, so any-hit over the list is the brute force's verdict.
// Built on the device (rt_setup.hip SCOUNT .. SSORT); oracle/rt.c sl_build
// restates it.
#define RT_SLIST_N 128              // default cells per face side (the oracle's SL_N); A/B r04g (nearest-first bounded lists): config 3 128 0.01836 / 256 0.0182 / 64 0.02072 ms, config 4 128 0.14286 / 256 0.14324; the lists build 4x fewer cells (set_light 0.137 -> 0.113 ms)
#define RT_SLIST_EPS (1.0f / 512.0f)

// ---- per-8x8-block candidate lists (primary visibility) -------------------
// For every 8x8 pixel block of the shard's tiles (local block lb = local
// tile * 16 + block of the tile), the geometry primitives whose covered-pixel
// rectangle reaches the block, ascending (depth lower bound, geometry index):
// the finer-grained form of draw3d's per-tile primitive lists
// (gfxutil.cpp:237-271).  Each entry carries the union rectangle (corners) of
// itself and the entries after it, so a wave stops scanning once no lane can
// change its winner.  Built on the device (rt_setup.hip, BCOUNT .. BSORT) or by
// the host restatement (rt_app.cpp BuildBlockLists); oracle/rt.c
// vis_build_lists restates them.
typedef struct {
  uint32_t k;              // geometry index (rt_vtri_t vgeom[k])
  uint32_t lo, hi;         // union rectangle of this entry and the rest: corners x | y << 16
  uint32_t zmin;           // this entry's depth lower bound (the smallest of the rest)
} rt_bentry_t;
// padding entries after the last list: block_primary loads the next pair of
// entries with each round's records, so the last round of an odd-length list
// ending at the end of the array reads up to 3 entries past it
#define RT_BLIST_PAD 3u
#define RT_BLIST_PAD_LO 0xffffffffu   // padding entries: a rectangle no pixel is in
#define RT_BLIST_PAD_HI 0xfffefffeu
#define RT_BLIST_MAX_LIST 1024u       // longest list the device sort takes (else: tree walk)
