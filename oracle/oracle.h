/*
 * oracle.h -- CPU restatement of the reference's draw3d pipeline and of the
 * north-star ray-tracing path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / CPU baseline.  The product
 * (skybox_rt_amd/) never links or calls anything here.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - raster path: pinned against the reference's committed golden images
 *     tests/regression/draw3d/triangle_ref_{8..128}.png, tekkaman_ref_128.png,
 *     box_ref_128.png and tests/regression/raster/triangle_ref_*.png (copied as
 *     data into tests/golden/).  The reference itself cannot be built here
 *     (cocogfx/softfloat/ramulator submodules are empty, no RISC-V toolchain).
 *   - ray-tracing path (MT visibility, shadow, bounce): NO REFERENCE EXISTS
 *      -> "parity unpinned" beyond primary visibility,
 *     which is cross-checked against the pinned raster path.
 *
 * Numerics: compiled with -ffp-contract=off; every fused multiply-add is an
 * explicit fmaf() so the HIP kernel (which uses the same explicit fmaf()s)
 * can be compared bit-for-bit.
 */
#ifndef ORACLE_H
#define ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- flattened scene (produced by oracle/cgltrace.py) -------------------- */
typedef struct {
  int32_t prim_offset, prim_count;
  int32_t tex_slot;                 /* index into textures[], -1 = none */
  float   znear, zfar;
  int32_t color_enabled;
  uint32_t color_writemask;
  int32_t depth_test, depth_writemask, depth_func;
  int32_t stencil_test, stencil_func, stencil_zpass, stencil_zfail, stencil_fail;
  int32_t stencil_ref, stencil_mask, stencil_writemask;
  int32_t texture_enabled, texture_envmode, texture_minfilter, texture_magfilter;
  int32_t texture_addressU, texture_addressV;
  int32_t blend_enabled, blend_src, blend_dst;
} orc_drawcall_t;

typedef struct {
  int32_t format, width, height, pad;
  int64_t offset;                   /* byte offset into texels blob */
} orc_texture_t;

typedef struct {
  int32_t num_drawcalls;
  const orc_drawcall_t* drawcalls;
  int32_t num_prims;
  const float* prim_verts;          /* [num_prims][3][10]: xyzw rgba uv */
  int32_t num_textures;
  const orc_texture_t* textures;
  const uint8_t* texels;
} orc_scene_t;

/* ---- fixed-point primitive record: graphics.h:38-64 rast_prim_t (120 B) --- */
typedef struct {
  int32_t edges[3][3];              /* Q15.16, [edge][a,b,c] */
  int32_t attribs[7][3];            /* Q7.24,  [z,r,g,b,a,u,v][x=a0-a2, y=a1-a2, z=a2] */
} orc_rast_prim_t;

/* Setup one primitive at W x H (gfxutil.cpp:131-251).  Returns 0 = ok,
 * 1 = degenerate (rejected), 2 = outside the viewport (rejected by bbox).
 * bbox = {left, right, top, bottom} in pixels when status != 1. */
int orc_setup_prim(const float* v /*[3][10]*/, uint32_t width, uint32_t height,
                   float znear, float zfar, orc_rast_prim_t* out, int32_t bbox[4]);

/* Full draw3d software path (Binning + Rasterizer + shader + OM) over all
 * drawcalls; color/depth must be pre-cleared by the caller (0xff000000 /
 * 0xffffffff in the reference, draw3d/main.cpp:47-48).  Row 0 = NDC y=-1.
 * pid_out (optional): per-pixel global primitive index of the last fragment
 * that passed the depth/stencil test and was written, -1 if none. */
int orc_raster_render(const orc_scene_t* scene, uint32_t width, uint32_t height,
                      uint32_t tile_logsize, uint32_t* color, uint32_t* depth,
                      int32_t* pid_out);
/* The raster regression app (tests/regression/raster): the same binning and
 * coverage, every covered pixel written 0xffffffff over the caller's clear
 * (0xff000000 in the reference, raster/main.cpp:40,245-250). */
int orc_raster_coverage(const orc_scene_t* scene, uint32_t width, uint32_t height,
                        uint32_t tile_logsize, uint32_t* color);

/* The rasterizer's per-pixel coverage of one primitive over a w x h pixel
 * window at (x0, y0): mask[j * w + i] = 1 iff all three edge values
 * a*x + b*y + c (int32 wrap, graphics.cpp:640-642) at (x0 + i, y0 + j) are
 * >= 0 (inclusive, no top-left rule, graphics.cpp:813-825).  `edges` holds
 * (a, b, c) per edge.  The RTL raster slice's known-answer test
 * (hw/unit_tests/raster_unit/raster_slice/testbench.cpp:53-66) pins it. */
void orc_edge_cover(const int32_t edges[9], uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                    uint8_t* mask);

/* ---- ray tracing -------------------------------------------------------- */
typedef struct {
  uint32_t width, height;
  uint32_t flags;                   /* RT_FLAG_* below */
  float    light[3];                /* point light in clip (x,y,w) space */
  uint32_t clear_color;
  uint32_t bounces;                 /* path-trace depth for RT_FLAG_BOUNCE */
  uint32_t seed;
  uint32_t nthreads;                /* CPU worker threads (timing baseline) */
  uint32_t row_begin, row_end;      /* render rows [begin,end) (0,0 = all) */
  uint32_t row_step;                /* every row_step-th row (0/1 = all) */
  uint32_t vis_per_lane;            /* BVH mode: 1 = primary rays walk the tree one pixel
                                       at a time (RT_VIS_PACKET=0 images), 0 = per wave packet
                                       (the default images; full frames only) */
  uint32_t vis_lists;               /* BVH mode: 1 = primary visibility from the per-8x8-block
                                       candidate lists (rt_app.cpp build_block_lists, the
                                       kernels' block_primary) */
  uint32_t shadow_lists;            /* primary+shadow: shadow rays test the light-space cell
                                       lists (rt.c sl_build, the kernels' occluded_list) */
  uint32_t path_queue;              /* path trace in two kernels (pt_primary + pt_queue): the
                                       primary pass runs 8x8 blocks everywhere (no 32-pixel
                                       waves in geometry tiles) */
  uint32_t split_log;               /* path trace: 2^split_log pixels per wave in the geometry
                                       tiles (the renderer's split_log; 0 = 5, 32 pixels) */
} orc_rt_params_t;

#define ORC_RT_SHADOWS 0x1u
#define ORC_RT_PATH    0x8u   /* diffuse path trace, `bounces` segments */

typedef struct {
  uint64_t primary_rays, shadow_rays, geometry_hits, occluded;
  uint64_t node_visits, tri_tests, layer_tests, shaded, texel_bytes;  /* layer_tests: per wave */
  uint64_t bounce_rays;
} orc_rt_counters_t;

/* path-trace constants (synthetic: the reference has no lights or
 * materials) -- identical in the HIP kernel */
#define ORC_PT_SKY 0.25f        /* radiance of an escaped bounce ray */
#define ORC_PT_TRIES 8          /* disk rejection-sampling attempts */

/* BVH in the device layout produced by the product's builder
 * (skybox_rt_amd/csrc/app/bvh.cpp, DESIGN.md "BVH layout"). */
typedef struct {
  int32_t num_nodes;
  const float* nodes;               /* [num_nodes][16] (4 x float4) */
  int32_t num_tris;
  const float* tris;                /* [num_tris][12]  (v0,pid | e1,- | e2,-) */
  int32_t num_nodes4;               /* > 0: traverse the 4-wide BVH instead */
  const float* nodes4;              /* [num_nodes4][32] (lo.x[4] hi.x[4] lo.y hi.y lo.z hi.z
                                       child[4] pad[4]) */
  /* the primary rays' tree (rt_renderer_export_vis_tree; NULL / 0: walk the
   * BVH above): child refs [num_vis_nodes][4], leaf record pids [num_vis_leaves] */
  int32_t num_vis_nodes;
  const int32_t* vis_refs;
  int32_t num_vis_leaves;
  const int32_t* vis_pids;
} orc_bvh_t;

/* Brute-force (no BVH) reference: closest hit over every geometry triangle,
 * any-hit shadows.  pid/t optional (may be NULL). */
int orc_rt_render_bruteforce(const orc_scene_t* scene, const orc_rt_params_t* p,
                             uint32_t* color, int32_t* pid, float* t,
                             orc_rt_counters_t* counters);

/* BVH traversal restatement of the HIP kernel's traversal order (for the
 * algorithmic byte counts and the multi-threaded CPU baseline). */
int orc_rt_render_bvh(const orc_scene_t* scene, const orc_bvh_t* bvh,
                      const orc_rt_params_t* p, uint32_t* color, int32_t* pid,
                      float* t, orc_rt_counters_t* counters);

/* Primary visibility (vis.c): per primitive at W x H, out[num_prims][3] =
 * covered-pixel rectangle x0|x1<<16, y0|y1<<16 (inclusive; empty 0x0000ffff)
 * and depth-word lower bound -- the product's rt_scene_setup_vis restated
 * by brute force over the binned tiles. */
int orc_vis_prims(const orc_scene_t* scene, uint32_t width, uint32_t height, uint32_t* out);

/* The per-8x8-block candidate lists of one shard (the product's
 * rt_bentry_t layout, rt.c vis_build_lists): idx [nlb][2] (first entry,
 * count), ent [total][4] (geometry index, union corners lo, hi, depth
 * bound); NULL arrays: sizes only. */
int orc_vis_block_lists(const orc_scene_t* scene, uint32_t width, uint32_t height, uint32_t shard_index,
                        uint32_t shard_count, uint32_t* idx, uint32_t* ent, uint64_t* total, uint32_t* nlb);

/* The light-space shadow lists for a point light (rt.c sl_build; the device
 * build rt_setup.hip SCOUNT .. SSORT): idx [6 * 128 * 128][2] (first entry,
 * count; cell = (face * 128 + cy) * 128 + cx), ent [total] geometry indices
 * (ascending within a cell); NULL arrays: total only. */
int orc_shadow_lists(const orc_scene_t* scene, const float light[3], uint32_t* idx, int32_t* ent,
                     uint64_t* total);

/* Möller–Trumbore as used by both sides (exposed for unit tests). */
int orc_mt(const float o[3], const float d[3], const float v0[3],
           const float e1[3], const float e2[3], float tmin, float* t_out);

/* ---- linear BVH (oracle/lbvh.c, restating kernels/bvh_build.hip) -------- */
/* verts: [n][3][3] clip (x, y, w); geom: [n][12] rt_tri_t records of the same
 * triangles; out: nodes [max(n-1,1)][16], tris [n+3][12], depth. */
int orc_lbvh_build(const float* verts, const float* geom, uint32_t n, float* nodes, float* tris,
                   uint32_t* depth);
/* BVH4 collapse of an LBVH node array (bvh_build.hip phase_collapse): every
 * reachable internal node at even depth becomes a BVH4 node at its own index
 * with its internal (odd-depth) children replaced by their children; nodes:
 * [nn][16] rt_node_t, out nodes4 [nn][32] rt_node4_t (zeros elsewhere) and
 * the worst-case near-first traversal stack. */
int orc_lbvh_collapse4(const float* nodes, uint32_t nn, float* nodes4, uint32_t* stack);
/* binary16 planes of a BVH4 node array: planes rounded outward in place,
 * 64-B rt_node4h_t records (24 halves + 4 child refs) to `half` (nn * 64 B) */
int orc_half4(float* nodes4, uint32_t nn, void* half);

/* ---- texture regression app (tests/regression/tex; oracle/tex.c) ------ */
/* LoadImage format conversion of one A8R8G8B8 pixel (VX_TEX_FORMAT_*) */
uint32_t orc_tex_encode(uint32_t argb, uint32_t format);
/* converted image + mip chain; out NULL = size query; mipoff[16] */
size_t orc_tex_build(const uint32_t* argb, uint32_t w, uint32_t h, uint32_t format, uint8_t* out,
                     uint32_t* mipoff, uint32_t* levels);
/* tex/kernel.cpp main(): lod + blend fraction for a dst size */
void orc_tex_lod(uint32_t logw, uint32_t logh, uint32_t dst_w, uint32_t dst_h, uint32_t* lod,
                 uint32_t* frac);
/* tex/kernel.cpp kernel_body over every task; filter 0/1/2 = -g */
void orc_tex_render(const uint8_t* tex, const uint32_t* mipoff, uint32_t logw, uint32_t logh,
                    uint32_t format, uint32_t wrap, uint32_t filter, uint32_t dst_w, uint32_t dst_h,
                    uint32_t num_tasks, uint32_t* dst);

#ifdef __cplusplus
}
#endif
#endif
