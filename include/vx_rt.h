/*
 * vx_rt.h -- C-ABI of the ray-tracing host app (librtapp.so).
 *
 * This is the host side of the north-star "tests/regression RT app": the
 * analog of tests/regression/draw3d/main.cpp (scene load, per-frame state
 * setup, upload, vx_start/vx_ready_wait, framebuffer read-back), built on the
 * public vortex.h API and therefore on whatever driver VORTEX_DRIVER selects
 * (libvortex-hip.so on MI355X).  The rtapp executable is its CLI with
 * draw3d's flags; Python (skybox_rt_amd.rt) and bench.py bind it via ctypes.
 *
 * All functions return 0 on success and a negative value on error; the last
 * error message of the calling thread is available from rt_last_error().
 */
#ifndef VX_RT_H
#define VX_RT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_scene* rt_scene_h;
typedef struct rt_renderer* rt_renderer_h;

typedef struct {
  uint32_t num_drawcalls, num_prims, num_geometry, num_layer, num_textures;
  uint32_t bvh_nodes, bvh_tris, bvh_leaves, bvh_depth;
  uint32_t bvh4_nodes, bvh4_depth, bvh4_stack;  /* the 4-wide BVH collapsed from it */
  uint32_t bvh4_f16;  /* 1: BVH4 boxes rounded outward to binary16, the kernel reads 64-B nodes */
  double parse_ms, bvh_ms;
} rt_scene_info_t;

#define RT_RENDER_SHADOWS 0x1u
#define RT_RENDER_PATH 0x8u            /* diffuse path trace (pt_kernel), `bounces` segments */
#define RT_RENDER_FLAT 0x10u           /* flat triangle list, no BVH (config 2; rt_flat) */
#define RT_RENDER_RASTER 0x20u         /* the draw3d raster pipeline (raster_kernel): any
                                          scene incl. blending/stencil; shard_count 1 */
#define RT_RENDER_BVH2 0x40u           /* traverse the binary BVH (default: the 4-wide one;
                                          env RT_BVH_WIDTH=2 flips the default) */
#define RT_RENDER_INSTRUMENTED 0x100u  /* use the counting kernel variant */
#define RT_RENDER_COMPACT 0x200u       /* compact tile-order output (the shard layout,
                                          implied by shard_count > 1) for one shard too */
#define RT_RENDER_COUNTERS 0x400u      /* per-workgroup counter rows on (vx_hip_set_counters):
                                          rt_render_stats' ray / hit counts; implied by
                                          RT_RENDER_INSTRUMENTED.  Off, a frame writes only
                                          its framebuffer (and one task-count word) */
#define RT_RENDER_HOST_SETUP 0x800u    /* build the per-resolution records (shading and
                                          visibility records, primary tree, tile order,
                                          clears) with the host loops instead of on the
                                          device (kernels/rt_setup.hip, the default; env
                                          RT_SETUP=host does the same) */
#define RT_RENDER_COVERAGE 0x1000u     /* with RT_RENDER_RASTER: the raster regression app's
                                          coverage image (tests/regression/raster/kernel.cpp:
                                          covered pixels 0xffffffff, no shading, no OM state) */
#define RT_RENDER_BVH_WALK 0x2000u     /* primary+shadow / path frames without the per-block
                                          and light-space lists: primary visibility by the BVH4
                                          packet walk, shadow rays by the BVH (BASELINE config 3's
                                          "full BVH traversal"); primary+shadow frames run their
                                          own image (rt_bvh: entry vx_main_rt_bvh).  Env
                                          RT_BLOCK_LISTS=0 RT_SHADOW_LISTS=0 give the same frames
                                          on the default image */

typedef struct {
  uint32_t width, height;
  uint32_t flags;             /* RT_RENDER_* */
  float light[3];             /* point light, clip (x, y, w) space */
  uint32_t clear_color;       /* ARGB8888, 0xff000000 in draw3d */
  uint32_t shard_index;       /* this device renders 32x32 tiles t with */
  uint32_t shard_count;       /*   t % shard_count == shard_index */
  uint32_t bounces;           /* RT_RENDER_PATH: bounce segments per path (config 4: 4) */
  uint32_t seed;              /* RT_RENDER_PATH: RNG seed (config 4: 0x5EED) */
  uint32_t tile_logsize;      /* RT_RENDER_RASTER: binning tile side 2^k (draw3d / raster -k,
                                 gfxutil.cpp:237-250; 2..15), 0 = RASTER_TILE_LOGSIZE (5) */
} rt_render_params_t;

typedef struct {
  uint64_t primary_rays, shadow_rays, geometry_hits, occluded;      /* RT_RENDER_COUNTERS */
  uint64_t node_visits, tri_tests, layer_tests, shaded, texel_bytes; /* instrumented only */
  uint64_t tasks;             /* VX_CSR_MINSTRET */
  double kernel_ms;           /* HIP-event time of the last launch */
  uint32_t grid, block;       /* launch geometry chosen by the driver */
  uint32_t num_tasks, local_tiles;
  uint64_t bounce_rays;       /* RT_RENDER_PATH: bounce segments traced */
  uint64_t rect_tests;        /* RT_RENDER_FLAT, instrumented: list entries whose rectangle a
                                 wave tested (per wave, the work executed) */
  uint64_t edge_tests;        /* RT_RENDER_FLAT, instrumented: entries some lane of the wave
                                 lay in, whose edges and depth the wave evaluated */
} rt_stats_t;

const char* rt_last_error(void);

int rt_scene_load(const char* path, rt_scene_h* out);
/* draw3d's -s start / -e end (tests/regression/draw3d/main.cpp:179-181): only
 * drawcalls start <= d <= end are drawn (rt_scene_load = 0, 0xffffffff) */
int rt_scene_load_range(const char* path, uint32_t start_draw, uint32_t end_draw, rt_scene_h* out);
int rt_scene_free(rt_scene_h scene);
int rt_scene_info(rt_scene_h scene, rt_scene_info_t* info);
/* flattened triangles, float[num_prims][3][10] (x,y,z,w, r,g,b,a, u,v) */
int rt_scene_export_prims(rt_scene_h scene, float* out, uint64_t count);
/* BVH arrays: float[bvh_nodes][16], float[bvh_tris][12] */
int rt_scene_export_bvh(rt_scene_h scene, float* nodes, float* tris);
/* 4-wide BVH nodes: float[bvh4_nodes][32] (rt_node4_t); leaves index the same tris */
int rt_scene_export_bvh4(rt_scene_h scene, float* nodes4);
/* fixed-point shading records (rt_prim_t) at width x height: int32[num_prims][32] */
int rt_scene_setup_prims(rt_scene_h scene, uint32_t width, uint32_t height, int32_t* out,
                         uint64_t count);
/* primary-visibility record of every primitive at width x height (the RT
 * kernels' raster-exact primary rays, rt_common.h): uint32[num_prims][3] =
 * covered-pixel rectangle x0 | x1 << 16, y0 | y1 << 16 (inclusive; empty:
 * 0x0000ffff) and the lower bound of its 24-bit depth word.  NO REFERENCE
 * (derived from draw3d's coverage rule; oracle/vis.c restates it). */
int rt_scene_setup_vis(rt_scene_h scene, uint32_t width, uint32_t height, uint32_t* out,
                       uint64_t count);
/* the screen-space BVH4 the primary rays walk at width x height (what
 * rt_renderer_configure builds; depth_scale 0 = the default 2D SAH):
 * int32 refs[num_nodes][4], leaf_pids[num_leaf], worst-case stack; NULL
 * arrays = counts only.  NO REFERENCE. */
int rt_scene_vis_tree(rt_scene_h scene, uint32_t width, uint32_t height, float depth_scale,
                      int32_t* refs, uint32_t* num_nodes, int32_t* leaf_pids, uint32_t* num_leaf,
                      uint32_t* stack4);

/* kernel_dir: directory holding rt_kernel.vxbin / rt_kernel_stats.vxbin
 * (NULL = next to librtapp.so).  Opens its own vortex device.  Scenes the
 * RT path cannot trace (blending, stencil, layers after geometry) get a
 * renderer that accepts only RT_RENDER_RASTER. */
int rt_renderer_create(rt_scene_h scene, const char* kernel_dir, rt_renderer_h* out);
int rt_renderer_free(rt_renderer_h r);
int rt_renderer_configure(rt_renderer_h r, const rt_render_params_t* params);
int rt_render_start(rt_renderer_h r);
int rt_render_wait(rt_renderer_h r);
int rt_render(rt_renderer_h r);  /* start + wait */
int rt_render_stats(rt_renderer_h r, rt_stats_t* stats);
/* HIP-event duration of the last launch only (no counter read-back) */
int rt_render_kernel_ms(rt_renderer_h r, double* kernel_ms);
/* waits for every started frame, then, since the renderer's device opened:
 * the summed HIP-event kernel time of the timed launches, their number, and
 * the number of all launches.  Back-to-back rt_render_start calls queue
 * behind the in-flight frame (the driver's VX_HIP_QUEUE_DEPTH) and are timed
 * one in VX_HIP_TIME_EVERY: kernel_ms_sum / timed is their average. */
int rt_render_run_totals(rt_renderer_h r, double* kernel_ms_sum, uint64_t* timed,
                         uint64_t* launches);
/* 1: launches timed by HIP events as above (the default); 0: untimed -- no
 * events and no queue bound, so a run of rt_render_start calls reaches the
 * GPU back to back (bench.py's stream clock: wall time of K such frames / K).
 * Waits for the in-flight frames. */
int rt_render_set_timing(rt_renderer_h r, int timed);
/* linear W*H framebuffer (shard_count == 1) or compact tile buffer
 * (local_tiles * 1024 pixels in task order) */
int rt_read_framebuffer(rt_renderer_h r, uint32_t* out, uint64_t count);

/* RT_RENDER_RASTER: the depth/stencil buffer (stencil << 24 | depth), W*H */
int rt_read_depthbuffer(rt_renderer_h r, uint32_t* out, uint64_t count);

/* Build the BVH on the device (Morton codes, radix
 * sort, binary radix tree, bottom-up boxes -- kernels/bvh_build.hip) from
 * the scene's triangles and make it this renderer's tree (binary traversal;
 * a configured renderer is reconfigured).  Stats optional. */
typedef struct {
  uint32_t nodes, depth, launches;
  uint32_t stack4;      /* worst-case stack of the device BVH4 collapse (traversed by the
                           RT/PT kernels), RT_BVH_STACK4_UNUSED if it exceeds the deep
                           images' stack and the BVH2 is traversed instead */
  double build_ms;      /* host wall time of the whole build (upload + launches) */
  double kernel_ms;     /* LBVH: sum of the build kernels' HIP-event times; SAH: host wall time
                           of the launch sequence and its one read-back (per-launch event
                           times under env RT_SAH_TRACE) */
  uint32_t nodes4;      /* rt_node4_t records (LBVH: one per BVH2 index, zeros at absorbed nodes) */
  uint32_t depth4;      /* BVH4 depth (SAH build; 0 for the LBVH) */
  uint32_t method;      /* RT_BVH_BUILD_* */
  uint32_t pad;
} rt_bvh_build_stats_t;
int rt_renderer_build_bvh(rt_renderer_h r, rt_bvh_build_stats_t* stats);  /* = _ex(LBVH) */
/* RT_BVH_BUILD_LBVH: Morton codes + radix tree (kernels/bvh_build.hip, 19
 * launches, fastest build).  RT_BVH_BUILD_SAH: the host builder's binned-SAH
 * tree, BVH4 collapse and binary16 planes restated on the device
 * (kernels/bvh_sah.hip): one stream-ordered launch sequence -- the init, a
 * split launch per tree level for a budget of log2(n) + 4 levels, 7
 * finishing launches -- with one read-back at the end (a deeper tree
 * continues once per further budget); the same arrays as the scene's host
 * build, bit for bit.  The build image and its scratch stay with the
 * renderer, so a rebuild loads nothing. */
#define RT_BVH_BUILD_LBVH 0u
#define RT_BVH_BUILD_SAH 1u
#define RT_BVH_BUILD_HOST 2u  /* the scene's host build (app/bvh.cpp) uploaded: env RT_BVH=host */
int rt_renderer_build_bvh_ex(rt_renderer_h r, uint32_t method, rt_bvh_build_stats_t* stats);
/* How the renderer's current tree was built: rt_renderer_create builds it on
 * the device with RT_BVH_BUILD_SAH (the host builder's tree bit for bit;
 * RT_BVH_BUILD_HOST under env RT_BVH=host or for a scene without geometry),
 * or the last rt_renderer_build_bvh_ex. */
int rt_renderer_bvh_stats(rt_renderer_h r, rt_bvh_build_stats_t* stats);
#define RT_BVH_STACK4_UNUSED 0xFFFFFFFFu
/* the renderer's current BVH4 (float[num_nodes4][32], rt_node4_t: the host
 * tree's collapse, or after rt_renderer_build_bvh the device collapse --
 * BVH4 node i at the BVH2 index of every even-depth internal node, zeros
 * elsewhere).  NO REFERENCE. */
int rt_renderer_export_bvh4(rt_renderer_h r, float* nodes4, uint32_t* num_nodes4);
/* the same nodes as 64-B rt_node4h_t records (binary16 planes, the layout the
 * kernels read), num_nodes4 * 64 bytes */
int rt_renderer_export_bvh4h(rt_renderer_h r, void* nodes4h, uint32_t* num_nodes4);
/* the renderer's current BVH (float[num_nodes][16], float[num_tris][12]) */
int rt_renderer_export_bvh(rt_renderer_h r, float* nodes, float* tris, uint32_t* num_nodes,
                           uint32_t* num_tris);

/* the primary rays' tree of the current configuration (NO REFERENCE): child
 * references int32[num_nodes][4] (rt_node4_t child encoding; leaf refs index
 * leaf_pids) and the pid of every leaf record -- by default a per-resolution
 * screen-space BVH4 over the covered-pixel rectangles (app/vis.h
 * BuildScreenTree).  NULL arrays: counts only. */
int rt_renderer_export_vis_tree(rt_renderer_h r, int32_t* refs, uint32_t* num_nodes,
                                int32_t* leaf_pids, uint32_t* num_leaf);

/* How the last rt_renderer_configure built its per-resolution records.  The
 * reference builds them per drawcall on the host (draw3d/main.cpp:179-211 ->
 * graphics::Binning, gfxutil.cpp:103-276); here kernels/rt_setup.hip builds
 * them unless RT_RENDER_HOST_SETUP. */
typedef struct {
  uint32_t device;        /* 1: device setup, 0: host loops */
  uint32_t launches;      /* device setup launches */
  uint32_t heavy_tiles;   /* local tiles whose weight (covering geometry primitives) > 0 */
  uint32_t blist_blocks;  /* local 8x8 blocks with candidate lists (0: primary rays walk the tree) */
  double setup_ms;        /* host wall time of the record build (uploads / launches included) */
  double configure_ms;    /* host wall time of the whole rt_renderer_configure */
  uint64_t blist_entries; /* candidate-list entries (0 when not built) */
  uint32_t blist_max;     /* the longest list */
  uint32_t slist_on;      /* 1: shadow rays test the light-space lists (rt_common.h) */
  uint64_t slist_entries; /* light-space shadow list entries */
  uint32_t path_queue;    /* 1: RT_RENDER_PATH runs in two kernels (pt_primary + pt_queue: a
                             frame is one launch group of 2, vortex_hip.h) */
  uint32_t slist_built;   /* 1: the last configure / set_light built shadow lists for a new light
                             (0: the lists of an unchanged light were kept) */
  uint32_t slist_stale;   /* 1: the light moved since its lists were built and none are queued:
                             frames walk the BVH for their shadow rays (rt_renderer_set_list_policy) */
} rt_setup_stats_t;
/* (reads back the status of shadow lists queued by rt_renderer_set_light:
 * waits for the device) */
int rt_renderer_setup_stats(rt_renderer_h r, rt_setup_stats_t* stats);

/* Move the point light of the current configuration (primary+shadow or path
 * frames; clip (x, y, w)): the light in the render arguments, queued behind
 * the frames already started, with no host wait; the frames started after it
 * see the new light.  When the configuration's shadow rays use the
 * light-space lists, the lists for the new light are a stream-ordered chain
 * of setup launches (kernels/rt_setup.hip SPROJ .. SSORT, ~0.1 ms at 1024^2)
 * whose last launch decides on the device whether they fit (else the frames'
 * shadow rays walk the BVH).  By default (rt_renderer_set_list_policy) the
 * chain is deferred: the frames after the change trace their shadow rays by
 * the BVH packet walk -- the same verdicts, no wait for lists -- and the
 * lists are queued once the light has stayed for `defer_frames` frames.  The
 * reference re-bins its scene on the host for every render
 * (tests/regression/draw3d/main.cpp:179-211 -> gfxutil.cpp:103-276); this
 * is the per-frame handling of the only light-dependent structure. */
int rt_renderer_set_light(rt_renderer_h r, const float light[3]);
/* When set_light queues a light's shadow lists: 0 = at once (set_light);
 * n > 0 = before the (n + 1)-th frame started with that light, the n frames
 * before walking the BVH for their shadow rays (default 8, env
 * RT_SLIST_DEFER; a build costs about as much as that many frames save).
 * NO REFERENCE. */
int rt_renderer_set_list_policy(rt_renderer_h r, uint32_t defer_frames);

/* Read back one per-resolution record array of the current configuration
 * (layouts: kernels/rt_common.h; NO REFERENCE).  out NULL = size query
 * (*size = bytes). */
#define RT_REC_PRIMS 0u     /* rt_prim_t per primitive (128 B) */
#define RT_REC_BBOX 1u      /* rt_bbox_t per primitive (raster mode or device setup) */
#define RT_REC_VIS 2u       /* uint32[4] per primitive: rectangle x, y, depth bound, any */
#define RT_REC_VNODES 3u    /* rt_vnode_t per node of the primary rays' tree */
#define RT_REC_VTRIS 4u     /* rt_vtri_t per leaf record (+3 pads) */
#define RT_REC_VLAYERS 5u   /* rt_vtri_t per screen layer, last drawn first */
#define RT_REC_VGEOM 6u     /* rt_vtri_t per geometry primitive, ascending pid */
#define RT_REC_ORDER 7u     /* u32 per local tile: the work order */
#define RT_REC_PTRIS 8u     /* rt_tri_t per primitive (clip v0 + pid, e1, e2) */
#define RT_REC_GEOM 9u      /* rt_tri_t per geometry primitive */
#define RT_REC_BIDX 10u     /* uint32[2] per local 8x8 block: first list entry, count */
#define RT_REC_BLIST 11u    /* rt_bentry_t per list entry (+3 padding entries, RT_BLIST_PAD) */
#define RT_REC_SIDX 12u     /* uint32[2] per light-space cell: first entry, count */
#define RT_REC_SLIST 13u    /* rt_tri_t per light-space list entry (+1 padding record) */
int rt_renderer_export_records(rt_renderer_h r, uint32_t which, void* out, uint64_t bytes,
                               uint64_t* size);

/* raw per-workgroup counter rows of the last launch (16 u32 each; the
 * RT_STAMPS diagnostic images put wave timestamps in slots 12-15) */
int rt_launch_rows(rt_renderer_h r, uint32_t* rows, uint64_t max_rows, uint64_t* nrows);

/* Multi-GPU frame exchange for C hosts (include/rt_shard.h, librt_shard.so,
 * RCCL): after rt_render, gather every rank's compact tile buffer to rank 0
 * and assemble the frame there, on the renderer's stream; rank 0 copies it
 * to `image` (W*H ARGB8888, row 0 = NDC y = -1) when not NULL.  The
 * renderer must be configured with shard_index / shard_count = the
 * communicator's rank / size.  Collective.  NO REFERENCE. */
struct rt_shard_comm;
int rt_render_gather(rt_renderer_h r, struct rt_shard_comm* comm, uint32_t* image);

/* device pointer + byte size of the output buffer (for RCCL gathers) and the
 * HIP stream the kernel runs on (for stream-ordered consumers) */
int rt_framebuffer_device(rt_renderer_h r, void** device_ptr, uint64_t* bytes);
int rt_device_stream(rt_renderer_h r, void** hip_stream);
int rt_device_caps(rt_renderer_h r, uint64_t caps[8]);

#ifdef __cplusplus
}
#endif

#endif /* VX_RT_H */
