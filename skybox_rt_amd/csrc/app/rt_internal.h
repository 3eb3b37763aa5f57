// rt_internal.h -- the RT host app's scene / renderer state (librtapp.so
// internals shared by rt_app.cpp and device_setup.cpp; not part of the ABI).
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "app_util.h"
#include "bvh.h"
#include "cgltrace.h"
#include "rt_common.h"
#include "vortex.h"
#include "vortex_hip.h"
#include "vx_rt.h"

struct rt_scene {
  rt::Scene scene;
  rt::Bvh bvh;                    // the host build: on request only (host_bvh)
  std::vector<rt::BuildTri> build_tris;  // its input: the depth-tested triangles, clip (x, y, w)
  bool bvh_built = false;
  std::vector<int32_t> geometry;  // depth-tested prims (BVH input), ascending
  std::vector<int32_t> layers;    // screen-layer prims, descending pid
  std::string unsupported;        // non-empty: the RT path cannot render it
  bool tie_high = false;
  double parse_ms = 0, bvh_ms = 0;
};

// a device buffer of the setup that persists across configurations and only
// grows (device_setup.cpp ensure)
struct DevScratch {
  vx_buffer_h h = nullptr;
  uint64_t addr = 0;
};
// the device setup's argument block, status words and scratch arrays
struct SetupScratch {
  DevScratch args, status, parent, count, weight, hist, bcnt, bpart, btmp;
  DevScratch scnt, spart, sproj, soff, skey, stmp;
  DevScratch sah, sah_args;  // the SAH build's arrays (one buffer) and argument block
  uint64_t bcap = 0;   // block-list entry capacity of btmp / blist
  uint32_t scap = 0;   // shadow-list entry capacity of stmp / slist
  uint64_t sah_bytes = 0;
  void release() {
    for (DevScratch* d : {&args, &status, &parent, &count, &weight, &hist, &bcnt, &bpart, &btmp, &scnt, &spart,
                          &sproj, &soff, &skey, &stmp, &sah, &sah_args})
      if (d->h) {
        vx_mem_free(d->h);
        d->h = nullptr;
      }
  }
};

struct rt_renderer {
  rt_scene* sc = nullptr;
  vx_device_h dev = nullptr;
  // kernel images [mode][instrumented]: mode 0 = primary+shadow (BVH),
  // 1 = path trace, 2 = flat list, 3 = raster (no instrumented image)
  vx_buffer_h krnl[4][2] = {};
  // path tracing in two kernels (the default with the binary16 BVH4): [0]
  // pt_primary (primary pass, path queue), [1] pt_queue (the queued paths);
  // [.][1] the instrumented images
  vx_buffer_h krnl_pq[2][2] = {};
  // RT_RENDER_BVH_WALK primary+shadow frames (binary16 BVH4 images only):
  // rt_bvh / rt_bvh_stats, the packet walks without the list code paths
  vx_buffer_h krnl_bvh[2] = {};
  vx_buffer_h sah_krnl = nullptr;  // bvh_sah.vxbin, loaded by the first device build
  vx_buffer_h pathq = nullptr, pathq_ctr = nullptr;
  bool pq = false;          // the configuration runs the two-kernel path tracer
  vx_buffer_h nodes = nullptr, nodes4 = nullptr, tris = nullptr, layers = nullptr, dcs = nullptr, tex = nullptr;
  vx_buffer_h ptris = nullptr, geom = nullptr, oms = nullptr, bbox = nullptr, zbuf = nullptr;
  vx_buffer_h order = nullptr;
  vx_buffer_h vnodes = nullptr, vtris = nullptr, vlayers = nullptr, vgeom = nullptr;
  vx_buffer_h blist = nullptr, bidx = nullptr;  // per-block candidate lists (rt_bentry_t)
  vx_buffer_h sidx = nullptr, slist = nullptr;  // light-space shadow lists (built for sl_light)
  bool sl_mode = false;     // this configuration's shadow rays use the light-space lists
  bool sl_pending = false;  // lists queued by rt_renderer_set_light, status not read yet
  // the moving light (rt_renderer_set_list_policy): after a light change the
  // frames trace their shadow rays by the BVH packet walk (slist_on = 0, no
  // wait for lists) until the light has stayed for sl_defer frames; then the
  // lists are queued before the next frame.  0: set_light queues them at once
  uint32_t sl_defer = 8;
  bool sl_stale = false;    // the light moved since the lists were built; lists not queued yet
  uint32_t sl_static = 0;   // frames started since that light change
  SetupScratch su;
  vx_hip_copy_to_dev_async_t copy_async = nullptr;
  vx_hip_set_launch_tag_t set_tag = nullptr;
  vx_hip_set_launch_words_t set_words = nullptr;  // a frame's light + flags (RT_LW_*)
  vx_hip_host_mem_t host_mem = nullptr;
  volatile uint32_t* stat_host = nullptr;  // pinned status words (+ nonce) of the setup sequences
  uint64_t stat_dev = 0;
  uint32_t stat_nonce = 0;
  uint32_t stat_pending = 0;  // nonce of the last sequence issued with the pinned status copy (0: none)
  float sl_light[3] = {0, 0, 0};
  uint32_t sl_n = 0;        // the cube-map resolution they were built at
  bool sl_built = false;
  bool sl_rejected = false;  // built for sl_light / sl_n and too large (block_lists_fit)
  uint64_t sl_entries = 0;
  vx_buffer_h gather_recv = nullptr, gather_image = nullptr;  // rank 0 of rt_render_gather
  vx_buffer_h prims = nullptr, cbuf = nullptr, args = nullptr;
  // device-side setup (device_setup.cpp, kernels/rt_setup.hip): the image,
  // the resolution-independent inputs uploaded once at creation, and the
  // per-primitive visibility records of the current configuration
  vx_buffer_h setup_krnl = nullptr, verts = nullptr, pdc = nullptr, dcz = nullptr;
  vx_buffer_h layer_list = nullptr, geometry_list = nullptr, vis = nullptr;
  uint64_t cbuf_bytes = 0;
  rt_render_params_t params{};
  rt_kernel_arg_t arg{};
  bool configured = false;
  uint32_t local_tiles = 0;
  vx_hip_mem_ptr_t mem_ptr = nullptr;
  vx_hip_stream_t stream = nullptr;
  vx_hip_last_run_t last_run = nullptr;
  vx_hip_mpm_rows_t mpm_rows = nullptr;
  vx_hip_run_totals_t run_totals = nullptr;
  vx_hip_set_counters_t set_counters = nullptr;
  vx_hip_launch_group_t launch_group = nullptr;
  vx_hip_set_timing_t set_timing = nullptr;
  std::string kdir;         // kernel directory (images missing there come from lib_dir)
  bool deep = false;        // generic RT/PT images (every BVH layout, 32-entry stack)
  // the primary rays' tree of the current configuration (rt_renderer_export_vis_tree;
  // host setup only -- after a device setup it is read back on request)
  std::vector<std::array<int32_t, 4>> vis_refs;
  std::vector<int32_t> vis_pids;
  bool use_bvh4 = true;     // the configured traversal reads the BVH4
  bool gpu_bvh = false;     // nodes/tris were built on the device (rt_renderer_build_bvh)
  bool gpu_bvh4 = false;    // ... and collapsed to a BVH4 there whose stack fits the images
  uint32_t num_tris = 0;    // leaf triangle records (without the 3 padding records)
  rt_setup_stats_t setup{};  // the last configuration's setup (rt_renderer_setup_stats)
  rt_bvh_build_stats_t bvh_stats{};  // how the current tree was built (rt_renderer_bvh_stats)

  ~rt_renderer() {
    vx_buffer_h* bufs[] = {&krnl[0][0], &krnl[0][1], &krnl[1][0], &krnl[1][1], &krnl[2][0],
                           &krnl[2][1], &krnl[3][0], &nodes, &nodes4, &tris, &layers, &dcs, &tex,
                           &ptris, &geom, &oms, &bbox, &zbuf, &order, &vnodes, &vtris, &vlayers,
                           &vgeom, &gather_recv, &gather_image, &prims, &cbuf, &args,
                           &setup_krnl, &verts, &pdc, &dcz, &layer_list, &geometry_list, &vis,
                           &blist, &bidx, &sidx, &slist, &krnl_pq[0][0], &krnl_pq[0][1],
                           &krnl_pq[1][0], &krnl_pq[1][1], &pathq, &pathq_ctr,
                           &krnl_bvh[0], &krnl_bvh[1], &sah_krnl};
    for (auto* b : bufs) {
      if (*b) vx_mem_free(*b);
      *b = nullptr;
    }
    su.release();
    if (dev) vx_dev_close(dev);
  }
};

namespace rtapp {

// the scene's host BVH (app/bvh.cpp), built on first use: the renderer
// builds its tree on the device (bvh_sah.hip) unless env RT_BVH=host
int host_bvh(rt_scene* s);

// (re)allocate *buf (size bytes, or 64 when 0), copy `data` when given; the
// device address must lie below 4 GiB (the kernels' 32-bit arena offsets)
int upload(vx_device_h dev, const void* data, uint64_t size, vx_buffer_h* buf, uint64_t* addr);
// kernel image `name` from the renderer's kernel directory (else the library's)
int load_image(rt_renderer* r, const std::string& name, vx_buffer_h* out);

struct DevBuf {  // scratch buffer freed at scope exit
  vx_buffer_h h = nullptr;
  uint64_t addr = 0;
  ~DevBuf() {
    if (h) vx_mem_free(h);
  }
};

// device_setup.cpp: the resolution-independent inputs of the device setup
// and the triangle records built from them (ptris, geom) at renderer creation
int device_ingest(rt_renderer* r, bool records);
// the per-resolution records of rt_renderer_configure on the device: prims
// (+ bbox, zbuf clear for raster), vis / vtris / vlayers / vgeom / vnodes,
// the tile order (heavy = local tiles with weight > 0), the cleared cbuf.
// r->arg holds the layout fields (tiles, shard, flags, the tree); the
// record buffers grow as needed and their addresses are set in r->arg.
// lists: also the per-block candidate lists (rt_bentry_t, the bidx / blist
// buffers and arg.blist_blocks; 0 when they do not fit, block_lists_fit);
// slists: the light-space shadow lists for a.light unless current (kept
// while the light is unchanged; arg.slist_on 0 when they do not fit).  One
// stream-ordered launch sequence, one status read-back.
int device_setup(rt_renderer* r, bool raster, bool order_on, bool lists, bool slists, uint32_t* heavy,
                 uint32_t* launches);
// rt_renderer_set_light: the new light into the render arguments and, when
// the configuration uses them, its shadow lists -- all queued on the
// driver's stream behind the in-flight frames, no host wait
int set_light(rt_renderer* r, const float light[3], uint32_t* launches);
// the shadow lists for the current light, queued on the driver's stream (the
// set_light policy 0, or a deferred build once the light stays)
int queue_lists(rt_renderer* r, uint32_t* launches);
// read the status of lists queued by set_light (waits for the device): their
// size, an overflow refill, r->sl_built
int settle_lists(rt_renderer* r);
// whether lists with this longest list and this many entries are built
// (RT_BLIST_MAX_LIST, the device sort's limit; env RT_BLIST_MAX_ENTRIES,
// default 16 M entries = 512 MiB of list and sort buffers)
bool block_lists_fit(uint64_t longest, uint64_t entries);

}  // namespace rtapp
