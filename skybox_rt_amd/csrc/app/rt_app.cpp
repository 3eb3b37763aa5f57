// rt_app.cpp -- librtapp.so: the RT host app behind include/vx_rt.h.
//
// Mirrors the host structure of tests/regression/draw3d/main.cpp:
//   scene load (:428-455) -> kernel upload (:459) -> buffer allocation and
//   clears (:461-490) -> per-frame state + kernel_arg upload (:179-347) ->
//   vx_start / vx_ready_wait (:349-361) -> vx_mpm_query (:367-372) ->
//   framebuffer read-back (:380-387).
// The acceleration structure differs (BVH over clip space instead of
// per-frame screen-tile binning, gfxutil.cpp:103-276): the BVH is built once
// per scene at load time and is resolution independent.
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <map>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "VX_types.h"
#include "app_util.h"
#include "bvh.h"
#include "bvh_common.h"
#include "cgltrace.h"
#include "rt_internal.h"
#include "sah_common.h"
#include "setup_common.h"
#include "setup.h"
#include "vis.h"
#include "vortex.h"
#include "rt_shard.h"
#include "vortex_hip.h"
#include "vx_rt.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& m, int code = -1) {
  g_err = m;
  return code;
}

std::string lib_dir() {
  Dl_info info;
  if (dladdr((void*)&lib_dir, &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    auto pos = p.rfind('/');
    if (pos != std::string::npos) return p.substr(0, pos);
  }
  return ".";
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

namespace rtapp {
int set_error(const std::string& message, int code) { return fail(message, code); }
std::string library_dir() { return lib_dir(); }
}  // namespace rtapp

using rtapp::DevBuf;
using rtapp::load_image;
using rtapp::upload;

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }

int rt_scene_load(const char* path, rt_scene_h* out) {
  return rt_scene_load_range(path, 0u, 0xffffffffu, out);
}

int rt_scene_load_range(const char* path, uint32_t start_draw, uint32_t end_draw, rt_scene_h* out) {
  if (path == nullptr || out == nullptr) return fail("null argument");
  auto sc = std::make_unique<rt_scene>();
  auto t0 = std::chrono::steady_clock::now();
  std::string err;
  if (rt::LoadCGLTrace(path, &sc->scene, &err) != 0) return fail(err);
  if (start_draw != 0u || end_draw != 0xffffffffu) {
    // draw3d -s / -e (main.cpp:179-181): drawcalls outside [start, end] are
    // not drawn; the kept ones keep their order (and so every tie rule)
    rt::Scene all = std::move(sc->scene);
    sc->scene = rt::Scene();
    sc->scene.textures = std::move(all.textures);
    for (uint32_t d = 0; d < (uint32_t)all.drawcalls.size(); ++d) {
      if (d < start_draw || d > end_draw) continue;
      rt::DrawCall dc = all.drawcalls[d];
      dc.prim_offset = (uint32_t)sc->scene.prims.size();
      sc->scene.prims.insert(sc->scene.prims.end(), all.prims.begin() + all.drawcalls[d].prim_offset,
                             all.prims.begin() + all.drawcalls[d].prim_offset + dc.prim_count);
      sc->scene.drawcalls.push_back(dc);
    }
  }
  sc->parse_ms = ms_since(t0);
  // classify drawcalls (DESIGN.md "Scope"): screen layers (depth test off)
  // must precede geometry; geometry shares one LESS/LEQUAL depth function.
  bool seen_geom = false;
  int geom_func = -1;
  std::vector<rt::BuildTri> build;
  for (size_t d = 0; d < sc->scene.drawcalls.size(); ++d) {
    const rt::DrawCall& dc = sc->scene.drawcalls[d];
    const rt::States& st = dc.states;
    if (st.blend_enabled || st.stencil_test || (st.color_writemask & 0xf) != 0xf)
      sc->unsupported = "drawcall " + std::to_string(d) + " uses blending/stencil/partial writes";
    if (st.depth_test) {
      // the depth test's winner is the closest hit only while every
      // geometry fragment that passes also writes its depth
      if (!(st.depth_writemask & 1)) sc->unsupported = "depth-tested drawcall without depth writes";
      const int f = (int)rt::ToVXCompare(st.depth_func);
      if (f != VX_OM_DEPTH_FUNC_LESS && f != VX_OM_DEPTH_FUNC_LEQUAL)
        sc->unsupported = "depth function other than LESS/LEQUAL";
      if (geom_func >= 0 && f != geom_func) sc->unsupported = "mixed depth functions";
      geom_func = f;
      seen_geom = true;
    } else if (seen_geom) {
      sc->unsupported = "screen layer drawn after depth-tested geometry";
    }
    for (uint32_t i = 0; i < dc.prim_count; ++i) {
      const int32_t g = (int32_t)(dc.prim_offset + i);
      if (st.depth_test) {
        rt::BuildTri bt;
        const auto& p = sc->scene.prims[g];
        for (int c = 0; c < 3; ++c) {
          bt.v[c][0] = p[c].pos[0];
          bt.v[c][1] = p[c].pos[1];
          bt.v[c][2] = p[c].pos[3];  // clip (x, y, w)
        }
        bt.pid = g;
        build.push_back(bt);
        sc->geometry.push_back(g);
      } else {
        sc->layers.push_back(g);
      }
    }
  }
  std::reverse(sc->layers.begin(), sc->layers.end());
  sc->tie_high = geom_func == VX_OM_DEPTH_FUNC_LEQUAL;
  sc->build_tris = std::move(build);
  *out = sc.release();
  return 0;
}

int rt_scene_free(rt_scene_h s) {
  delete s;
  return 0;
}

int rt_scene_info(rt_scene_h s, rt_scene_info_t* info) {
  if (!s || !info) return fail("null argument");
  if (rtapp::host_bvh(s) != 0) return -1;
  std::memset(info, 0, sizeof(*info));
  info->num_drawcalls = (uint32_t)s->scene.drawcalls.size();
  info->num_prims = (uint32_t)s->scene.prims.size();
  info->num_geometry = (uint32_t)s->geometry.size();
  info->num_layer = (uint32_t)s->layers.size();
  info->num_textures = (uint32_t)s->scene.textures.size();
  info->bvh_nodes = (uint32_t)s->bvh.nodes.size();
  info->bvh_tris = (uint32_t)s->bvh.tris.size();
  info->bvh_leaves = s->bvh.leaves;
  info->bvh_depth = s->bvh.depth;
  info->bvh4_nodes = (uint32_t)s->bvh.nodes4.size();
  info->bvh4_depth = s->bvh.depth4;
  info->bvh4_stack = s->bvh.stack4;
  info->bvh4_f16 = s->bvh.nodes4h.empty() ? 0u : 1u;
  info->parse_ms = s->parse_ms;
  info->bvh_ms = s->bvh_ms;
  return 0;
}

int rt_scene_export_prims(rt_scene_h s, float* out, uint64_t count) {
  if (!s || !out) return fail("null argument");
  if (count < s->scene.prims.size()) return fail("buffer too small");
  for (size_t i = 0; i < s->scene.prims.size(); ++i)
    for (int c = 0; c < 3; ++c) {
      const rt::Vertex& v = s->scene.prims[i][c];
      float* o = out + (i * 3 + c) * 10;
      std::memcpy(o, v.pos, 16);
      std::memcpy(o + 4, v.color, 16);
      std::memcpy(o + 8, v.uv, 8);
    }
  return 0;
}

int rt_scene_export_bvh(rt_scene_h s, float* nodes, float* tris) {
  if (!s) return fail("null argument");
  if (rtapp::host_bvh(s) != 0) return -1;
  if (nodes) std::memcpy(nodes, s->bvh.nodes.data(), s->bvh.nodes.size() * sizeof(rt_node_t));
  if (tris) std::memcpy(tris, s->bvh.tris.data(), s->bvh.tris.size() * sizeof(rt_tri_t));
  return 0;
}

int rt_scene_export_bvh4(rt_scene_h s, float* nodes4) {
  if (!s || !nodes4) return fail("null argument");
  if (rtapp::host_bvh(s) != 0) return -1;
  std::memcpy(nodes4, s->bvh.nodes4.data(), s->bvh.nodes4.size() * sizeof(rt_node4_t));
  return 0;
}

}  // extern "C"

int rtapp::host_bvh(rt_scene* s) {
  if (s->bvh_built) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  std::string err;
  if (rt::BuildBvh(s->build_tris, &s->bvh, &err) != 0) return fail(err);
  s->bvh_ms = ms_since(t0);
  s->bvh_built = true;
  return 0;
}

bool rtapp::block_lists_fit(uint64_t longest, uint64_t entries) {
  uint64_t cap = 16ull << 20;
  if (const char* e = std::getenv("RT_BLIST_MAX_ENTRIES")) cap = std::strtoull(e, nullptr, 0);
  return longest <= RT_BLIST_MAX_LIST && entries <= cap;
}

int rtapp::upload(vx_device_h dev, const void* data, uint64_t size, vx_buffer_h* buf,
                  uint64_t* addr) {
  const uint64_t sz = size ? size : 64;
  if (*buf) vx_mem_free(*buf);
  *buf = nullptr;
  if (vx_mem_alloc(dev, sz, VX_MEM_READ, buf) != 0) return fail("vx_mem_alloc failed");
  if (data && size && vx_copy_to_dev(*buf, data, 0, size) != 0) return fail("vx_copy_to_dev failed");
  if (vx_mem_address(*buf, addr) != 0) return fail("vx_mem_address failed");
  // the kernel addresses every buffer with 32-bit offsets into one arena
  // descriptor (vx_arena in vx_spawn.h)
  if (*addr + sz > (1ull << 32)) return fail("buffer beyond the 4 GiB kernel address range");
  return 0;
}

static int build_sah(rt_renderer_h r, rt_bvh_build_stats_t* st);

extern "C" {

int rt_renderer_create(rt_scene_h s, const char* kernel_dir, rt_renderer_h* out) {
  if (!s || !out) return fail("null argument");
  auto r = std::make_unique<rt_renderer>();
  r->sc = s;
  if (vx_dev_open(&r->dev) != 0) {
    r->dev = nullptr;
    return fail("vx_dev_open failed (no GPU or driver missing)");
  }
  const std::string dir = kernel_dir ? kernel_dir : lib_dir();
  r->kdir = dir;
  // the tree: built on the device from the ingested triangles (bvh_sah.hip,
  // the host builder's binned SAH restated, equal to it bit for bit) unless
  // env RT_BVH=host asks for the host build (app/bvh.cpp) uploaded; so does
  // the host builder's fp32-box BVH4 variant (env RT_BVH_F16=0)
  const char* bv = std::getenv("RT_BVH");
  const char* f16 = std::getenv("RT_BVH_F16");
  const bool host_tree = (bv && std::string(bv) == "host") || (f16 && std::atoi(f16) == 0) ||
                         s->geometry.empty();
  if (host_tree && rtapp::host_bvh(s) != 0) return -1;
  static const rt::Bvh kEmpty{};
  const rt::Bvh& bvh = host_tree ? s->bvh : kEmpty;
  // the regular image's LDS stack holds RT_STACK_SHALLOW (24) entries; a BVH whose traversal may
  // need more (BVH2: its depth, BVH4: its stack bound) uses the deep image
  // (32 entries, lower occupancy); build_sah decides for a device tree
  const bool deep = std::max(bvh.depth, bvh.stack4) > RT_STACK_SHALLOW;
  if (std::max(bvh.depth, bvh.stack4) > RT_STACK_DEEP)
    return fail("BVH too deep for the traversal stack");
  r->deep = deep;
  const char* names[4][2] = {
      {deep ? "rt_kernel_deep.vxbin" : "rt_kernel.vxbin",
       deep ? "rt_kernel_deep_stats.vxbin" : "rt_kernel_stats.vxbin"},
      {deep ? "pt_kernel_deep.vxbin" : "pt_kernel.vxbin",
       deep ? "pt_kernel_deep_stats.vxbin" : "pt_kernel_stats.vxbin"},
      {"rt_flat.vxbin", "rt_flat_stats.vxbin"},
      {"raster_kernel.vxbin", nullptr}};
  // images missing from kernel_dir (e.g. an A/B variant directory holding
  // only rt_kernel*) come from the library directory
  for (int m = 0; m < 4; ++m)
    for (int i = 0; i < 2; ++i) {
      if (!names[m][i]) continue;
      std::string path = dir + "/" + names[m][i];
      if (FILE* f = std::fopen(path.c_str(), "rb")) std::fclose(f);
      else path = lib_dir() + "/" + names[m][i];
      if (vx_upload_kernel_file(r->dev, path.c_str(), &r->krnl[m][i]) != 0)
        return fail("cannot upload kernel " + path);
    }
  r->mem_ptr = (vx_hip_mem_ptr_t)vx_driver_symbol("vx_hip_mem_ptr");
  r->stream = (vx_hip_stream_t)vx_driver_symbol("vx_hip_stream");
  r->last_run = (vx_hip_last_run_t)vx_driver_symbol("vx_hip_last_run");
  r->mpm_rows = (vx_hip_mpm_rows_t)vx_driver_symbol("vx_hip_mpm_rows");
  r->run_totals = (vx_hip_run_totals_t)vx_driver_symbol("vx_hip_run_totals");
  r->set_counters = (vx_hip_set_counters_t)vx_driver_symbol("vx_hip_set_counters");
  r->launch_group = (vx_hip_launch_group_t)vx_driver_symbol("vx_hip_launch_group");
  r->set_timing = (vx_hip_set_timing_t)vx_driver_symbol("vx_hip_set_timing");
  r->copy_async = (vx_hip_copy_to_dev_async_t)vx_driver_symbol("vx_hip_copy_to_dev_async");
  // the moving-light policy (rt_renderer_set_list_policy); env RT_SLIST_DEFER
  if (const char* e = std::getenv("RT_SLIST_DEFER")) r->sl_defer = (uint32_t)std::atoi(e);
  r->set_tag = (vx_hip_set_launch_tag_t)vx_driver_symbol("vx_hip_set_launch_tag");
  r->set_words = (vx_hip_set_launch_words_t)vx_driver_symbol("vx_hip_set_launch_words");
  r->host_mem = (vx_hip_host_mem_t)vx_driver_symbol("vx_hip_host_mem");
  if (r->host_mem) {
    void* h = nullptr;
    if (r->host_mem(r->dev, 64, &h, &r->stat_dev) == 0) r->stat_host = (volatile uint32_t*)h;
  }
  // the two-kernel path tracer's images (binary16 BVH4 only; the others run
  // the one-kernel pt_kernel images), from the kernel directory itself: a
  // directory without them (e.g. lib/pt_compact) runs its own pt_kernel
  if (!deep) {
    const char* pq_names[2][2] = {{"pt_primary.vxbin", "pt_primary_stats.vxbin"},
                                  {"pt_queue.vxbin", "pt_queue_stats.vxbin"}};
    bool all = true;
    for (int m = 0; m < 2; ++m)
      for (int i = 0; i < 2; ++i)
        if (FILE* f = std::fopen((dir + "/" + pq_names[m][i]).c_str(), "rb")) std::fclose(f);
        else all = false;
    for (int m = 0; m < 2 && all; ++m)
      for (int i = 0; i < 2; ++i)
        if (vx_upload_kernel_file(r->dev, (dir + "/" + pq_names[m][i]).c_str(), &r->krnl_pq[m][i]) != 0)
          return fail("cannot upload kernel " + dir + "/" + pq_names[m][i]);
    // the BVH-walk primary+shadow images (RT_RENDER_BVH_WALK), from the
    // kernel directory or the library's
    const char* bvh_names[2] = {"rt_bvh.vxbin", "rt_bvh_stats.vxbin"};
    for (int i = 0; i < 2; ++i) {
      std::string path = dir + "/" + bvh_names[i];
      if (FILE* f = std::fopen(path.c_str(), "rb")) std::fclose(f);
      else path = lib_dir() + "/" + bvh_names[i];
      if (vx_upload_kernel_file(r->dev, path.c_str(), &r->krnl_bvh[i]) != 0)
        return fail("cannot upload kernel " + path);
    }
  }
  rt_kernel_arg_t& a = r->arg;
  std::memset(&a, 0, sizeof(a));
  // 3 padding records: the kernel fetches all 4 slots of a leaf at once
  std::vector<rt_tri_t> tris(bvh.tris);
  tris.resize(tris.size() + 3);
  std::memset(tris.data() + bvh.tris.size(), 0, 3 * sizeof(rt_tri_t));
  // BVH4: rt_node4_t array, then (binary16 boxes) the rt_node4h_t array
  std::vector<uint8_t> nodes4(bvh.nodes4.size() * sizeof(rt_node4_t) +
                              bvh.nodes4h.size() * sizeof(rt_node4h_t));
  if (!bvh.nodes4.empty()) {
    std::memcpy(nodes4.data(), bvh.nodes4.data(), bvh.nodes4.size() * sizeof(rt_node4_t));
    if (!bvh.nodes4h.empty())
      std::memcpy(nodes4.data() + bvh.nodes4.size() * sizeof(rt_node4_t), bvh.nodes4h.data(),
                  bvh.nodes4h.size() * sizeof(rt_node4h_t));
  }
  if (upload(r->dev, bvh.nodes.data(), bvh.nodes.size() * sizeof(rt_node_t), &r->nodes, &a.nodes_addr) ||
      upload(r->dev, nodes4.data(), nodes4.size(), &r->nodes4, &a.nodes4_addr) ||
      upload(r->dev, tris.data(), tris.size() * sizeof(rt_tri_t), &r->tris, &a.tris_addr))
    return -1;
  a.num_nodes = (uint32_t)bvh.nodes.size();
  a.num_nodes4 = (uint32_t)bvh.nodes4.size();
  r->num_tris = (uint32_t)bvh.tris.size();
  a.num_geom = (uint32_t)s->geometry.size();
  // the resolution-independent device-setup inputs, and every primitive's
  // clip-space triangle by pid (path-trace bounce hits) + the geometry
  // triangles in ascending pid order (flat-list mode) -- built on the device
  // unless env RT_SETUP=host
  const char* sv = std::getenv("RT_SETUP");
  const bool host_records = sv && std::string(sv) == "host";
  if (rtapp::device_ingest(r.get(), !host_records) != 0) return -1;
  if (host_records) {
    std::vector<rt_tri_t> pt(s->scene.prims.size());
    for (size_t g = 0; g < pt.size(); ++g) {
      const auto& p = s->scene.prims[g];
      std::memset(&pt[g], 0, sizeof(rt_tri_t));
      for (int k = 0; k < 3; ++k) {
        const int src = k == 2 ? 3 : k;
        pt[g].v[k] = p[0].pos[src];
        pt[g].v[4 + k] = p[1].pos[src] - p[0].pos[src];
        pt[g].v[8 + k] = p[2].pos[src] - p[0].pos[src];
      }
      const int32_t pid = (int32_t)g;
      std::memcpy(&pt[g].v[3], &pid, 4);
    }
    if (upload(r->dev, pt.data(), pt.size() * sizeof(rt_tri_t), &r->ptris, &a.ptris_addr)) return -1;
    std::vector<rt_tri_t> gl;
    for (int32_t g : s->geometry) gl.push_back(pt[g]);
    if (upload(r->dev, gl.data(), gl.size() * sizeof(rt_tri_t), &r->geom, &a.geom_addr)) return -1;
  }
  a.num_layer_tris = (uint32_t)s->layers.size();
  // textures: one buffer, each texture 256-B aligned
  std::vector<uint8_t> texels;
  std::map<int32_t, uint64_t> tex_off;
  for (auto& kv : s->scene.textures) {
    tex_off[kv.first] = texels.size();
    texels.insert(texels.end(), kv.second.pixels.begin(), kv.second.pixels.end());
    texels.resize((texels.size() + 255) & ~size_t(255));
  }
  uint64_t tex_addr = 0;
  if (upload(r->dev, texels.data(), texels.size(), &r->tex, &tex_addr)) return -1;
  std::vector<rt_dcstate_t> dcs;
  for (const rt::DrawCall& dc : s->scene.drawcalls) {
    rt_dcstate_t st = rt::DrawcallState(dc, s->scene);
    if (st.flags & RT_DC_TEX) st.tex_addr = tex_addr + tex_off[dc.texture_id];
    dcs.push_back(st);
  }
  if (upload(r->dev, dcs.data(), dcs.size() * sizeof(rt_dcstate_t), &r->dcs, &a.dcs_addr)) return -1;
  // output-merger state per drawcall (raster pipeline)
  std::vector<rt_omstate_t> oms;
  for (const rt::DrawCall& dc : s->scene.drawcalls) oms.push_back(rt::OmState(dc));
  if (upload(r->dev, oms.data(), oms.size() * sizeof(rt_omstate_t), &r->oms, &a.oms_addr)) return -1;
  a.num_drawcalls = (uint32_t)oms.size();
  std::memset(&r->bvh_stats, 0, sizeof(r->bvh_stats));
  if (!host_tree) {
    if (build_sah(r.get(), &r->bvh_stats) != 0) return -1;
  } else {
    r->bvh_stats.nodes = (uint32_t)bvh.nodes.size();
    r->bvh_stats.depth = bvh.depth;
    r->bvh_stats.stack4 = bvh.stack4;
    r->bvh_stats.nodes4 = (uint32_t)bvh.nodes4.size();
    r->bvh_stats.depth4 = bvh.depth4;
    r->bvh_stats.build_ms = s->bvh_ms;
    r->bvh_stats.method = RT_BVH_BUILD_HOST;
  }
  *out = r.release();
  return 0;
}

int rt_renderer_bvh_stats(rt_renderer_h r, rt_bvh_build_stats_t* st) {
  if (!r || !st) return fail("null argument");
  *st = r->bvh_stats;
  return 0;
}

static int tree_refs(rt_renderer* r, bool use_bvh4, std::vector<std::array<int32_t, 4>>* out_refs,
                     std::vector<int32_t>* out_pids);

int rt_renderer_export_vis_tree(rt_renderer_h r, int32_t* refs, uint32_t* num_nodes,
                                int32_t* leaf_pids, uint32_t* num_leaf) {
  if (!r || !r->configured) return fail("renderer not configured");
  // a device setup keeps no host copy: the traversed tree's references
  if (r->setup.device && !(r->params.flags & RT_RENDER_RASTER) && r->vis_refs.empty() &&
      tree_refs(r, r->use_bvh4, &r->vis_refs, &r->vis_pids) != 0)
    return -1;
  if (num_nodes) *num_nodes = (uint32_t)r->vis_refs.size();
  if (num_leaf) *num_leaf = (uint32_t)r->vis_pids.size();
  if (refs && !r->vis_refs.empty()) std::memcpy(refs, r->vis_refs.data(), r->vis_refs.size() * 16);
  if (leaf_pids && !r->vis_pids.empty())
    std::memcpy(leaf_pids, r->vis_pids.data(), r->vis_pids.size() * 4);
  return 0;
}

int rt_renderer_setup_stats(rt_renderer_h r, rt_setup_stats_t* st) {
  if (!r || !st) return fail("null argument");
  if (!r->configured) return fail("renderer not configured");
  if (rtapp::settle_lists(r) != 0) return -1;
  r->setup.slist_on = r->arg.slist_on;
  r->setup.slist_stale = r->sl_stale ? 1u : 0u;
  *st = r->setup;
  return 0;
}

int rt_renderer_set_light(rt_renderer_h r, const float light[3]) {
  if (!r || !light) return fail("null argument");
  if (!r->configured) return fail("renderer not configured");
  if (!(r->params.flags & (RT_RENDER_SHADOWS | RT_RENDER_PATH)) || (r->params.flags & RT_RENDER_RASTER))
    return fail("rt_renderer_set_light: the configuration traces no shadow rays");
  uint32_t launches = 0;
  if (rtapp::set_light(r, light, &launches) != 0) return -1;
  r->setup.slist_built = r->sl_mode ? 1u : 0u;
  return 0;
}

int rt_renderer_export_records(rt_renderer_h r, uint32_t which, void* out, uint64_t bytes,
                               uint64_t* size) {
  if (!r || !r->configured) return fail("renderer not configured");
  // lists queued by rt_renderer_set_light: their entry count (and slist_on)
  // are known once their status is read, before the exports are sized
  if ((which == RT_REC_SIDX || which == RT_REC_SLIST) && rtapp::settle_lists(r) != 0) return -1;
  const rt_kernel_arg_t& a = r->arg;
  const bool raster = (r->params.flags & RT_RENDER_RASTER) != 0;
  const uint64_t np = r->sc->scene.prims.size();
  vx_buffer_h b = nullptr;
  uint64_t n = 0;
  switch (which) {
    case RT_REC_PRIMS: b = r->prims; n = np * sizeof(rt_prim_t); break;
    case RT_REC_BBOX: b = r->bbox; n = np * sizeof(rt_bbox_t); break;
    case RT_REC_VIS: b = raster ? nullptr : r->vis; n = np * 16; break;
    case RT_REC_VNODES: b = raster ? nullptr : r->vnodes; n = (uint64_t)a.num_vnodes * sizeof(rt_vnode_t); break;
    case RT_REC_VTRIS: b = raster ? nullptr : r->vtris; n = ((uint64_t)r->num_tris + 3) * sizeof(rt_vtri_t); break;
    case RT_REC_VLAYERS: b = raster ? nullptr : r->vlayers; n = (uint64_t)r->sc->layers.size() * sizeof(rt_vtri_t); break;
    case RT_REC_VGEOM: b = raster ? nullptr : r->vgeom; n = (uint64_t)r->sc->geometry.size() * sizeof(rt_vtri_t); break;
    case RT_REC_ORDER: b = a.order_addr ? r->order : nullptr; n = (uint64_t)r->local_tiles * 4; break;
    case RT_REC_PTRIS: b = r->ptris; n = np * sizeof(rt_tri_t); break;
    case RT_REC_GEOM: b = r->geom; n = (uint64_t)r->sc->geometry.size() * sizeof(rt_tri_t); break;
    case RT_REC_BIDX: b = a.blist_blocks ? r->bidx : nullptr; n = (uint64_t)a.blist_blocks * 8; break;
    case RT_REC_BLIST:
      b = a.blist_blocks ? r->blist : nullptr;
      n = (r->setup.blist_entries + RT_BLIST_PAD) * sizeof(rt_bentry_t);
      break;
    case RT_REC_SIDX: b = a.slist_on ? r->sidx : nullptr; n = 6ull * a.slist_n * a.slist_n * 8; break;
    case RT_REC_SLIST: b = a.slist_on ? r->slist : nullptr; n = (r->sl_entries + 1) * sizeof(rt_tri_t); break;
    default: return fail("unknown record array");
  }
  if (!b) return fail("record array not present in this configuration");
  if (size) *size = n;
  if (!out) return 0;
  if (bytes < n) return fail("buffer too small");
  return (n == 0 || vx_copy_from_dev(out, b, 0, n) == 0) ? 0 : fail("vx_copy_from_dev failed");
}

int rt_renderer_free(rt_renderer_h r) {
  delete r;
  return 0;
}

int rt_scene_setup_prims(rt_scene_h s, uint32_t width, uint32_t height, int32_t* out,
                         uint64_t count) {
  if (!s || !out || width == 0 || height == 0) return fail("bad argument");
  if (count < s->scene.prims.size()) return fail("buffer too small");
  for (size_t d = 0; d < s->scene.drawcalls.size(); ++d) {
    const rt::DrawCall& dc = s->scene.drawcalls[d];
    for (uint32_t i = 0; i < dc.prim_count; ++i) {
      rt_prim_t p;
      rt::PrimSetup(s->scene.prims[dc.prim_offset + i], width, height, dc.viewport[4],
                    dc.viewport[5], &p);
      p.dc = (uint32_t)d;
      std::memcpy(out + (size_t)(dc.prim_offset + i) * 32, &p, sizeof(p));
    }
  }
  return 0;
}

int rt_scene_setup_vis(rt_scene_h s, uint32_t width, uint32_t height, uint32_t* out,
                       uint64_t count) {
  if (!s || !out || width == 0 || height == 0) return fail("bad argument");
  if (count < s->scene.prims.size()) return fail("buffer too small");
  for (size_t d = 0; d < s->scene.drawcalls.size(); ++d) {
    const rt::DrawCall& dc = s->scene.drawcalls[d];
    for (uint32_t i = 0; i < dc.prim_count; ++i) {
      const uint32_t g = dc.prim_offset + i;
      rt_prim_t p;
      rt_bbox_t bb{0, 0};
      const bool ok = rt::PrimSetup(s->scene.prims[g], width, height, dc.viewport[4],
                                    dc.viewport[5], &p) == rt::kSetupOk &&
                      rt::PrimBBox(s->scene.prims[g], width, height, &bb) == rt::kSetupOk;
      const rt::VisPrim v = rt::ComputeVisPrim(p, ok, bb, width, height);
      out[3 * g + 0] = v.rx;
      out[3 * g + 1] = v.ry;
      out[3 * g + 2] = v.zmin;
    }
  }
  return 0;
}

int rt_scene_vis_tree(rt_scene_h s, uint32_t width, uint32_t height, float depth_scale,
                      int32_t* refs, uint32_t* num_nodes, int32_t* leaf_pids, uint32_t* num_leaf,
                      uint32_t* stack4) {
  if (!s || width == 0 || height == 0) return fail("bad argument");
  std::vector<rt::VisPrim> vis(s->scene.prims.size());
  for (size_t d = 0; d < s->scene.drawcalls.size(); ++d) {
    const rt::DrawCall& dc = s->scene.drawcalls[d];
    for (uint32_t i = 0; i < dc.prim_count; ++i) {
      const uint32_t g = dc.prim_offset + i;
      rt_prim_t p;
      rt_bbox_t bb{0, 0};
      const bool ok = rt::PrimSetup(s->scene.prims[g], width, height, dc.viewport[4],
                                    dc.viewport[5], &p) == rt::kSetupOk &&
                      rt::PrimBBox(s->scene.prims[g], width, height, &bb) == rt::kSetupOk;
      vis[g] = rt::ComputeVisPrim(p, ok, bb, width, height);
    }
  }
  std::vector<std::array<int32_t, 4>> rf;
  std::vector<int32_t> lp;
  uint32_t st = 0;
  if (rt::BuildScreenTree(vis, s->geometry, depth_scale, &rf, &lp, &st) != 0)
    return fail("screen tree build failed");
  if (num_nodes) *num_nodes = (uint32_t)rf.size();
  if (num_leaf) *num_leaf = (uint32_t)lp.size();
  if (stack4) *stack4 = st;
  if (refs && !rf.empty()) std::memcpy(refs, rf.data(), rf.size() * 16);
  if (leaf_pids && !lp.empty()) std::memcpy(leaf_pids, lp.data(), lp.size() * 4);
  return 0;
}

}  // extern "C"

int rtapp::load_image(rt_renderer* r, const std::string& name, vx_buffer_h* out) {
  std::string path = r->kdir + "/" + name;
  if (FILE* f = std::fopen(path.c_str(), "rb")) std::fclose(f);
  else path = lib_dir() + "/" + name;
  if (*out) vx_mem_free(*out);
  *out = nullptr;
  return vx_upload_kernel_file(r->dev, path.c_str(), out) == 0 ? 0 : fail("cannot upload kernel " + path);
}

extern "C" {

namespace {

// the generic RT / PT images: every BVH layout, the 32-entry traversal stack
int load_deep_images(rt_renderer* r) {
  if (load_image(r, "rt_kernel_deep.vxbin", &r->krnl[0][0]) ||
      load_image(r, "rt_kernel_deep_stats.vxbin", &r->krnl[0][1]) ||
      load_image(r, "pt_kernel_deep.vxbin", &r->krnl[1][0]) ||
      load_image(r, "pt_kernel_deep_stats.vxbin", &r->krnl[1][1]))
    return -1;
  r->deep = true;
  return 0;
}

}  // namespace

// child references (4 per node; a BVH2 uses slots 0-1) and leaf-record pids
// of the tree the kernels traverse: the host tree, or the device tree read back
static int tree_refs(rt_renderer* r, bool use_bvh4, std::vector<std::array<int32_t, 4>>* out_refs,
                     std::vector<int32_t>* out_pids) {
  const rt_scene* s = r->sc;
  const rt_kernel_arg_t& a = r->arg;
  std::vector<std::array<int32_t, 4>>& refs = *out_refs;
  std::vector<int32_t>& leaf_pids = *out_pids;
  refs.clear();
  leaf_pids.clear();
  std::vector<rt_node4_t> n4;
  std::vector<rt_node_t> n2;
  std::vector<rt_tri_t> tr;
  if (r->gpu_bvh) {
    tr.resize(r->num_tris);
    if (r->num_tris && vx_copy_from_dev(tr.data(), r->tris, 0, tr.size() * sizeof(rt_tri_t)) != 0)
      return fail("vx_copy_from_dev failed");
    if (use_bvh4) {
      n4.resize(a.num_nodes4);
      if (!n4.empty() && vx_copy_from_dev(n4.data(), r->nodes4, 0, n4.size() * sizeof(rt_node4_t)) != 0)
        return fail("vx_copy_from_dev failed");
    } else {
      n2.resize(a.num_nodes);
      if (!n2.empty() && vx_copy_from_dev(n2.data(), r->nodes, 0, n2.size() * sizeof(rt_node_t)) != 0)
        return fail("vx_copy_from_dev failed");
    }
  } else {
    if (rtapp::host_bvh(r->sc) != 0) return -1;
    tr = s->bvh.tris;
    if (use_bvh4) n4 = s->bvh.nodes4;
    else n2 = s->bvh.nodes;
  }
  for (const rt_tri_t& t : tr) {
    int32_t pid;
    std::memcpy(&pid, &t.v[3], 4);
    leaf_pids.push_back(pid);
  }
  if (use_bvh4) {
    for (const rt_node4_t& n : n4) {
      std::array<int32_t, 4> c;
      std::memcpy(c.data(), &n.v[24], 16);
      refs.push_back(c);
    }
  } else {
    for (const rt_node_t& n : n2) {
      std::array<int32_t, 4> c = {RT_EMPTY_REF, RT_EMPTY_REF, RT_EMPTY_REF, RT_EMPTY_REF};
      std::memcpy(c.data(), &n.v[12], 8);
      refs.push_back(c);
    }
  }
  return 0;
}

// Per-resolution primary-visibility records (app/vis.h): every primitive's
// covered-pixel rectangle and depth bound, the leaf / layer / flat-list
// rt_vtri_t records and the rt_vnode_t of the tree the kernels traverse
// (host tree, or the device tree read back).
static int configure_vis(rt_renderer* r, const std::vector<rt_prim_t>& prims,
                         const std::vector<rt::VisPrim>& vis, bool use_bvh4) {
  const rt_scene* s = r->sc;
  rt_kernel_arg_t& a = r->arg;
  // the primary rays' tree: the secondary rays' tree (the host tree or the
  // device tree read back), whose nodes get the pixel rectangles and depth
  // bounds of their subtrees.  Env RT_VIS_TREE=screen: a per-resolution
  // screen-space BVH4 over the rectangles (rt::BuildScreenTree) -- fewer
  // visits per ray (tekkaman 1024^2: 8.6 vs 9.3) but measured 6 % slower
  // (profiles/r02f_ab.json)
  std::vector<std::array<int32_t, 4>> refs;
  std::vector<int32_t> leaf_pids;
  const char* vt = std::getenv("RT_VIS_TREE");
  if (vt && std::string(vt) == "screen") {
    float dscale = 0.0f;
    if (const char* e = std::getenv("RT_VIS_DEPTH_SCALE")) dscale = (float)std::atof(e);
    uint32_t stack = 0;
    if (rt::BuildScreenTree(vis, s->geometry, dscale, &refs, &leaf_pids, &stack) != 0)
      return fail("screen tree build failed");
    if (stack > RT_STACK_DEEP) return fail("screen tree deeper than the traversal stack");
    if (stack > RT_STACK_SHALLOW && !r->deep && load_deep_images(r) != 0) return -1;
  } else if (tree_refs(r, use_bvh4, &refs, &leaf_pids) != 0) {
    return -1;
  }
  r->vis_refs = refs;
  r->vis_pids = leaf_pids;
  std::vector<rt_vnode_t> vnodes;
  if (rt::BuildVisNodes(refs, leaf_pids, vis, &vnodes) != 0) return fail("malformed BVH");
  std::vector<rt_vtri_t> vtris;
  for (int32_t pid : leaf_pids) vtris.push_back(rt::MakeVisTri(prims[pid], vis[pid], pid));
  for (int i = 0; i < 3; ++i)  // padding: the kernel loads all 4 slots of a leaf
    vtris.push_back(rt::MakeVisTri(rt_prim_t{}, rt::VisPrim{}, -1));
  std::vector<rt_vtri_t> vl, vg;
  for (int32_t g : s->layers) vl.push_back(rt::MakeVisTri(prims[g], vis[g], g));
  for (int32_t g : s->geometry) vg.push_back(rt::MakeVisTri(prims[g], vis[g], g));
  a.num_vnodes = (uint32_t)vnodes.size();
  if (upload(r->dev, vnodes.data(), vnodes.size() * sizeof(rt_vnode_t), &r->vnodes, &a.vnodes_addr) ||
      upload(r->dev, vtris.data(), vtris.size() * sizeof(rt_vtri_t), &r->vtris, &a.vtris_addr) ||
      upload(r->dev, vl.data(), vl.size() * sizeof(rt_vtri_t), &r->vlayers, &a.vlayers_addr) ||
      upload(r->dev, vg.data(), vg.size() * sizeof(rt_vtri_t), &r->vgeom, &a.vgeom_addr))
    return -1;
  return 0;
}


// Per-8x8-block candidate lists (rt_common.h rt_bentry_t), the host
// restatement of the device build (rt_setup.hip BCOUNT .. BSORT; oracle/rt.c
// vis_build_lists): for every local block of the shard, the geometry
// primitives whose covered rectangle reaches it, ascending (depth bound,
// geometry index), each with the union rectangle of itself and the rest.
static int build_block_lists(rt_renderer* r, const std::vector<rt::VisPrim>& vis) {
  const rt_scene* s = r->sc;
  rt_kernel_arg_t& a = r->arg;
  const uint32_t nblk = r->local_tiles * 16u, sc = a.shard_count, si = a.shard_index;
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> lists(nblk);  // (zmin, k)
  for (uint32_t k = 0; k < (uint32_t)s->geometry.size(); ++k) {
    const rt::VisPrim& v = vis[s->geometry[k]];
    if (!v.any) continue;
    for (uint32_t by = (v.ry & 0xffffu) >> 3; by <= (v.ry >> 16) >> 3; ++by)
      for (uint32_t bx = (v.rx & 0xffffu) >> 3; bx <= (v.rx >> 16) >> 3; ++bx) {
        const uint32_t t = (by >> 2) * a.tiles_x + (bx >> 2);
        if (t % sc != si) continue;
        lists[((t / sc) << 4) | ((by & 3u) << 2) | (bx & 3u)].push_back({v.zmin, k});
      }
  }
  uint64_t total = 0, longest = 0;
  for (const auto& l : lists) {
    total += l.size();
    longest = std::max<uint64_t>(longest, l.size());
  }
  r->setup.blist_max = (uint32_t)longest;
  r->setup.blist_entries = total;
  a.blist_blocks = 0;
  if (!rtapp::block_lists_fit(longest, total)) return 0;
  std::vector<rt_bentry_t> ent;
  std::vector<uint32_t> idx;
  ent.reserve(total + RT_BLIST_PAD);
  idx.reserve(2 * (size_t)nblk);
  for (auto& l : lists) {
    std::sort(l.begin(), l.end());
    idx.push_back((uint32_t)ent.size());
    idx.push_back((uint32_t)l.size());
    const size_t base = ent.size();
    ent.resize(base + l.size());
    uint32_t x0 = 0xffffu, y0 = 0xffffu, x1 = 0, y1 = 0;
    for (size_t i = l.size(); i-- > 0;) {
      const rt::VisPrim& v = vis[s->geometry[l[i].second]];
      x0 = std::min(x0, v.rx & 0xffffu); x1 = std::max(x1, v.rx >> 16);
      y0 = std::min(y0, v.ry & 0xffffu); y1 = std::max(y1, v.ry >> 16);
      ent[base + i] = rt_bentry_t{l[i].second, x0 | (y0 << 16), x1 | (y1 << 16), l[i].first};
    }
  }
  for (uint32_t i = 0; i < RT_BLIST_PAD; ++i)
    ent.push_back(rt_bentry_t{0u, RT_BLIST_PAD_LO, RT_BLIST_PAD_HI, RT_VIS_ZMIN_NONE});
  if (upload(r->dev, ent.data(), ent.size() * sizeof(rt_bentry_t), &r->blist, &a.blist_addr) ||
      upload(r->dev, idx.data(), idx.size() * 4, &r->bidx, &a.bidx_addr))
    return -1;
  a.blist_blocks = nblk;
  return 0;
}

// Tile layout, work order and kernel flags of a configuration; the
// per-resolution records come from the device setup (device_setup.cpp,
// kernels/rt_setup.hip; the default) or from the host loops below
// (RT_RENDER_HOST_SETUP / env RT_SETUP=host, and the RT_VIS_TREE=screen
// variant, which needs the visibility records on the host).
static int host_setup(rt_renderer* r, const rt_render_params_t* p, bool raster, bool order_on, bool lists,
                      uint32_t* heavy) {
  const rt_scene* s = r->sc;
  rt_kernel_arg_t& a = r->arg;
  // per-resolution shading records (rast_prim_t + drawcall id)
  std::vector<rt_prim_t> prims(s->scene.prims.size());
  std::vector<uint8_t> setup_ok(prims.size(), 0);
  for (size_t d = 0; d < s->scene.drawcalls.size(); ++d) {
    const rt::DrawCall& dc = s->scene.drawcalls[d];
    for (uint32_t i = 0; i < dc.prim_count; ++i) {
      rt_prim_t& q = prims[dc.prim_offset + i];
      const int st = rt::PrimSetup(s->scene.prims[dc.prim_offset + i], p->width, p->height,
                                   dc.viewport[4], dc.viewport[5], &q);
      q.dc = (uint32_t)d;
      setup_ok[dc.prim_offset + i] = st == rt::kSetupOk;
    }
  }
  if (upload(r->dev, prims.data(), prims.size() * sizeof(rt_prim_t), &r->prims, &a.prims_addr))
    return -1;
  // screen boxes (PrimBBox; degenerate / culled primitives get an empty box
  // and are never binned, gfxutil.cpp:155-192) and primary visibility per
  // primitive (app/vis.h): covered-pixel rectangle + depth bound
  std::vector<rt_bbox_t> bb(prims.size());
  std::vector<rt::VisPrim> vis(prims.size());
  for (size_t g = 0; g < prims.size(); ++g) {
    const bool ok = setup_ok[g] &&
                    rt::PrimBBox(s->scene.prims[g], p->width, p->height, &bb[g]) == rt::kSetupOk;
    if (!ok) bb[g].x = bb[g].y = 0;
    if (!raster) vis[g] = rt::ComputeVisPrim(prims[g], ok, bb[g], p->width, p->height);
  }
  if (raster) {
    if (upload(r->dev, bb.data(), bb.size() * sizeof(rt_bbox_t), &r->bbox, &a.bbox_addr)) return -1;
    std::vector<uint32_t> zclear((size_t)p->width * p->height, 0xffffffffu);  // main.cpp:48
    if (upload(r->dev, zclear.data(), zclear.size() * 4, &r->zbuf, &a.zbuf_addr)) return -1;
  } else {
    // the visibility records as the device setup keeps them (uint4: rx, ry, zmin, any)
    std::vector<uint32_t> v4(4 * vis.size());
    for (size_t g = 0; g < vis.size(); ++g) {
      v4[4 * g] = vis[g].rx;
      v4[4 * g + 1] = vis[g].ry;
      v4[4 * g + 2] = vis[g].zmin;
      v4[4 * g + 3] = vis[g].any ? 1u : 0u;
    }
    uint64_t va = 0;
    if (upload(r->dev, v4.data(), v4.size() * 4, &r->vis, &va)) return -1;
  }
  // Work order of this shard's 32x32 tiles: heaviest first (longest
  // processing time first) -- weight = geometry primitives whose
  // covered-pixel rectangle reaches the tile, capped at 255 (the device
  // sort's 8-bit key) -- so the long model waves start with the frame
  // rather than trailing it.  Output is order independent.
  *heavy = 0;
  if (order_on) {
    std::vector<uint32_t> weight((size_t)a.tiles_x * a.tiles_y, 0);
    for (int32_t g : s->geometry) {
      const rt::VisPrim& v = vis[g];
      if (!v.any) continue;
      const uint32_t tx0 = (v.rx & 0xffffu) >> RT_TILE_LOG, tx1 = (v.rx >> 16) >> RT_TILE_LOG;
      const uint32_t ty0 = (v.ry & 0xffffu) >> RT_TILE_LOG, ty1 = (v.ry >> 16) >> RT_TILE_LOG;
      for (uint32_t ty = ty0; ty <= ty1 && ty < a.tiles_y; ++ty)
        for (uint32_t tx = tx0; tx <= tx1 && tx < a.tiles_x; ++tx) ++weight[ty * a.tiles_x + tx];
    }
    const uint32_t shards = a.shard_count;
    std::vector<uint32_t> ord(r->local_tiles);
    for (uint32_t i = 0; i < r->local_tiles; ++i) ord[i] = i;
    auto w = [&](uint32_t lt) { return std::min(weight[a.shard_index + lt * shards], RTS_WEIGHT_CAP); };
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return w(x) > w(y); });
    if (upload(r->dev, ord.data(), ord.size() * 4, &r->order, &a.order_addr)) return -1;
    while (*heavy < r->local_tiles && w(ord[*heavy]) > 0) ++*heavy;
  }
  if (!raster && configure_vis(r, prims, vis, r->use_bvh4) != 0) return -1;
  if (lists && build_block_lists(r, vis) != 0) return -1;
  // output buffer, pre-filled with the clear colour (draw3d/main.cpp:485-490)
  std::vector<uint32_t> clear(r->cbuf_bytes / 4 ? r->cbuf_bytes / 4 : 1, p->clear_color);
  if (upload(r->dev, clear.data(), r->cbuf_bytes, &r->cbuf, &a.cbuf_addr)) return -1;
  return 0;
}

int rt_renderer_configure(rt_renderer_h r, const rt_render_params_t* p) {
  if (!r || !p) return fail("null argument");
  if (p->width == 0 || p->height == 0 || p->width > 32768 || p->height > 32768)
    return fail("bad resolution");
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t shards = p->shard_count ? p->shard_count : 1;
  const uint32_t modes = p->flags & (RT_RENDER_PATH | RT_RENDER_FLAT | RT_RENDER_RASTER);
  if (modes & (modes - 1)) return fail("RT_RENDER_PATH / FLAT / RASTER are exclusive");
  const bool raster = (p->flags & RT_RENDER_RASTER) != 0;
  if (!raster && !r->sc->unsupported.empty())
    return fail("scene not supported by the RT path (use RT_RENDER_RASTER): " + r->sc->unsupported, -2);
  const bool compact = shards > 1 || (p->flags & RT_RENDER_COMPACT);
  if (raster && (compact || (p->flags & RT_RENDER_INSTRUMENTED)))
    return fail("RT_RENDER_RASTER renders whole frames, uninstrumented");
  if (p->shard_index >= shards) return fail("shard_index >= shard_count");
  const rt_scene* s = r->sc;
  r->configured = false;
  r->params = *p;
  r->params.shard_count = shards;
  for (vx_buffer_h* b : {&r->gather_recv, &r->gather_image})  // sized per configuration
    if (*b) { vx_mem_free(*b); *b = nullptr; }
  rt_kernel_arg_t& a = r->arg;
  a.width = p->width;
  a.height = p->height;
  // raster workgroups own 2^log x 2^log tiles (16x16 by default; env
  // RT_RASTER_TILE_LOG=5 selects the reference's 32x32), 256 tasks each
  uint32_t tlog = RT_TILE_LOG;
  if (raster) {
    tlog = RT_RASTER_TILE_LOG;
    if (const char* e = std::getenv("RT_RASTER_TILE_LOG")) tlog = std::atoi(e) == 5 ? 5u : 4u;
  }
  a.raster_tile_log = tlog;
  // binning granularity (draw3d / raster -k): semantic, fixed-point coverage
  // reaching past a primitive's bbox counts only inside its binned tiles
  a.raster_bin_log = p->tile_logsize ? p->tile_logsize : RT_TILE_LOG;
  if (raster && (a.raster_bin_log < 2 || a.raster_bin_log > 15))
    return fail("tile_logsize must be in [2, 15] (raster_unit.cpp:92)");
  if (!raster && a.raster_bin_log != RT_TILE_LOG)
    return fail("the RT modes bin at RASTER_TILE_LOGSIZE 5; other tile sizes need RT_RENDER_RASTER");
  if ((p->flags & RT_RENDER_COVERAGE) && !raster) return fail("RT_RENDER_COVERAGE needs RT_RENDER_RASTER");
  a.tiles_y = (p->height + (1u << tlog) - 1) >> tlog;
  a.tiles_x = (p->width + (1u << tlog) - 1) >> tlog;
  a.tiles_x_magic = rt_tiles_x_magic(a.tiles_x);
  const uint32_t tiles = a.tiles_x * a.tiles_y;
  r->local_tiles = (tiles > p->shard_index) ? (tiles - p->shard_index + shards - 1) / shards : 0;
  a.num_tasks = r->local_tiles * (raster ? 256u : RT_TILE_PIXELS);
  a.shard_index = p->shard_index;
  a.shard_count = shards;
  a.order_addr = 0;
  a.split_tiles = 0;
  a.split_log = 5;
  a.quad_tiles = 0;
  const bool order_on = !raster && r->local_tiles > 0 &&
                        !(std::getenv("RT_TILE_ORDER") && std::atoi(std::getenv("RT_TILE_ORDER")) == 0);
  bool use_bvh4 = !(p->flags & RT_RENDER_BVH2) && (!r->gpu_bvh || r->gpu_bvh4);
  if (const char* e = std::getenv("RT_BVH_WIDTH")) use_bvh4 = use_bvh4 && std::atoi(e) != 2;
  r->use_bvh4 = use_bvh4;
  a.flags = ((p->flags & RT_RENDER_SHADOWS) ? RT_FLAG_SHADOWS : 0u) |
            ((p->flags & RT_RENDER_PATH) ? RT_FLAG_PATH : 0u) |
            ((p->flags & RT_RENDER_FLAT) ? RT_FLAG_FLAT : 0u) |
            (raster ? RT_FLAG_RASTER : 0u) |
            ((p->flags & RT_RENDER_COVERAGE) ? RT_FLAG_COVERAGE : 0u) |
            (s->tie_high ? RT_FLAG_TIE_HIGH : 0u) | (compact ? RT_FLAG_COMPACT : 0u) |
            (use_bvh4 ? RT_FLAG_BVH4 : 0u) |
            // binary16 node records: the host tree's, or the device tree's (BVHB_HALF)
            (use_bvh4 && (r->gpu_bvh || !s->bvh.nodes4h.empty()) ? RT_FLAG_BVH4H : 0u);
  // the regular RT / PT images walk only the binary16 BVH4 (RT_ONLY_BVH4H);
  // any other layout runs the generic images (the deep ones: every layout,
  // 32-entry stack)
  if (!raster && !(p->flags & RT_RENDER_FLAT) && !(a.flags & RT_FLAG_BVH4H) && !r->deep &&
      load_deep_images(r) != 0)
    return -1;
  // path tracing in two kernels (pt_primary, pt_queue: the compacted path
  // queue) on the binary16 BVH4 images when env RT_PT_QUEUE=1; the default is
  // the one-kernel pt_kernel (0.155 vs 0.235 ms at config 4)
  const char* pqe = std::getenv("RT_PT_QUEUE");
  r->pq = (p->flags & RT_RENDER_PATH) && !r->deep && (a.flags & RT_FLAG_BVH4H) && r->krnl_pq[0][0] &&
          r->launch_group && pqe && std::atoi(pqe) == 1;
  a.bounces = p->bounces;
  a.seed = p->seed;
  a.clear_color = p->clear_color;
  a.sx = 2.0f / (float)p->width;
  a.sy = 2.0f / (float)p->height;
  a.light[0] = p->light[0];
  a.light[1] = p->light[1];
  a.light[2] = p->light[2];
  const uint64_t npx = compact ? (uint64_t)r->local_tiles * RT_TILE_PIXELS
                                  : (uint64_t)p->width * p->height;
  r->cbuf_bytes = npx * 4;
  // the per-resolution records: on the device unless the host path is asked
  // for (or needed: the screen-space primary tree is built on the host)
  const char* sv = std::getenv("RT_SETUP");
  const char* vt = std::getenv("RT_VIS_TREE");
  const bool device = !(p->flags & RT_RENDER_HOST_SETUP) && !(sv && std::string(sv) == "host") &&
                      !(!raster && vt && std::string(vt) == "screen");
  uint32_t heavy = 0, launches = 0;
  // primary visibility of primary+shadow and path frames from per-block
  // candidate lists (rt_bentry_t; env RT_BLOCK_LISTS=0 keeps the tree walk)
  const char* bl = std::getenv("RT_BLOCK_LISTS");
  const bool bvh_walk = (p->flags & RT_RENDER_BVH_WALK) != 0;
  const bool lists = !raster && !(p->flags & RT_RENDER_FLAT) && !(bl && std::atoi(bl) == 0) && !bvh_walk &&
                     a.num_geom > 0 && r->local_tiles > 0;
  a.blist_blocks = 0;
  a.blist_addr = a.bidx_addr = 0;
  r->setup.blist_entries = 0;
  r->setup.blist_max = 0;
  // shadow rays (primary+shadow frames, every path vertex): light-space
  // lists (built on the device for this light; env RT_SHADOW_LISTS=0 keeps
  // the BVH walks; the host setup path walks the BVH)
  const char* sle = std::getenv("RT_SHADOW_LISTS");
  const bool slists = device && !raster && !(p->flags & RT_RENDER_FLAT) &&
                      (p->flags & (RT_RENDER_SHADOWS | RT_RENDER_PATH)) && a.num_geom > 0 &&
                      !(sle && std::atoi(sle) == 0) && !bvh_walk;
  r->sl_mode = slists;
  r->sl_stale = false;  // the configure builds the lists for its light
  a.slist_on = 0;
  r->setup.slist_entries = 0;
  const auto t1 = std::chrono::steady_clock::now();
  if (device) {
    r->vis_refs.clear();
    r->vis_pids.clear();
    if (rtapp::device_setup(r, raster, order_on, lists, slists, &heavy, &launches) != 0) return -1;
  } else if (host_setup(r, p, raster, order_on, lists, &heavy) != 0) {
    return -1;
  }
  const double setup_ms = ms_since(t1);
  if (order_on) {
    // path tracing: tiles that geometry covers (first in the order;
    // oracle/rt.c tile_split restates the rule) run 32 pixels per wave
    // (task_map in rt_trace.h): 0.34 -> 0.30 ms at 1024^2; for primary +
    // shadow rays it measured slower (0.071 -> 0.086 ms: the shadow rays then
    // also trace in half-empty waves), so off there.  RT_SPLIT_TILES=n
    // overrides the count, 0 disables.
    uint32_t split = (p->flags & RT_RENDER_PATH) && !r->pq ? heavy : 0u;
    if (const char* e = std::getenv("RT_SPLIT_TILES"))
      split = std::min<uint32_t>((uint32_t)std::atoi(e), r->local_tiles);
    a.split_tiles = split;
    a.split_log = 5;  // 32 pixels per wave
    if (const char* e = std::getenv("RT_SPLIT_LOG")) a.split_log = std::min(6u, std::max(3u, (uint32_t)std::atoi(e)));
    const uint32_t extra = RT_TILE_PIXELS * ((64u >> a.split_log) - 1u);  // per split tile
    a.num_tasks += split * extra;
    // the heaviest split tiles at 16 pixels per wave (a path on four lanes)
    a.quad_tiles = 0;
    if (const char* e = std::getenv("RT_QUAD_TILES")) a.quad_tiles = std::min<uint32_t>((uint32_t)std::atoi(e), split);
    const uint32_t qextra = RT_TILE_PIXELS * 3u - extra;  // per quad tile beyond a split tile's
    a.num_tasks += a.quad_tiles * qextra;
    // timing probe only (the frame is incomplete): render just the first n
    // tiles of the work order, e.g. the geometry tiles without the background
    if (const char* e = std::getenv("RT_TILE_LIMIT")) {
      const uint32_t n = std::min<uint32_t>((uint32_t)std::atoi(e), r->local_tiles);
      a.num_tasks = std::min(a.num_tasks, n * RT_TILE_PIXELS + std::min(n, split) * extra +
                                              std::min(n, a.quad_tiles) * qextra);
    }
  }
  uint64_t args_addr = 0;
  if (r->pq) {
    // the path queue: RT_PQ_SEGS segments (chunk c -> segment c % RT_PQ_SEGS),
    // each holding up to 64 paths per chunk it gets; the counters, one 128-B
    // line each (rt_common.h)
    const uint32_t chunks = (a.num_tasks + 63u) / 64u;
    a.pathq_seg_cap = ((chunks + RT_PQ_SEGS - 1) / RT_PQ_SEGS) * 64u;
    const std::vector<uint32_t> zero(32u * (2u * RT_PQ_SEGS + 1u), 0u);
    uint64_t qa = 0, ca = 0;
    if (upload(r->dev, nullptr, (uint64_t)RT_PQ_SEGS * a.pathq_seg_cap * 16, &r->pathq, &qa) ||
        upload(r->dev, zero.data(), zero.size() * 4, &r->pathq_ctr, &ca))
      return -1;
    a.pathq_addr = qa;
    a.pathq_ctr_addr = ca;
    // paths per pt_queue wave (env RT_PQ_LANES: 64, 32 or 16)
    a.pathq_lanes = 64;
    if (const char* e = std::getenv("RT_PQ_LANES")) {
      const uint32_t l = (uint32_t)std::atoi(e);
      a.pathq_lanes = (l == 16 || l == 32) ? l : 64u;
    }
  } else {
    a.pathq_addr = a.pathq_ctr_addr = 0;
  }
  // the render arguments: one buffer for the renderer's life (its address,
  // the launches' STARTUP_ARG, stays put), rewritten in stream order behind
  // the setup just queued -- no wait for the device
  if (!r->args && upload(r->dev, nullptr, sizeof(a), &r->args, &args_addr)) return -1;
  if (r->copy_async ? r->copy_async(r->args, &a, 0, sizeof(a)) != 0
                    : vx_copy_to_dev(r->args, &a, 0, sizeof(a)) != 0)
    return fail("render argument upload failed");
  r->setup.device = device ? 1u : 0u;
  r->setup.launches = launches;
  r->setup.heavy_tiles = heavy;
  r->setup.blist_blocks = a.blist_blocks;
  r->setup.slist_on = a.slist_on;
  r->setup.path_queue = r->pq ? 1u : 0u;
  r->setup.setup_ms = setup_ms;
  r->setup.configure_ms = ms_since(t0);
  r->configured = true;
  return 0;
}

int rt_renderer_set_list_policy(rt_renderer_h r, uint32_t defer_frames) {
  if (!r) return fail("null argument");
  r->sl_defer = defer_frames;
  return 0;
}

int rt_render_start(rt_renderer_h r) {
  if (!r || !r->configured) return fail("renderer not configured");
  // the moving light: the lists of a light that stayed for sl_defer frames
  // are queued before this frame (the frames before walked the BVH)
  if (r->sl_stale && ++r->sl_static > r->sl_defer) {
    uint32_t launches = 0;
    if (rtapp::queue_lists(r, &launches) != 0) return -1;
  }
  const uint32_t f = r->params.flags;
  const int mode = (f & RT_RENDER_PATH) ? 1 : (f & RT_RENDER_FLAT) ? 2 : (f & RT_RENDER_RASTER) ? 3 : 0;
  const int k = (f & RT_RENDER_INSTRUMENTED) && mode != 3 ? 1 : 0;
  // every launch of the frame carries its light (and, while the lists wait
  // for a light that stays, the switch to the BVH walk) in its launch words:
  // rt_renderer_set_light queues no copy
  uint32_t lw[4] = {0, 0, 0, 0};
  if (r->set_words) {
    std::memcpy(lw, r->arg.light, sizeof(r->arg.light));
    lw[3] = RT_LW_LIGHT | (r->sl_stale ? RT_LW_NO_SLIST : 0u);
  }
  auto start = [&](vx_buffer_h img) {
    return (!r->set_words || r->set_words(r->dev, lw, 4) == 0) && vx_start(r->dev, img, r->args) == 0;
  };
  // counter rows only when the caller wants rt_render_stats' counts
  if (r->set_counters &&
      r->set_counters(r->dev, (f & (RT_RENDER_COUNTERS | RT_RENDER_INSTRUMENTED)) ? 1 : 0) != 0)
    return fail("vx_hip_set_counters failed");
  // a frame of the two-kernel path tracer is one launch group of 2
  if (mode == 1 && r->pq) {
    if (r->launch_group(r->dev, 2) != 0) return fail("vx_hip_launch_group failed");
    if (start(r->krnl_pq[0][k]) && start(r->krnl_pq[1][k])) return 0;
    r->launch_group(r->dev, 0);  // abandon the half-issued group: later launches stand alone
    return fail("vx_start failed");
  }
  // BVH-walk primary+shadow frames: their own image on the binary16 BVH4
  // (the deep images walk every layout with the list code paths idle)
  const bool bvh = mode == 0 && (f & RT_RENDER_BVH_WALK) && !r->deep && (r->arg.flags & RT_FLAG_BVH4H) &&
                   r->krnl_bvh[k];
  vx_buffer_h img = bvh ? r->krnl_bvh[k] : r->krnl[mode][k];
  return start(img) ? 0 : fail("vx_start failed");
}

int rt_render_wait(rt_renderer_h r) {
  if (!r) return fail("null argument");
  return vx_ready_wait(r->dev, VX_MAX_TIMEOUT) == 0 ? 0 : fail("vx_ready_wait failed");
}

int rt_render(rt_renderer_h r) {
  int e = rt_render_start(r);
  return e ? e : rt_render_wait(r);
}

int rt_render_stats(rt_renderer_h r, rt_stats_t* st) {
  if (!r || !st) return fail("null argument");
  std::memset(st, 0, sizeof(*st));
  uint64_t v[RT_STAT_COUNT] = {};
  for (int i = 0; i <= RT_STAT_EDGE_TESTS; ++i)
    if (vx_mpm_query(r->dev, VX_CSR_MPM_BASE + RT_MPM_USER + i, 0, &v[i]) != 0)
      return fail("vx_mpm_query failed");
  st->primary_rays = v[RT_STAT_PRIMARY];
  st->shadow_rays = v[RT_STAT_SHADOW];
  st->geometry_hits = v[RT_STAT_HITS];
  st->occluded = v[RT_STAT_OCCLUDED];
  st->node_visits = v[RT_STAT_NODE_VISITS];
  st->tri_tests = v[RT_STAT_TRI_TESTS];
  st->layer_tests = v[RT_STAT_LAYER_TESTS];
  st->shaded = v[RT_STAT_SHADED];
  st->texel_bytes = v[RT_STAT_TEXEL_BYTES];
  st->bounce_rays = v[RT_STAT_BOUNCE];
  st->rect_tests = v[RT_STAT_RECT_TESTS];
  st->edge_tests = v[RT_STAT_EDGE_TESTS];
  vx_mpm_query(r->dev, VX_CSR_MINSTRET, 0, &st->tasks);
  uint64_t ns = 0;
  vx_mpm_query(r->dev, VX_CSR_MCYCLE, 0, &ns);
  st->kernel_ms = (double)ns * 1e-6;
  if (r->last_run) r->last_run(r->dev, &st->kernel_ms, &st->grid, &st->block);
  st->num_tasks = r->arg.num_tasks;
  st->local_tiles = r->local_tiles;
  return 0;
}

int rt_render_kernel_ms(rt_renderer_h r, double* kernel_ms) {
  if (!r || !kernel_ms) return fail("null argument");
  uint32_t grid = 0, block = 0;
  if (!r->last_run || r->last_run(r->dev, kernel_ms, &grid, &block) != 0)
    return fail("vx_hip_last_run failed");
  return 0;
}

int rt_render_set_timing(rt_renderer_h r, int timed) {
  if (!r) return fail("null argument");
  if (!r->set_timing || r->set_timing(r->dev, timed) != 0) return fail("vx_hip_set_timing failed");
  return 0;
}

int rt_render_run_totals(rt_renderer_h r, double* kernel_ms_sum, uint64_t* timed,
                         uint64_t* launches) {
  if (!r || !kernel_ms_sum || !timed || !launches) return fail("null argument");
  if (!r->run_totals || r->run_totals(r->dev, kernel_ms_sum, timed, launches) != 0)
    return fail("vx_hip_run_totals failed");
  return 0;
}

int rt_read_framebuffer(rt_renderer_h r, uint32_t* out, uint64_t count) {
  if (!r || !out || !r->configured) return fail("renderer not configured");
  if (count * 4 < r->cbuf_bytes) return fail("buffer too small");
  return vx_copy_from_dev(out, r->cbuf, 0, r->cbuf_bytes) == 0 ? 0 : fail("vx_copy_from_dev failed");
}

int rt_read_depthbuffer(rt_renderer_h r, uint32_t* out, uint64_t count) {
  if (!r || !out || !r->configured) return fail("renderer not configured");
  if (!r->zbuf || !(r->params.flags & RT_RENDER_RASTER)) return fail("no depth buffer (raster mode only)");
  const uint64_t n = (uint64_t)r->params.width * r->params.height;
  if (count < n) return fail("buffer too small");
  return vx_copy_from_dev(out, r->zbuf, 0, n * 4) == 0 ? 0 : fail("vx_copy_from_dev failed");
}

int rt_launch_rows(rt_renderer_h r, uint32_t* rows, uint64_t max_rows, uint64_t* nrows) {
  if (!r || !r->mpm_rows) return fail("not available");
  return r->mpm_rows(r->dev, rows, max_rows, nrows) == 0 ? 0 : fail("vx_hip_mpm_rows failed");
}

int rt_render_gather(rt_renderer_h r, struct rt_shard_comm* comm, uint32_t* image) {
  if (!r || !comm || !r->configured || !r->mem_ptr || !r->stream) return fail("renderer not configured");
  // librt_shard.so (HIP + RCCL) is loaded on first use: librtapp itself
  // does not depend on RCCL
  static void* lib = nullptr;
  using gather_fn = int (*)(rt_shard_comm_h, const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t,
                            uint32_t, void*);
  using info_fn = int (*)(rt_shard_comm_h, uint32_t*, uint32_t*);
  using sync_fn = int (*)(void*);
  if (!lib) lib = dlopen((lib_dir() + "/librt_shard.so").c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!lib) return fail(std::string("cannot load librt_shard.so: ") + dlerror());
  auto gather = (gather_fn)dlsym(lib, "rt_frame_gather");
  auto info = (info_fn)dlsym(lib, "rt_shard_comm_info");
  auto sync = (sync_fn)dlsym(lib, "rt_shard_stream_sync");
  if (!gather || !info || !sync) return fail("librt_shard.so lacks the gather API");
  uint32_t rank = 0, world = 0;
  if (info(comm, &rank, &world) != 0) return fail("rt_shard_comm_info failed");
  const rt_render_params_t& p = r->params;
  if (rank != p.shard_index || world != p.shard_count || !(r->arg.flags & RT_FLAG_COMPACT))
    return fail("renderer shard (index/count, compact output) does not match the communicator");
  const uint64_t ntiles = (uint64_t)r->arg.tiles_x * r->arg.tiles_y;
  const uint64_t slots = ((ntiles + world - 1) / world) * RT_TILE_PIXELS;  // rank 0's buffer
  void *local = nullptr, *recv = nullptr, *img = nullptr, *stream = nullptr;
  if (r->mem_ptr(r->cbuf, &local) != 0 || r->stream(r->dev, &stream) != 0)
    return fail("driver extension failed");
  if (rank == 0) {
    uint64_t a1 = 0, a2 = 0;
    const uint64_t rbytes = world * slots * 4, ibytes = (uint64_t)p.width * p.height * 4;
    if (!r->gather_recv && upload(r->dev, nullptr, rbytes, &r->gather_recv, &a1)) return -1;
    if (!r->gather_image && upload(r->dev, nullptr, ibytes, &r->gather_image, &a2)) return -1;
    if (r->mem_ptr(r->gather_recv, &recv) != 0 || r->mem_ptr(r->gather_image, &img) != 0)
      return fail("driver extension failed");
  }
  // every render this host started is on the stream ahead of the exchange
  if (gather(comm, (const uint32_t*)local, (uint32_t*)recv, slots, (uint32_t*)img, p.width, p.height,
             stream) != 0)
    return fail("rt_frame_gather failed");
  if (sync(stream) != 0) return fail("stream synchronize failed");
  if (rank == 0 && image &&
      vx_copy_from_dev(image, r->gather_image, 0, (uint64_t)p.width * p.height * 4) != 0)
    return fail("vx_copy_from_dev failed");
  return 0;
}

int rt_framebuffer_device(rt_renderer_h r, void** ptr, uint64_t* bytes) {
  if (!r || !ptr || !r->configured || !r->mem_ptr) return fail("not available");
  if (bytes) *bytes = r->cbuf_bytes;
  return r->mem_ptr(r->cbuf, ptr) == 0 ? 0 : fail("vx_hip_mem_ptr failed");
}

int rt_device_stream(rt_renderer_h r, void** stream) {
  if (!r || !stream || !r->stream) return fail("not available");
  return r->stream(r->dev, stream) == 0 ? 0 : fail("vx_hip_stream failed");
}

int rt_device_caps(rt_renderer_h r, uint64_t caps[8]) {
  if (!r || !caps) return fail("null argument");
  for (uint32_t i = 0; i < 8; ++i)
    if (vx_dev_caps(r->dev, i, &caps[i]) != 0) return fail("vx_dev_caps failed");
  return 0;
}

}  // extern "C"

// ---- GPU BVH build (kernels/bvh_build.hip) --------

namespace {

int alloc_buf(vx_device_h dev, uint64_t size, DevBuf* b, const void* init = nullptr) {
  return upload(dev, init, size, &b->h, &b->addr);
}

}  // namespace

static int build_lbvh(rt_renderer_h r, rt_bvh_build_stats_t* st) {
  rt_scene* s = r->sc;
  const uint32_t n = (uint32_t)s->geometry.size();
  if (n == 0) return fail("no depth-tested geometry to build a BVH over");
  const auto t0 = std::chrono::steady_clock::now();
  vx_buffer_h krnl = nullptr;
  if (load_image(r, "bvh_build.vxbin", &krnl)) return -1;
  DevBuf kimg;
  kimg.h = krnl;
  // ingestion: the clip-space (x, y, w) corners, one float4 each
  std::vector<float> verts((size_t)n * 12, 0.0f);
  for (uint32_t i = 0; i < n; ++i) {
    const auto& p = s->scene.prims[s->geometry[i]];
    for (int c = 0; c < 3; ++c) {
      verts[(size_t)i * 12 + 4 * c + 0] = p[c].pos[0];
      verts[(size_t)i * 12 + 4 * c + 1] = p[c].pos[1];
      verts[(size_t)i * 12 + 4 * c + 2] = p[c].pos[3];
    }
  }
  const uint32_t nblocks = (n + BVHB_ITEMS - 1) / BVHB_ITEMS;
  const uint32_t bounds_init[10] = {~0u, ~0u, ~0u, 0, 0, 0, 0, 0, 0, 0};
  DevBuf vb, cen, keys[2], vals[2], hist, bounds, parent, flags, boxes, range, child, argb;
  vx_buffer_h nodes_h = nullptr, tris_h = nullptr, nodes4_h = nullptr;
  uint64_t nodes_addr = 0, tris_addr = 0, nodes4_addr = 0;
  const uint32_t nn = n > 1 ? n - 1 : 1;
  if (alloc_buf(r->dev, verts.size() * 4, &vb, verts.data()) ||
      alloc_buf(r->dev, (uint64_t)n * 16, &cen) || alloc_buf(r->dev, (uint64_t)n * 4, &keys[0]) ||
      alloc_buf(r->dev, (uint64_t)n * 4, &keys[1]) || alloc_buf(r->dev, (uint64_t)n * 4, &vals[0]) ||
      alloc_buf(r->dev, (uint64_t)n * 4, &vals[1]) ||
      alloc_buf(r->dev, (uint64_t)256 * nblocks * 4, &hist) ||
      alloc_buf(r->dev, sizeof(bounds_init), &bounds, bounds_init) ||
      alloc_buf(r->dev, (uint64_t)n * 8, &parent) || alloc_buf(r->dev, (uint64_t)n * 4, &flags) ||
      alloc_buf(r->dev, (uint64_t)n * 64, &boxes) || alloc_buf(r->dev, (uint64_t)n * 8, &range) ||
      alloc_buf(r->dev, (uint64_t)n * 8, &child) ||
      alloc_buf(r->dev, sizeof(bvh_build_arg_t), &argb) ||
      upload(r->dev, nullptr, (uint64_t)nn * sizeof(rt_node_t), &nodes_h, &nodes_addr) ||
      upload(r->dev, nullptr, (uint64_t)(n + 3) * sizeof(rt_tri_t), &tris_h, &tris_addr) ||
      upload(r->dev, nullptr, (uint64_t)nn * (sizeof(rt_node4_t) + sizeof(rt_node4h_t)), &nodes4_h,
             &nodes4_addr)) {
    if (nodes_h) vx_mem_free(nodes_h);
    if (tris_h) vx_mem_free(tris_h);
    if (nodes4_h) vx_mem_free(nodes4_h);
    return -1;
  }
  DevBuf nodes_out, tris_out, nodes4_out;  // owned here until handed to the renderer
  nodes_out.h = nodes_h;
  tris_out.h = tris_h;
  nodes4_out.h = nodes4_h;
  bvh_build_arg_t a;
  std::memset(&a, 0, sizeof(a));
  a.verts_addr = vb.addr;
  a.geom_addr = r->arg.geom_addr;
  a.cen_addr = cen.addr;
  a.keys_addr[0] = keys[0].addr;
  a.keys_addr[1] = keys[1].addr;
  a.vals_addr[0] = vals[0].addr;
  a.vals_addr[1] = vals[1].addr;
  a.hist_addr = hist.addr;
  a.bounds_addr = bounds.addr;
  a.parent_addr = parent.addr;
  a.flags_addr = flags.addr;
  a.boxes_addr = boxes.addr;
  a.range_addr = range.addr;
  a.child_addr = child.addr;
  a.nodes_addr = nodes_addr;
  a.tris_addr = tris_addr;
  a.nodes4_addr = nodes4_addr;
  a.n = n;
  a.nblocks = nblocks;
  double kernel_ms = 0.0;
  uint32_t launches = 0;
  auto launch = [&](uint32_t phase, uint32_t pass) -> int {
    a.phase = phase;
    a.pass = pass;
    if (vx_copy_to_dev(argb.h, &a, 0, sizeof(a)) != 0) return fail("vx_copy_to_dev failed");
    if (vx_start(r->dev, krnl, argb.h) != 0) return fail("vx_start failed");
    if (vx_ready_wait(r->dev, VX_MAX_TIMEOUT) != 0) return fail("vx_ready_wait failed");
    double ms = 0.0;
    uint32_t g = 0, b = 0;
    if (r->last_run && r->last_run(r->dev, &ms, &g, &b) == 0) kernel_ms += ms;
    ++launches;
    return 0;
  };
  if (launch(BVHB_BOUNDS, 0) || launch(BVHB_MORTON, 0)) return -1;
  for (uint32_t pass = 0; pass < 4; ++pass)  // 30-bit codes: 4 passes of 8 bits
    if (launch(BVHB_HIST, pass) || launch(BVHB_SCAN, pass) || launch(BVHB_SCATTER, pass)) return -1;
  if (launch(BVHB_TREE, 0) || launch(BVHB_BOXES, 0) || launch(BVHB_EMIT, 0) ||
      launch(BVHB_COLLAPSE, 0) || launch(BVHB_HALF, 0))
    return -1;
  uint32_t bres[10];
  if (vx_copy_from_dev(bres, bounds.h, 0, sizeof(bres)) != 0) return fail("vx_copy_from_dev failed");
  const uint32_t depth = bres[7], stack4 = bres[8];
  if (depth == 0 || depth > RT_STACK_DEEP) return fail("GPU BVH deeper than the traversal stack");
  // the device BVH4 is traversed when its worst-case stack fits the deep
  // images (else the BVH2, whose depth bound was just checked)
  const bool use4 = stack4 <= RT_STACK_DEEP;
  // traversal images with a stack deep enough for this tree
  if (std::max(depth, use4 ? stack4 : 0u) > RT_STACK_SHALLOW && !r->deep && load_deep_images(r) != 0)
    return -1;
  if (r->nodes) vx_mem_free(r->nodes);
  if (r->tris) vx_mem_free(r->tris);
  if (r->nodes4) vx_mem_free(r->nodes4);
  r->nodes = nodes_out.h;
  r->tris = tris_out.h;
  r->nodes4 = nodes4_out.h;
  nodes_out.h = tris_out.h = nodes4_out.h = nullptr;
  r->arg.nodes_addr = nodes_addr;
  r->arg.tris_addr = tris_addr;
  r->arg.num_nodes = nn;
  r->arg.nodes4_addr = nodes4_addr;
  r->arg.num_nodes4 = nn;
  r->num_tris = n;
  r->gpu_bvh = true;
  r->gpu_bvh4 = use4;
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->nodes = nn;
    st->depth = depth;
    st->stack4 = use4 ? stack4 : RT_BVH_STACK4_UNUSED;
    st->launches = launches;
    st->kernel_ms = kernel_ms;
    st->build_ms = ms_since(t0);
    st->nodes4 = nn;
    st->method = RT_BVH_BUILD_LBVH;
  }
  // a configured renderer picks up the new tree (and the BVH2 traversal) now
  if (r->configured) {
    const rt_render_params_t p = r->params;
    return rt_renderer_configure(r, &p);
  }
  return 0;
}

// The host builder (app/bvh.cpp) restated on the device (kernels/bvh_sah.hip):
// the same binned-SAH tree, BVH4 collapse and binary16 planes bit for bit.
// One stream-ordered launch sequence (launch i runs seq[i], its launch tag):
// the init, one split launch per tree level for a level budget, then the
// numbering, emission and collapse (7 launches) -- every count a launch needs is read on
// the device, so the host waits once, for the control words.  A tree deeper
// than the budget continues with the next levels and the finishing phases
// again.  The image and the scratch arrays stay with the renderer (a free
// waits for the device).  env RT_SAH_TRACE: every launch its own timed run,
// per-launch times to stderr (scripts/sah_trace.py).
static int build_sah(rt_renderer_h r, rt_bvh_build_stats_t* st) {
  rt_scene* s = r->sc;
  const uint32_t n = (uint32_t)s->geometry.size();
  const auto t0 = std::chrono::steady_clock::now();
  if (!r->set_tag) return fail("the driver has no vx_hip_set_launch_tag");
  if (!r->sah_krnl && load_image(r, "bvh_sah.vxbin", &r->sah_krnl)) return -1;
  std::vector<float> verts((size_t)n * 12, 0.0f);
  for (uint32_t i = 0; i < n; ++i) {
    const auto& p = s->scene.prims[s->geometry[i]];
    for (int c = 0; c < 3; ++c) {
      verts[(size_t)i * 12 + 4 * c + 0] = p[c].pos[0];
      verts[(size_t)i * 12 + 4 * c + 1] = p[c].pos[1];
      verts[(size_t)i * 12 + 4 * c + 2] = p[c].pos[3];
    }
  }
  sah_arg_t a;
  std::memset(&a, 0, sizeof(a));
  const uint64_t N = n;
  // the arrays (sah_common.h), 256-B aligned in one scratch buffer
  const std::pair<uint64_t*, uint64_t> parts[] = {
      {&a.verts_addr, N * 48},     {&a.tbox_addr, N * 32},      {&a.cen_addr, N * 16},
      {&a.idx_addr[0], N * 4},     {&a.idx_addr[1], N * 4},     {&a.final_addr, N * 4},
      {&a.segs_addr[0], N * 16},   {&a.segs_addr[1], N * 16},   {&a.small_addr[0], N * 16},
      {&a.small_addr[1], N * 16},  {&a.nrec_addr, N * 16},      {&a.nbox_addr, N * 64},
      {&a.cnt_addr, (N + 1) * 4},  {&a.d0_addr, N * 4},         {&a.parent_addr, N * 4},
      {&a.cs_addr, N * 32},        {&a.is4_addr, (N + 1) * 4},  {&a.ctl_addr, SAH_CTL_WORDS * 4}};
  uint64_t total = 0;
  for (const auto& pt : parts) total += (pt.second + 255) & ~255ull;
  if (r->su.sah_bytes < total || !r->su.sah.h) {
    if (upload(r->dev, nullptr, total, &r->su.sah.h, &r->su.sah.addr)) return -1;
    r->su.sah_bytes = total;
  }
  if (!r->su.sah_args.h && upload(r->dev, nullptr, sizeof(sah_arg_t), &r->su.sah_args.h, &r->su.sah_args.addr))
    return -1;
  uint64_t off = 0;
  for (const auto& pt : parts) {
    *pt.first = r->su.sah.addr + off;
    off += (pt.second + 255) & ~255ull;
  }
  const uint64_t ctl_off = a.ctl_addr - r->su.sah.addr;
  // the outputs, sized for the largest tree n triangles make (BFS ids < n)
  vx_buffer_h nodes_h = nullptr, tris_h = nullptr, nodes4_h = nullptr;
  uint64_t nodes_addr = 0, tris_addr = 0, nodes4_addr = 0;
  DevBuf nodes_out, tris_out, nodes4_out;  // owned here until handed to the renderer
  const uint64_t nmax = std::max<uint64_t>(N, 1);
  if (upload(r->dev, nullptr, nmax * sizeof(rt_node_t), &nodes_h, &nodes_addr)) return -1;
  nodes_out.h = nodes_h;
  if (upload(r->dev, nullptr, (N + 3) * sizeof(rt_tri_t), &tris_h, &tris_addr)) return -1;
  tris_out.h = tris_h;
  if (upload(r->dev, nullptr, nmax * (sizeof(rt_node4_t) + sizeof(rt_node4h_t)), &nodes4_h, &nodes4_addr))
    return -1;
  nodes4_out.h = nodes4_h;
  a.geom_addr = r->arg.geom_addr;
  a.nodes_addr = nodes_addr;
  a.tris_addr = tris_addr;
  a.nodes4_addr = nodes4_addr;
  a.n = n;
  auto copy = [&](vx_buffer_h h, const void* src, uint64_t o, uint64_t size) -> int {
    const int rc = r->copy_async ? r->copy_async(h, src, o, size) : vx_copy_to_dev(h, src, o, size);
    return rc == 0 ? 0 : fail("vx_copy_to_dev failed");
  };
  const std::vector<uint32_t> ctl0(SAH_CTL_WORDS, 0u);
  if (copy(r->su.sah.h, verts.data(), a.verts_addr - r->su.sah.addr, verts.size() * 4) ||
      copy(r->su.sah.h, ctl0.data(), ctl_off, ctl0.size() * 4))
    return -1;
  const bool trace = std::getenv("RT_SAH_TRACE") != nullptr;
  double kernel_ms = 0.0;
  uint32_t launches = 0;
  auto run = [&](const std::vector<uint32_t>& seq) -> int {
    if (seq.size() > SAH_MAX_SEQ) return fail("SAH build sequence too long");
    a.nseq = (uint32_t)seq.size();
    std::memset(a.seq, 0, sizeof(a.seq));
    std::copy(seq.begin(), seq.end(), a.seq);
    if (copy(r->su.sah_args.h, &a, 0, sizeof(a))) return -1;
    for (uint32_t i = 0; i < a.nseq;) {
      // untimed groups of up to 16 launches (the driver's queue slots bound a group)
      uint32_t k = trace ? 1u : std::min<uint32_t>(16u, a.nseq - i);
      bool grouped = false;
      while (!trace && k > 1 && !(grouped = r->launch_group && r->launch_group(r->dev, k | VX_HIP_GROUP_UNTIMED) == 0))
        k >>= 1;
      for (uint32_t j = i; j < i + k; ++j) {
        if (r->set_tag(r->dev, j) != 0 || vx_start(r->dev, r->sah_krnl, r->su.sah_args.h) != 0) {
          if (grouped) r->launch_group(r->dev, 0);
          return fail("vx_start failed");
        }
        ++launches;
        if (trace) {
          double ms = 0.0;
          uint32_t g = 0, b = 0;
          if (vx_ready_wait(r->dev, VX_MAX_TIMEOUT) != 0) return fail("vx_ready_wait failed");
          if (r->last_run && r->last_run(r->dev, &ms, &g, &b) == 0) kernel_ms += ms;
          std::fprintf(stderr, "sah phase %u level %u: %.4f ms\n", seq[j] & 0xffu, seq[j] >> 8, ms);
        }
      }
      i += k;
    }
    return 0;
  };
  // the level budget: a binned-SAH tree over n triangles is rarely deeper
  // than log2(n) + 4 (r04: the deepest of the reference scenes is log2(n) + 3); a
  // deeper one costs a second round trip
  uint32_t lg = 0;
  while ((1ull << lg) < N + 1) ++lg;
  const uint32_t budget = lg + 4;
  uint32_t c[SAH_CTL_WORDS];
  std::vector<uint32_t> seq{SAH_SEQ(SAH_INIT, 0)};
  for (uint32_t L = 0;;) {
    const uint32_t lend = std::min<uint32_t>(L + budget, SAH_MAX_LEVELS - 1);
    for (; L < lend; ++L) seq.push_back(SAH_SEQ(SAH_SPLIT, L));
    // the finishing phases carry level lend: on the device they do nothing
    // while that level still holds segments (a partial tree, bvh_sah.hip)
    for (const uint32_t ph : {SAH_NUMBER, SAH_SCAN, SAH_EMIT, SAH_CS, SAH_MARK, SAH_SCAN4, SAH_EMIT4})
      seq.push_back(SAH_SEQ(ph, lend));
    const auto tr = std::chrono::steady_clock::now();
    if (run(seq) || vx_copy_from_dev(c, r->su.sah.h, ctl_off, sizeof(c)) != 0)
      return fail("SAH build: launch or read-back failed");
    if (!trace) kernel_ms += ms_since(tr);
    if (c[SAH_CTL_ERR] & 1u) return fail("SAH build overflowed its node / segment capacity");
    if (c[SAH_CTL_SEG + L] == 0 && c[SAH_CTL_SMALL + L] == 0) break;  // level L is empty: the tree is whole
    if (L + 1 >= SAH_MAX_LEVELS) return fail("SAH build deeper than its level table");
    seq.assign(1, SAH_SEQ(SAH_RESET, 0));
  }
  const uint32_t nn = c[SAH_CTL_NODES], depth = c[SAH_CTL_DEPTH], nn4 = c[SAH_CTL_NODES4];
  if (depth > RT_STACK_DEEP) return fail("BVH deeper than RT_STACK_DEEP");
  if (c[SAH_CTL_ERR]) return fail("SAH build: BVH4 walk deeper than its path table");
  const uint32_t stack4 = c[SAH_CTL_STACK4];
  const bool use4 = stack4 <= RT_STACK_DEEP;
  if (std::max(depth, use4 ? stack4 : 0u) > RT_STACK_SHALLOW && !r->deep && load_deep_images(r) != 0)
    return -1;
  if (r->nodes) vx_mem_free(r->nodes);
  if (r->tris) vx_mem_free(r->tris);
  if (r->nodes4) vx_mem_free(r->nodes4);
  r->nodes = nodes_out.h;
  r->tris = tris_out.h;
  r->nodes4 = nodes4_out.h;
  nodes_out.h = tris_out.h = nodes4_out.h = nullptr;
  r->arg.nodes_addr = nodes_addr;
  r->arg.tris_addr = tris_addr;
  r->arg.num_nodes = nn;
  r->arg.nodes4_addr = nodes4_addr;
  r->arg.num_nodes4 = nn4;
  r->num_tris = n;
  r->gpu_bvh = true;
  r->gpu_bvh4 = use4;
  if (st) {
    std::memset(st, 0, sizeof(*st));
    st->nodes = nn;
    st->depth = depth;
    st->stack4 = use4 ? stack4 : RT_BVH_STACK4_UNUSED;
    st->launches = launches;
    st->kernel_ms = kernel_ms;
    st->build_ms = ms_since(t0);
    st->nodes4 = nn4;
    st->depth4 = c[SAH_CTL_DEPTH4];
    st->method = RT_BVH_BUILD_SAH;
  }
  if (r->configured) {
    const rt_render_params_t p = r->params;
    return rt_renderer_configure(r, &p);
  }
  return 0;
}

int rt_renderer_build_bvh_ex(rt_renderer_h r, uint32_t method, rt_bvh_build_stats_t* st) {
  if (!r) return fail("null argument");
  if (r->sc->geometry.empty()) return fail("no depth-tested geometry to build a BVH over");
  if (method != RT_BVH_BUILD_SAH && method != RT_BVH_BUILD_LBVH) return fail("unknown BVH build method");
  rt_bvh_build_stats_t tmp;
  const int rc = method == RT_BVH_BUILD_SAH ? build_sah(r, &tmp) : build_lbvh(r, &tmp);
  if (rc == 0) {
    r->bvh_stats = tmp;
    if (st) *st = tmp;
  }
  return rc;
}

int rt_renderer_build_bvh(rt_renderer_h r, rt_bvh_build_stats_t* st) {
  return rt_renderer_build_bvh_ex(r, RT_BVH_BUILD_LBVH, st);
}

int rt_renderer_export_bvh4(rt_renderer_h r, float* nodes4, uint32_t* num_nodes4) {
  if (!r) return fail("null argument");
  if (num_nodes4) *num_nodes4 = r->arg.num_nodes4;
  // the fp32 rt_node4_t records (a host tree's buffer carries its binary16
  // copy behind them)
  if (nodes4 && r->arg.num_nodes4 &&
      vx_copy_from_dev(nodes4, r->nodes4, 0, (uint64_t)r->arg.num_nodes4 * sizeof(rt_node4_t)) != 0)
    return fail("vx_copy_from_dev failed");
  return 0;
}

int rt_renderer_export_bvh4h(rt_renderer_h r, void* nodes4h, uint32_t* num_nodes4) {
  if (!r) return fail("null argument");
  if (num_nodes4) *num_nodes4 = r->arg.num_nodes4;
  // the binary16 records behind the fp32 ones (host tree: BuildBvh; device
  // tree: BVHB_HALF)
  const uint64_t n4 = r->arg.num_nodes4;
  if (nodes4h && n4 &&
      vx_copy_from_dev(nodes4h, r->nodes4, n4 * sizeof(rt_node4_t), n4 * sizeof(rt_node4h_t)) != 0)
    return fail("vx_copy_from_dev failed");
  return 0;
}

int rt_renderer_export_bvh(rt_renderer_h r, float* nodes, float* tris, uint32_t* num_nodes,
                           uint32_t* num_tris) {
  if (!r) return fail("null argument");
  if (num_nodes) *num_nodes = r->arg.num_nodes;
  if (num_tris) *num_tris = r->num_tris;
  if (nodes && r->arg.num_nodes &&
      vx_copy_from_dev(nodes, r->nodes, 0, (uint64_t)r->arg.num_nodes * sizeof(rt_node_t)) != 0)
    return fail("vx_copy_from_dev failed");
  if (tris && r->num_tris &&
      vx_copy_from_dev(tris, r->tris, 0, (uint64_t)r->num_tris * sizeof(rt_tri_t)) != 0)
    return fail("vx_copy_from_dev failed");
  return 0;
}
