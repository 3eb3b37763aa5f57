// device_setup.cpp -- host side of the device-built per-resolution records
// (kernels/rt_setup.hip, argument block kernels/setup_common.h).
//
// The reference rebuilds its per-drawcall records on the host every frame
// (draw3d/main.cpp:179-211 -> graphics::Binning, gfxutil.cpp:103-276).  Here
// the host uploads the scene's triangles once (device_ingest) and every
// rt_renderer_configure builds the records the RT kernels read with a short
// chain of launches of one image (device_setup); app/setup.cpp, app/vis.cpp
// and rt_app.cpp host_setup remain the host restatement (RT_SETUP=host) that
// the GPU tests compare against bit for bit.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_internal.h"
#include "setup_common.h"

namespace rtapp {
namespace {

// one setup launch: argument block, start, wait (the next launch and the
// host's read-backs depend on it)
int run(rt_renderer* r, DevBuf* argb, const rt_setup_arg_t& a, uint32_t* launches) {
  static const bool trace = std::getenv("RT_SETUP_TRACE") != nullptr;  // per-launch phases to stderr
  const auto t0 = std::chrono::steady_clock::now();
  if (vx_copy_to_dev(argb->h, &a, 0, sizeof(a)) != 0) return set_error("vx_copy_to_dev failed");
  if (vx_start(r->dev, r->setup_krnl, argb->h) != 0) return set_error("vx_start failed");
  if (vx_ready_wait(r->dev, VX_MAX_TIMEOUT) != 0) return set_error("vx_ready_wait failed");
  ++*launches;
  if (trace)
    std::fprintf(stderr, "rt_setup launch phases 0x%05x host %.1f us\n", a.phases,
                 std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  return 0;
}

int alloc(rt_renderer* r, uint64_t bytes, vx_buffer_h* h, uint64_t* addr) {
  return upload(r->dev, nullptr, bytes, h, addr);
}

int alloc_tmp(rt_renderer* r, uint64_t bytes, DevBuf* b, const void* init = nullptr) {
  return upload(r->dev, init, bytes, &b->h, &b->addr);
}

void base_arg(const rt_renderer* r, rt_setup_arg_t* g) {
  std::memset(g, 0, sizeof(*g));
  uint64_t x = 0;
  if (vx_mem_address(r->verts, &x) == 0) g->verts_addr = x;
  if (vx_mem_address(r->pdc, &x) == 0) g->pdc_addr = x;
  if (vx_mem_address(r->dcz, &x) == 0) g->dcz_addr = x;
  if (vx_mem_address(r->layer_list, &x) == 0) g->layers_addr = x;
  if (vx_mem_address(r->geometry_list, &x) == 0) g->geometry_addr = x;
  g->num_prims = (uint32_t)r->sc->scene.prims.size();
  g->num_layers = (uint32_t)r->sc->layers.size();
  g->num_geom = (uint32_t)r->sc->geometry.size();
}

void add_fill(rt_setup_arg_t* g, uint64_t addr, uint64_t words, uint32_t value) {
  if (words == 0 || g->nfills >= RTS_MAX_FILLS) return;
  g->fills[g->nfills++] = rts_fill_t{addr, words, value, 0};
}

}  // namespace

int device_ingest(rt_renderer* r, bool records) {
  const rt_scene* s = r->sc;
  if (load_image(r, "rt_setup.vxbin", &r->setup_krnl)) return -1;
  const size_t np = s->scene.prims.size();
  std::vector<float> verts(np * 32, 0.0f);
  std::vector<uint32_t> pdc(np, 0);
  std::vector<float> dcz(2 * s->scene.drawcalls.size() + 2, 0.0f);
  for (size_t d = 0; d < s->scene.drawcalls.size(); ++d) {
    const rt::DrawCall& dc = s->scene.drawcalls[d];
    dcz[2 * d] = dc.viewport[4];
    dcz[2 * d + 1] = dc.viewport[5];
    for (uint32_t i = 0; i < dc.prim_count; ++i) pdc[dc.prim_offset + i] = (uint32_t)d;
  }
  for (size_t g = 0; g < np; ++g)
    for (int c = 0; c < 3; ++c) {
      const rt::Vertex& v = s->scene.prims[g][c];
      float* o = &verts[32 * g + 10 * c];
      std::memcpy(o, v.pos, 16);
      std::memcpy(o + 4, v.color, 16);
      std::memcpy(o + 8, v.uv, 8);
    }
  uint64_t x = 0;
  if (upload(r->dev, verts.data(), verts.size() * 4, &r->verts, &x) ||
      upload(r->dev, pdc.data(), pdc.size() * 4, &r->pdc, &x) ||
      upload(r->dev, dcz.data(), dcz.size() * 4, &r->dcz, &x) ||
      upload(r->dev, s->layers.data(), s->layers.size() * 4, &r->layer_list, &x) ||
      upload(r->dev, s->geometry.data(), s->geometry.size() * 4, &r->geometry_list, &x))
    return -1;
  if (!records) return 0;
  rt_kernel_arg_t& a = r->arg;
  if (alloc(r, np * sizeof(rt_tri_t), &r->ptris, &a.ptris_addr) ||
      alloc(r, s->geometry.size() * sizeof(rt_tri_t), &r->geom, &a.geom_addr))
    return -1;
  rt_setup_arg_t g;
  base_arg(r, &g);
  g.phases = RTS_RECORDS;
  g.ptris_addr = a.ptris_addr;
  g.geom_addr = a.geom_addr;
  DevBuf argb;
  uint32_t launches = 0;
  if (alloc_tmp(r, sizeof(g), &argb)) return -1;
  return run(r, &argb, g, &launches);
}

int device_setup(rt_renderer* r, bool raster, bool order_on, bool lists, uint32_t* heavy,
                 uint32_t* launches) {
  const rt_scene* s = r->sc;
  rt_kernel_arg_t& a = r->arg;
  *heavy = 0;
  *launches = 0;
  const uint64_t np = s->scene.prims.size();
  uint64_t bbox_addr = 0;
  if (alloc(r, np * sizeof(rt_prim_t), &r->prims, &a.prims_addr) ||
      alloc(r, np * sizeof(rt_bbox_t), &r->bbox, &bbox_addr) ||
      alloc(r, r->cbuf_bytes, &r->cbuf, &a.cbuf_addr))
    return -1;
  const uint32_t zero4[4] = {0, 0, 0, 0};
  DevBuf argb, status;
  if (alloc_tmp(r, sizeof(rt_setup_arg_t), &argb) || alloc_tmp(r, sizeof(zero4), &status, zero4))
    return -1;
  rt_setup_arg_t g;
  base_arg(r, &g);
  g.prims_addr = a.prims_addr;
  g.bbox_addr = bbox_addr;
  g.status_addr = status.addr;
  g.width = a.width;
  g.height = a.height;
  g.raster = raster ? 1u : 0u;
  // output buffer, cleared to the clear colour (draw3d/main.cpp:485-490)
  add_fill(&g, a.cbuf_addr, r->cbuf_bytes / 4, a.clear_color);
  if (raster) {
    a.bbox_addr = bbox_addr;
    if (alloc(r, (uint64_t)a.width * a.height * 4, &r->zbuf, &a.zbuf_addr)) return -1;
    add_fill(&g, a.zbuf_addr, (uint64_t)a.width * a.height, 0xffffffffu);  // main.cpp:48
    g.phases = RTS_FILL | RTS_PRIMVIS;
    return run(r, &argb, g, launches);
  }
  // primary-visibility records and the traversed tree's vnodes
  const bool bvh4 = r->use_bvh4;
  const uint32_t nn = bvh4 ? a.num_nodes4 : a.num_nodes;
  uint64_t vis_addr = 0;
  if (alloc(r, np * 16, &r->vis, &vis_addr) ||
      alloc(r, ((uint64_t)r->num_tris + 3) * sizeof(rt_vtri_t), &r->vtris, &a.vtris_addr) ||
      alloc(r, s->layers.size() * sizeof(rt_vtri_t), &r->vlayers, &a.vlayers_addr) ||
      alloc(r, s->geometry.size() * sizeof(rt_vtri_t), &r->vgeom, &a.vgeom_addr) ||
      alloc(r, (uint64_t)nn * sizeof(rt_vnode_t), &r->vnodes, &a.vnodes_addr))
    return -1;
  a.num_vnodes = nn;
  DevBuf parent, count, weight, hist, bcnt, bpart, btmp;
  if (alloc_tmp(r, (uint64_t)nn * 4, &parent) || alloc_tmp(r, (uint64_t)nn * 8, &count)) return -1;
  // per-block candidate lists: one count / cursor word and one (first, count)
  // pair per local 8x8 block, one partial sum per RTS_BLOCKS_PER_PART blocks
  const uint32_t nblk = lists ? r->local_tiles * 16u : 0u;
  const uint32_t nbpart = (nblk + RTS_BLOCKS_PER_PART - 1) / RTS_BLOCKS_PER_PART;
  if (lists && (alloc_tmp(r, (uint64_t)nblk * 4, &bcnt) || alloc_tmp(r, (uint64_t)nbpart * 4, &bpart) ||
                alloc(r, (uint64_t)nblk * 8, &r->bidx, &a.bidx_addr)))
    return -1;
  const uint64_t wwords = (uint64_t)(a.tiles_x + 1) * (a.tiles_y + 1);
  const uint32_t nblocks = (r->local_tiles + RTS_ITEMS - 1) / RTS_ITEMS;
  if (order_on && (alloc_tmp(r, wwords * 4, &weight) || alloc_tmp(r, 256ull * nblocks * 4, &hist) ||
                   alloc(r, (uint64_t)r->local_tiles * 4, &r->order, &a.order_addr)))
    return -1;
  g.vis_addr = vis_addr;
  g.tris_addr = a.tris_addr;
  g.nodes_addr = bvh4 ? a.nodes4_addr : a.nodes_addr;
  g.vnodes_addr = a.vnodes_addr;
  g.vtris_addr = a.vtris_addr;
  g.vlayers_addr = a.vlayers_addr;
  g.vgeom_addr = a.vgeom_addr;
  g.parent_addr = parent.addr;
  g.count_addr = count.addr;
  g.weight_addr = weight.addr;
  g.hist_addr = hist.addr;
  g.order_addr = a.order_addr;
  g.num_tris = r->num_tris;
  g.num_nodes = nn;
  g.bvh4 = bvh4 ? 1u : 0u;
  g.tiles_x = a.tiles_x;
  g.tiles_y = a.tiles_y;
  g.shard_index = a.shard_index;
  g.shard_count = a.shard_count;
  g.local_tiles = r->local_tiles;
  g.nblocks = nblocks;
  g.nblk = nblk;
  g.nbpart = nbpart;
  g.bcnt_addr = bcnt.addr;
  g.bpart_addr = bpart.addr;
  g.bidx_addr = a.bidx_addr;
  add_fill(&g, parent.addr, nn, 0xffffffffu);
  if (order_on) add_fill(&g, weight.addr, wwords, 0u);
  if (lists) add_fill(&g, bcnt.addr, nblk, 0u);
  const uint32_t ord = order_on ? 1u : 0u;
  uint32_t bl = lists ? 1u : 0u;
  const uint32_t steps[] = {
      RTS_FILL | RTS_PRIMVIS,                                     // records, clears
      RTS_VTRIS | (ord ? RTS_WEIGHT : 0u) | (bl ? RTS_BCOUNT : 0u),  // vtris; tile weights; block counts
      RTS_LINK | (ord ? RTS_ROWSUM : 0u) | (bl ? RTS_BSUM : 0u),     // tree parents; rows; block sums
      RTS_CLIMB | (ord ? RTS_COLSUM : 0u) | (bl ? RTS_BSCAN : 0u),   // vnodes; columns; sums scanned
      (ord ? RTS_HIST : 0u) | (bl ? RTS_BOFF : 0u),                // tile histograms; list offsets
      0u,                                                          // (list sizes read back here)
      (ord ? RTS_SCAN : 0u) | (bl ? RTS_BFILL : 0u),               // digit scan; list entries
      (ord ? RTS_SCATTER : 0u) | (bl ? RTS_BSORT : 0u)};           // tile order; lists sorted
  uint32_t st[4] = {0, 0, 0, 0};
  for (uint32_t ph : steps) {
    if (ph == 0u && bl) {
      // the list sizes: the longest list and the entries in total decide
      // whether the lists are built (else the kernels walk the tree)
      if (vx_copy_from_dev(st, status.h, 0, sizeof(st)) != 0) return set_error("vx_copy_from_dev failed");
      r->setup.blist_max = st[1];
      r->setup.blist_entries = st[2];
      if (!rtapp::block_lists_fit(st[1], st[2])) {
        bl = 0u;
        continue;
      }
      const uint64_t total = st[2];
      if (alloc_tmp(r, total * 16 + 16, &btmp) || alloc(r, (total + RT_BLIST_PAD) * 16, &r->blist, &a.blist_addr))
        return -1;
      g.btmp_addr = btmp.addr;
      g.blist_addr = a.blist_addr;
      g.blist_entries = st[2];
      continue;
    }
    if (!bl) ph &= ~(RTS_BFILL | RTS_BSORT);
    if (!ph) continue;
    g.phases = ph;
    if (run(r, &argb, g, launches) != 0) return -1;
  }
  a.blist_blocks = bl ? nblk : 0u;
  if (vx_copy_from_dev(st, status.h, 0, sizeof(st)) != 0) return set_error("vx_copy_from_dev failed");
  if (st[0] & RTS_ERR_REF) return set_error("malformed BVH (reference out of range)");
  if (st[0] & RTS_ERR_PID) return set_error("malformed BVH (leaf pid out of range)");
  if (st[0] & RTS_ERR_CLIMB) return set_error("malformed BVH (deeper than 64 levels)");
  // local tiles with weight > 0 = items whose digit is below 255 = the
  // exclusive-scan offset of digit 255 in block 0
  if (order_on &&
      vx_copy_from_dev(heavy, hist.h, 255ull * nblocks * 4, 4) != 0)
    return set_error("vx_copy_from_dev failed");
  return 0;
}

int shadow_lists(rt_renderer* r, uint32_t* launches) {
  rt_kernel_arg_t& a = r->arg;
  uint32_t N = RT_SLIST_N;
  if (const char* e = std::getenv("RT_SLIST_N")) N = std::min(1024u, std::max(1u, (uint32_t)std::atoi(e)));
  if (r->sl_built && std::memcmp(r->sl_light, a.light, sizeof(a.light)) == 0 && a.slist_n == N) {
    r->setup.slist_entries = r->sl_entries;
    return 0;
  }
  r->sl_built = false;
  a.slist_on = 0;
  a.slist_n = N;
  const uint32_t cells = 6u * N * N, nbpart = (cells + RTS_BLOCKS_PER_PART - 1) / RTS_BLOCKS_PER_PART;
  const uint32_t zero4[4] = {0, 0, 0, 0};
  DevBuf argb, status, cnt, part, tmp;
  if (alloc_tmp(r, sizeof(rt_setup_arg_t), &argb) || alloc_tmp(r, sizeof(zero4), &status, zero4) ||
      alloc_tmp(r, (uint64_t)cells * 4, &cnt) || alloc_tmp(r, (uint64_t)nbpart * 4, &part) ||
      alloc(r, (uint64_t)cells * 8, &r->sidx, &a.sidx_addr))
    return -1;
  rt_setup_arg_t g;
  base_arg(r, &g);
  g.geom_addr = a.geom_addr;
  g.status_addr = status.addr;
  g.bcnt_addr = cnt.addr;
  g.bpart_addr = part.addr;
  g.bidx_addr = a.sidx_addr;
  g.nblk = cells;
  g.nbpart = nbpart;
  g.slist_n = N;
  for (int i = 0; i < 3; ++i) g.light[i] = a.light[i];
  add_fill(&g, cnt.addr, cells, 0u);
  for (uint32_t ph : {RTS_FILL, RTS_SCOUNT, RTS_BSUM, RTS_BSCAN, RTS_BOFF}) {
    g.phases = ph;
    if (run(r, &argb, g, launches) != 0) return -1;
  }
  uint32_t st[4];
  if (vx_copy_from_dev(st, status.h, 0, sizeof(st)) != 0) return set_error("vx_copy_from_dev failed");
  r->sl_entries = st[2];
  r->setup.slist_entries = st[2];
  if (!block_lists_fit(st[1], st[2])) return 0;  // the packet walk, as without lists
  // tmp: the entries' geometry indices, then their sort keys
  if (alloc_tmp(r, (uint64_t)st[2] * 8 + 8, &tmp) || alloc(r, ((uint64_t)st[2] + 1) * 48, &r->slist, &a.slist_addr))
    return -1;
  g.btmp_addr = tmp.addr;
  g.slist_addr = a.slist_addr;
  g.blist_entries = st[2];
  g.nfills = 0;
  for (uint32_t ph : {RTS_SFILL, RTS_SSORT}) {
    g.phases = ph;
    if (run(r, &argb, g, launches) != 0) return -1;
  }
  std::memcpy(r->sl_light, a.light, sizeof(a.light));
  r->sl_built = true;
  a.slist_on = 1;
  return 0;
}

}  // namespace rtapp
