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
#include <cstddef>
#include <cstring>
#include <vector>

#include "rt_internal.h"
#include "setup_common.h"

namespace rtapp {
namespace {

int ensure(rt_renderer* r, uint64_t bytes, DevScratch* d);

// one setup launch (renderer creation): argument block, start, wait -- in
// the buffer the configure sequences use, so their first launch finds the
// image's start arguments unchanged (no constant re-upload before it)
int run(rt_renderer* r, vx_buffer_h argb, const rt_setup_arg_t& a, uint32_t* launches) {
  static const bool trace = std::getenv("RT_SETUP_TRACE") != nullptr;  // per-launch phases to stderr
  const auto t0 = std::chrono::steady_clock::now();
  if (vx_copy_to_dev(argb, &a, 0, sizeof(a)) != 0) return set_error("vx_copy_to_dev failed");
  if (vx_start(r->dev, r->setup_krnl, argb) != 0) return set_error("vx_start failed");
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
  uint32_t launches = 0;
  if (ensure(r, sizeof(g), &r->su.args) != 0) return -1;
  return run(r, r->su.args.h, g, &launches);
}

namespace {

// a persistent buffer holding at least `bytes`: kept while it is large
// enough (vx_mem_access checks the range), else reallocated -- a free waits
// for the device, so the setup's buffers only ever grow
int ensure(rt_renderer* r, uint64_t bytes, vx_buffer_h* h, uint64_t* addr) {
  const uint64_t b = bytes ? bytes : 64;
  if (*h && vx_mem_access(*h, 0, b, VX_MEM_READ_WRITE) == 0)
    return vx_mem_address(*h, addr) == 0 ? 0 : set_error("vx_mem_address failed");
  return alloc(r, b, h, addr);
}
int ensure(rt_renderer* r, uint64_t bytes, DevScratch* d) { return ensure(r, bytes, &d->h, &d->addr); }

// a launch sequence of the setup image (setup_common.h): launch i runs
// ph[i] on every workgroup, then last[i] (the scans) on the last one
struct Seq {
  uint32_t ph[RTS_MAX_SEQ] = {}, last[RTS_MAX_SEQ] = {};
  uint32_t n = 0;
  void add(uint32_t p, uint32_t l = 0u) {
    if (p == 0u && l == 0u) return;
    ph[n] = p;
    last[n] = l;
    ++n;
  }
};

// the scans the launches do themselves (setup_common.h RTS_FOLD_*): the list
// and tile-order scans always, the candidate-count scan while its items fit
// the workgroup's LDS copy
uint32_t fold_flags(const rt_renderer* r) {
  const char* fe = std::getenv("RT_SETUP_FOLD");
  const bool off = fe && std::atoi(fe) == 0;
  if (off) return 0u;
  uint32_t f = RTS_FOLD_LISTS | RTS_FOLD_ORDER;
  if (6ull * r->sc->geometry.size() <= RTS_SOFF_LDS) f |= RTS_FOLD_SOFF;
  return f;
}

// The argument block goes through the driver's stream (vx_hip_copy_to_dev_async)
// and the n launches are queued behind it: no host wait before, between or
// after them -- the caller reads the status words back when it needs them.
int run_seq(rt_renderer* r, rt_setup_arg_t& g, const Seq& q, uint32_t* launches) {
  static const bool trace = std::getenv("RT_SETUP_TRACE") != nullptr;  // the sequence to stderr
  if (q.n == 0) return 0;
  // a step's scans (one workgroup) read what the whole grid wrote in that
  // step: they run as a launch of their own right behind it
  // (env RT_SETUP_SPLIT=1, profiling: every sub-phase a launch of its own,
  // in the same order -- rocprofv3 then times each; RT_SETUP_TRACE names them)
  static const bool split = std::getenv("RT_SETUP_SPLIT") && std::atoi(std::getenv("RT_SETUP_SPLIT")) == 1;
  Seq x;
  for (uint32_t i = 0; i < q.n; ++i) {
    for (const uint32_t ph : {q.ph[i], q.last[i]}) {
      if (!split) {
        x.add(ph);
        continue;
      }
      for (uint32_t b = 1; b != 0 && b <= ph; b <<= 1)
        if (ph & b) x.add(b);
    }
  }
  if (x.n > RTS_MAX_SEQ) return set_error("setup sequence too long");
  g.phases = 0;
  g.nseq = x.n;
  // the last launch leaves the status words in pinned host memory (read_status)
  g.status_host = 0;
  g.status_nonce = 0;
  r->stat_pending = 0;
  if (r->stat_host && x.n >= 2) {
    g.status_host = r->stat_dev;
    g.status_nonce = ++r->stat_nonce;
    r->stat_pending = g.status_nonce;
  }
  // a launch's sub-phases side by side on slices of the grid (env RT_SETUP_PART=0: in turn)
  const char* pe = std::getenv("RT_SETUP_PART");
  g.part = (pe && std::atoi(pe) == 0) ? 0u : 1u;
  for (uint32_t i = 0; i < RTS_MAX_SEQ; ++i) g.seq_phases[i] = i < x.n ? x.ph[i] : 0u;
  if (ensure(r, sizeof(g), &r->su.args) != 0) return -1;
  const int rc = r->copy_async ? r->copy_async(r->su.args.h, &g, 0, sizeof(g))
                               : vx_copy_to_dev(r->su.args.h, &g, 0, sizeof(g));
  if (rc != 0) return set_error("setup argument upload failed");
  if (!r->set_tag) return set_error("the driver has no vx_hip_set_launch_tag");
  // one untimed run: no timing events between the steps (each costs the
  // device ~5 us idle) and no queue bound stalling the host mid-sequence
  // (the driver refuses groups longer than its slots allow: then one run each)
  const bool grouped = r->launch_group && r->launch_group(r->dev, x.n | VX_HIP_GROUP_UNTIMED) == 0;
  for (uint32_t i = 0; i < x.n; ++i)
    if (r->set_tag(r->dev, i) != 0 || vx_start(r->dev, r->setup_krnl, r->su.args.h) != 0) {
      if (grouped) r->launch_group(r->dev, 0);  // abandon the half-issued group
      return set_error("vx_start failed");
    }
  *launches += x.n;
  if (trace)
    for (uint32_t i = 0; i < x.n; ++i)
      std::fprintf(stderr, "rt_setup seq launch %u/%u phases 0x%07x\n", i + 1, x.n, x.ph[i]);
  return 0;
}

int read_status(rt_renderer* r, uint32_t st[RTS_STATUS_WORDS]) {
  // the last sequence's copy in pinned host memory: wait for the device,
  // then read it (no copy back); else the device words
  if (r->stat_pending != 0) {
    // the last launch stores the words, fences, then the nonce: spin on the
    // nonce (a host-memory read; no device sync, no wake-up latency) -- the
    // launch's own sub-phases may still run, later work is stream-ordered
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false;
    while (!(seen = r->stat_host[RTS_STATUS_WORDS] == r->stat_pending)) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
      __builtin_ia32_pause();
    }
    if (!seen && vx_ready_wait(r->dev, VX_MAX_TIMEOUT) != 0) return set_error("vx_ready_wait failed");
    if (seen || r->stat_host[RTS_STATUS_WORDS] == r->stat_pending) {
      for (int i = 0; i < RTS_STATUS_WORDS; ++i) st[i] = r->stat_host[i];
      return 0;
    }
  }
  if (vx_copy_from_dev(st, r->su.status.h, 0, RTS_STATUS_WORDS * 4) != 0)
    return set_error("vx_copy_from_dev failed");
  return 0;
}

uint32_t slist_res() {
  uint32_t N = RT_SLIST_N;
  if (const char* e = std::getenv("RT_SLIST_N")) N = std::min(1024u, std::max(1u, (uint32_t)std::atoi(e)));
  return N;
}

// the shadow-list fields of the setup argument block for the light in r->arg
// (buffers grown to the light-space cells and the entry capacity r->su.scap)
int slist_args(rt_renderer* r, rt_setup_arg_t* g) {
  rt_kernel_arg_t& a = r->arg;
  const uint32_t N = slist_res(), cells = 6u * N * N;
  const uint32_t ncpart = (cells + RTS_BLOCKS_PER_PART - 1) / RTS_BLOCKS_PER_PART;
  const uint64_t items = 6ull * r->sc->geometry.size();
  if (r->su.scap == 0) {
    // initial entry capacity (env RT_SETUP_SCAP: tests force the overflow refill)
    r->su.scap = 1u << 19;
    if (const char* e = std::getenv("RT_SETUP_SCAP")) r->su.scap = std::max(1u, (uint32_t)std::atoi(e));
  }
  if (ensure(r, (uint64_t)cells * 4, &r->su.scnt) || ensure(r, (uint64_t)ncpart * 4, &r->su.spart) ||
      ensure(r, (uint64_t)cells * 8, &r->sidx, &a.sidx_addr) ||
      ensure(r, items * RTS_SPROJ_WORDS * 4, &r->su.sproj) || ensure(r, (items + 1) * 4, &r->su.soff) ||
      ensure(r, r->sc->geometry.size() * 4, &r->su.skey) ||
      ensure(r, 3ull * r->su.scap * 4, &r->su.stmp) ||
      ensure(r, ((uint64_t)r->su.scap + 1) * sizeof(rt_tri_t), &r->slist, &a.slist_addr))
    return -1;
  a.slist_n = N;
  g->geom_addr = a.geom_addr;
  g->slist_n = N;
  for (int i = 0; i < 3; ++i) g->light[i] = a.light[i];
  g->scnt_addr = r->su.scnt.addr;
  g->spart_addr = r->su.spart.addr;
  g->sidx_addr = a.sidx_addr;
  g->sproj_addr = r->su.sproj.addr;
  g->soff_addr = r->su.soff.addr;
  g->skey_addr = r->su.skey.addr;
  g->stmp_addr = r->su.stmp.addr;
  g->slist_addr = a.slist_addr;
  g->ncells = cells;
  g->ncpart = ncpart;
  g->scap = r->su.scap;
  g->fold = fold_flags(r);  // a refill reads the counts the way the chain left them
  return 0;
}

// the lists' size limits (block_lists_fit) for the device's own verdict
void list_limits(rt_setup_arg_t* g) {
  g->max_list = RT_BLIST_MAX_LIST;
  uint64_t cap = 16ull << 20;
  if (const char* e = std::getenv("RT_BLIST_MAX_ENTRIES")) cap = std::strtoull(e, nullptr, 0);
  g->max_entries = (uint32_t)std::min<uint64_t>(cap, 0xffffffffu);
}

// after a chain that built the shadow lists: their verdict from the status
// words; an overflow of the entry capacity (only when the lists would be
// used) grows it to the exact size and refills: cursors zeroed, SFILL, SSORT
int slist_finish(rt_renderer* r, rt_setup_arg_t& g, uint32_t st[RTS_STATUS_WORDS], uint32_t* launches) {
  r->sl_entries = st[5];
  r->setup.slist_entries = st[5];
  const bool fit = block_lists_fit(st[4], st[5]);
  if (fit && st[7] != 0) {
    r->su.scap = st[5];
    if (slist_args(r, &g) != 0) return -1;
    g.nfills = 0;
    add_fill(&g, r->su.scnt.addr, g.ncells, 0u);
    add_fill(&g, r->su.status.addr + 28, 1, 0u);  // the overflow word
    Seq q;
    q.add(RTS_FILL);
    q.add(RTS_SFILL);
    q.add(RTS_SSORT);
    if (run_seq(r, g, q, launches) != 0 || read_status(r, st) != 0) return -1;
    if (st[7] != 0) return set_error("shadow-list refill overflowed its exact capacity");
  }
  r->sl_pending = false;
  r->sl_built = fit;
  r->sl_rejected = !fit;
  return 0;
}

}  // namespace

int device_setup(rt_renderer* r, bool raster, bool order_on, bool lists, bool slists, uint32_t* heavy,
                 uint32_t* launches) {
  const rt_scene* s = r->sc;
  rt_kernel_arg_t& a = r->arg;
  *heavy = 0;
  *launches = 0;
  r->setup.slist_built = 0;
  if (r->sl_pending && settle_lists(r) != 0) return -1;  // lists queued by set_light
  const uint64_t np = s->scene.prims.size();
  uint64_t bbox_addr = 0;
  if (ensure(r, np * sizeof(rt_prim_t), &r->prims, &a.prims_addr) ||
      ensure(r, np * sizeof(rt_bbox_t), &r->bbox, &bbox_addr) ||
      ensure(r, r->cbuf_bytes, &r->cbuf, &a.cbuf_addr) ||
      ensure(r, RTS_STATUS_WORDS * 4, &r->su.status))
    return -1;
  rt_setup_arg_t g;
  base_arg(r, &g);
  list_limits(&g);
  g.prims_addr = a.prims_addr;
  g.bbox_addr = bbox_addr;
  g.status_addr = r->su.status.addr;
  g.width = a.width;
  g.height = a.height;
  g.raster = raster ? 1u : 0u;
  // output buffer, cleared to the clear colour (draw3d/main.cpp:485-490)
  add_fill(&g, a.cbuf_addr, r->cbuf_bytes / 4, a.clear_color);
  add_fill(&g, g.status_addr, RTS_STATUS_WORDS, 0u);
  uint32_t st[RTS_STATUS_WORDS] = {};
  if (raster) {
    a.bbox_addr = bbox_addr;
    if (ensure(r, (uint64_t)a.width * a.height * 4, &r->zbuf, &a.zbuf_addr)) return -1;
    add_fill(&g, a.zbuf_addr, (uint64_t)a.width * a.height, 0xffffffffu);  // main.cpp:48
    Seq q;
    q.add(RTS_FILL | RTS_PRIMVIS);
    return run_seq(r, g, q, launches) != 0 || read_status(r, st) != 0 ? -1 : 0;
  }
  // primary-visibility records and the traversed tree's vnodes
  const bool bvh4 = r->use_bvh4;
  const uint32_t nn = bvh4 ? a.num_nodes4 : a.num_nodes;
  uint64_t vis_addr = 0;
  if (ensure(r, np * 16, &r->vis, &vis_addr) ||
      ensure(r, ((uint64_t)r->num_tris + 3) * sizeof(rt_vtri_t), &r->vtris, &a.vtris_addr) ||
      ensure(r, s->layers.size() * sizeof(rt_vtri_t), &r->vlayers, &a.vlayers_addr) ||
      ensure(r, s->geometry.size() * sizeof(rt_vtri_t), &r->vgeom, &a.vgeom_addr) ||
      ensure(r, (uint64_t)nn * sizeof(rt_vnode_t), &r->vnodes, &a.vnodes_addr) ||
      ensure(r, (uint64_t)nn * 4, &r->su.parent) || ensure(r, (uint64_t)nn * 8, &r->su.count))
    return -1;
  a.num_vnodes = nn;
  // per-block candidate lists: one count / cursor word and one (first, count)
  // pair per local 8x8 block, one partial sum per RTS_BLOCKS_PER_PART blocks;
  // the entries at a capacity that only grows (the exact size after an overflow)
  const uint32_t nblk = lists ? r->local_tiles * 16u : 0u;
  const uint32_t nbpart = (nblk + RTS_BLOCKS_PER_PART - 1) / RTS_BLOCKS_PER_PART;
  if (lists) {
    uint64_t bcap0 = 2ull * nblk + 16ull * s->geometry.size();
    if (const char* e = std::getenv("RT_SETUP_BCAP")) bcap0 = std::max(1ull, std::strtoull(e, nullptr, 0));  // tests
    r->su.bcap = std::max<uint64_t>(r->su.bcap, bcap0);
    if (ensure(r, (uint64_t)nblk * 4, &r->su.bcnt) || ensure(r, (uint64_t)nbpart * 4, &r->su.bpart) ||
        ensure(r, (uint64_t)nblk * 8, &r->bidx, &a.bidx_addr) || ensure(r, r->su.bcap * 16, &r->su.btmp) ||
        ensure(r, (r->su.bcap + RT_BLIST_PAD) * 16, &r->blist, &a.blist_addr))
      return -1;
  }
  const uint64_t wwords = (uint64_t)(a.tiles_x + 1) * (a.tiles_y + 1);
  const uint32_t nblocks = (r->local_tiles + RTS_ITEMS - 1) / RTS_ITEMS;
  if (order_on && (ensure(r, wwords * 4, &r->su.weight) || ensure(r, 256ull * nblocks * 4, &r->su.hist) ||
                   ensure(r, (uint64_t)r->local_tiles * 4, &r->order, &a.order_addr)))
    return -1;
  g.vis_addr = vis_addr;
  g.tris_addr = a.tris_addr;
  g.nodes_addr = bvh4 ? a.nodes4_addr : a.nodes_addr;
  g.vnodes_addr = a.vnodes_addr;
  g.vtris_addr = a.vtris_addr;
  g.vlayers_addr = a.vlayers_addr;
  g.vgeom_addr = a.vgeom_addr;
  g.parent_addr = r->su.parent.addr;
  g.count_addr = r->su.count.addr;
  g.weight_addr = r->su.weight.addr;
  g.hist_addr = r->su.hist.addr;
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
  g.bcnt_addr = r->su.bcnt.addr;
  g.bpart_addr = r->su.bpart.addr;
  g.bidx_addr = a.bidx_addr;
  g.btmp_addr = r->su.btmp.addr;
  g.blist_addr = a.blist_addr;
  g.bcap = lists ? (uint32_t)r->su.bcap : 0u;
  add_fill(&g, g.parent_addr, nn, 0xffffffffu);
  if (order_on) add_fill(&g, g.weight_addr, wwords, 0u);
  if (lists) add_fill(&g, g.bcnt_addr, nblk, 0u);
  // the shadow lists for this light unless the ones built (or found too
  // large) for it are current
  const uint32_t N = slist_res();
  const bool sl_now = slists && !((r->sl_built || r->sl_rejected) && r->sl_n == N &&
                                  std::memcmp(r->sl_light, a.light, sizeof(a.light)) == 0);
  r->setup.slist_built = sl_now ? 1u : 0u;
  if (sl_now) {
    if (slist_args(r, &g) != 0) return -1;
    add_fill(&g, g.scnt_addr, g.ncells, 0u);
  }
  const uint32_t ord = order_on ? 1u : 0u, bl = lists ? 1u : 0u, sl = sl_now ? 1u : 0u;
  // the per-resolution records, the block lists, the work order and the
  // shadow lists in one stream-ordered sequence: six launches, one
  // read-back of the status words at the end
  // the scans folded into the launches that read them (setup_common.h
  // RTS_FOLD_*; env RT_SETUP_FOLD=0 keeps the one-workgroup scan launches)
  g.fold = fold_flags(r);
  const bool fl = (g.fold & RTS_FOLD_LISTS) != 0, fo = (g.fold & RTS_FOLD_ORDER) != 0,
             fs = (g.fold & RTS_FOLD_SOFF) != 0;
  Seq q;
  q.add(RTS_FILL | RTS_PRIMVIS | (sl ? RTS_SPROJ : 0u), sl && !fs ? RTS_SOSCAN : 0u);
  q.add(RTS_VTRIS | (ord ? RTS_WEIGHT : 0u) | (bl ? RTS_BCOUNT : 0u) | (sl ? RTS_SCOUNT : 0u));
  q.add(RTS_LINK | (ord ? RTS_ROWSUM : 0u) | (bl ? RTS_BSUM : 0u) | (sl ? RTS_SSUM : 0u), fl ? 0u :
        (bl ? RTS_BSCAN : 0u) | (sl ? RTS_SSCAN : 0u));
  q.add(RTS_CLIMB | (ord ? RTS_COLSUM : 0u) | (bl ? RTS_BOFF : 0u) | (sl ? RTS_SOFF : 0u));
  q.add((ord ? RTS_HIST : 0u) | (bl ? RTS_BFILL : 0u) | (sl ? RTS_SFILL : 0u), ord && !fo ? RTS_SCAN : 0u);
  q.add((ord ? RTS_SCATTER : 0u) | (bl ? RTS_BSORT : 0u) | (sl ? RTS_SSORT : 0u));
  if (run_seq(r, g, q, launches) != 0 || read_status(r, st) != 0) return -1;
  if (st[0] & RTS_ERR_REF) return set_error("malformed BVH (reference out of range)");
  if (st[0] & RTS_ERR_PID) return set_error("malformed BVH (leaf pid out of range)");
  if (st[0] & RTS_ERR_CLIMB) return set_error("malformed BVH (deeper than 64 levels)");
  *heavy = order_on ? st[3] : 0u;
  a.blist_blocks = 0;
  if (lists) {
    r->setup.blist_max = st[1];
    r->setup.blist_entries = st[2];
    const bool fit = block_lists_fit(st[1], st[2]);
    if (fit && st[6] != 0) {
      // more entries than the capacity: grow it to the exact size and refill
      r->su.bcap = st[2];
      if (ensure(r, r->su.bcap * 16, &r->su.btmp) ||
          ensure(r, (r->su.bcap + RT_BLIST_PAD) * 16, &r->blist, &a.blist_addr))
        return -1;
      g.btmp_addr = r->su.btmp.addr;
      g.blist_addr = a.blist_addr;
      g.bcap = (uint32_t)r->su.bcap;
      g.nfills = 0;
      add_fill(&g, g.bcnt_addr, nblk, 0u);
      add_fill(&g, g.status_addr + 24, 1, 0u);
      Seq f;
      f.add(RTS_FILL);
      f.add(RTS_BFILL);
      f.add(RTS_BSORT);
      if (run_seq(r, g, f, launches) != 0 || read_status(r, st) != 0) return -1;
      if (st[6] != 0) return set_error("block-list refill overflowed its exact capacity");
    }
    a.blist_blocks = fit ? nblk : 0u;
  }
  if (sl_now) {
    std::memcpy(r->sl_light, a.light, sizeof(a.light));
    r->sl_n = N;
    if (slist_finish(r, g, st, launches) != 0) return -1;
  } else if (slists) {
    r->setup.slist_entries = r->sl_entries;
    a.slist_n = N;
  }
  a.slist_on = slists && r->sl_built ? 1u : 0u;
  return 0;
}

int set_light(rt_renderer* r, const float light[3], uint32_t* launches) {
  rt_kernel_arg_t& a = r->arg;
  for (int i = 0; i < 3; ++i) {
    a.light[i] = light[i];
    r->params.light[i] = light[i];
  }
  // the render arguments' light, in stream order behind the queued frames --
  // unless every frame carries it in its launch words (rt_render_start)
  const int rc = r->set_words ? 0
                 : r->copy_async
                     ? r->copy_async(r->args, a.light, offsetof(rt_kernel_arg_t, light), sizeof(a.light))
                     : vx_copy_to_dev(r->args, a.light, offsetof(rt_kernel_arg_t, light), sizeof(a.light));
  if (rc != 0) return set_error("light upload failed");
  if (!r->sl_mode) return 0;  // this configuration's shadow rays walk the BVH
  if (r->sl_defer > 0) {
    // the moving light: the next frames walk the BVH for their shadow rays
    // (the same verdicts as the lists) and the lists wait until the light
    // stays (queue_lists from rt_render_start).  A build still unsettled
    // from before is settled first: its last launch writes slist_on.
    if (r->sl_pending && settle_lists(r) != 0) return -1;
    // the frames' launch words switch the stale lists off (RT_LW_NO_SLIST);
    // without them the argument block's slist_on is cleared in stream order
    if (a.slist_on && !r->set_words) {
      a.slist_on = 0;
      const size_t o = offsetof(rt_kernel_arg_t, slist_on);
      const int rs = r->copy_async ? r->copy_async(r->args, &a.slist_on, o, sizeof(a.slist_on))
                                   : vx_copy_to_dev(r->args, &a.slist_on, o, sizeof(a.slist_on));
      if (rs != 0) return set_error("slist_on upload failed");
    }
    a.slist_on = 0;  // (the host's view: the lists are not in use)
    r->sl_stale = true;
    r->sl_static = 0;
    return 0;
  }
  return queue_lists(r, launches);
}

int queue_lists(rt_renderer* r, uint32_t* launches) {
  rt_kernel_arg_t& a = r->arg;
  r->sl_stale = false;
  // the shadow lists for the current light, queued behind it: the chain's last
  // launch writes the render arguments' slist_on (the lists' own verdict),
  // so no host wait anywhere; the status words are read when asked for
  // (rt_renderer_setup_stats) or by the next configure
  rt_setup_arg_t g;
  base_arg(r, &g);
  list_limits(&g);
  g.status_addr = r->su.status.addr;
  if (slist_args(r, &g) != 0) return -1;
  uint64_t rargs = 0;
  if (vx_mem_address(r->args, &rargs) != 0) return set_error("vx_mem_address failed");
  g.rargs_addr = rargs;
  add_fill(&g, g.scnt_addr, g.ncells, 0u);
  add_fill(&g, g.status_addr + 16, 4, 0u);  // status words 4..7: the shadow lists
  g.fold = fold_flags(r);
  Seq q;
  q.add(RTS_FILL | RTS_SPROJ, (g.fold & RTS_FOLD_SOFF) ? 0u : RTS_SOSCAN);
  q.add(RTS_SCOUNT);
  q.add(RTS_SSUM, (g.fold & RTS_FOLD_LISTS) ? 0u : RTS_SSCAN);
  q.add(RTS_SOFF);
  q.add(RTS_SFILL);
  q.add(RTS_SSORT);
  if (run_seq(r, g, q, launches) != 0) return -1;
  std::memcpy(r->sl_light, a.light, sizeof(a.light));
  r->sl_n = a.slist_n;
  r->sl_pending = true;
  return 0;
}

int settle_lists(rt_renderer* r) {
  if (!r->sl_pending) return 0;
  uint32_t st[RTS_STATUS_WORDS];
  if (read_status(r, st) != 0) return -1;
  rt_setup_arg_t g;
  base_arg(r, &g);
  list_limits(&g);
  g.status_addr = r->su.status.addr;
  uint64_t rargs = 0;
  if (vx_mem_address(r->args, &rargs) != 0) return set_error("vx_mem_address failed");
  g.rargs_addr = rargs;
  uint32_t launches = 0;
  const uint64_t sidx0 = r->arg.sidx_addr, slist0 = r->arg.slist_addr;
  if (slist_finish(r, g, st, &launches) != 0) return -1;
  r->arg.slist_on = r->sl_built ? 1u : 0u;
  if (r->arg.sidx_addr != sidx0 || r->arg.slist_addr != slist0) {
    // a refill moved the lists: the render arguments' addresses follow (the
    // refill's SSORT wrote their slist_on)
    const size_t o = offsetof(rt_kernel_arg_t, slist_n);
    const size_t n = offsetof(rt_kernel_arg_t, slist_addr) + sizeof(uint64_t) - o;
    if (vx_copy_to_dev(r->args, reinterpret_cast<const uint8_t*>(&r->arg) + o, o, n) != 0)
      return set_error("vx_copy_to_dev failed");
  }
  return 0;
}

}  // namespace rtapp
