// hip_driver.cpp -- libvortex-hip.so: the MI355X driver plugin.
//
// Implements the 16-entry callbacks_t ABI (callbacks.h; reference
// runtime/common/callbacks.h:23-75 and callbacks.inc:20-225) on HIP.  It takes
// the place of the simx driver (runtime/simx/vortex.cpp:32-246):
//   * device memory   = one hipMalloc'd HBM arena + ArenaAllocator; device
//                       addresses are arena offsets >= USER_BASE_ADDR;
//   * kernel image    = vxbin header + gfx950 code object; start() loads it
//                       once (hipModuleLoadData, cached) and launches
//                       `vx_main` over an oversubscribed grid (16 blocks per
//                       CU: the hardware dispatcher balances the load);
//   * DCRs            = host store, mirrored into the module's __vx_dcrs
//                       constant block at every start();
//   * start/ready_wait = asynchronous launch on the driver's stream, bracketed
//                       by HIP events; ready_wait polls the stop event with a
//                       timeout (the simx driver polls a std::future at 1 s).
//                       simx's start() first waits for the in-flight run
//                       (vortex.cpp:174-176); here a start() behind a run
//                       queues on the stream instead -- the device still runs
//                       them one after the other, the host just does not
//                       idle between them (VX_HIP_QUEUE_DEPTH runs in flight,
//                       default 2; 1 = simx's synchronous behaviour).  Every
//                       call that touches memory, DCRs or counters still
//                       waits for all of them first.  Queued runs carry HIP
//                       events (kernel time) one in VX_HIP_TIME_EVERY (4);
//                       a run started on an idle queue (the apps' start +
//                       wait) is followed by its image's completion kernel
//                       (vx_spawn.h <entry>_done) instead: it stores a nonce
//                       and the launch's start / end stamps to pinned host
//                       words, and ready_wait spins on that word with no HIP
//                       call (VX_HIP_TAIL=0: events as for queued runs);
//   * mpm_query       = device ns (MCYCLE: events, or the completion
//                       kernel's stamps) and task count (MINSTRET) of the
//                       last run;
//   * __vx_state      = per-launch device state: one counter row per block,
//                       written by the block at exit (no per-launch memset)
//                       only while counters are on -- VORTEX_PROFILING set
//                       (the stub's MPM_CLASS DCR, as the reference gates its
//                       perf classes, runtime/stub/utils.cpp:25-47), env
//                       VX_HIP_COUNTERS=1 or vx_hip_set_counters(); without
//                       them a launch writes only its task count (MINSTRET)
//                       and the other counters read 0.
// Error behaviour mirrors callbacks.inc: null handles / zero sizes / ranges
// past the buffer -> -1; unknown caps id -> -1 (simx aborts).
#include <hip/hip_runtime.h>

#include <elf.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "VX_types.h"
#include "arena.h"
#include "callbacks.h"
#include "common.h"
#include "vortex_hip.h"

#define HIP_CHECK(_expr)                                                              \
  do {                                                                                \
    hipError_t _e = (_expr);                                                          \
    if (_e != hipSuccess) {                                                           \
      std::printf("[VXDRV] HIP error: '%s' -> %s\n", #_expr, hipGetErrorString(_e));  \
      return -1;                                                                      \
    }                                                                                 \
  } while (false)

namespace {

constexpr uint64_t kBlockSize = 256;      // allocation granule (>= 64 B DCR blocks)
constexpr uint64_t kDefaultArenaMB = 4096;
// __vx_state layout (include/vx_spawn.h): uint32 mpm[kMaxGrid][kMpmRow],
// one row of the first kMpmRow counters per block, written at block exit
constexpr uint32_t kMaxGrid = 32768;
constexpr uint32_t kMpmRow = 16;
constexpr size_t kTasksOffset = (size_t)kMaxGrid * kMpmRow * sizeof(uint32_t);  // vx_state_t::tasks
constexpr int kGridWavesPerCU = 64;  // 4x the 16 resident waves/CU of the RT kernel
// the pinned host buffer (vx_hip_host_mem): the app's words below
// kHostMemApp, then one 64-B completion slot per in-flight run (<entry>_done:
// nonce, start and end stamps)
constexpr uint64_t kHostMemBytes = 65536, kHostMemApp = 32768, kTailSlot = 64;

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* s = std::getenv(name);
  return (s && *s) ? std::strtoull(s, nullptr, 0) : dflt;
}

uint64_t fnv1a(const uint8_t* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

// The kernel entry of a code object: every image defines one VX_MAIN entry
// named vx_main or vx_main_<image> (include/vx_spawn.h VX_ENTRY; distinct
// names let a rocprofv3 kernel trace tell the images apart).  Read from the
// ELF symbol table: the kernel descriptor symbol "<entry>.kd".
std::string entry_name(const std::vector<uint8_t>& img) {
  const std::string dflt = "vx_main";
  if (img.size() < sizeof(Elf64_Ehdr) || std::memcmp(img.data(), ELFMAG, SELFMAG) != 0) return dflt;
  Elf64_Ehdr eh;
  std::memcpy(&eh, img.data(), sizeof(eh));
  if (eh.e_shoff == 0 || eh.e_shentsize != sizeof(Elf64_Shdr) ||
      eh.e_shoff + (uint64_t)eh.e_shnum * sizeof(Elf64_Shdr) > img.size())
    return dflt;
  auto shdr = [&](uint32_t i) {
    Elf64_Shdr sh;
    std::memcpy(&sh, img.data() + eh.e_shoff + (uint64_t)i * sizeof(Elf64_Shdr), sizeof(sh));
    return sh;
  };
  for (uint32_t i = 0; i < eh.e_shnum; ++i) {
    const Elf64_Shdr sym = shdr(i);
    if (sym.sh_type != SHT_SYMTAB || sym.sh_link >= eh.e_shnum) continue;
    const Elf64_Shdr str = shdr(sym.sh_link);
    if (sym.sh_offset + sym.sh_size > img.size() || str.sh_offset + str.sh_size > img.size()) continue;
    for (uint64_t o = 0; o + sizeof(Elf64_Sym) <= sym.sh_size; o += sizeof(Elf64_Sym)) {
      Elf64_Sym e;
      std::memcpy(&e, img.data() + sym.sh_offset + o, sizeof(e));
      if (e.st_name >= str.sh_size) continue;
      const char* nm = (const char*)img.data() + str.sh_offset + e.st_name;
      const size_t len = strnlen(nm, str.sh_size - e.st_name);
      const std::string n(nm, len);
      // (the image's completion kernel <entry>_done is not the entry)
      if (n.size() > 3 && n.compare(n.size() - 3, 3, ".kd") == 0 && n.rfind("vx_main", 0) == 0 &&
          !(n.size() > 8 && n.compare(n.size() - 8, 8, "_done.kd") == 0))
        return n.substr(0, n.size() - 3);
    }
  }
  return dflt;
}

struct Module {
  hipModule_t module = nullptr;
  hipFunction_t entry = nullptr;
  hipFunction_t done = nullptr;  // <entry>_done: the completion kernel (vx_spawn.h), if the image has one
  std::string name;  // the entry's symbol
  hipDeviceptr_t dcrs = nullptr, mem_base = nullptr, mpm = nullptr;
  size_t dcrs_size = 0, mpm_size = 0;
  uint32_t block = 0, grid = 0;
  uint32_t dcrs_sent[VX_DCR_MIRROR_SIZE] = {};  // host copies kept alive for async H2D
  uint64_t base_value = 0;
  bool dcrs_set = false, base_set = false;
};

}  // namespace

// hip/hip_ext.h's launch templates need the HIP compiler; this file is
// host C++, so the one extension used is declared here (libamdhip64 exports it)
extern "C" hipError_t hipExtModuleLaunchKernel(hipFunction_t f, uint32_t gx, uint32_t gy,
                                               uint32_t gz, uint32_t lx, uint32_t ly, uint32_t lz,
                                               size_t shmem, hipStream_t stream, void** params,
                                               void** extra, hipEvent_t start, hipEvent_t stop,
                                               uint32_t flags);

class vx_device {
 public:
  vx_device() : alloc_(0, 0, kBlockSize) {}

  ~vx_device() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (auto& kv : modules_) (void)hipModuleUnload(kv.second.module);
    for (int i = 0; i < kMaxQueue; ++i) {
      if (ev_start_[i]) (void)hipEventDestroy(ev_start_[i]);
      if (ev_stop_[i]) (void)hipEventDestroy(ev_stop_[i]);
    }
    for (int i = 0; i < kStageSlots; ++i)
      if (stage_ev_[i]) (void)hipEventDestroy(stage_ev_[i]);
    if (stage_) (void)hipHostFree(stage_);
    if (hostmem_) (void)hipHostFree(hostmem_);
    if (stream_) (void)hipStreamDestroy(stream_);
    if (arena_) (void)hipFree(arena_);
  }

  int init() {
    int ndev = 0;
    HIP_CHECK(hipGetDeviceCount(&ndev));
    if (ndev <= 0) {
      std::printf("[VXDRV] no HIP device visible\n");
      return -1;
    }
    int dev = -1;
    if (const char* s = std::getenv("VX_HIP_DEVICE")) dev = std::atoi(s);
    else if (const char* s = std::getenv("LOCAL_RANK")) dev = std::atoi(s) % ndev;
    if (dev < 0) HIP_CHECK(hipGetDevice(&dev));
    device_id_ = dev;
    HIP_CHECK(hipSetDevice(dev));
    HIP_CHECK(hipGetDeviceProperties(&props_, dev));
    const uint64_t arena_bytes = env_u64("VX_HIP_ARENA_MB", kDefaultArenaMB) << 20;
    HIP_CHECK(hipMalloc(&arena_, arena_bytes));
    arena_size_ = arena_bytes;
    alloc_ = ArenaAllocator(USER_BASE_ADDR, arena_bytes - USER_BASE_ADDR, kBlockSize);
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (int i = 0; i < kMaxQueue; ++i) {
      HIP_CHECK(hipEventCreate(&ev_start_[i]));
      HIP_CHECK(hipEventCreate(&ev_stop_[i]));
    }
    HIP_CHECK(hipHostMalloc((void**)&stage_, (size_t)kStageSlots * kStageSlot, hipHostMallocDefault));
    for (int i = 0; i < kStageSlots; ++i)
      HIP_CHECK(hipEventCreateWithFlags(&stage_ev_[i], hipEventDisableTiming));
    const uint64_t qd = env_u64("VX_HIP_QUEUE_DEPTH", 2);
    depth_ = qd < 1 ? 1 : qd > 16 ? 16 : (int)qd;
    const uint64_t te = env_u64("VX_HIP_TIME_EVERY", 4);
    time_every_ = te < 1 ? 1 : te > 16 ? 16 : (int)te;
    launch_mode_ = (int)env_u64("VX_HIP_EXT_LAUNCH", 1);
    launch_mode_timed_ = launch_mode_;
    counters_env_ = env_u64("VX_HIP_COUNTERS", 0) != 0;
    tail_on_ = env_u64("VX_HIP_TAIL", 1) != 0;
    return 0;
  }

  int get_caps(uint32_t id, uint64_t* v) {
    switch (id) {
    case VX_CAPS_VERSION: *v = 1; break;
    case VX_CAPS_NUM_THREADS: *v = 64; break;  // wave64
    case VX_CAPS_NUM_WARPS:
      *v = (uint64_t)props_.maxThreadsPerMultiProcessor / 64;  // 32 waves per CU
      break;
    case VX_CAPS_NUM_CORES: *v = (uint64_t)props_.multiProcessorCount; break;  // 256 CUs
    case VX_CAPS_CACHE_LINE_SIZE: *v = 128; break;
    case VX_CAPS_GLOBAL_MEM_SIZE: *v = arena_size_; break;
    case VX_CAPS_LOCAL_MEM_SIZE: *v = (uint64_t)props_.maxSharedMemoryPerMultiProcessor; break;
    case VX_CAPS_ISA_FLAGS:
      // XLEN 64 (log2(64)-4 = 2 at bit 30); caches, local memory and the
      // graphics extensions (provided by the device library of vx_gfx.h)
      *v = (2ull << 30) | VX_ISA_EXT_ICACHE | VX_ISA_EXT_DCACHE | VX_ISA_EXT_L2CACHE |
           VX_ISA_EXT_L3CACHE | VX_ISA_EXT_LMEM | VX_ISA_EXT_TEX | VX_ISA_EXT_RASTER |
           VX_ISA_EXT_OM;
      break;
    default:
      std::printf("[VXDRV] invalid caps id: %u\n", id);
      return -1;
    }
    return 0;
  }

  int mem_alloc(uint64_t size, int flags, uint64_t* addr) {
    if (alloc_.allocate(size, addr) != 0) return -1;
    acl_[*addr] = flags;
    return 0;
  }
  int mem_reserve(uint64_t addr, uint64_t size, int flags) {
    if (addr + size > arena_size_) return -1;
    if (alloc_.reserve(addr, size) != 0) return -1;
    acl_[addr] = flags;
    shadow_[addr].assign(size, 0);  // kernel images: keep a host copy to load
    return 0;
  }
  int mem_free(uint64_t addr) {
    wait_idle();  // a queued run may still read it
    acl_.erase(addr);
    shadow_.erase(addr);
    image_key_.erase(addr);
    return alloc_.release(addr);
  }
  int mem_access(uint64_t addr, uint64_t size, int flags) {
    uint64_t start = 0;
    const uint64_t asz = alloc_.find(addr, &start);
    if (asz == 0 || addr + size > start + asz) return -1;
    acl_[addr] = flags;  // bookkeeping only: gfx950 has no per-range ACL
    return 0;
  }
  int mem_info(uint64_t* fr, uint64_t* used) const {
    if (fr) *fr = alloc_.free_bytes();
    if (used) *used = alloc_.used_bytes();
    return 0;
  }

  int upload(uint64_t addr, const void* src, uint64_t size) {
    if (addr + size > arena_size_) return -1;
    if (size == 0) return 0;
    wait_idle();
    HIP_CHECK(hipMemcpyAsync(arena_ + addr, src, size, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (auto& kv : shadow_) {  // keep kernel-image shadows coherent
      const uint64_t a = kv.first, e = a + kv.second.size();
      if (addr >= a && addr + size <= e) {
        std::memcpy(kv.second.data() + (addr - a), src, size);
        image_key_.erase(a);
      }
    }
    return 0;
  }
  // stream-ordered upload (vx_hip_copy_to_dev_async): the bytes are staged
  // in a pinned slot at once and copied when the driver's stream reaches
  // the copy, so the host does not wait for queued runs; a slot is reused
  // once its copy has completed (its event).  Larger copies, and copies into
  // a kernel image (whose host shadow must stay coherent), are synchronous.
  int upload_async(uint64_t addr, const void* src, uint64_t size) {
    if (addr + size > arena_size_) return -1;
    if (size == 0) return 0;
    bool image = false;
    for (auto& kv : shadow_)
      image |= addr < kv.first + kv.second.size() && kv.first < addr + size;
    if (size > kStageSlot || image) return upload(addr, src, size);
    const int slot = (int)(stage_next_++ % kStageSlots);
    if (stage_busy_[slot]) HIP_CHECK(hipEventSynchronize(stage_ev_[slot]));
    uint8_t* st = stage_ + (size_t)slot * kStageSlot;
    std::memcpy(st, src, size);
    HIP_CHECK(hipMemcpyAsync(arena_ + addr, st, size, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipEventRecord(stage_ev_[slot], stream_));
    stage_busy_[slot] = true;
    return 0;
  }
  int download(void* dst, uint64_t addr, uint64_t size) {
    if (addr + size > arena_size_) return -1;
    if (size == 0) return 0;
    wait_idle();
    HIP_CHECK(hipMemcpyAsync(dst, arena_ + addr, size, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    return 0;
  }

  int start(uint64_t krnl_addr, uint64_t args_addr) {
    // DCR writes already waited for the device (dcr_write); the STARTUP
    // words below only differ from the in-flight run's when another image
    // or argument block is started, which the constant upload check catches
    if (depth_ <= 1) wait_idle();
    dcr_set(VX_DCR_BASE_STARTUP_ADDR0, (uint32_t)(krnl_addr & 0xffffffffu));
    dcr_set(VX_DCR_BASE_STARTUP_ADDR1, (uint32_t)(krnl_addr >> 32));
    dcr_set(VX_DCR_BASE_STARTUP_ARG0, (uint32_t)(args_addr & 0xffffffffu));
    dcr_set(VX_DCR_BASE_STARTUP_ARG1, (uint32_t)(args_addr >> 32));
    // per-block counter rows only when counters are wanted (vx_spawn.h)
    const bool rows = counters_ || counters_env_ ||
                      (dcr_valid_[VX_DCR_BASE_MPM_CLASS] && dcrs_[VX_DCR_BASE_MPM_CLASS] != 0);
    dcr_set(VX_DCR_HIP_MPM_ROWS, rows ? 1u : 0u);
    Module* m = nullptr;
    if (load_module(krnl_addr, &m) != 0) return -1;
    // constant blocks are only re-sent when they changed since this module's
    // last launch (a steady-state frame loop issues memset + launch only)
    const bool upload = !m->base_set || !m->dcrs_set ||
                        std::memcmp(m->dcrs_sent, dcrs_, sizeof(dcrs_)) != 0;
    // constant uploads read host memory: only with the device idle
    if (upload) wait_idle();
    // bounded queue: with depth_ + time_every_ - 1 runs in flight, retire up
    // to the oldest timed one (at least depth_ - 1 stay queued behind it)
    while (launch_mode_ != 2 && group_pos_ == 0 &&
           issued_ - retired_ >= (uint64_t)(depth_ + time_every_ - 1) * group_n_) {
      uint64_t j = retired_ + 1;
      while (j <= issued_ && !timed_[(j - 1) % kMaxQueue]) ++j;
      if (retire(j <= issued_ ? j : issued_, VX_MAX_TIMEOUT) != 0) return -1;
    }
    if (!m->base_set) {
      m->base_value = (uint64_t)(uintptr_t)arena_;
      HIP_CHECK(hipMemcpyHtoDAsync(m->mem_base, (void*)&m->base_value, sizeof(m->base_value), stream_));
      m->base_set = true;
    }
    if (!m->dcrs_set || std::memcmp(m->dcrs_sent, dcrs_, sizeof(dcrs_)) != 0) {
      std::memcpy(m->dcrs_sent, dcrs_, sizeof(dcrs_));
      HIP_CHECK(hipMemcpyHtoDAsync(m->dcrs, m->dcrs_sent, sizeof(dcrs_), stream_));
      m->dcrs_set = true;
    }
    // the entry's one kernel argument (vx_spawn.h VX_MAIN: vx_launch_tag),
    // copied into the dispatch's kernarg segment by the launch call
    uint32_t tag = launch_tag_;
    launch_tag_ = 0;
    // and its four launch words (vx_hip_set_launch_words), after the tag
    uint32_t words[4];
    std::memcpy(words, launch_words_, sizeof(words));
    std::memset(launch_words_, 0, sizeof(launch_words_));
    void* kparams[2] = {&tag, words};
    const int slot = (int)(issued_ % kMaxQueue);
    // a run is timed (events) when it starts on an idle queue -- every run of
    // a start + wait loop -- and then every time_every_-th run: an event
    // costs ~5 us of idle device between back-to-back runs (measured).  A
    // run is a group of group_n_ launches (vx_hip_launch_group: one frame of
    // several kernels): timed as a whole, the start event on its first
    // launch, the stop event on its last.
    const bool first = group_pos_ == 0, last = group_pos_ + 1 == group_n_;
    // a single launch started on an idle queue -- the synchronous start +
    // wait of the reference's apps (draw3d/main.cpp:353-357) -- is followed by
    // its image's completion kernel instead of carrying events: the wait spins
    // on a pinned host word (no hipEventQuery), the duration comes from the
    // device's own stamps (launch_probe: +6.6 vs +14.5 us over the kernel)
    const bool tail = tail_on_ && m->done && group_n_ == 1 && !group_untimed_ && launch_mode_ != 2 &&
                      issued_ == retired_ && ensure_hostmem() == 0;
    if (first) {
      group_timed_ = !group_untimed_ && launch_mode_ != 2 &&
                     (issued_ == retired_ || runs_issued_ % time_every_ == 0);
      group_slot_ = slot;
      group_mods_.clear();
      ++runs_issued_;
    }
    group_mods_.push_back({m, m->grid, rows});
    const bool timed = group_timed_ && !tail;
    timed_[slot] = (timed || tail) && last;  // the run completes (and is timed) with its last launch
    tail_[slot] = tail;
    group_last_[slot] = last;
    group_first_slot_[slot] = group_slot_;
    group_pos_ = last ? 0 : group_pos_ + 1;
    if (last) {  // a group covers the launches it was declared for
      group_n_ = 1;
      group_untimed_ = false;
    }
    if (tail) {
      HIP_CHECK(hipExtModuleLaunchKernel(m->entry, m->grid * m->block, 1, 1, m->block, 1, 1, 0,
                                         stream_, kparams, nullptr, nullptr, nullptr, 0));
      const uint32_t nonce = ++tail_nonce_;
      tail_nonce_slot_[slot] = nonce;
      volatile uint32_t* w = tail_word(slot);
      w[0] = 0u;
      uint64_t hp = hostmem_dev_ + kHostMemApp + (uint64_t)slot * kTailSlot;
      uint32_t nv = nonce;
      void* dparams[2] = {&hp, &nv};
      HIP_CHECK(hipModuleLaunchKernel(m->done, 1, 1, 1, 64, 1, 1, 0, stream_, dparams, nullptr));
    } else if (!timed) {
      HIP_CHECK(hipExtModuleLaunchKernel(m->entry, m->grid * m->block, 1, 1, m->block, 1, 1, 0,
                                         stream_, kparams, nullptr, nullptr, nullptr, 0));
    } else if (launch_mode_ == 2) {
      HIP_CHECK(hipExtModuleLaunchKernel(m->entry, m->grid * m->block, 1, 1, m->block, 1, 1, 0,
                                         stream_, kparams, nullptr, nullptr, nullptr, 0));
    } else if (launch_mode_ == 1) {
      // the dispatch packet itself carries the start/stop timestamps: no
      // separate event packets between back-to-back frames
      HIP_CHECK(hipExtModuleLaunchKernel(m->entry, m->grid * m->block, 1, 1, m->block, 1, 1, 0,
                                         stream_, kparams, nullptr,
                                         first ? ev_start_[slot] : nullptr,
                                         last ? ev_stop_[slot] : nullptr, 0));
    } else {
      if (first) HIP_CHECK(hipEventRecord(ev_start_[slot], stream_));
      HIP_CHECK(hipModuleLaunchKernel(m->entry, m->grid, 1, 1, m->block, 1, 1, 0, stream_,
                                      kparams, nullptr));
      if (last) HIP_CHECK(hipEventRecord(ev_stop_[slot], stream_));
    }
    ++issued_;
    mpm_dirty_ = true;  // read back lazily by mpm_query (after wait_idle)
    last_rows_ = rows;
    last_module_ = m;
    last_grid_ = m->grid;
    last_block_ = m->block;
    return 0;
  }

  int ready_wait(uint64_t timeout_ms) { return retire(issued_, timeout_ms); }

  // wait until run number `upto` (1-based issue count) has finished, then
  // retire every run up to it: per-run event time into last_ms_ and the
  // running totals (vx_hip_run_totals)
  int retire(uint64_t upto, uint64_t timeout_ms) {
    if (upto <= retired_) return 0;
    // an untimed run has no event: its completion is the stream's; a run
    // with a completion kernel is complete when its pinned word holds its nonce
    const int us = (int)((upto - 1) % kMaxQueue);
    const bool by_tail = tail_[us] && timed_[us];
    const bool by_event = timed_[us] && !by_tail;
    if (!by_event && !by_tail) upto = issued_;
    hipEvent_t stop = ev_stop_[(upto - 1) % kMaxQueue];
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      if (by_tail) {
        if (*tail_word(us) == tail_nonce_slot_[us]) break;
        // (no HIP call on this path: a fault still ends the wait at the timeout)
        const auto dt = std::chrono::steady_clock::now() - t0;
        if ((uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(dt).count() > timeout_ms) {
          const hipError_t e = hipStreamQuery(stream_);
          if (e != hipSuccess && e != hipErrorNotReady) {
            std::printf("[VXDRV] kernel failed: %s\n", hipGetErrorString(e));
            retired_ = issued_;
          }
          return -1;
        }
        if (spin > 4096 && dt > std::chrono::milliseconds(5)) {
          // a long run: check the stream for a fault now and then, then sleep
          const hipError_t e = hipStreamQuery(stream_);
          if (e != hipSuccess && e != hipErrorNotReady) {
            std::printf("[VXDRV] kernel failed: %s\n", hipGetErrorString(e));
            retired_ = issued_;
            return -1;
          }
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        continue;
      }
      hipError_t e = by_event ? hipEventQuery(stop) : hipStreamQuery(stream_);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) {
        std::printf("[VXDRV] kernel failed: %s\n", hipGetErrorString(e));
        retired_ = issued_;
        return -1;
      }
      const auto dt = std::chrono::steady_clock::now() - t0;
      if ((uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(dt).count() > timeout_ms)
        return -1;
      // spin (a frame is ~0.1 ms; a sleep costs its timer slack, ~60 us),
      // back off to sleeping only for long runs
      if (spin > 1024 && dt > std::chrono::milliseconds(5))
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    for (; retired_ < upto; ++retired_) {
      const int slot = (int)(retired_ % kMaxQueue);
      if (!group_last_[slot]) continue;  // a run = a whole launch group
      ++runs_total_;
      if (!timed_[slot]) continue;
      float ms = 0.0f;
      if (tail_[slot]) {
        // block 0's start to the completion kernel's start (100 MHz stamps):
        // the kernel plus the launch boundary behind it
        volatile uint32_t* w = tail_word(slot);
        std::atomic_thread_fence(std::memory_order_acquire);
        const uint64_t a = ((uint64_t)w[3] << 32) | w[2], b = ((uint64_t)w[5] << 32) | w[4];
        ms = b > a ? (float)((double)(b - a) * 1.0e-5) : 0.0f;
      } else {
        HIP_CHECK(hipEventElapsedTime(&ms, ev_start_[group_first_slot_[slot]], ev_stop_[slot]));
      }
      last_ms_ = ms;
      last_stamped_ = tail_[slot];
      run_ms_total_ += ms;
      ++runs_timed_;
      runs_stamped_ += tail_[slot] ? 1u : 0u;
    }
    return 0;
  }

  int dcr_write(uint32_t addr, uint32_t value) {
    if (addr >= VX_DCR_MIRROR_SIZE) return -1;
    wait_idle();  // simx: ensure the prior run completed (vortex.cpp:211-214)
    dcr_set(addr, value);
    return 0;
  }
  int dcr_read(uint32_t addr, uint32_t* value) const {
    if (addr >= VX_DCR_MIRROR_SIZE || !dcr_valid_[addr]) return -1;
    *value = dcrs_[addr];
    return 0;
  }

  int mpm_query(uint32_t addr, uint32_t core_id, uint64_t* value) {
    const uint32_t off = addr - VX_CSR_MPM_BASE;
    if (off >= VX_MPM_COUNT) return -1;
    if (core_id != 0) { *value = 0; return 0; }  // device totals live on core 0
    wait_idle();
    if (addr == VX_CSR_MCYCLE) {
      *value = (uint64_t)(last_ms_ * 1.0e6 + 0.5);
      return 0;
    }
    if (mpm_dirty_ && last_module_) {
      for (uint32_t i = 0; i < VX_MPM_COUNT; ++i) mpm_[i] = 0;
      // every launch of the last run (launch group): their modules are
      // distinct images, each with its own counter slab
      for (const GroupLaunch& g : group_mods_) {
        if (g.rows) {  // sum the per-block counter rows of the launch
          rows_.resize((size_t)g.grid * kMpmRow);
          HIP_CHECK(hipMemcpyAsync(rows_.data(), g.m->mpm, rows_.size() * sizeof(uint32_t),
                                   hipMemcpyDeviceToHost, stream_));
          HIP_CHECK(hipStreamSynchronize(stream_));
          for (size_t b = 0; b < g.grid; ++b)
            for (uint32_t i = 0; i < kMpmRow; ++i) mpm_[i] += rows_[b * kMpmRow + i];
        } else {  // counters off: the task count the launch declared
          uint32_t tasks = 0;
          HIP_CHECK(hipMemcpyAsync(&tasks, (uint8_t*)g.m->mpm + kTasksOffset, 4,
                                   hipMemcpyDeviceToHost, stream_));
          HIP_CHECK(hipStreamSynchronize(stream_));
          mpm_[VX_CSR_MINSTRET - VX_CSR_MPM_BASE] += tasks;
        }
      }
      mpm_dirty_ = false;
    }
    *value = mpm_[off];
    return 0;
  }

  // ---- extensions (vortex_hip.h) ----
  int mpm_rows(uint32_t* rows, uint64_t max_rows, uint64_t* nrows) {
    wait_idle();
    if (nrows) *nrows = last_grid_;
    if (!last_module_ || !rows) return last_module_ ? 0 : -1;
    const uint64_t n = max_rows < last_grid_ ? max_rows : last_grid_;
    HIP_CHECK(hipMemcpyAsync(rows, last_module_->mpm, n * kMpmRow * sizeof(uint32_t),
                             hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    return 0;
  }
  void set_counters(bool on) { counters_ = on; }  // applies from the next start()
  // timed (1: events on one run in time_every_, the default) or untimed (0:
  // no events, no queue bound -- back-to-back launches for a host clock)
  int set_timing(int timed) {
    if (group_pos_ != 0) return -1;
    wait_idle();
    launch_mode_ = timed ? (launch_mode_timed_ == 2 ? 1 : launch_mode_timed_) : 2;
    return 0;
  }
  // the next n launches form one run (then single launches again).  The
  // event and slot arrays must hold every launch the queue bound lets into
  // flight, (depth_ + time_every_ - 1) * n, plus the one being issued.
  // n = 0 abandons an open group (a launch inside it failed): the launches
  // already issued retire as one untimed run, and single launches resume.
  int launch_group(uint32_t n) {
    const bool untimed = (n & VX_HIP_GROUP_UNTIMED) != 0;
    n &= ~VX_HIP_GROUP_UNTIMED;
    if (n == 0) {
      if (group_pos_ != 0) {
        const int slot = (int)((issued_ + kMaxQueue - 1) % kMaxQueue);
        group_last_[slot] = true;
        timed_[slot] = false;
      }
      group_pos_ = 0;
      group_n_ = 1;
      group_untimed_ = false;
      return 0;
    }
    if ((n > 4 && !untimed) || group_pos_ != 0) return -1;  // not inside a group
    if ((uint64_t)(depth_ + time_every_) * n > (uint64_t)kMaxQueue) return -1;
    group_n_ = n;
    group_untimed_ = untimed;
    return 0;
  }
  void set_launch_tag(uint32_t tag) { launch_tag_ = tag; }  // the next start()'s kernel argument
  void set_launch_words(const uint32_t* w, uint32_t n) {       // and its launch words
    std::memset(launch_words_, 0, sizeof(launch_words_));
    std::memcpy(launch_words_, w, n * sizeof(uint32_t));
  }
  // one pinned host buffer mapped into the device's address space (allocated
  // on first use, at most 64 KiB): kernels store to it, the host reads it
  // after waiting for the device -- no copy back
  int host_mem(uint64_t size, void** host, uint64_t* dev) {
    if (size == 0 || size > kHostMemApp) return -1;
    if (ensure_hostmem() != 0) return -1;
    *host = hostmem_;
    *dev = hostmem_dev_;
    return 0;
  }
  int ensure_hostmem() {
    if (hostmem_) return 0;
    HIP_CHECK(hipHostMalloc(&hostmem_, kHostMemBytes, hipHostMallocMapped));
    std::memset(hostmem_, 0, kHostMemBytes);
    void* d = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&d, hostmem_, 0));
    hostmem_dev_ = (uint64_t)(uintptr_t)d;
    return 0;
  }
  // a run's completion word in the pinned block.  Guarded (r06, VERDICT r05
  // item 5): the r05c / r05d work-in-progress trees died with SIGSEGV in
  // rt_renderer_create while this block was being introduced -- the tree of
  // those runs was never committed, and a completion word touched before the
  // block existed (or past it) fits the trace; a slot outside the block or a
  // block not yet allocated now ends the process with a message instead
  volatile uint32_t* tail_word(int slot) const {
    if (!hostmem_ || slot < 0 || slot >= kMaxQueue) {
      std::fprintf(stderr, "[VXDRV] completion slot %d outside the pinned block (%p)\n", slot, hostmem_);
      std::abort();
    }
    return reinterpret_cast<volatile uint32_t*>(static_cast<uint8_t*>(hostmem_) + kHostMemApp +
                                                (uint64_t)slot * kTailSlot);
  }
  bool counters() const { return counters_ || counters_env_; }
  void* mem_ptr(uint64_t addr) { return arena_ + addr; }
  hipStream_t stream() const { return stream_; }
  int device_id() const { return device_id_; }
  double last_ms() const { return last_ms_; }
  // which clock timed the runs: the completion kernel's stamps
  // (a run started on an idle queue: kernel + launch boundary) or HIP events
  // on the dispatch (queued runs: kernel only)
  void timing_source(int* last_stamped, uint64_t* stamped, uint64_t* evented) const {
    if (last_stamped) *last_stamped = last_stamped_ ? 1 : 0;
    if (stamped) *stamped = runs_stamped_;
    if (evented) *evented = runs_timed_ - runs_stamped_;
  }
  void run_totals(double* ms, uint64_t* timed, uint64_t* runs) {
    wait_idle();
    if (ms) *ms = run_ms_total_;
    if (timed) *timed = runs_timed_;
    if (runs) *runs = runs_total_;
  }
  uint32_t last_grid() const { return last_grid_; }
  uint32_t last_block() const { return last_block_; }

 private:
  void dcr_set(uint32_t addr, uint32_t v) {
    dcrs_[addr] = v;
    dcr_valid_[addr] = true;
  }
  void wait_idle() {
    if (issued_ > retired_) ready_wait(VX_MAX_TIMEOUT);
  }

  int load_module(uint64_t krnl_addr, Module** out) {
    auto it = shadow_.find(krnl_addr);
    if (it == shadow_.end()) {
      std::printf("[VXDRV] no kernel image at 0x%llx (use vx_upload_kernel_*)\n",
                  (unsigned long long)krnl_addr);
      return -1;
    }
    // the image is hashed only after an upload touched it (not per launch)
    auto hit = image_key_.find(krnl_addr);
    if (hit == image_key_.end()) {
      const std::vector<uint8_t>& img = it->second;
      hit = image_key_.emplace(krnl_addr, fnv1a(img.data(), img.size()) ^ krnl_addr).first;
    }
    const uint64_t key = hit->second;
    auto mit = modules_.find(key);
    if (mit != modules_.end()) {
      *out = &mit->second;
      return 0;
    }
    const std::vector<uint8_t>& img = it->second;
    Module m;
    HIP_CHECK(hipModuleLoadData(&m.module, img.data()));
    m.name = entry_name(img);
    HIP_CHECK(hipModuleGetFunction(&m.entry, m.module, m.name.c_str()));
    // its completion kernel (vx_spawn.h VX_MAIN), when the image has one
    if (hipModuleGetFunction(&m.done, m.module, (m.name + "_done").c_str()) != hipSuccess) {
      m.done = nullptr;
      (void)hipGetLastError();
    }
    HIP_CHECK(hipModuleGetGlobal(&m.dcrs, &m.dcrs_size, m.module, "__vx_dcrs"));
    size_t sz = 0;
    HIP_CHECK(hipModuleGetGlobal(&m.mem_base, &sz, m.module, "__vx_mem_base"));
    HIP_CHECK(hipModuleGetGlobal(&m.mpm, &m.mpm_size, m.module, "__vx_state"));  // mpm + queues
    int max_threads = 0;
    HIP_CHECK(hipFuncGetAttribute(&max_threads, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, m.entry));
    m.block = (uint32_t)(max_threads > 0 ? max_threads : 256);
    // Grid = kGridWavesPerCU waves per CU, several times what is resident:
    // vx_spawn deals 64-task chunks to waves by global wave id, so the blocks
    // waiting for a slot are the load balancer (the hardware dispatcher hands
    // a CU its next block when one retires, as simx's cores pull warps).
    int per_cu = kGridWavesPerCU / (int)((m.block + 63) / 64);
    // an image may carry its own measured grid (u32 __vx_grid_per_cu, in
    // 64-thread blocks per CU); the env knob still overrides it
    hipDeviceptr_t gp = nullptr;
    size_t gsz = 0;
    if (hipModuleGetGlobal(&gp, &gsz, m.module, "__vx_grid_per_cu") == hipSuccess && gsz == 4) {
      // read on the driver's stream (frames of another image may be queued
      // on it; the null stream would not be ordered with them)
      uint32_t v = 0;
      HIP_CHECK(hipMemcpyAsync(&v, gp, 4, hipMemcpyDeviceToHost, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
      if (v > 0) per_cu = (int)v;
    } else {
      (void)hipGetLastError();
    }
    if (const char* s = std::getenv("VX_HIP_BLOCKS_PER_CU")) per_cu = std::atoi(s);
    if (per_cu < 1) per_cu = 1;
    m.grid = (uint32_t)(props_.multiProcessorCount * per_cu);
    if (m.grid > kMaxGrid) m.grid = kMaxGrid;
    if (m.mpm_size < kTasksOffset + sizeof(uint32_t)) {
      std::printf("[VXDRV] kernel image has no per-block counter slab\n");
      return -1;
    }
    auto ins = modules_.emplace(key, m);
    *out = &ins.first->second;
    return 0;
  }

  hipDeviceProp_t props_{};
  int device_id_ = 0;
  uint8_t* arena_ = nullptr;
  uint64_t arena_size_ = 0;
  ArenaAllocator alloc_;
  std::map<uint64_t, int> acl_;
  std::map<uint64_t, std::vector<uint8_t>> shadow_;
  std::map<uint64_t, Module> modules_;
  // pinned staging slots of upload_async
  static constexpr int kStageSlots = 64;
  static constexpr uint64_t kStageSlot = 4096;
  uint8_t* stage_ = nullptr;
  void* hostmem_ = nullptr;  // vx_hip_host_mem: pinned, device-mapped words (+ completion slots)
  uint64_t hostmem_dev_ = 0;
  // completion kernels (<entry>_done): per queue slot whether the run has
  // one and the nonce it stores; VX_HIP_TAIL=0 keeps events on idle-queue runs
  bool tail_[64] = {};
  uint32_t tail_nonce_slot_[64] = {};
  uint32_t tail_nonce_ = 0;
  bool tail_on_ = true;
  hipEvent_t stage_ev_[kStageSlots] = {};
  bool stage_busy_[kStageSlots] = {};
  uint64_t stage_next_ = 0;
  uint32_t launch_tag_ = 0;
  uint32_t launch_words_[4] = {};
  std::map<uint64_t, uint64_t> image_key_;  // image address -> module key
  hipStream_t stream_ = nullptr;
  static constexpr int kMaxQueue = 64;  // >= (depth_ + time_every_) * group_n_
  static_assert(kHostMemApp + (uint64_t)kMaxQueue * kTailSlot <= kHostMemBytes,
                "a completion slot per queue slot in the pinned block");
  static_assert(kMaxQueue == 64, "tail_ / tail_nonce_slot_ are sized by it");
  static_assert(kHostMemApp + kMaxQueue * kTailSlot <= kHostMemBytes, "completion slots fit");
  hipEvent_t ev_start_[kMaxQueue] = {}, ev_stop_[kMaxQueue] = {};
  bool timed_[kMaxQueue] = {};
  // launch groups (vx_hip_launch_group): group_n_ consecutive launches form
  // one run (a frame of several kernels)
  struct GroupLaunch {
    Module* m;
    uint32_t grid;
    bool rows;
  };
  uint32_t group_n_ = 1, group_pos_ = 0;
  bool group_untimed_ = false;  // the declared group runs without events
  uint64_t runs_issued_ = 0;
  bool group_timed_ = false;
  int group_slot_ = 0;
  bool group_last_[kMaxQueue] = {};
  int group_first_slot_[kMaxQueue] = {};
  std::vector<GroupLaunch> group_mods_;
  int time_every_ = 4;
  uint64_t runs_timed_ = 0;
  uint64_t issued_ = 0, retired_ = 0;  // runs started / retired (events read)
  int depth_ = 2;
  // 0: hipModuleLaunchKernel between two hipEventRecord packets;
  // 1: hipExtModuleLaunchKernel, start/stop timestamps on the dispatch packet;
  // 2: diagnostic -- every run untimed (no events, no queue bound)
  int launch_mode_ = 1;
  int launch_mode_timed_ = 1;  // the mode set_timing(1) restores
  double run_ms_total_ = 0.0;
  uint64_t runs_total_ = 0;
  Module* last_module_ = nullptr;
  bool mpm_dirty_ = false;
  bool counters_ = false, counters_env_ = false, last_rows_ = false;
  double last_ms_ = 0.0;
  bool last_stamped_ = false;
  uint64_t runs_stamped_ = 0;
  uint32_t last_grid_ = 0, last_block_ = 0;
  uint32_t dcrs_[VX_DCR_MIRROR_SIZE] = {};
  bool dcr_valid_[VX_DCR_MIRROR_SIZE] = {};
  unsigned long long mpm_[VX_MPM_COUNT] = {};
  std::vector<uint32_t> rows_;
};

struct vx_buffer {
  vx_device* device;
  uint64_t addr;
  uint64_t size;
};

extern "C" {

__attribute__((visibility("default"))) int vx_dev_init(callbacks_t* cb) {
  if (cb == nullptr) return -1;
  cb->dev_open = [](vx_device_h* hdevice) -> int {
    if (hdevice == nullptr) return -1;
    auto* d = new vx_device();
    VX_CHECK_ERR(d->init(), { delete d; return err; });
    *hdevice = d;
    return 0;
  };
  cb->dev_close = [](vx_device_h hdevice) -> int {
    if (hdevice == nullptr) return -1;
    delete (vx_device*)hdevice;
    return 0;
  };
  cb->dev_caps = [](vx_device_h hdevice, uint32_t id, uint64_t* value) -> int {
    if (hdevice == nullptr || value == nullptr) return -1;
    return ((vx_device*)hdevice)->get_caps(id, value);
  };
  cb->mem_alloc = [](vx_device_h hdevice, uint64_t size, int flags, vx_buffer_h* hbuf) -> int {
    if (hdevice == nullptr || hbuf == nullptr || size == 0) return -1;
    auto* d = (vx_device*)hdevice;
    uint64_t addr = 0;
    VX_CHECK_ERR(d->mem_alloc(size, flags, &addr), { return err; });
    *hbuf = new vx_buffer{d, addr, size};
    return 0;
  };
  cb->mem_reserve = [](vx_device_h hdevice, uint64_t address, uint64_t size, int flags,
                       vx_buffer_h* hbuf) -> int {
    if (hdevice == nullptr || hbuf == nullptr || size == 0) return -1;
    auto* d = (vx_device*)hdevice;
    VX_CHECK_ERR(d->mem_reserve(address, size, flags), { return err; });
    *hbuf = new vx_buffer{d, address, size};
    return 0;
  };
  cb->mem_free = [](vx_buffer_h hbuf) -> int {
    if (hbuf == nullptr) return 0;
    auto* b = (vx_buffer*)hbuf;
    const int err = b->device->mem_free(b->addr);
    delete b;
    return err;
  };
  cb->mem_access = [](vx_buffer_h hbuf, uint64_t off, uint64_t size, int flags) -> int {
    if (hbuf == nullptr) return -1;
    auto* b = (vx_buffer*)hbuf;
    if (off + size > b->size) return -1;
    return b->device->mem_access(b->addr + off, size, flags);
  };
  cb->mem_address = [](vx_buffer_h hbuf, uint64_t* address) -> int {
    if (hbuf == nullptr || address == nullptr) return -1;
    *address = ((vx_buffer*)hbuf)->addr;
    return 0;
  };
  cb->mem_info = [](vx_device_h hdevice, uint64_t* fr, uint64_t* used) -> int {
    if (hdevice == nullptr) return -1;
    return ((vx_device*)hdevice)->mem_info(fr, used);
  };
  cb->copy_to_dev = [](vx_buffer_h hbuf, const void* src, uint64_t off, uint64_t size) -> int {
    if (hbuf == nullptr || src == nullptr) return -1;
    auto* b = (vx_buffer*)hbuf;
    if (off + size > b->size) return -1;
    return b->device->upload(b->addr + off, src, size);
  };
  cb->copy_from_dev = [](void* dst, vx_buffer_h hbuf, uint64_t off, uint64_t size) -> int {
    if (hbuf == nullptr || dst == nullptr) return -1;
    auto* b = (vx_buffer*)hbuf;
    if (off + size > b->size) return -1;
    return b->device->download(dst, b->addr + off, size);
  };
  cb->start = [](vx_device_h hdevice, vx_buffer_h hkernel, vx_buffer_h hargs) -> int {
    if (hdevice == nullptr || hkernel == nullptr || hargs == nullptr) return -1;
    return ((vx_device*)hdevice)->start(((vx_buffer*)hkernel)->addr, ((vx_buffer*)hargs)->addr);
  };
  cb->ready_wait = [](vx_device_h hdevice, uint64_t timeout) -> int {
    if (hdevice == nullptr) return -1;
    return ((vx_device*)hdevice)->ready_wait(timeout);
  };
  cb->dcr_read = [](vx_device_h hdevice, uint32_t addr, uint32_t* value) -> int {
    if (hdevice == nullptr || value == nullptr) return -1;
    return ((vx_device*)hdevice)->dcr_read(addr, value);
  };
  cb->dcr_write = [](vx_device_h hdevice, uint32_t addr, uint32_t value) -> int {
    if (hdevice == nullptr) return -1;
    return ((vx_device*)hdevice)->dcr_write(addr, value);
  };
  cb->mpm_query = [](vx_device_h hdevice, uint32_t addr, uint32_t core, uint64_t* value) -> int {
    if (hdevice == nullptr || value == nullptr) return -1;
    return ((vx_device*)hdevice)->mpm_query(addr, core, value);
  };
  return 0;
}

// ---- extensions (vortex_hip.h) ----
__attribute__((visibility("default"))) int vx_hip_mem_ptr(vx_buffer_h hbuf, void** ptr) {
  if (hbuf == nullptr || ptr == nullptr) return -1;
  auto* b = (vx_buffer*)hbuf;
  *ptr = b->device->mem_ptr(b->addr);
  return 0;
}
__attribute__((visibility("default"))) int vx_hip_stream(vx_device_h hdevice, void** stream) {
  if (hdevice == nullptr || stream == nullptr) return -1;
  *stream = (void*)((vx_device*)hdevice)->stream();
  return 0;
}
__attribute__((visibility("default"))) int vx_hip_last_run(vx_device_h hdevice, double* ms,
                                                           uint32_t* grid, uint32_t* block) {
  if (hdevice == nullptr) return -1;
  auto* d = (vx_device*)hdevice;
  d->run_totals(nullptr, nullptr, nullptr);  // retires every queued run
  if (ms) *ms = d->last_ms();
  if (grid) *grid = d->last_grid();
  if (block) *block = d->last_block();
  return 0;
}
__attribute__((visibility("default"))) int vx_hip_run_totals(vx_device_h hdevice, double* ms,
                                                             uint64_t* timed, uint64_t* runs) {
  if (hdevice == nullptr) return -1;
  ((vx_device*)hdevice)->run_totals(ms, timed, runs);
  return 0;
}
__attribute__((visibility("default"))) int vx_hip_mpm_rows(vx_device_h hdevice, uint32_t* rows,
                                                           uint64_t max_rows, uint64_t* nrows) {
  if (hdevice == nullptr) return -1;
  return ((vx_device*)hdevice)->mpm_rows(rows, max_rows, nrows);
}
__attribute__((visibility("default"))) int vx_hip_set_counters(vx_device_h hdevice, int enable) {
  if (hdevice == nullptr) return -1;
  ((vx_device*)hdevice)->set_counters(enable != 0);
  return 0;
}
__attribute__((visibility("default"))) int vx_hip_set_timing(vx_device_h hdevice, int timed) {
  if (hdevice == nullptr) return -1;
  return ((vx_device*)hdevice)->set_timing(timed);
}
__attribute__((visibility("default"))) int vx_hip_launch_group(vx_device_h hdevice, uint32_t n) {
  if (hdevice == nullptr) return -1;
  return ((vx_device*)hdevice)->launch_group(n);
}
__attribute__((visibility("default"))) int vx_hip_copy_to_dev_async(vx_buffer_h hbuf, const void* src,
                                                                    uint64_t off, uint64_t size) {
  if (hbuf == nullptr || (src == nullptr && size != 0)) return -1;
  auto* b = (vx_buffer*)hbuf;
  if (off + size > b->size) return -1;
  return b->device->upload_async(b->addr + off, src, size);
}
__attribute__((visibility("default"))) int vx_hip_host_mem(vx_device_h hdevice, uint64_t size, void** host,
                                                           uint64_t* device_addr) {
  if (hdevice == nullptr || host == nullptr || device_addr == nullptr) return -1;
  return ((vx_device*)hdevice)->host_mem(size, host, device_addr);
}
__attribute__((visibility("default"))) int vx_hip_timing_source(vx_device_h hdevice, int* last_stamped,
                                                                uint64_t* stamped_runs, uint64_t* event_runs) {
  if (hdevice == nullptr) return -1;
  ((vx_device*)hdevice)->timing_source(last_stamped, stamped_runs, event_runs);
  return 0;
}

__attribute__((visibility("default"))) int vx_hip_set_launch_words(vx_device_h hdevice, const uint32_t* words,
                                                                   uint32_t n) {
  if (hdevice == nullptr || (n > 0 && words == nullptr) || n > 4) return -1;
  ((vx_device*)hdevice)->set_launch_words(words, n);
  return 0;
}

__attribute__((visibility("default"))) int vx_hip_set_launch_tag(vx_device_h hdevice, uint32_t tag) {
  if (hdevice == nullptr) return -1;
  ((vx_device*)hdevice)->set_launch_tag(tag);
  return 0;
}
__attribute__((visibility("default"))) int vx_hip_device_id(vx_device_h hdevice, int* id) {
  if (hdevice == nullptr || id == nullptr) return -1;
  *id = ((vx_device*)hdevice)->device_id();
  return 0;
}

}  // extern "C"
