// aql_probe.cpp -- the synchronous-frame cost of a direct AQL dispatch (DESIGN
// 1), next to launch_probe.hip's HIP mechanisms: the frame
// kernel of launch_probe (aql_probe_kernel.hip, a code object loaded through
// the HSA loader) dispatched by writing one kernel-dispatch packet into a
// user-mode queue of our own and ringing its doorbell, completion by the
// packet's completion signal (host spins on it) -- no HIP launch call and no
// second kernel per frame.  Also times hipModuleLaunchKernel + the one-wave
// tail kernel on the same frame (the driver's current mechanism) in the same
// process, so the two are compared on one box.
//   aql_probe <kernel.co> [frames] [ticks]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#define HK(x)                                                                           \
  do {                                                                                  \
    hsa_status_t s_ = (x);                                                              \
    if (s_ != HSA_STATUS_SUCCESS) {                                                     \
      const char* m_ = nullptr;                                                         \
      hsa_status_string(s_, &m_);                                                       \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, m_ ? m_ : "?"); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)
#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                       \
    }                                                                                     \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

struct Found {
  hsa_agent_t gpu{};
  bool have_gpu = false;
  hsa_region_t kernarg{};
  bool have_kernarg = false;
};
static hsa_status_t find_gpu(hsa_agent_t a, void* d) {
  Found* f = (Found*)d;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !f->have_gpu) {
    f->gpu = a;
    f->have_gpu = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kernarg(hsa_region_t r, void* d) {
  Found* f = (Found*)d;
  hsa_region_segment_t seg;
  hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg);
  if (seg != HSA_REGION_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_REGION_GLOBAL_FLAG_KERNARG) && !f->have_kernarg) {
    f->kernarg = r;
    f->have_kernarg = true;
  }
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: aql_probe <kernel.co> [frames] [ticks]\n");
    return 2;
  }
  const int frames = argc > 2 ? std::atoi(argv[2]) : 400;
  const uint32_t ticks = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 1200;
  const uint32_t nblocks = 8192, block = 128;
  std::ifstream in(argv[1], std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (co.empty()) {
    std::fprintf(stderr, "aql_probe: cannot read %s\n", argv[1]);
    return 2;
  }
  CK(hipSetDevice(0));
  uint32_t *host_word = nullptr, *dev_word = nullptr;
  CK(hipHostMalloc((void**)&host_word, 64, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&dev_word, host_word, 0));
  volatile uint32_t* hw = host_word;

  HK(hsa_init());
  Found f;
  HK(hsa_iterate_agents(find_gpu, &f));
  if (!f.have_gpu) return 3;
  HK(hsa_agent_iterate_regions(f.gpu, find_kernarg, &f));
  if (!f.have_kernarg) return 3;
  hsa_queue_t* q = nullptr;
  HK(hsa_queue_create(f.gpu, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  hsa_code_object_reader_t rdr;
  HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rdr));
  hsa_executable_t exe;
  HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  HK(hsa_executable_load_agent_code_object(exe, f.gpu, rdr, nullptr, nullptr));
  HK(hsa_executable_freeze(exe, nullptr));
  auto kernel = [&](const char* name, uint64_t* obj, uint32_t* ka, uint32_t* grp, uint32_t* prv) {
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(exe, name, &f.gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, obj));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, ka));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, grp));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, prv));
  };
  uint64_t kobj = 0;
  uint32_t kasz = 0, grp = 0, prv = 0;
  kernel("aql_frame_kernel.kd", &kobj, &kasz, &grp, &prv);
  // explicit arguments (ticks, counter, host_word, nonce, nblocks) then the
  // hidden block counts / group sizes (code object v5: at the first 8-B
  // boundary after the explicit ones)
  void* kargs = nullptr;
  HK(hsa_memory_allocate(f.kernarg, kasz < 256 ? 256 : kasz, &kargs));
  std::memset(kargs, 0, kasz < 256 ? 256 : kasz);
  uint8_t* kb = (uint8_t*)kargs;
  auto put32 = [&](size_t off, uint32_t v) { std::memcpy(kb + off, &v, 4); };
  auto put64 = [&](size_t off, uint64_t v) { std::memcpy(kb + off, &v, 8); };
  auto put16 = [&](size_t off, uint16_t v) { std::memcpy(kb + off, &v, 2); };
  put32(0, ticks);
  put64(8, 0);
  put64(16, (uint64_t)(uintptr_t)dev_word);
  put32(24, 0);
  put32(28, nblocks);
  put32(32, nblocks); put32(36, 1); put32(40, 1);         // hidden_block_count_x/y/z
  put16(44, (uint16_t)block); put16(46, 1); put16(48, 1);  // hidden_group_size_x/y/z
  uint64_t tobj = 0;
  uint32_t tkasz = 0, tgrp = 0, tprv = 0;
  kernel("aql_tail_kernel.kd", &tobj, &tkasz, &tgrp, &tprv);
  void* targs = nullptr;
  HK(hsa_memory_allocate(f.kernarg, 256, &targs));
  std::memset(targs, 0, 256);
  std::memcpy((uint8_t*)targs, &dev_word, 8);
  hsa_signal_t sig, sig_gpu;
  HK(hsa_signal_create(1, 0, nullptr, &sig));
  HK(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &sig_gpu));
  hsa_signal_t none{};
  none.handle = 0;
  auto dispatch = [&](uint64_t obj, uint32_t grid, uint32_t blk, void* ka, uint32_t g, uint32_t pr,
                      hsa_signal_t cs, int acq, int rel) {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {}
    hsa_kernel_dispatch_packet_t* p = (hsa_kernel_dispatch_packet_t*)q->base_address + (idx & (q->size - 1));
    p->workgroup_size_x = (uint16_t)blk;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = grid * blk;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = pr;
    p->group_segment_size = g;
    p->kernel_object = obj;
    p->kernarg_address = ka;
    p->reserved2 = 0;
    p->completion_signal = cs;
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                       (1u << HSA_PACKET_HEADER_BARRIER) |
                                       (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = 1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n((uint32_t*)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
  };
  const char* names[] = {"aql_signal_sys", "aql_signal_agent", "aql_gpuonly_signal_agent", "aql_tail_agent",
                         "aql_tail_sys"};
  std::printf("{");
  uint32_t nonce = 0;
  for (int m = 0; m < 5; ++m) {
    std::vector<double> tot, iss;
    for (int i = 0; i < frames + 20; ++i) {
      ++nonce;
      const double t0 = now_us();
      const int rel = (m == 0 || m == 4) ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT;
      if (m <= 2) {
        hsa_signal_t cs = m == 2 ? sig_gpu : sig;
        hsa_signal_store_relaxed(cs, 1);
        dispatch(kobj, nblocks, block, kargs, grp, prv, cs, HSA_FENCE_SCOPE_SYSTEM, rel);
      } else {
        std::memcpy((uint8_t*)targs + 8, &nonce, 4);
        dispatch(kobj, nblocks, block, kargs, grp, prv, none, HSA_FENCE_SCOPE_SYSTEM, rel);
        dispatch(tobj, 1, 64, targs, tgrp, tprv, none, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT);
      }
      const double t1 = now_us();
      if (m <= 2) {
        hsa_signal_t cs = m == 2 ? sig_gpu : sig;
        while (hsa_signal_load_scacquire(cs) != 0) {
          if (now_us() - t1 > 1e6) {
            std::fprintf(stderr, "aql_probe: no completion (%s)\n", names[m]);
            return 3;
          }
        }
      } else {
        while (*hw != nonce) {
          if (now_us() - t1 > 1e6) {
            std::fprintf(stderr, "aql_probe: no tail word (%s)\n", names[m]);
            return 3;
          }
        }
      }
      const double t2 = now_us();
      if (i >= 20) {
        tot.push_back(t2 - t0);
        iss.push_back(t1 - t0);
      }
    }
    // drain (tail modes: the tail packet has no signal; wait for the queue)
    while (hsa_queue_load_read_index_scacquire(q) != hsa_queue_load_write_index_relaxed(q)) {}
    std::printf("%s\"%s\": {\"frame_us\": %.2f, \"issue_us\": %.2f}", m ? ", " : "", names[m], median(tot),
                median(iss));
  }
  std::vector<double> tot, iss;
  // HIP on the same kernel image: hipModuleLaunchKernel + tail kernel
  hipModule_t mod;
  CK(hipModuleLoadData(&mod, co.data()));
  hipFunction_t fk, tk;
  CK(hipModuleGetFunction(&fk, mod, "aql_frame_kernel"));
  CK(hipModuleGetFunction(&tk, mod, "aql_tail_kernel"));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  tot.clear();
  iss.clear();
  for (int i = 0; i < frames + 20; ++i) {
    ++nonce;
    uint32_t tk_ticks = ticks, nb = nblocks, nv = nonce;
    uint32_t* ctr = nullptr;
    uint32_t* dw = dev_word;
    void* a[5] = {&tk_ticks, &ctr, &dw, &nv, &nb};
    const double t0 = now_us();
    CK(hipModuleLaunchKernel(fk, nblocks, 1, 1, block, 1, 1, 0, s, a, nullptr));
    void* b[2] = {&dw, &nv};
    CK(hipModuleLaunchKernel(tk, 1, 1, 1, 64, 1, 1, 0, s, b, nullptr));
    const double t1 = now_us();
    while (*hw != nonce) {
      if (now_us() - t1 > 1e6) {
        std::fprintf(stderr, "aql_probe: no tail word\n");
        return 3;
      }
    }
    const double t2 = now_us();
    if (i >= 20) {
      tot.push_back(t2 - t0);
      iss.push_back(t1 - t0);
    }
  }
  CK(hipStreamSynchronize(s));
  std::printf(", \"hip_tail_kernel\": {\"frame_us\": %.2f, \"issue_us\": %.2f}", median(tot), median(iss));
  // back-to-back device time of the frame kernel (events around 50 launches)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t tk_ticks = ticks, nb = nblocks, nv = 0;
  uint32_t* ctr = nullptr;
  uint32_t* dw = dev_word;
  void* a[5] = {&tk_ticks, &ctr, &dw, &nv, &nb};
  for (int i = 0; i < 10; ++i) CK(hipModuleLaunchKernel(fk, nblocks, 1, 1, block, 1, 1, 0, s, a, nullptr));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < 50; ++i) CK(hipModuleLaunchKernel(fk, nblocks, 1, 1, block, 1, 1, 0, s, a, nullptr));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::printf(", \"frame_kernel_us_back_to_back\": %.2f, \"frames\": %d}\n", ms * 1000.0 / 50, frames);
  hsa_signal_destroy(sig);
  hsa_signal_destroy(sig_gpu);
  hsa_queue_destroy(q);
  hsa_executable_destroy(exe);
  hsa_code_object_reader_destroy(rdr);
  return 0;
}
