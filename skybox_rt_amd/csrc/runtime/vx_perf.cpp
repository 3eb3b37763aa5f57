// vx_perf.cpp -- libvx_perf.so: the reference's vx_dump_perf counter classes
// (VORTEX_PROFILING = VX_DCR_MPM_CLASS_CORE 1 / MEM 2 / TEX 3 / RASTER 4 /
// OM 5; runtime/stub/utils.cpp:159-805) collected IN PROCESS on MI355X.
//
// The reference's classes are simulator counters; here they are the gfx950
// hardware counters (the mapping of scripts/vx_perf.py, which collects the
// same sets out of process with rocprofv3).  The stub (runtime/stub.cpp)
// dlopens this library only when VORTEX_PROFILING is set, before the HIP
// runtime starts: vx_perf_init registers a rocprofiler-sdk tool whose
// dispatch-counting service attaches one counter set to every `vx_main`
// dispatch, rotating through the class's sets (the hardware collects a
// limited number of counters per pass, so a class with several sets needs
// as many launches); vx_dump_perf prints the per-launch averages in the
// reference's "PERF: ..." format.  The product path never loads it.
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kXcds = 8;  // GRBM_GUI_ACTIVE is summed over the 8 XCDs

// counter sets per class; every set fits one pass (<= 8 SQ, 4 TCC, 4 TCP,
// 2 TA, 2 GRBM counters); set 0 of every class: instructions, waves, cycles
const std::vector<std::vector<std::string>>& Sets(int cls) {
  static const std::map<int, std::vector<std::vector<std::string>>> kSets = {
      {1, {{"SQ_INSTS", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
           {"SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_SALU",
            "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS"},
           {"SQ_IFETCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_WR"}}},
      {2, {{"SQ_INSTS", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
           {"SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"},
           {"TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"},
           {"TCC_READ_sum", "TCC_WRITE_sum"},
           {"TCC_MISS_sum", "TCC_HIT_sum"},
           {"TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"}}},
      {3, {{"SQ_INSTS", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
           {"TA_BUFFER_READ_WAVEFRONTS_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum"},
           {"TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"}}},
      {4, {{"SQ_INSTS", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
           {"SQ_INSTS_SMEM"},
           {"SQC_DCACHE_REQ", "SQC_DCACHE_MISSES"}}},
      {5, {{"SQ_INSTS", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
           {"TA_BUFFER_WRITE_WAVEFRONTS_sum", "TA_BUFFER_READ_WAVEFRONTS_sum"},
           {"TCP_TOTAL_WRITE_sum", "TCP_TCC_WRITE_REQ_sum"},
           {"TCP_PENDING_STALL_CYCLES_sum"}}},
  };
  static const std::vector<std::vector<std::string>> kNone;
  auto it = kSets.find(cls);
  return it == kSets.end() ? kNone : it->second;
}

struct State {
  std::mutex mu;
  int cls = 0;
  bool configured = false, started = false;
  rocprofiler_context_id_t ctx{0};
  std::unordered_map<uint64_t, std::string> kernel_names;  // kernel_id -> symbol
  // per agent: one config per counter set (built on first use)
  std::map<std::pair<uint64_t, size_t>, rocprofiler_counter_config_id_t> configs;
  uint64_t dispatches = 0;                    // vx_main dispatches seen
  std::map<std::string, double> sum;          // counter -> sum over collecting dispatches
  std::map<std::string, uint64_t> launches;   // counter -> collecting dispatches
};

State& St() {
  static State s;
  return s;
}

bool IsMain(const std::string& name) {
  // vx_main, vx_main_<image> (VX_ENTRY); not an image's completion kernel <entry>_done
  return name.rfind("vx_main", 0) == 0 && !(name.size() > 5 && name.compare(name.size() - 5, 5, "_done") == 0);
}

void CodeObjectCb(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (rec.kind != ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT ||
      rec.operation != ROCPROFILER_CODE_OBJECT_DEVICE_KERNEL_SYMBOL_REGISTER ||
      rec.phase != ROCPROFILER_CALLBACK_PHASE_LOAD)
    return;
  auto* d = static_cast<rocprofiler_callback_tracing_code_object_kernel_symbol_register_data_t*>(
      rec.payload);
  State& s = St();
  std::lock_guard<std::mutex> lk(s.mu);
  s.kernel_names[d->kernel_id] = d->kernel_name ? d->kernel_name : "";
}

// the counter ids of `names` on `agent` (names the agent lacks are skipped)
std::vector<rocprofiler_counter_id_t> CounterIds(rocprofiler_agent_id_t agent,
                                                 const std::vector<std::string>& names) {
  std::vector<rocprofiler_counter_id_t> all, out;
  rocprofiler_iterate_agent_supported_counters(
      agent,
      [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
        auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud);
        v->insert(v->end(), c, c + n);
        return ROCPROFILER_STATUS_SUCCESS;
      },
      &all);
  for (const std::string& want : names)
    for (rocprofiler_counter_id_t c : all) {
      rocprofiler_counter_info_v0_t info{};
      if (rocprofiler_query_counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_0, &info) ==
              ROCPROFILER_STATUS_SUCCESS &&
          info.name && want == info.name) {
        out.push_back(c);
        break;
      }
    }
  return out;
}

void DispatchCb(rocprofiler_dispatch_counting_service_data_t d, rocprofiler_counter_config_id_t* cfg,
                rocprofiler_user_data_t* ud, void*) {
  ud->value = 0;
  State& s = St();
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.kernel_names.find(d.dispatch_info.kernel_id);
  if (it == s.kernel_names.end() || !IsMain(it->second)) return;  // not ours: no counters
  const auto& sets = Sets(s.cls);
  if (sets.empty()) return;
  const size_t k = (size_t)(s.dispatches++ % sets.size());
  const auto key = std::make_pair(d.dispatch_info.agent_id.handle, k);
  auto c = s.configs.find(key);
  if (c == s.configs.end()) {
    const auto ids = CounterIds(d.dispatch_info.agent_id, sets[k]);
    rocprofiler_counter_config_id_t id{0};
    if (ids.empty() || rocprofiler_create_counter_config(d.dispatch_info.agent_id,
                                                         const_cast<rocprofiler_counter_id_t*>(ids.data()),
                                                         ids.size(), &id) != ROCPROFILER_STATUS_SUCCESS)
      id.handle = 0;
    c = s.configs.emplace(key, id).first;
  }
  if (c->second.handle == 0) return;
  *cfg = c->second;
  ud->value = k + 1;
}

void RecordCb(rocprofiler_dispatch_counting_service_data_t, rocprofiler_counter_record_t* rec,
              size_t n, rocprofiler_user_data_t ud, void*) {
  if (ud.value == 0) return;
  std::map<std::string, double> per;  // this dispatch: counter -> sum over its instances
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_id_t cid{0};
    if (rocprofiler_query_record_counter_id(rec[i].id, &cid) != ROCPROFILER_STATUS_SUCCESS) continue;
    rocprofiler_counter_info_v0_t info{};
    if (rocprofiler_query_counter_info(cid, ROCPROFILER_COUNTER_INFO_VERSION_0, &info) !=
            ROCPROFILER_STATUS_SUCCESS ||
        info.name == nullptr)
      continue;
    per[info.name] += rec[i].counter_value;
  }
  State& s = St();
  std::lock_guard<std::mutex> lk(s.mu);
  for (const auto& kv : per) {
    s.sum[kv.first] += kv.second;
    ++s.launches[kv.first];
  }
}

int ToolInit(rocprofiler_client_finalize_t, void*) {
  State& s = St();
  if (rocprofiler_create_context(&s.ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  if (rocprofiler_configure_callback_tracing_service(s.ctx, ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT,
                                                     nullptr, 0, CodeObjectCb, nullptr) !=
      ROCPROFILER_STATUS_SUCCESS)
    return -1;
  if (rocprofiler_configure_callback_dispatch_counting_service(s.ctx, DispatchCb, nullptr, RecordCb,
                                                                nullptr) !=
      ROCPROFILER_STATUS_SUCCESS)
    return -1;
  if (rocprofiler_start_context(s.ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  s.started = true;
  return 0;
}

void ToolFini(void*) {
  State& s = St();
  if (s.started) rocprofiler_stop_context(s.ctx);
  s.started = false;
}

rocprofiler_tool_configure_result_t* Configure(uint32_t, const char*, uint32_t,
                                               rocprofiler_client_id_t* id) {
  id->name = "vx_perf";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t),
                                                 &ToolInit, &ToolFini, nullptr};
  return &cfg;
}

double Avg(const State& s, const char* name) {
  auto it = s.sum.find(name);
  if (it == s.sum.end()) return 0.0;
  auto n = s.launches.find(name);
  return n == s.launches.end() || n->second == 0 ? 0.0 : it->second / (double)n->second;
}

int Pct(double a, double b) { return b > 0.0 ? (int)(100.0 * a / b) : 0; }

}  // namespace

#define VX_PERF_API extern "C" __attribute__((visibility("default")))

// Register the counter tool for class `cls` (1-5).  Must run before the HIP
// runtime initialises in this process.  0 = registered, -1 = unavailable
// (bad class, or the runtime already started).
VX_PERF_API int vx_perf_init(int cls) {
  State& s = St();
  if (Sets(cls).empty()) return -1;
  if (s.configured) return s.cls == cls ? 0 : -1;
  int inited = 0;
  if (rocprofiler_is_initialized(&inited) == ROCPROFILER_STATUS_SUCCESS && inited) return -1;
  s.cls = cls;
  if (rocprofiler_force_configure(&Configure) != ROCPROFILER_STATUS_SUCCESS) return -1;
  s.configured = true;
  return 0;
}

// vx_main dispatches that carried counters so far (all sets)
VX_PERF_API uint64_t vx_perf_dispatches(void) {
  State& s = St();
  std::lock_guard<std::mutex> lk(s.mu);
  return s.dispatches;
}

// Per-launch averages of the class's counters, as the reference's PERF lines
// (utils.cpp:262-800 wording).  0, or -1 when nothing was collected.
VX_PERF_API int vx_perf_dump(FILE* out, int cls) {
  State& s = St();
  std::lock_guard<std::mutex> lk(s.mu);
  if (!s.configured || s.dispatches == 0 || cls != s.cls) return -1;
  auto g = [&](const char* k) { return (unsigned long long)Avg(s, k); };
  auto v = [&](const char* k) { return Avg(s, k); };
  if (cls == 1) {
    const double wc = v("SQ_WAVE_CYCLES");
    std::fprintf(out, "PERF: scheduler idle=%llu (%d%%)\n", g("SQ_WAIT_ANY"), Pct(v("SQ_WAIT_ANY"), wc));
    std::fprintf(out, "PERF: scheduler stalls=%llu (%d%%)\n", g("SQ_WAIT_INST_ANY"),
                 Pct(v("SQ_WAIT_INST_ANY"), wc));
    const double act = v("SQ_ACTIVE_INST_SALU") + v("SQ_ACTIVE_INST_VALU") + v("SQ_ACTIVE_INST_VMEM") +
                       v("SQ_ACTIVE_INST_LDS");
    std::fprintf(out,
                 "PERF: scoreboard stalls=%llu (%d%%) (alu=%d%%, fpu=%d%%, lsu=%d%%, lmem=%d%%)\n",
                 (unsigned long long)act, Pct(act, wc), Pct(v("SQ_ACTIVE_INST_SALU"), act),
                 Pct(v("SQ_ACTIVE_INST_VALU"), act), Pct(v("SQ_ACTIVE_INST_VMEM"), act),
                 Pct(v("SQ_ACTIVE_INST_LDS"), act));
    std::fprintf(out, "PERF: ifetches=%llu\n", g("SQ_IFETCH"));
    std::fprintf(out, "PERF: loads=%llu\n", g("SQ_INSTS_VMEM_RD") + g("SQ_INSTS_SMEM"));
    std::fprintf(out, "PERF: stores=%llu\n", g("SQ_INSTS_VMEM_WR"));
  } else if (cls == 2) {
    std::fprintf(out, "PERF: lmem reads=%llu\n", g("SQ_INSTS_LDS"));
    std::fprintf(out, "PERF: lmem bank stalls=%llu (utilization=%d%%)\n", g("SQ_LDS_BANK_CONFLICT"),
                 100 - Pct(v("SQ_LDS_BANK_CONFLICT"), v("SQ_ACTIVE_INST_LDS")));
    const double acc = v("TCP_TOTAL_CACHE_ACCESSES_sum"), miss = v("TCP_TCC_READ_REQ_sum");
    std::fprintf(out, "PERF: dcache reads=%llu\n", (unsigned long long)acc);
    std::fprintf(out, "PERF: dcache read misses=%llu (hit ratio=%d%%)\n", (unsigned long long)miss,
                 100 - Pct(miss, acc));
    const double hit = v("TCC_HIT_sum"), mis = v("TCC_MISS_sum");
    std::fprintf(out, "PERF: l2cache reads=%llu\n", g("TCC_READ_sum"));
    std::fprintf(out, "PERF: l2cache writes=%llu\n", g("TCC_WRITE_sum"));
    std::fprintf(out, "PERF: l2cache read misses=%llu (hit ratio=%d%%)\n", (unsigned long long)mis,
                 Pct(hit, hit + mis));
    const unsigned long long r = g("TCC_EA0_RDREQ_sum"), w = g("TCC_EA0_WRREQ_sum");
    std::fprintf(out, "PERF: memory requests=%llu (reads=%llu, writes=%llu)\n", r + w, r, w);
  } else if (cls == 3) {
    std::fprintf(out, "PERF: tex memory reads=%llu\n", g("TA_BUFFER_READ_WAVEFRONTS_sum"));
    std::fprintf(out, "PERF: tex stalls=%llu (%d%%)\n", g("TA_DATA_STALLED_BY_TC_CYCLES_sum"),
                 Pct(v("TA_DATA_STALLED_BY_TC_CYCLES_sum"), v("GRBM_GUI_ACTIVE")));
    const double acc = v("TCP_TOTAL_CACHE_ACCESSES_sum"), miss = v("TCP_TCC_READ_REQ_sum");
    std::fprintf(out, "PERF: tcache reads=%llu\n", (unsigned long long)acc);
    std::fprintf(out, "PERF: tcache read misses=%llu (hit ratio=%d%%)\n", (unsigned long long)miss,
                 100 - Pct(miss, acc));
  } else if (cls == 4) {
    std::fprintf(out, "PERF: raster memory reads=%llu\n", g("SQ_INSTS_SMEM"));
    const double req = v("SQC_DCACHE_REQ"), miss = v("SQC_DCACHE_MISSES");
    std::fprintf(out, "PERF: rcache reads=%llu\n", (unsigned long long)req);
    std::fprintf(out, "PERF: rcache read misses=%llu (hit ratio=%d%%)\n", (unsigned long long)miss,
                 100 - Pct(miss, req));
  } else if (cls == 5) {
    std::fprintf(out, "PERF: om memory reads=%llu\n", g("TA_BUFFER_READ_WAVEFRONTS_sum"));
    std::fprintf(out, "PERF: om memory writes=%llu\n", g("TA_BUFFER_WRITE_WAVEFRONTS_sum"));
    std::fprintf(out, "PERF: om stalls=%llu\n", g("TCP_PENDING_STALL_CYCLES_sum"));
    std::fprintf(out, "PERF: ocache writes=%llu\n", g("TCP_TOTAL_WRITE_sum"));
    std::fprintf(out, "PERF: ocache write requests=%llu\n", g("TCP_TCC_WRITE_REQ_sum"));
  }
  const unsigned long long instrs = g("SQ_INSTS");
  const unsigned long long cycles = g("GRBM_GUI_ACTIVE") / kXcds;
  std::fprintf(out, "PERF: instrs=%llu, cycles=%llu, IPC=%f\n", instrs, cycles,
               cycles ? (double)instrs / (double)cycles : 0.0);
  std::fprintf(out, "PERF: class %d: %llu vx_main launches profiled, %zu counter set(s) rotated\n",
               cls, (unsigned long long)s.dispatches, Sets(cls).size());
  return 0;
}
