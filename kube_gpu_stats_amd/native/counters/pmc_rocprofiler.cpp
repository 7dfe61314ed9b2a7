// libkgs_pmc.so — agent-wide hardware-counter reader for MI355X (gfx950).
//
// The exporter process registers itself as a rocprofiler-sdk tool
// (rocprofiler_force_configure) *before* HSA comes up, brings HSA up with
// hsa_init(), and opens one device-counting context per GPU agent.  Each
// kgs_pmc_sample() asks the counting service for the current values of the
// programmed counters (SQ/TCC/GRBM perfmon registers read by the command
// processor; no kernel is dispatched and no application queue is touched) and
// reduces the per-XCC / per-SE / per-channel instances to one value per counter.
//
// C ABI (consumed by native/src/pmc.cpp via dlopen):
//   int  kgs_pmc_init(char* err, int errlen);
//   int  kgs_pmc_open(uint64_t kfd_gpu_id, const char* const* names, const int* is_max, int n,
//                     char* err, int errlen);                       -> handle >= 0
//   int  kgs_pmc_sample(int handle, uint64_t* out, int n, uint32_t* read_ns);
//   void kgs_pmc_close(int handle);
//   int  kgs_pmc_mode(int handle);   // 1 = service returns cumulative values, 2 = deltas
#include <hsa/hsa.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int kMaxCounters = 16;
constexpr size_t kMaxRecords = 8192;

struct Agent {
  rocprofiler_agent_id_t id{};
  uint64_t gpu_id = 0;
  rocprofiler_context_id_t ctx{};
  bool configured = false;
  bool started = false;
  std::vector<std::string> names;
  std::vector<int> is_max;
  std::vector<uint64_t> ids;          // rocprofiler counter id handle per name (0 = missing)
  std::vector<rocprofiler_counter_record_t> recs;
  std::vector<double> acc;            // running totals (delta mode)
  int mode = 0;                       // 1 cumulative, 2 delta
  std::string err;
  std::vector<int> instances;         // records seen per counter in the last read
  size_t last_records = 0;
  std::vector<int> rec_map;           // record index -> counter index (-1 = not ours)
  std::vector<rocprofiler_counter_instance_id_t> rec_ids;
};

std::mutex g_mu;
std::vector<Agent*> g_agents;        // every GPU agent seen at tool init
std::atomic<bool> g_tool_init{false};
std::string g_init_err;

void set_err(char* err, int len, const std::string& s) {
  if (err && len > 0) {
    std::snprintf(err, static_cast<size_t>(len), "%s", s.c_str());
  }
}

const char* st_str(rocprofiler_status_t s) { return rocprofiler_get_status_string(s); }

// Called by the counting service when the context starts: program our counters.
void profile_cb(rocprofiler_context_id_t ctx, rocprofiler_agent_id_t agent_id,
                rocprofiler_device_counting_agent_cb_t set_config, void* user_data) {
  Agent* a = static_cast<Agent*>(user_data);
  struct Q {
    Agent* a;
  } q{a};
  a->ids.assign(a->names.size(), 0);
  rocprofiler_iterate_agent_supported_counters(
      agent_id,
      [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* counters, size_t n, void* ud) -> rocprofiler_status_t {
        Agent* ag = static_cast<Q*>(ud)->a;
        for (size_t i = 0; i < n; ++i) {
          rocprofiler_counter_info_v0_t info{};
          if (rocprofiler_query_counter_info(counters[i], ROCPROFILER_COUNTER_INFO_VERSION_0, &info) !=
              ROCPROFILER_STATUS_SUCCESS || !info.name)
            continue;
          for (size_t k = 0; k < ag->names.size(); ++k)
            if (ag->names[k] == info.name) ag->ids[k] = counters[i].handle;
        }
        return ROCPROFILER_STATUS_SUCCESS;
      },
      &q);
  std::vector<rocprofiler_counter_id_t> list;
  for (size_t k = 0; k < a->ids.size(); ++k) {
    if (a->ids[k]) {
      rocprofiler_counter_id_t c;
      c.handle = a->ids[k];
      list.push_back(c);
    }
  }
  if (list.empty()) {
    a->err = "none of the requested counters is supported on this agent";
    return;
  }
  rocprofiler_counter_config_id_t cfg{};
  rocprofiler_status_t s = rocprofiler_create_counter_config(agent_id, list.data(), list.size(), &cfg);
  if (s != ROCPROFILER_STATUS_SUCCESS) {
    a->err = std::string("create_counter_config: ") + st_str(s);
    return;
  }
  s = set_config(ctx, cfg);
  if (s != ROCPROFILER_STATUS_SUCCESS) a->err = std::string("set_config: ") + st_str(s);
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  std::lock_guard<std::mutex> g(g_mu);
  rocprofiler_status_t s = rocprofiler_query_available_agents(
      ROCPROFILER_AGENT_INFO_VERSION_0,
      [](rocprofiler_agent_version_t, const void** agents, size_t n, void*) -> rocprofiler_status_t {
        for (size_t i = 0; i < n; ++i) {
          const auto* ag = static_cast<const rocprofiler_agent_v0_t*>(agents[i]);
          if (ag->type != ROCPROFILER_AGENT_TYPE_GPU) continue;
          Agent* a = new Agent();
          a->id = ag->id;
          a->gpu_id = ag->gpu_id;
          g_agents.push_back(a);
        }
        return ROCPROFILER_STATUS_SUCCESS;
      },
      sizeof(rocprofiler_agent_v0_t), nullptr);
  if (s != ROCPROFILER_STATUS_SUCCESS) {
    g_init_err = std::string("query_available_agents: ") + st_str(s);
    return 0;
  }
  for (Agent* a : g_agents) {
    s = rocprofiler_create_context(&a->ctx);
    if (s != ROCPROFILER_STATUS_SUCCESS) {
      a->err = std::string("create_context: ") + st_str(s);
      continue;
    }
    rocprofiler_buffer_id_t nobuf{};
    nobuf.handle = 0;
    s = rocprofiler_configure_device_counting_service(a->ctx, nobuf, a->id, profile_cb, a);
    if (s != ROCPROFILER_STATUS_SUCCESS) {
      a->err = std::string("configure_device_counting_service: ") + st_str(s);
      continue;
    }
    a->configured = true;
  }
  g_tool_init.store(true);
  return 0;
}

void tool_fini(void*) {}

rocprofiler_tool_configure_result_t* configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "kube_gpu_stats_amd";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// Read all programmed counters and reduce instances -> vals[k].
int read_raw(Agent* a, std::vector<double>& vals) {
  size_t n = a->recs.size();
  rocprofiler_user_data_t ud{};
  rocprofiler_status_t s =
      rocprofiler_sample_device_counting_service(a->ctx, ud, ROCPROFILER_COUNTER_FLAG_NONE, a->recs.data(), &n);
  if (s != ROCPROFILER_STATUS_SUCCESS) return -static_cast<int>(s) - 1;
  vals.assign(a->names.size(), 0.0);
  a->instances.assign(a->names.size(), 0);
  a->last_records = n;
  if (n > a->recs.size()) n = a->recs.size();
  // The service returns the same instances in the same order every read, so
  // the record → counter map is resolved once and then only validated by
  // instance id (saves one SDK lookup per record: ≈600 per read with TA/TD).
  bool cached = a->rec_map.size() == n;
  for (size_t i = 0; cached && i < n; ++i) cached = a->rec_ids[i] == a->recs[i].id;
  if (!cached) {
    a->rec_map.assign(n, -1);
    a->rec_ids.assign(n, 0);
    for (size_t i = 0; i < n; ++i) {
      a->rec_ids[i] = a->recs[i].id;
      rocprofiler_counter_id_t cid{};
      if (rocprofiler_query_record_counter_id(a->recs[i].id, &cid) != ROCPROFILER_STATUS_SUCCESS) continue;
      for (size_t k = 0; k < a->ids.size(); ++k)
        if (a->ids[k] == cid.handle) a->rec_map[i] = static_cast<int>(k);
    }
  }
  for (size_t i = 0; i < n; ++i) {
    const int k = a->rec_map[i];
    if (k < 0) continue;
    const double v = a->recs[i].counter_value;
    if (a->is_max[k] == 1) vals[k] = std::max(vals[k], v);
    else vals[k] += v;  // sum, or sum then mean below
    a->instances[k]++;
  }
  for (size_t k = 0; k < vals.size(); ++k)
    if (a->is_max[k] == 2 && a->instances[k] > 0) vals[k] /= a->instances[k];
  return 0;
}

}  // namespace

extern "C" {

// Tool-library entry point.  Normally the exporter registers itself with
// rocprofiler_force_configure() before HSA starts; when the exporter process
// runs under another rocprofiler tool (e.g. rocprofv3 tracing a benchmark),
// configuration is closed by the time we are dlopen'd, so the parent lists this
// library in ROCP_TOOL_LIBRARIES and sets KGS_PMC_AS_TOOL=1 instead.
rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t version, const char* runtime_version,
                                                           uint32_t priority, rocprofiler_client_id_t* id) {
  const char* as_tool = std::getenv("KGS_PMC_AS_TOOL");
  if (!as_tool || std::strcmp(as_tool, "1") != 0) return nullptr;
  return configure(version, runtime_version, priority, id);
}

int kgs_pmc_init(char* err, int errlen) {
  static std::once_flag once;
  static int rc = 0;
  std::call_once(once, [&] {
    const char* as_tool = std::getenv("KGS_PMC_AS_TOOL");
    const bool tool_mode = as_tool && std::strcmp(as_tool, "1") == 0;
    rocprofiler_status_t s = tool_mode ? ROCPROFILER_STATUS_SUCCESS : rocprofiler_force_configure(&configure);
    if (s != ROCPROFILER_STATUS_SUCCESS) {
      g_init_err = std::string("rocprofiler_force_configure: ") + st_str(s) +
                   " (HSA already initialised in this process? run the exporter in its own process)";
      rc = -1;
      return;
    }
    hsa_status_t hs = hsa_init();
    if (hs != HSA_STATUS_SUCCESS) {
      g_init_err = "hsa_init failed: " + std::to_string(static_cast<int>(hs));
      rc = -2;
      return;
    }
    if (!g_tool_init.load()) {
      g_init_err = "rocprofiler tool initialisation did not run";
      rc = -3;
      return;
    }
    if (!g_init_err.empty()) rc = -4;
  });
  if (rc != 0) set_err(err, errlen, g_init_err);
  return rc;
}

int kgs_pmc_open(uint64_t kfd_gpu_id, const char* const* names, const int* is_max, int n, char* err, int errlen) {
  if (n <= 0 || n > kMaxCounters) {
    set_err(err, errlen, "bad counter count");
    return -1;
  }
  std::lock_guard<std::mutex> g(g_mu);
  for (size_t h = 0; h < g_agents.size(); ++h) {
    Agent* a = g_agents[h];
    if (a->gpu_id != kfd_gpu_id) continue;
    if (!a->configured) {
      set_err(err, errlen, a->err);
      return -1;
    }
    if (a->started) {
      set_err(err, errlen, "agent already open");
      return -1;
    }
    a->names.assign(names, names + n);
    a->is_max.assign(is_max, is_max + n);
    a->recs.resize(kMaxRecords);
    a->acc.assign(static_cast<size_t>(n), 0.0);
    rocprofiler_status_t s = rocprofiler_start_context(a->ctx);
    if (s != ROCPROFILER_STATUS_SUCCESS) {
      set_err(err, errlen, std::string("start_context: ") + st_str(s) + (a->err.empty() ? "" : " / " + a->err));
      return -1;
    }
    if (!a->err.empty()) {
      set_err(err, errlen, a->err);
      rocprofiler_stop_context(a->ctx);
      return -1;
    }
    a->started = true;
    // Learn whether the service reports cumulative values or per-read deltas
    // from the free-running GRBM_COUNT-like first counter.
    std::vector<double> v0, v1, v2;
    if (read_raw(a, v0) != 0 || (std::this_thread::sleep_for(std::chrono::milliseconds(20)), read_raw(a, v1)) != 0 ||
        (std::this_thread::sleep_for(std::chrono::milliseconds(20)), read_raw(a, v2)) != 0) {
      set_err(err, errlen, "initial counter reads failed");
      rocprofiler_stop_context(a->ctx);
      a->started = false;
      return -1;
    }
    const char* force = std::getenv("KGS_PMC_MODE");
    if (force && std::strcmp(force, "cumulative") == 0) a->mode = 1;
    else if (force && std::strcmp(force, "delta") == 0) a->mode = 2;
    else {
      // Measured on MI355X / ROCm 7.2: the device counting service returns values
      // accumulated since the context started (a stopped MFMA load leaves
      // SQ_VALU_MFMA_BUSY_CYCLES constant across reads).  The first reads after
      // start can all be 0, so the warm-up reads only prime the agent.
      a->mode = 1;
    }
    if (a->mode == 2)
      for (size_t k = 0; k < a->acc.size(); ++k) a->acc[k] = v0[k] + v1[k] + v2[k];
    return static_cast<int>(h);
  }
  set_err(err, errlen, "no rocprofiler GPU agent with kfd gpu_id " + std::to_string(kfd_gpu_id));
  return -1;
}

int kgs_pmc_sample(int handle, uint64_t* out, int n, uint32_t* read_ns) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  if (!a->started) return -1;
  std::vector<double> v;
  const int64_t t0 = mono_ns();
  const int rc = read_raw(a, v);
  if (read_ns) *read_ns = static_cast<uint32_t>(mono_ns() - t0);
  if (rc != 0) return rc;
  for (int k = 0; k < n && static_cast<size_t>(k) < v.size(); ++k) {
    if (a->mode == 2) {
      a->acc[static_cast<size_t>(k)] += v[static_cast<size_t>(k)];
      out[k] = static_cast<uint64_t>(a->acc[static_cast<size_t>(k)]);
    } else {
      out[k] = static_cast<uint64_t>(v[static_cast<size_t>(k)]);
    }
  }
  return 0;
}

// "mode=cumulative;records=N;NAME=instances,...;missing=A,B"
int kgs_pmc_info(int handle, char* buf, int len) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  std::string o = std::string("mode=") + (a->mode == 1 ? "cumulative" : a->mode == 2 ? "delta" : "unknown") +
                  ";records=" + std::to_string(a->last_records);
  std::string missing;
  for (size_t k = 0; k < a->names.size(); ++k) {
    if (!a->ids.empty() && a->ids[k] == 0) missing += (missing.empty() ? "" : ",") + a->names[k];
    o += ";" + a->names[k] + "=" + std::to_string(k < a->instances.size() ? a->instances[k] : 0);
  }
  if (!missing.empty()) o += ";missing=" + missing;
  set_err(buf, len, o);
  return 0;
}

int kgs_pmc_mode(int handle) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  return g_agents[static_cast<size_t>(handle)]->mode;
}

void kgs_pmc_close(int handle) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  if (a->started) {
    rocprofiler_stop_context(a->ctx);
    a->started = false;
  }
}

}  // extern "C"
