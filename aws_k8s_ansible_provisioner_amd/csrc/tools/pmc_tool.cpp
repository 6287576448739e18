// In-process GPU hardware-counter sampler for the serving engine: a rocprofiler-sdk tool
// library (loaded at process start through ROCP_TOOL_LIBRARIES=<this .so>) that configures the
// DEVICE counting service on every GPU agent of the process with a fixed counter set and lets
// the engine read device-wide counter values whenever it wants (exporter/pmc_sampler.py, every
// few seconds) -> akap_gpu_pmc_* series on the engine's /metrics -> the OTel collector.
//
// Why device counting (not dispatch counting, what `rocprofv3 --pmc` uses): it samples the
// agent's counters between arbitrary points in time without serialising or instrumenting
// kernel dispatches, so it can stay on in production, including inside hipGraph replays.
//
// The counter set stays inside one pass of the hardware's per-block limits (<= 8 SQ, <= 4 TCC,
// <= 2 GRBM counters; MI355X_MICROARCH / the gpurun notes): GRBM_COUNT + GRBM_GUI_ACTIVE
// (GPU busy), SQ_WAVES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES (matrix-core
// busy), SQ_LDS_BANK_CONFLICT, SQ_INSTS_VALU, TCC_EA0_RDREQ_sum + TCC_EA0_WRREQ_sum (memory-side
// read / write requests: HBM + Infinity-Cache traffic).  Counters an agent does not offer are
// skipped (akap_pmc_name lists what is collected).
//
// C ABI for ctypes: akap_pmc_status, akap_pmc_count, akap_pmc_name, akap_pmc_sample.
#include <rocprofiler-sdk/agent.h>
#include <rocprofiler-sdk/context.h>
#include <rocprofiler-sdk/counter_config.h>
#include <rocprofiler-sdk/counters.h>
#include <rocprofiler-sdk/device_counting_service.h>
#include <rocprofiler-sdk/fwd.h>
#include <rocprofiler-sdk/registration.h>

// from rocprofiler.h, which is not included whole: it pulls in the HIP runtime headers
extern "C" const char* rocprofiler_get_status_string(rocprofiler_status_t status);

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

const char* const kWanted[] = {
    "GRBM_COUNT",          "GRBM_GUI_ACTIVE",          "SQ_WAVES",
    "SQ_BUSY_CYCLES",      "SQ_WAVE_CYCLES",           "SQ_VALU_MFMA_BUSY_CYCLES",
    "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VALU",           "TCC_EA0_RDREQ_sum",
    "TCC_EA0_WRREQ_sum"};

struct AgentState {
  rocprofiler_agent_id_t agent{};
  rocprofiler_context_id_t ctx{};
  rocprofiler_counter_config_id_t config{};
  std::vector<rocprofiler_counter_id_t> ids;
  std::vector<std::string> names;
  int node = -1;
  bool started = false;
};

struct Tool {
  std::mutex mu;
  std::vector<AgentState> agents;
  std::string status = "not initialised (ROCP_TOOL_LIBRARIES not set?)";
  rocprofiler_client_id_t* client = nullptr;
} g;

#define PMC_CHECK(call, what)                                          \
  do {                                                                 \
    rocprofiler_status_t st_ = (call);                                 \
    if (st_ != ROCPROFILER_STATUS_SUCCESS) {                           \
      g.status = std::string(what) + ": " + rocprofiler_get_status_string(st_); \
      return -1;                                                       \
    }                                                                  \
  } while (0)

rocprofiler_status_t collect_agents(rocprofiler_agent_version_t, const void** agents, size_t n,
                                    void* user) {
  auto* out = static_cast<std::vector<AgentState>*>(user);
  for (size_t i = 0; i < n; ++i) {
    const auto* a = static_cast<const rocprofiler_agent_v0_t*>(agents[i]);
    if (a->type != ROCPROFILER_AGENT_TYPE_GPU) continue;
    AgentState s;
    s.agent = a->id;
    s.node = a->logical_node_type_id;
    out->push_back(s);
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

rocprofiler_status_t pick_counters(rocprofiler_agent_id_t, rocprofiler_counter_id_t* counters,
                                   size_t n, void* user) {
  auto* s = static_cast<AgentState*>(user);
  std::map<std::string, rocprofiler_counter_id_t> by_name;
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_info_v0_t info{};
    if (rocprofiler_query_counter_info(counters[i], ROCPROFILER_COUNTER_INFO_VERSION_0,
                                       &info) == ROCPROFILER_STATUS_SUCCESS && info.name)
      by_name[info.name] = counters[i];
  }
  for (const char* w : kWanted) {
    auto it = by_name.find(w);
    if (it == by_name.end()) continue;
    s->ids.push_back(it->second);
    s->names.push_back(w);
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

void set_profile(rocprofiler_context_id_t, rocprofiler_agent_id_t,
                 rocprofiler_device_counting_agent_cb_t set_config, void* user) {
  auto* s = static_cast<AgentState*>(user);
  set_config(s->ctx, s->config);
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  std::lock_guard<std::mutex> lk(g.mu);
  PMC_CHECK(rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0, collect_agents,
                                               sizeof(rocprofiler_agent_v0_t), &g.agents),
            "query agents");
  if (g.agents.empty()) {
    g.status = "no GPU agent";
    return 0;
  }
  for (auto& s : g.agents) {
    PMC_CHECK(rocprofiler_iterate_agent_supported_counters(s.agent, pick_counters, &s),
              "list counters");
    if (s.ids.empty()) continue;
    PMC_CHECK(rocprofiler_create_counter_config(s.agent, s.ids.data(), s.ids.size(), &s.config),
              "counter config");
    PMC_CHECK(rocprofiler_create_context(&s.ctx), "create context");
    PMC_CHECK(rocprofiler_configure_device_counting_service(
                  s.ctx, rocprofiler_buffer_id_t{0}, s.agent, set_profile, &s),
              "device counting service");
  }
  g.status = "configured";
  return 0;
}

void tool_fini(void*) {
  std::lock_guard<std::mutex> lk(g.mu);
  for (auto& s : g.agents)
    if (s.started) rocprofiler_stop_context(s.ctx);
}

// The contexts start lazily on the first sample: the HSA runtime is up by then (the engine
// has launched kernels), which the device counting service needs.
int start_locked() {
  for (auto& s : g.agents) {
    if (s.started || s.ids.empty()) continue;
    PMC_CHECK(rocprofiler_start_context(s.ctx), "start context");
    s.started = true;
  }
  g.status = "ok";
  return 0;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) rocprofiler_tool_configure_result_t* rocprofiler_configure(
    uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "akap-pmc";
  g.client = id;
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t),
                                                 &tool_init, &tool_fini, nullptr};
  return &cfg;
}

__attribute__((visibility("default"))) const char* akap_pmc_status() { return g.status.c_str(); }

// counters collected on GPU agent `agent` (0-based among this process's GPU agents)
__attribute__((visibility("default"))) int akap_pmc_count(int agent) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (agent < 0 || agent >= (int)g.agents.size()) return 0;
  return (int)g.agents[agent].names.size();
}

__attribute__((visibility("default"))) const char* akap_pmc_name(int agent, int i) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (agent < 0 || agent >= (int)g.agents.size()) return "";
  const auto& n = g.agents[agent].names;
  return i >= 0 && i < (int)n.size() ? n[i].c_str() : "";
}

// Read the device counters of GPU agent `agent` now (synchronous): out[i] = value of counter i
// summed over its instances (XCDs, SEs, channels).  Returns the number of values or -1.
__attribute__((visibility("default"))) int akap_pmc_sample(int agent, double* out, int n) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (agent < 0 || agent >= (int)g.agents.size()) return -1;
  if (start_locked() != 0) return -1;
  AgentState& s = g.agents[agent];
  std::vector<rocprofiler_counter_record_t> recs(4096);
  size_t cnt = recs.size();
  rocprofiler_status_t st = rocprofiler_sample_device_counting_service(
      s.ctx, rocprofiler_user_data_t{}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &cnt);
  if (st != ROCPROFILER_STATUS_SUCCESS) {
    g.status = std::string("sample: ") + rocprofiler_get_status_string(st);
    return -1;
  }
  const int m = (int)s.ids.size() < n ? (int)s.ids.size() : n;
  for (int i = 0; i < m; ++i) out[i] = 0.0;
  for (size_t r = 0; r < cnt; ++r) {
    rocprofiler_counter_id_t cid{};
    if (rocprofiler_query_record_counter_id(recs[r].id, &cid) != ROCPROFILER_STATUS_SUCCESS)
      continue;
    for (int i = 0; i < m; ++i)
      if (s.ids[i].handle == cid.handle) out[i] += recs[r].counter_value;
  }
  return m;
}

}  // extern "C"
