// libkgs_pmc_aql.so — device-wide hardware counters straight from the CP, with
// no profiler framework in between.
//
// Same C ABI as pmc_rocprofiler.cpp (kgs_pmc_init/open/sample/info/mode/close),
// so the exporter's dlopen bridge (src/pmc.cpp) loads either.  Why a second
// reader: once rocprofiler-sdk's device-counting context is started, HSA's
// async-events thread re-arms a KFD event wait in a tight loop and burns one
// full CPU core per exporter, whatever the sample rate (measured: profiles/r1/
// pmc_helper_thread.md).  This reader registers no async handler at all:
//
//   * one private AQL queue per GPU (HSA_QUEUE_TYPE_SINGLE, no error callback);
//   * aqlprofile (hsa_ven_amd_aqlprofile.h, the v1 packet builder that ships
//     with ROCm) fills vendor-specific PM4-IB AQL packets: START once (programs
//     and enables the counters), then READ per sample (copies the running
//     counters into a fine-grained host buffer);
//   * READs are pipelined over two slots: each sample collects the READ
//     submitted on the previous tick (its completion signal is normally set
//     already) and submits the next, so the sampler never waits out the CP
//     round trip; a READ that is not done yet is waited for in
//     HSA_WAIT_STATE_BLOCKED;
//   * the READ IB is made lean (no per-XCC CS_PARTIAL_FLUSH, an L2 writeback
//     instead of the full cache invalidate) and its AQL header has no acquire
//     fence, only the system-scope release that orders the completion signal
//     after the results (profiles/launch_overhead.md);
//   * batched publication (--pmc-batch, default 8; read_batched and
//     include/kgs/aql_batch.h): the READs rotate over 2B slots and only the last
//     READ of each half keeps the L2 writeback and the release fence, at most
//     1 ms after the half's first READ; its completion publishes the whole half
//     (packets run in order), so at 8 kHz the L2 is written back 1000 times a
//     second instead of 8000 (profiles/r3/README.md r3i-r3k);
//   * results are folded per counter over every block instance / XCC sample
//     (max for GRBM clocks, sum for SQ busy cycles, mean for TA busy), the same
//     reductions as the rocprofiler path, and reported cumulative since START;
//   * every wait is bounded (fault boundary): a queue slot is
//     reserved only when there is room (include/kgs/aql_ring.h), a completion is
//     waited for at most --pmc-timeout-ms, and kgs_pmc_abort() makes a blocked
//     call return at once (Sampler::stop()).  A wedged command processor costs the
//     caller one timeout per call, never a spin; kgs_pmc_reset() destroys the
//     agent's queue so the next open starts on a fresh one.
//
// Threading: every call on one handle comes from one thread (the device's
// sampler thread); handles of different GPUs share no lock, so a slow or hung
// GPU never delays another's READs.  kgs_pmc_info() may be called from any
// thread: it reads atomics, plus the error string and a snapshot of the session
// layout under a lock that is never held across a wait.
//
// Counter selects for gfx950 (block, event) come from ROCm's own definitions
// (/opt/rocm/share/rocprofiler-sdk/counter_defs.yaml); any other counter can be
// asked for as "BLOCK:event" (e.g. "SQ:4" for SQ_WAVES).
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_aqlprofile.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "kgs/aql_batch.h"
#include "kgs/aql_ib.h"
#include "kgs/aql_ring.h"

namespace {

constexpr int kMaxCounters = 16;

struct Sel {
  const char* name;
  hsa_ven_amd_aqlprofile_block_name_t block;
  const char* block_name;  // aqlprofile block-id query name
  uint32_t event;
};

// gfx950 selects (counter_defs.yaml, architectures: gfx950).
const Sel kGfx950[] = {
    {"GRBM_COUNT", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, "GRBM", 0},
    {"GRBM_GUI_ACTIVE", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, "GRBM", 2},
    {"GRBM_SPI_BUSY", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, "GRBM", 11},
    {"SQ_BUSY_CYCLES", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, "SQ", 3},
    {"SQ_WAVES", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, "SQ", 4},
    {"SQ_VALU_MFMA_BUSY_CYCLES", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, "SQ", 93},
    {"TA_TA_BUSY", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TA, "TA", 13},
    {"TCC_HIT", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC, "TCC", 21},
    {"CPC_ADC_DISPATCH_ALLOC_DONE", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_CPC, "CPC", 4},
    {"CPC_TG_SEND", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_CPC, "CPC", 62},
    {"CPC_CPC_STAT_BUSY", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_CPC, "CPC", 25},
    {"CPF_CPF_STAT_BUSY", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_CPF, "CPF", 23},
    {"TCC_EA0_RDREQ", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC, "TCC", 42},
};

struct BlockNameId {
  const char* name;
  hsa_ven_amd_aqlprofile_block_name_t id;
};
const BlockNameId kBlocks[] = {
    {"GRBM", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM}, {"SQ", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ},
    {"TA", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TA},     {"TD", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TD},
    {"TCC", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC},   {"TCP", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCP},
    {"SPI", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI},   {"CPC", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_CPC},
    {"CPF", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_CPF},   {"GRBMSE", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBMSE},
    // memory-side blocks, probed for a counter-tier HBM bandwidth (tools/aql_probe.py umc_* / mmea / gcea)
    {"UMC", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_UMC},   {"MMEA", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_MMEA},
    {"GCEA", HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GCEA},
};

constexpr int kMaxBatch = kgs::BatchPlan::kMaxBatch;
constexpr int kMaxSlots = 2 * kMaxBatch;  // pipelined READ slots (2 × the largest batch)

struct Agent {
  hsa_agent_t agent{};
  uint32_t gpu_id = 0;  // KFD gpu_id (== HSA_AMD_AGENT_INFO_DRIVER_UID)
  uint32_t cu_count = 0;  // enabled CUs (256 on MI355X)
  hsa_queue_t* queue = nullptr;
  hsa_signal_t sig{};                                // START/STOP and synchronous READs
  hsa_signal_t stall_sig{};                          // kgs_pmc_inject_stall: never signalled (test hook)
  std::vector<std::string> names;
  std::vector<int> reduce;                           // 0 sum, 1 max, 2 mean
  std::vector<char> per_cu;                          // counter's block has one instance per CU
  std::vector<char> per_se;                          // counter read per SE (SQ, TA/TD/TCP): lite READs skip it
  // Lite READs (kgs_pmc_configure("lite")): the batch's non-publishing READs leave
  // the per-SE counters out; their values are the last read ones (se_*).
  bool plite[kMaxSlots] = {};                        // slot k's READ IB is lite
  void* plib[kMaxSlots] = {};                        // ... its compacted IB (kgs/aql_ib.h)
  uint32_t plib_sz[kMaxSlots] = {};
  std::string lite_why;                              // why a slot kept the full IB; guarded by info_mu
  bool se_have = false;                              // se_* hold a full READ's values since the last START
  std::vector<double> se_vals, se_vals_xcd;
  std::vector<uint32_t> se_seen, se_inst;
  bool last_se_fresh = true;                         // the last returned sample read the per-SE counters
  std::atomic<uint64_t> lite_reads{0};
  std::vector<hsa_ven_amd_aqlprofile_event_t> events;
  std::vector<int> ev_counter;                       // event index -> counter index
  hsa_ven_amd_aqlprofile_profile_t prof{};
  void* cmd = nullptr;
  void* out = nullptr;
  hsa_ext_amd_aql_pm4_packet_t start_pkt{}, read_pkt{}, stop_pkt{};
  bool started = false;
  // Pipelined mode: two READ slots, each with its own command/output buffer and
  // completion signal.  A sample() collects the READ submitted on the previous
  // call (normally finished long ago) and submits the next one without waiting,
  // so the sampler thread never blocks on the CP round trip.
  bool pipelined = false;
  hsa_ven_amd_aqlprofile_profile_t pprof[kMaxSlots]{};
  void* pcmd[kMaxSlots] = {};
  void* pout[kMaxSlots] = {};
  hsa_ext_amd_aql_pm4_packet_t pread[kMaxSlots]{};
  hsa_signal_t psig[kMaxSlots]{};
  uint32_t pcmd_sz = 0, pout_sz = 0;                 // allocated sizes of the slot buffers
  std::vector<hsa_ven_amd_aqlprofile_event_t> pipe_events;  // event list the slot packets were built for
  bool pipe_lite = false;                                    // ... and whether their non-publishers are lite
  int64_t psubmit_ns[kMaxSlots] = {};
  // Batched publication (kgs_pmc_configure("batch", B), B >= 2; see read_batched
  // and include/kgs/aql_batch.h): 2B slots in two halves of B; only a half's
  // publisher writes the L2 back.
  int batch = 1;                                     // B of the current slot set (1 = every READ publishes)
  int nslots = 2;
  kgs::BatchPlan plan;
  std::vector<volatile uint32_t*> pdst[kMaxSlots];   // each slot's COPY_DATA destination dwords
  bool bprimed = false;
  struct Ready {
    std::vector<double> vals, vals_xcd;
    std::vector<uint32_t> xcd_seen;
    int64_t ts = 0;
    bool se_fresh = true;
  };
  std::deque<Ready> bready;                          // folded samples not yet returned
  std::atomic<uint64_t> land_waits{0}, land_timeouts{0};  // collections that had to wait / gave up waiting
  std::atomic<uint64_t> publishes{0};                // READs that wrote the L2 back (all, unless batched)
  // KGS_AQL_PROFILE=<n>: CP timestamps of every pipelined READ (queue profiling on):
  // queueing delay (submit → CP start) and execution (start → end), reported on
  // stderr every n READs.  How long the CP makes a READ wait says how busy it
  // is dispatching other queues' work (profiles/launch_overhead.md).
  uint64_t prof_n = 0, prof_bad = 0;
  int64_t prof_q_sum = 0, prof_q_max = 0, prof_x_sum = 0, prof_x_max = 0;
  int inflight = -1;                                 // slot with a READ on the queue, -1 none
  // Written by the handle's thread only, read by kgs_pmc_info from any thread:
  // relaxed atomics (single writer, load + store, no locked RMW on the hot path).
  std::atomic<int64_t> rtt_ns{0};                    // CP round trip of a synchronous READ (EWMA)
  std::atomic<uint64_t> ready_on_poll{0}, waited_on_poll{0};  // pipelined: READ already done / had to wait
  std::atomic<int64_t> host_ns{0};                   // host time spent inside sample()
  uint32_t cmd_sz = 0, out_sz = 0;
  int lean_changed = 0;                              // packets rewritten by lean_read_ib
  std::string err;                                   // guarded by info_mu (read by kgs_pmc_info from any thread)
  // Session layout for kgs_pmc_info (events, results per counter, XCD placement,
  // batch, lean, pipelined), rebuilt by the handle's thread (snap_info) whenever it
  // changes, guarded by info_mu: info never touches the vectors the hot path swaps
  // and refolds.
  std::string info_layout;
  std::mutex info_mu;                                // never held across a wait
  std::atomic<uint64_t> reads{0}, timeouts{0};
  std::atomic<uint64_t> enqueue_timeouts{0};         // no queue slot within the deadline (CP not consuming)
  std::atomic<uint64_t> aborted{0};                  // waits cut short by kgs_pmc_abort
  std::atomic<uint64_t> resets{0};                   // queues destroyed by kgs_pmc_reset
  std::atomic<int> abort{0};                         // kgs_pmc_abort: blocked / new waits return at once
  std::atomic<int> stall_injected{0};                // kgs_pmc_inject_stall: a never-signalled barrier is on the queue
  uint32_t last_results = 0;
  std::vector<uint32_t> instances;                   // results folded per counter (last read)
  std::vector<double> vals;
  // Per-XCD fold.  Each result's XCD coordinate is resolved once, on the first
  // READ, with hsa_ven_amd_aqlprofile_iterate_event_coord and cached by the
  // result's position in the output buffer (fixed by the event list, the same in
  // every READ slot).  -1 = no XCD coordinate.
  std::vector<int> res_xcd;
  std::vector<std::pair<int, uint32_t>> res_slot;     // result ordinal → (counter, index among its results)
  bool res_xcd_done = false;
  const char* xcd_from = "none";                     // "coord" | "order" | "none"
  uint32_t num_xcc = 1;                              // HSA_AMD_AGENT_INFO_NUM_XCC
  std::vector<double> vals_xcd;                      // [counter * kMaxXcd + xcd]
  std::vector<uint32_t> xcd_seen;                    // per counter: bit x = XCD x contributed
};

constexpr int kMaxXcd = 8;
int g_xcd_coord_id = -1;  // id of the "XCD" event coordinate (hsa_ven_amd_aqlprofile_iterate_event_ids)

hsa_status_t on_coord_id(int id, const char* name) {
  if (name && std::strcmp(name, "XCD") == 0) g_xcd_coord_id = id;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_coord(int, int id, int, int coordinate, const char*, void* ud) {
  if (id == g_xcd_coord_id) *static_cast<int*>(ud) = coordinate;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_coord_print(int pos, int id, int extent, int coordinate, const char* name, void*) {
  std::fprintf(stderr, " %s(%d)=%d/%d@%d", name ? name : "?", id, coordinate, extent, pos);
  return HSA_STATUS_SUCCESS;
}

// Bring-up aid (KGS_AQL_DUMP_RESULTS=<n>): every result of the n-th READ with its
// sample id and every event coordinate aqlprofile reports for it.
int64_t dump_results_at() {
  static const int64_t n = [] {
    const char* e = std::getenv("KGS_AQL_DUMP_RESULTS");
    return e ? std::atoll(e) : -1LL;
  }();
  return n;
}

std::vector<Agent*> g_agents;  // built once by kgs_pmc_init, never resized afterwards
// Upper bound of every wait on the command processor: a queue slot, a READ, a
// START / STOP.  A READ takes ≈10-200 µs; 250 ms is three orders of magnitude of
// slack and still lets a sampler notice a wedged CP within a second.
std::atomic<int64_t> g_timeout_ns{250000000};
hsa_amd_memory_pool_t g_host_pool{};
bool g_have_pool = false;
std::string g_init_err;

void set_err(char* err, int len, const std::string& s) {
  if (err && len > 0) std::snprintf(err, static_cast<size_t>(len), "%s", s.c_str());
}

std::string aql_error() {
  const char* s = nullptr;
  if (hsa_ven_amd_aqlprofile_error_string(&s) == HSA_STATUS_SUCCESS && s) return s;
  return "unknown";
}

bool debug() {
  static const bool on = std::getenv("KGS_AQL_DEBUG") != nullptr;
  return on;
}
#define KGS_DBG(...)                      \
  do {                                    \
    if (debug()) {                        \
      std::fprintf(stderr, "[aql] " __VA_ARGS__); \
      std::fflush(stderr);                \
    }                                     \
  } while (0)

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// Single-writer counters of an Agent (the handle's thread), read by kgs_pmc_info.
inline void bump(std::atomic<uint64_t>& c) { c.store(c.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed); }
inline int64_t half_rtt(const Agent* a) { return a->rtt_ns.load(std::memory_order_relaxed) / 2; }

hsa_status_t find_host_pool(hsa_amd_memory_pool_t pool, void*) {
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) || !(flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED))
    return HSA_STATUS_SUCCESS;
  g_host_pool = pool;
  g_have_pool = true;
  return HSA_STATUS_INFO_BREAK;
}

hsa_status_t on_agent(hsa_agent_t agent, void*) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !g_have_pool) {
    hsa_amd_agent_iterate_memory_pools(agent, find_host_pool, nullptr);
  } else if (t == HSA_DEVICE_TYPE_GPU) {
    Agent* a = new Agent();
    a->agent = agent;
    hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DRIVER_UID), &a->gpu_id);
    hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &a->cu_count);
    if (hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_XCC), &a->num_xcc) !=
            HSA_STATUS_SUCCESS || a->num_xcc == 0)
      a->num_xcc = 1;
    g_agents.push_back(a);
  }
  return HSA_STATUS_SUCCESS;
}

bool resolve(const std::string& name, hsa_ven_amd_aqlprofile_block_name_t& block, std::string& block_name,
             uint32_t& event) {
  for (const Sel& s : kGfx950)
    if (name == s.name) {
      block = s.block;
      block_name = s.block_name;
      event = s.event;
      return true;
    }
  const size_t c = name.find(':');
  if (c == std::string::npos) return false;
  block_name = name.substr(0, c);
  for (const BlockNameId& b : kBlocks)
    if (block_name == b.name) {
      block = b.id;
      event = static_cast<uint32_t>(std::strtoul(name.c_str() + c + 1, nullptr, 10));
      return true;
    }
  return false;
}

void* host_alloc(Agent* a, size_t bytes) {
  void* p = nullptr;
  if (hsa_amd_memory_pool_allocate(g_host_pool, bytes, 0, &p) != HSA_STATUS_SUCCESS) return nullptr;
  if (hsa_amd_agents_allow_access(1, &a->agent, nullptr, p) != HSA_STATUS_SUCCESS) {
    hsa_amd_memory_pool_free(p);
    return nullptr;
  }
  std::memset(p, 0, bytes);
  return p;
}

// AQL header fence scopes of the pipelined READ packets: KGS_AQL_FENCE =
// <scope> or <acquire>,<release> with scopes sys | agent | none; default
// none,sys.  A system-scope acquire makes every XCC's CP invalidate its caches
// before the packet; a READ reads only registers, so it needs none.  The release
// is what orders the completion signal after the COPY_DATA results: without it
// the host reads stale values (run r40: MFMA util 57 % for 91 %).  Dropping the
// acquire cuts the READ's cost to a dispatch-bound stream from ≈7 % to ≈5 % at
// 8 kHz with identical counter values (runs r40/r41, profiles/launch_overhead.md).
// START, STOP and synchronous READs keep system scope both ways.
int parse_scope(const char* s, size_t n) {
  if (n == 3 && std::strncmp(s, "sys", 3) == 0) return static_cast<int>(HSA_FENCE_SCOPE_SYSTEM);
  if (n == 5 && std::strncmp(s, "agent", 5) == 0) return static_cast<int>(HSA_FENCE_SCOPE_AGENT);
  return static_cast<int>(HSA_FENCE_SCOPE_NONE);
}
std::pair<int, int> read_fences() {
  static const std::pair<int, int> v = [] {
    const char* e = std::getenv("KGS_AQL_FENCE");
    if (!e) return std::make_pair(static_cast<int>(HSA_FENCE_SCOPE_NONE), static_cast<int>(HSA_FENCE_SCOPE_SYSTEM));
    const char* c = std::strchr(e, ',');
    if (!c) return std::make_pair(parse_scope(e, std::strlen(e)), parse_scope(e, std::strlen(e)));
    return std::make_pair(parse_scope(e, static_cast<size_t>(c - e)), parse_scope(c + 1, std::strlen(c + 1)));
  }();
  return v;
}
constexpr std::pair<int, int> kSystemFences{HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_SYSTEM};

// Completion signals of the pipelined READ slots (KGS_AQL_SIGNAL = interrupt |
// poll).  The pipelined reader polls the previous READ's signal, so it needs no
// interrupt; a signal whose only consumer is the GPU agent is a plain memory
// word (no KFD event, no interrupt per READ).
bool poll_signals() {
  static const bool on = [] {
    const char* e = std::getenv("KGS_AQL_SIGNAL");
    return e && std::strcmp(e, "poll") == 0;
  }();
  return on;
}

// (No READ-queue priority switch: low / normal / high changed nothing measurable
// against a dispatch-bound stream, profiles/launch_overhead.md r2af and
// profiles/r4/ r4c.  The cost is the CP's handling of each packet.)

// KGS_AQL_PROFILE=<n>: report READ timestamps every n pipelined READs (0/unset = off).
uint64_t profile_every() {
  static const uint64_t n = [] {
    const char* e = std::getenv("KGS_AQL_PROFILE");
    return e ? std::strtoull(e, nullptr, 10) : 0ull;
  }();
  return n;
}
bool profile_ts() { return profile_every() > 0; }
// HSA system clock → CLOCK_MONOTONIC ns, calibrated once (HSA timestamps are
// ticks at HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY).
struct ClockMap {
  double ns_per_tick = 1.0;
  int64_t off = 0;
  bool ok = false;
};
const ClockMap& hsa_clock() {
  static const ClockMap m = [] {
    ClockMap c;
    uint64_t f = 0, t = 0;
    if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) != HSA_STATUS_SUCCESS || f == 0) return c;
    const int64_t m0 = mono_ns();
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
    const int64_t m1 = mono_ns();
    c.ns_per_tick = 1e9 / static_cast<double>(f);
    c.off = (m0 + m1) / 2 - static_cast<int64_t>(static_cast<double>(t) * c.ns_per_tick);
    c.ok = true;
    return c;
  }();
  return m;
}

// Put one PM4-IB vendor packet on the agent's private queue.  Waits for a free
// slot at most g_timeout_ns (a full queue means the CP stopped consuming it);
// 0 = queued, -1 = no slot (timeout or abort; nothing was reserved).
int enqueue(Agent* a, const hsa_ext_amd_aql_pm4_packet_t& tmpl, hsa_signal_t sig,
            std::pair<int, int> fences = kSystemFences, bool barrier = true) {
  hsa_queue_t* q = a->queue;
  if (!q) return -1;
  uint64_t idx = 0;
  const kgs::SlotResult r = kgs::reserve_slot(
      q->size, mono_ns() + g_timeout_ns.load(std::memory_order_relaxed), &a->abort,
      [q] { return hsa_queue_load_read_index_scacquire(q); }, [q] { return hsa_queue_load_write_index_relaxed(q); },
      [q](uint64_t i) { hsa_queue_store_write_index_relaxed(q, i + 1); }, [] { return mono_ns(); },
      [] { sched_yield(); }, idx);
  if (r != kgs::SlotResult::kOk) {
    (r == kgs::SlotResult::kAborted ? a->aborted : a->enqueue_timeouts).fetch_add(1, std::memory_order_relaxed);
    return -1;
  }
  hsa_signal_store_relaxed(sig, 1);
  auto* slot = reinterpret_cast<hsa_ext_amd_aql_pm4_packet_t*>(q->base_address) + (idx & (q->size - 1));
  std::memcpy(slot->pm4_command, tmpl.pm4_command, sizeof slot->pm4_command);
  slot->completion_signal = sig;
  const uint16_t header = static_cast<uint16_t>(
      (HSA_PACKET_TYPE_VENDOR_SPECIFIC << HSA_PACKET_HEADER_TYPE) | ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
      (fences.first << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
      (fences.second << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  __atomic_store_n(&slot->header, header, __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
  return 0;
}

// Wait for a packet's completion signal, at most g_timeout_ns, in 10 ms slices so
// that kgs_pmc_abort() ends the wait promptly.  BLOCKED: ROCr spins briefly, then
// sleeps on the signal's KFD event.  0 = done, -1 = timeout, -3 = aborted.
int wait_done(Agent* a, hsa_signal_t sig) {
  const int64_t end = mono_ns() + g_timeout_ns.load(std::memory_order_relaxed);
  constexpr uint64_t kSliceNs = 10000000;
  while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, kSliceNs, HSA_WAIT_STATE_BLOCKED) != 0) {
    if (a->abort.load(std::memory_order_relaxed)) {
      a->aborted.fetch_add(1, std::memory_order_relaxed);
      return -3;
    }
    if (mono_ns() > end) {
      a->timeouts.fetch_add(1, std::memory_order_relaxed);
      return -1;
    }
  }
  return 0;
}

// Put one packet on the queue and wait for it (both bounded).
int submit(Agent* a, const hsa_ext_amd_aql_pm4_packet_t& tmpl) {
  if (enqueue(a, tmpl, a->sig) != 0) return -1;
  return wait_done(a, a->sig);
}

struct Fold {
  Agent* a;
  uint32_t n = 0;
};

hsa_status_t on_data(hsa_ven_amd_aqlprofile_info_type_t type, hsa_ven_amd_aqlprofile_info_data_t* d, void* ud) {
  if (type != HSA_VEN_AMD_AQLPROFILE_INFO_PMC_DATA) return HSA_STATUS_SUCCESS;
  Fold* f = static_cast<Fold*>(ud);
  Agent* a = f->a;
  const uint32_t ord = f->n++;
  if (!a->res_xcd_done) {
    int x = -1;
    if (g_xcd_coord_id >= 0)
      hsa_ven_amd_aqlprofile_iterate_event_coord(a->agent, d->pmc_data.event, d->sample_id, on_coord, &x);
    a->res_xcd.push_back(x);
    a->res_slot.emplace_back(-1, 0);
  }
  if (static_cast<int64_t>(a->reads.load(std::memory_order_relaxed)) == dump_results_at()) {
    std::fprintf(stderr, "[aql-res] ord=%u sid=%u block=%d idx=%u ev=%u val=%llu coords:", ord, d->sample_id,
                 static_cast<int>(d->pmc_data.event.block_name), d->pmc_data.event.block_index,
                 d->pmc_data.event.counter_id, static_cast<unsigned long long>(d->pmc_data.result));
    hsa_ven_amd_aqlprofile_iterate_event_coord(a->agent, d->pmc_data.event, d->sample_id, on_coord_print, nullptr);
    std::fprintf(stderr, "\n");
  }
  for (size_t e = 0; e < a->events.size(); ++e) {
    const auto& ev = a->events[e];
    if (ev.block_name != d->pmc_data.event.block_name || ev.block_index != d->pmc_data.event.block_index ||
        ev.counter_id != d->pmc_data.event.counter_id)
      continue;
    const size_t k = static_cast<size_t>(a->ev_counter[e]);
    const double v = static_cast<double>(d->pmc_data.result);
    const bool is_max = a->reduce[k] == 1;
    if (is_max) a->vals[k] = std::max(a->vals[k], v);
    else a->vals[k] += v;
    if (!a->res_xcd_done) a->res_slot.back() = {static_cast<int>(k), a->instances[k]};
    a->instances[k]++;
    const int x = ord < a->res_xcd.size() ? a->res_xcd[ord] : -1;
    if (x >= 0 && x < kMaxXcd) {  // within one XCD the same reduction, except mean → sum
      double& vx = a->vals_xcd[k * kMaxXcd + static_cast<size_t>(x)];
      vx = is_max ? std::max(vx, v) : vx + v;
      a->xcd_seen[k] |= 1u << x;
    }
    break;
  }
  return HSA_STATUS_SUCCESS;
}

// Bring-up aid (KGS_AQL_DUMP=1): decode the PM4 indirect buffer behind a vendor
// packet — type-3 opcode histogram plus the first packets verbatim — so the cost
// of START / READ on the command processor can be reasoned about.
void dump_packet(const char* name, const hsa_ext_amd_aql_pm4_packet_t& pkt) {
  // pm4_command[0] is the vendor format (AMD_AQL_FORMAT_PM4_IB); the 4-dword
  // INDIRECT_BUFFER jump command follows it.
  uint32_t dw[13];
  std::memcpy(dw, pkt.pm4_command + 1, sizeof dw);
  std::fprintf(stderr, "[aql-dump] %s pm4_command:", name);
  for (int i = 0; i < 13; ++i) std::fprintf(stderr, " %08x", dw[i]);
  std::fprintf(stderr, "\n");
  const uint32_t op = (dw[0] >> 8) & 0xFF;
  if (op != 0x3F && op != 0x33) {  // INDIRECT_BUFFER (0x3f) / INDIRECT_BUFFER_CONST (0x33)
    std::fprintf(stderr, "[aql-dump] %s: first packet opcode 0x%02x is not an IB\n", name, op);
    return;
  }
  const uint64_t addr = (static_cast<uint64_t>(dw[1]) | (static_cast<uint64_t>(dw[2] & 0xFFFF) << 32)) & ~3ull;
  const uint32_t ndw = dw[3] & 0xFFFFF;
  const uint32_t* ib = reinterpret_cast<const uint32_t*>(addr);
  std::fprintf(stderr, "[aql-dump] %s IB at %#llx, %u dwords\n", name, static_cast<unsigned long long>(addr), ndw);
  uint32_t hist[256] = {};
  uint32_t i = 0, shown = 0;
  while (i < ndw) {
    const uint32_t h = ib[i];
    const uint32_t type = h >> 30;
    if (type == 2) { ++i; continue; }  // type-2 filler
    if (type != 3) {
      std::fprintf(stderr, "[aql-dump] %s: non type-3 header %08x at dword %u\n", name, h, i);
      break;
    }
    const uint32_t opc = (h >> 8) & 0xFF, cnt = ((h >> 16) & 0x3FFF) + 2;
    ++hist[opc];
    if (shown < 16 || (opc != 0x40 && opc != 0x79 && shown < 200)) {
      std::fprintf(stderr, "[aql-dump] %s +%u op=0x%02x len=%u:", name, i, opc, cnt);
      for (uint32_t k = 1; k < cnt && k < 8; ++k) std::fprintf(stderr, " %08x", ib[i + k]);
      std::fprintf(stderr, "\n");
      ++shown;
    }
    i += cnt;
  }
  std::fprintf(stderr, "[aql-dump] %s opcode histogram:", name);
  for (int k = 0; k < 256; ++k)
    if (hist[k]) std::fprintf(stderr, " 0x%02x:%u", k, hist[k]);
  std::fprintf(stderr, "\n");
}

// Lean READ.  aqlprofile's READ IB (decoded with KGS_AQL_DUMP=1,
// profiles/read_packet.md) brackets the per-XCC register copies with a
// CS_PARTIAL_FLUSH on every XCC and ends with an ACQUIRE_MEM that invalidates
// the shader I$/K$, the vector L1 and the L2 (with writeback).  That is what a
// per-dispatch profiler needs; a device-wide sampler of free-running busy
// counters needs neither the flushes nor the invalidations, and both cost a
// dispatch-bound workload on the same GPU (profiles/launch_overhead.md).
// Modes: 0 = aqlprofile's packets as built; 1 = CS_PARTIAL_FLUSH → NOP;
// 2 (default) = 1 + ACQUIRE_MEM reduced to the L2 writeback that publishes the
// CP's COPY_DATA results; 3 = 1 + no ACQUIRE_MEM.  Cost-attribution modes
// (KGS_AQL_LEAN only; the counter values they return are stale): 4 = 3 + no
// COPY_DATA, 5 = every packet of the IB a NOP.  Returns packets changed.
int lean_read_ib(const hsa_ext_amd_aql_pm4_packet_t& pkt, int mode, std::vector<volatile uint32_t*>* dsts = nullptr,
                 const void* out = nullptr, size_t out_sz = 0) {
  if (mode <= 0) return 0;
  uint32_t dw[4];
  std::memcpy(dw, pkt.pm4_command + 1, sizeof dw);
  if (((dw[0] >> 8) & 0xFF) != 0x3F) return -1;
  const uint64_t addr = (static_cast<uint64_t>(dw[1]) | (static_cast<uint64_t>(dw[2] & 0xFFFF) << 32)) & ~3ull;
  const uint32_t ndw = dw[3] & 0xFFFFF;
  uint32_t* ib = reinterpret_cast<uint32_t*>(addr);
  auto nop = [&](uint32_t at, uint32_t len) { ib[at] = (3u << 30) | ((len - 2) << 16) | (0x10u << 8); };
  int changed = 0;
  for (uint32_t i = 0; i < ndw;) {
    const uint32_t h = ib[i];
    if ((h >> 30) == 2) { ++i; continue; }
    if ((h >> 30) != 3) return -2;
    const uint32_t opc = (h >> 8) & 0xFF, len = ((h >> 16) & 0x3FFF) + 2;
    if (mode >= 5 || (mode == 4 && opc == 0x40)) {  // cost attribution: NOP the packet
      if (opc != 0x10) {
        nop(i, len);
        ++changed;
      }
    } else if (opc == 0x40 && len == 6 && ((ib[i + 1] >> 8) & 0xF) == 5) {  // COPY_DATA → memory: note where
      const uint64_t dst = (static_cast<uint64_t>(ib[i + 4]) | (static_cast<uint64_t>(ib[i + 5]) << 32)) & ~3ull;
      const uint64_t lo = reinterpret_cast<uint64_t>(out);
      if (dsts && out && dst >= lo && dst + 4 <= lo + out_sz) dsts->push_back(reinterpret_cast<volatile uint32_t*>(dst));
    } else if (opc == 0x46 && (ib[i + 1] & 0x3F) == 7) {  // EVENT_WRITE CS_PARTIAL_FLUSH
      nop(i, len);
      ++changed;
    } else if (opc == 0x58 && mode == 2) {         // ACQUIRE_MEM: keep TC_WB_ACTION_ENA only
      ib[i + 1] &= (1u << 18);
      ++changed;
    } else if (opc == 0x58 && mode >= 3) {
      nop(i, len);
      ++changed;
    }
    i += len;
  }
  return changed;
}

int g_lean = 2;  // kgs_pmc_configure("lean", m) before kgs_pmc_open; KGS_AQL_LEAN overrides
int g_lite = 0;  // kgs_pmc_configure("lite", 1): batched non-publishing READs skip the per-SE counters
int g_batch = 1;  // kgs_pmc_configure("batch", B) before kgs_pmc_set_pipelined; KGS_AQL_BATCH overrides
// kgs_pmc_configure("publish_us", t): the longest a batched READ waits for its
// publisher (aql_batch.h); 0 = only a half's B-th READ publishes.
int64_t g_publish_ns = 1000000;

int lean_mode() {
  const char* e = std::getenv("KGS_AQL_LEAN");
  return e ? std::atoi(e) : g_lean;
}

bool lite_on() {
  const char* e = std::getenv("KGS_AQL_LITE");
  return e ? std::atoi(e) != 0 : g_lite != 0;
}

// Batched publication needs READs whose IB does no cache operation (lean ≥ 2 with
// the ACQUIRE_MEM dropped) next to the publishing one; below lean 2 it is off.
int batch_size() {
  const char* e = std::getenv("KGS_AQL_BATCH");
  const int b = e ? std::atoi(e) : g_batch;
  return lean_mode() >= 2 && lean_mode() <= 3 ? std::clamp(b, 1, kMaxBatch) : 1;
}

// Decide each result's XCD after the first fold.  Preferred: aqlprofile's XCD
// event coordinate, when it spreads the results over every XCC.  Fallback: the
// output order, XCC-major — a counter's i-th of m results sits on XCD
// i·num_xcc/m.  On MI355X / ROCm 7.2 the coordinate reads XCD 0 for all 48
// results, and the buffer holds 8 XCC-major groups of [GRBM_COUNT,
// GRBM_GUI_ACTIVE (now GRBM_SPI_BUSY), SQ MFMA busy × 4 SEs]; an MFMA load gated on HW_REG_XCC_ID
// to XCDs {0, 2} shows up on exactly those two under the order placement
// (profiles/r1/xcd/README.md, tests/test_gpu.py::test_per_xcd_counters_follow_xcc_gated_load).
void place_xcds(Agent* a) {
  uint32_t seen = 0;
  for (int x : a->res_xcd)
    if (x >= 0 && x < kMaxXcd) seen |= 1u << x;
  const uint32_t nx = a->num_xcc;
  if (nx > 1 && nx <= static_cast<uint32_t>(kMaxXcd) && static_cast<uint32_t>(__builtin_popcount(seen)) == nx) {
    a->xcd_from = "coord";
    return;
  }
  a->xcd_from = "none";
  if (nx < 2 || nx > static_cast<uint32_t>(kMaxXcd)) {
    a->res_xcd.assign(a->res_xcd.size(), -1);
    return;
  }
  for (size_t k = 0; k < a->instances.size(); ++k)
    if (a->instances[k] % nx != 0) {  // not a whole number of results per XCC: no guess
      a->res_xcd.assign(a->res_xcd.size(), -1);
      return;
    }
  for (size_t o = 0; o < a->res_slot.size() && o < a->res_xcd.size(); ++o) {
    const auto [k, i] = a->res_slot[o];
    a->res_xcd[o] = k < 0 ? -1 : static_cast<int>(i * nx / a->instances[static_cast<size_t>(k)]);
  }
  a->xcd_from = "order";
}

void snap_info(Agent* a);

// Fold one completed READ's output buffer into a->vals.
int fold(Agent* a, hsa_ven_amd_aqlprofile_profile_t* prof, bool lite = false) {
  a->reads.fetch_add(1, std::memory_order_relaxed);
  a->vals.assign(a->names.size(), 0.0);
  a->instances.assign(a->names.size(), 0);
  a->vals_xcd.assign(a->names.size() * kMaxXcd, 0.0);
  a->xcd_seen.assign(a->names.size(), 0);
  if (!a->res_xcd_done) {  // a failed first fold leaves no partial table
    a->res_xcd.clear();
    a->res_slot.clear();
  }
  Fold f{a};
  if (hsa_ven_amd_aqlprofile_iterate_data(prof, on_data, &f) != HSA_STATUS_SUCCESS) return -3;
  const bool first = !a->res_xcd_done;
  if (first) place_xcds(a);  // the first fold's per-XCD values are never returned (open's READ)
  a->res_xcd_done = true;
  a->last_results = f.n;
  if (first) snap_info(a);
  // Mean of a per-CU block (TA/TD/TCP): the packets read every instance slot of
  // every SE (16 per SE on gfx950), but only cu_count of them exist (8 per SE
  // on MI355X); the absent ones read 0.  Average over the CUs that exist.
  for (size_t k = 0; k < a->vals.size(); ++k)
    if (a->reduce[k] == 2 && a->instances[k] > 0)
      a->vals[k] /= (a->per_cu[k] && a->cu_count > 0) ? a->cu_count : a->instances[k];
  // Lite READ: its per-SE dwords were not written; carry the last read values (0
  // before the first full READ after a START: the counts restart there).  A full
  // READ keeps its per-SE values for the lite ones after it.
  const size_t nk = a->vals.size();
  if (a->se_vals.size() != nk) {
    a->se_vals.assign(nk, 0.0);
    a->se_vals_xcd.assign(nk * kMaxXcd, 0.0);
    a->se_seen.assign(nk, 0);
    a->se_inst.assign(nk, 0);
    a->se_have = false;
  }
  for (size_t k = 0; k < nk; ++k) {
    if (k >= a->per_se.size() || !a->per_se[k]) continue;
    double* vx = &a->vals_xcd[k * kMaxXcd];
    double* sx = &a->se_vals_xcd[k * kMaxXcd];
    if (lite) {
      a->vals[k] = a->se_have ? a->se_vals[k] : 0.0;
      std::copy(sx, sx + kMaxXcd, vx);
      a->xcd_seen[k] = a->se_seen[k];
      a->instances[k] = a->se_inst[k];
    } else {
      a->se_vals[k] = a->vals[k];
      std::copy(vx, vx + kMaxXcd, sx);
      a->se_seen[k] = a->xcd_seen[k];
      a->se_inst[k] = a->instances[k];
    }
  }
  if (lite) a->lite_reads.fetch_add(1, std::memory_order_relaxed);
  else a->se_have = true;
  a->last_se_fresh = !lite;
  return 0;
}

int read_values(Agent* a) {
  std::memset(a->out, 0, a->prof.output_buffer.size);
  const int64_t t0 = mono_ns();
  if (submit(a, a->read_pkt) != 0) return -2;
  const int64_t rtt = mono_ns() - t0;
  const int64_t prev = a->rtt_ns.load(std::memory_order_relaxed);
  a->rtt_ns.store(prev ? (7 * prev + rtt) / 8 : rtt, std::memory_order_relaxed);
  return fold(a, &a->prof);
}

// Pipelined sample: collect the READ in flight, submit the next one.  Returns the
// collected values' estimated CP read time in *ts (submit + half a round trip).
int read_pipelined(Agent* a, int64_t* ts) {
  if (a->inflight < 0) {  // first call (or after an error): one synchronous read to prime
    const int64_t t0 = mono_ns();
    const int rc = read_values(a);
    if (rc != 0) return rc;
    if (ts) *ts = t0 + half_rtt(a);
    std::memset(a->pout[0], 0, a->pprof[0].output_buffer.size);
    a->psubmit_ns[0] = mono_ns();
    a->inflight = enqueue(a, a->pread[0], a->psig[0], read_fences()) == 0 ? 0 : -1;
    return 0;
  }
  const int k = a->inflight;
  if (hsa_signal_load_scacquire(a->psig[k]) < 1) {
    bump(a->ready_on_poll);
  } else {
    bump(a->waited_on_poll);
    if (wait_done(a, a->psig[k]) != 0) {
      a->inflight = -1;  // the packet may still complete later; its slot is re-armed before reuse
      return -2;
    }
  }
  if (profile_ts()) {
    hsa_amd_profiling_dispatch_time_t t{};
    const ClockMap& c = hsa_clock();
    if (c.ok && hsa_amd_profiling_get_dispatch_time(a->agent, a->psig[k], &t) == HSA_STATUS_SUCCESS && t.start &&
        t.end >= t.start) {
      const int64_t st = static_cast<int64_t>(static_cast<double>(t.start) * c.ns_per_tick) + c.off;
      const int64_t q = st - a->psubmit_ns[k], x = static_cast<int64_t>(static_cast<double>(t.end - t.start) * c.ns_per_tick);
      ++a->prof_n;
      a->prof_q_sum += q;
      a->prof_x_sum += x;
      a->prof_q_max = std::max(a->prof_q_max, q);
      a->prof_x_max = std::max(a->prof_x_max, x);
    } else {
      ++a->prof_bad;
    }
    if (a->prof_n + a->prof_bad >= profile_every()) {
      const double n = a->prof_n ? static_cast<double>(a->prof_n) : 1.0;
      std::fprintf(stderr,
                   "kgs-aql-prof t=%.3f reads=%llu no_ts=%llu qdelay_us mean=%.2f max=%.1f exec_us mean=%.2f "
                   "max=%.1f\n",
                   mono_ns() * 1e-9, static_cast<unsigned long long>(a->prof_n), static_cast<unsigned long long>(a->prof_bad),
                   a->prof_q_sum / n / 1e3, a->prof_q_max / 1e3, a->prof_x_sum / n / 1e3, a->prof_x_max / 1e3);
      a->prof_n = a->prof_bad = 0;
      a->prof_q_sum = a->prof_q_max = a->prof_x_sum = a->prof_x_max = 0;
    }
  }
  const int rc = fold(a, &a->pprof[k]);
  if (ts) *ts = a->psubmit_ns[k] + half_rtt(a);
  const int n = k ^ 1;
  std::memset(a->pout[n], 0, a->pprof[n].output_buffer.size);
  a->psubmit_ns[n] = mono_ns();
  // No slot for the next READ: these values stand, the next call primes again
  // (and fails there if the CP is still not consuming).
  a->inflight = enqueue(a, a->pread[n], a->psig[n], read_fences()) == 0 ? n : -1;
  return rc;
}

// ---- batched publication ----------------------------------------------------
// Every READ writes its results into fine-grained host memory that the GPU's L2
// caches, so a READ must end with an L2 writeback before the host can see them,
// and that writeback is about half of what a READ costs a training step
// (profiles/r3/README.md, r3e / r3g).  With a batch of B the READs go round 2B
// slots in two halves (include/kgs/aql_batch.h); only a half's publisher keeps
// the writeback and the system-scope release fence.  Packets on the queue run in
// order (barrier bit), so when the publisher completes, its writeback has pushed
// every earlier READ of the half out of the L2 as well; the host then folds the
// half's READs in order, each with its own CP time.  At 8 kHz a sample comes out
// B to 2B ticks late and the L2 is written back once per B samples; a READ never
// waits more than the publish interval (1 ms) for its publisher, so at low rates
// every READ publishes.  Every result dword is pre-set to kUnlanded and checked
// before the fold (wait_landed): a dword the writeback missed is waited for,
// briefly; if it still reads kUnlanded the READ is dropped and counted.  The
// counters are cumulative, so the next sample's interval covers a dropped one and
// nothing is lost but resolution (a dword that really holds 0xFFFFFFFF, about one
// READ in 5·10^7, is dropped the same way).
constexpr uint32_t kUnlanded = 0xFFFFFFFFu;

bool is_publisher(const Agent* a, int k) { return a->batch < 2 || a->plan.is_publisher(k); }

// Every READ keeps the AQL barrier bit: dropping it on a batch's non-publisher
// READs (the round-3 KGS_AQL_NOBARRIER experiment) cost a µs-kernel stream the same
// 3.8 % at 8 kHz (profiles/r4/ r4c), and the publisher's writeback must follow
// every READ of its half anyway.

// Rebuild the session-layout part of kgs_pmc_info (handle's thread only; called
// when the layout changes: open, mode switch, the first fold of an event list).
void snap_info(Agent* a) {
  // XCDs the result layout places results on (place_xcds), not the XCDs one fold
  // happened to see: the first fold runs before the placement exists.
  uint32_t placed = 0;
  for (int x : a->res_xcd)
    if (x >= 0 && x < kMaxXcd) placed |= 1u << x;
  std::string o = ";events=" + std::to_string(a->events.size()) + ";results=" + std::to_string(a->last_results) +
                  ";pipelined=" + std::to_string(a->pipelined ? 1 : 0) + ";lean=" + std::to_string(lean_mode()) + ":" +
                  std::to_string(a->lean_changed) + ";batch=" + std::to_string(a->batch) +
                  ";xcd=" + std::to_string(__builtin_popcount(placed)) + ":" + a->xcd_from;
  for (size_t k = 0; k < a->names.size(); ++k)
    o += ";" + a->names[k] + "=" + std::to_string(k < a->instances.size() ? a->instances[k] : 0);
  std::lock_guard<std::mutex> g(a->info_mu);
  a->info_layout.swap(o);
}

// true = every result dword of slot k was written (fold it), false = drop the READ.
bool wait_landed(Agent* a, int k) {
  const int64_t t0 = mono_ns();
  bool waited = false;
  for (;;) {
    bool all = true;
    for (volatile uint32_t* p : a->pdst[k])
      if (*p == kUnlanded) {
        all = false;
        break;
      }
    if (all) break;
    if (!waited) {
      waited = true;
      a->land_waits.fetch_add(1, std::memory_order_relaxed);
    }
    if (mono_ns() - t0 > 200000) {
      a->land_timeouts.fetch_add(1, std::memory_order_relaxed);
      return false;
    }
    sched_yield();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return true;
}

void batch_reset(Agent* a) {
  a->plan.reset();
  a->bprimed = false;
  a->bready.clear();
}

// Wait (bounded) for the last READ submitted, then forget the batch state.
void batch_drain(Agent* a) {
  if (a->batch >= 2 && a->plan.last() >= 0) wait_done(a, a->psig[a->plan.last()]);
  batch_reset(a);
}

// Fold half h (its publisher has completed) into the ready queue.
void batch_collect(Agent* a, int h) {
  int ks[kMaxSlots];
  const int n = a->plan.slots(h, ks);
  for (int j = 0; j < n; ++j) {
    const int k = ks[j];
    if (!wait_landed(a, k) || fold(a, &a->pprof[k], a->plite[k]) != 0) continue;
    Agent::Ready r;
    r.vals = a->vals;
    r.vals_xcd = a->vals_xcd;
    r.xcd_seen = a->xcd_seen;
    r.se_fresh = !a->plite[k];
    r.ts = a->psubmit_ns[k] + half_rtt(a);
    a->bready.push_back(std::move(r));
  }
  a->plan.collected(h);
}

// One batched sample: collect a published half, submit the next READ, return the
// oldest folded sample.  0 = values in a->vals / *ts, 1 = none yet (the first
// half is still in flight), < 0 = error (the batch state is dropped).
int read_batched(Agent* a, int64_t* ts) {
  kgs::BatchPlan& p = a->plan;
  if (!a->bprimed) {  // first call (or after an error / mode switch): one synchronous READ
    batch_reset(a);
    const int64_t t0 = mono_ns();
    const int rc = read_values(a);
    if (rc != 0) return rc;
    ++a->publishes;  // a synchronous READ writes the L2 back
    if (ts) *ts = t0 + half_rtt(a);
    a->bprimed = true;
    return 0;  // the next call starts the slot rotation
  }
  // Fold closed halves oldest first (BatchPlan::collect_order): the half the next
  // READ reuses, if still closed, is older than the other one and is waited for;
  // the other half's publisher went out a tick or more ago and is usually done.
  const int other = p.current_half() ^ 1;
  const bool other_done = p.closed(other) && hsa_signal_load_scacquire(a->psig[p.publisher(other)]) < 1;
  int halves[2];
  bool waits[2];
  const int nh = p.collect_order(other_done, halves, waits);
  for (int i = 0; i < nh; ++i) {
    if (waits[i]) {  // reusing a half not yet collected: wait for its publisher
      bump(a->waited_on_poll);
      if (wait_done(a, a->psig[p.publisher(halves[i])]) != 0) {
        batch_reset(a);  // the packets may still complete later; their slots are re-armed before reuse
        return -2;
      }
    } else {
      bump(a->ready_on_poll);
    }
    batch_collect(a, halves[i]);
  }
  const int k = p.next_slot(mono_ns());
  for (volatile uint32_t* d : a->pdst[k]) *d = kUnlanded;
  std::atomic_thread_fence(std::memory_order_release);
  a->psubmit_ns[k] = mono_ns();
  const std::pair<int, int> none{HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE};
  const bool pub = p.is_publisher(k);
  if (enqueue(a, a->pread[k], a->psig[k], pub ? read_fences() : none) != 0) {
    if (p.last() >= 0) wait_done(a, a->psig[p.last()]);
    batch_reset(a);
    return -2;
  }
  p.submitted(k, a->psubmit_ns[k]);
  if (pub) ++a->publishes;
  if (a->bready.empty()) return 1;
  Agent::Ready& r = a->bready.front();
  a->vals.swap(r.vals);
  a->vals_xcd.swap(r.vals_xcd);
  a->xcd_seen.swap(r.xcd_seen);
  a->last_se_fresh = r.se_fresh;
  if (ts) *ts = r.ts;
  a->bready.pop_front();
  return 0;
}

bool same_events(const std::vector<hsa_ven_amd_aqlprofile_event_t>& x,
                 const std::vector<hsa_ven_amd_aqlprofile_event_t>& y) {
  if (x.size() != y.size()) return false;
  for (size_t i = 0; i < x.size(); ++i)
    if (x[i].block_name != y[i].block_name || x[i].block_index != y[i].block_index || x[i].counter_id != y[i].counter_id)
      return false;
  return true;
}

// Lite READ for slot k (--pmc-lite): point its READ packet at a compacted copy of
// its IB without the per-SE sections (kgs/aql_ib.h), and drop those results from
// the slot's landing check.  false (the slot keeps the full IB) if the IB does not
// compact cleanly; the reason goes to kgs_pmc_info.
bool make_lite(Agent* a, int k, uint32_t cmd_sz) {
  auto why = [a](const std::string& w) {
    std::lock_guard<std::mutex> g(a->info_mu);
    a->lite_why = w;
    return false;
  };
  uint32_t dw[4];
  std::memcpy(dw, a->pread[k].pm4_command + 1, sizeof dw);
  if (((dw[0] >> 8) & 0xFF) != 0x3F) {
    return why("READ packet is not an INDIRECT_BUFFER");
  }
  const uint64_t addr = (static_cast<uint64_t>(dw[1]) | (static_cast<uint64_t>(dw[2] & 0xFFFF) << 32)) & ~3ull;
  const uint32_t ndw = dw[3] & 0xFFFFF;
  std::vector<uint32_t> out;
  const kgs::IbCompact c = kgs::compact_se_sections(reinterpret_cast<const uint32_t*>(addr), ndw, out);
  if (!c.ok) {
    return why(c.why);
  }
  // fold() carries the last values over a lite READ only for the per_se counters
  // (SQ / TA / TD / TCP): every dropped result must be one of theirs.  A
  // session counter of another SE-indexed block (SPI, GRBMSE, ...) would have its
  // per-SE copies dropped too and then be read from dwords the lite IB never writes.
  // The output buffer holds the results in fold order, each `m` copies of one size
  // (gfx950: two 32-bit copies, LO and HI); the open READ's fold recorded each result
  // ordinal's counter (res_slot), so every dropped destination maps to its counter.
  const size_t n_res = a->res_slot.size(), copies = c.kept_copies + c.dropped_copies;
  if (!a->res_xcd_done || n_res == 0 || copies % n_res != 0 || c.copy_bytes == 0) {
    return why("cannot map " + std::to_string(copies) + " result copies onto " + std::to_string(n_res) + " results");
  }
  const uint64_t base = reinterpret_cast<uint64_t>(a->pout[k]), stride = c.copy_bytes * (copies / n_res);
  for (uint64_t dst : c.dropped_dsts) {
    const uint64_t ord = dst >= base ? (dst - base) / stride : n_res;
    const int ck = ord < n_res ? a->res_slot[ord].first : -1;
    if (ck < 0 || static_cast<size_t>(ck) >= a->per_se.size() || !a->per_se[static_cast<size_t>(ck)]) {
      return why("a dropped result (ordinal " + std::to_string(ord) + ") is not a per-SE counter's" +
                 (ck >= 0 && static_cast<size_t>(ck) < a->names.size() ? ": " + a->names[static_cast<size_t>(ck)] : ""));
    }
  }
  // the compacted IB only (≈1.5 KB for the base set), not a whole command buffer
  const uint32_t need = static_cast<uint32_t>((out.size() * 4 + 4095) & ~size_t{4095});
  if (a->plib[k] && a->plib_sz[k] < need) {
    hsa_amd_memory_pool_free(a->plib[k]);
    a->plib[k] = nullptr;
  }
  if (!a->plib[k]) {
    a->plib[k] = host_alloc(a, need);
    a->plib_sz[k] = a->plib[k] ? need : 0;
  }
  if (!a->plib[k] || out.size() * 4 > cmd_sz) {
    return why("no memory for the compacted IB");
  }
  std::memcpy(a->plib[k], out.data(), out.size() * 4);
  const uint64_t na = reinterpret_cast<uint64_t>(a->plib[k]);
  dw[1] = static_cast<uint32_t>(na) | (dw[1] & 3u);
  dw[2] = (dw[2] & ~0xFFFFu) | static_cast<uint32_t>((na >> 32) & 0xFFFF);
  dw[3] = (dw[3] & ~0xFFFFFu) | static_cast<uint32_t>(out.size());
  std::memcpy(a->pread[k].pm4_command + 1, dw, sizeof dw);
  auto& d = a->pdst[k];
  d.erase(std::remove_if(d.begin(), d.end(),
                         [&](volatile uint32_t* p) {
                           const uint64_t x = reinterpret_cast<uint64_t>(p);
                           return std::find(c.dropped_dsts.begin(), c.dropped_dsts.end(), x) != c.dropped_dsts.end();
                         }),
          d.end());
  return true;
}

// Two READ slots for pipelined mode: the session's events, own buffers and
// signals.  Only their READ packets are ever submitted (START/STOP come from the
// main profile).  Called again when a re-open changed the event list: the slot
// packets of the previous list would otherwise be folded against the new one.
bool setup_pipeline(Agent* a, uint32_t cmd_sz, uint32_t out_sz, std::string& err) {
  {  // a reason left by an earlier build of the slots no longer applies
    std::lock_guard<std::mutex> g(a->info_mu);
    a->lite_why.clear();
  }
  a->batch = batch_size();
  a->nslots = a->batch >= 2 ? 2 * a->batch : 2;
  if (a->batch >= 2) a->plan.configure(a->batch, g_publish_ns);
  batch_reset(a);
  for (int k = 0; k < a->nslots; ++k) {
    hsa_ven_amd_aqlprofile_profile_t& p = a->pprof[k];
    p = a->prof;
    if (a->pcmd[k] && a->pcmd_sz < cmd_sz) { hsa_amd_memory_pool_free(a->pcmd[k]); a->pcmd[k] = nullptr; }
    if (a->pout[k] && a->pout_sz < out_sz) { hsa_amd_memory_pool_free(a->pout[k]); a->pout[k] = nullptr; }
    if (!a->pcmd[k]) a->pcmd[k] = host_alloc(a, cmd_sz);
    if (!a->pout[k]) a->pout[k] = host_alloc(a, out_sz);
    hsa_status_t sc = HSA_STATUS_SUCCESS;
    if (!a->psig[k].handle)
      sc = poll_signals() ? hsa_amd_signal_create(1, 1, &a->agent, 0, &a->psig[k])
                          : hsa_signal_create(1, 0, nullptr, &a->psig[k]);
    if (!a->pcmd[k] || !a->pout[k] || sc != HSA_STATUS_SUCCESS) {
      err = "pipeline buffer allocation failed";
      return false;
    }
    p.command_buffer = {a->pcmd[k], cmd_sz};
    p.output_buffer = {a->pout[k], out_sz};
    hsa_ext_amd_aql_pm4_packet_t s{}, t{};
    if (hsa_ven_amd_aqlprofile_start(&p, &s) != HSA_STATUS_SUCCESS ||
        hsa_ven_amd_aqlprofile_read(&p, &a->pread[k]) != HSA_STATUS_SUCCESS ||
        hsa_ven_amd_aqlprofile_stop(&p, &t) != HSA_STATUS_SUCCESS) {
      err = "aqlprofile pipeline packet build: " + aql_error();
      return false;
    }
    // Batched: only the half's last READ writes the L2 back (lean 2); the others
    // drop the ACQUIRE_MEM (lean 3).  Every slot notes its result dwords.
    a->pdst[k].clear();
    const int mode = a->batch >= 2 && !is_publisher(a, k) ? 3 : lean_mode();
    if (mode > 0) lean_read_ib(a->pread[k], mode, &a->pdst[k], a->pout[k], out_sz);
    a->plite[k] = lite_on() && a->batch >= 2 && !is_publisher(a, k) && mode > 0 && make_lite(a, k, cmd_sz);
  }
  a->pcmd_sz = std::max(a->pcmd_sz, cmd_sz);
  a->pout_sz = std::max(a->pout_sz, out_sz);
  a->pipe_events = a->events;
  a->pipe_lite = lite_on();
  return true;
}

}  // namespace

extern "C" {

int kgs_pmc_sample_ts(int handle, uint64_t* out, int n, uint32_t* read_ns, int64_t* sample_ns);

// Reader options, applied to counter sessions opened afterwards.  Keys: "lean"
// (READ packet mode 0-3, see lean_read_ib), "batch" (1..16: READs per L2
// writeback, see read_batched), "publish_us" (0..10^6: the longest a batched READ
// waits for its publisher, default 1000; 0 = only the B-th READ publishes).
// "timeout_ms" (1..60000): bound of every wait on the CP (default 250).
// "lite" (0/1): a batch's non-publishing READs skip the per-SE counters.
// 0 = ok, -1 = unknown key / value.
int kgs_pmc_configure(const char* key, int value) {
  if (key && std::strcmp(key, "lean") == 0 && value >= 0 && value <= 3) {
    g_lean = value;
    return 0;
  }
  if (key && std::strcmp(key, "batch") == 0 && value >= 1 && value <= kMaxBatch) {
    g_batch = value;
    return 0;
  }
  if (key && std::strcmp(key, "publish_us") == 0 && value >= 0 && value <= 1000000) {
    g_publish_ns = static_cast<int64_t>(value) * 1000;
    return 0;
  }
  if (key && std::strcmp(key, "lite") == 0 && (value == 0 || value == 1)) {
    g_lite = value;
    return 0;
  }
  if (key && std::strcmp(key, "timeout_ms") == 0 && value >= 1 && value <= 60000) {
    g_timeout_ns.store(static_cast<int64_t>(value) * 1000000LL);
    return 0;
  }
  return -1;
}

int kgs_pmc_init(char* err, int errlen) {
  static std::once_flag once;
  static int rc = 0;
  std::call_once(once, [&] {
    if (hsa_init() != HSA_STATUS_SUCCESS) {
      g_init_err = "hsa_init failed";
      rc = -2;
      return;
    }
    hsa_iterate_agents(on_agent, nullptr);
    hsa_ven_amd_aqlprofile_iterate_event_ids(on_coord_id);  // finds the "XCD" coordinate for the per-XCD fold
    if (!g_have_pool) {
      g_init_err = "no fine-grained host memory pool";
      rc = -3;
      return;
    }
    if (g_agents.empty()) {
      g_init_err = "no GPU agents";
      rc = -4;
    }
  });
  if (rc != 0) set_err(err, errlen, g_init_err);
  return rc;
}

int kgs_pmc_open(uint64_t kfd_gpu_id, const char* const* names, const int* is_max, int n, char* err, int errlen) {
  if (n <= 0 || n > kMaxCounters) {
    set_err(err, errlen, "bad counter count");
    return -1;
  }
  for (size_t h = 0; h < g_agents.size(); ++h) {
    Agent* a = g_agents[h];
    if (a->gpu_id != kfd_gpu_id) continue;
    if (a->started) {
      set_err(err, errlen, "agent already open");
      return -1;
    }
    a->names.assign(names, names + n);
    a->reduce.assign(is_max, is_max + n);
    const std::vector<hsa_ven_amd_aqlprofile_event_t> prev_events = a->events;
    a->events.clear();
    a->ev_counter.clear();
    a->per_cu.assign(static_cast<size_t>(n), 0);
    a->per_se.assign(static_cast<size_t>(n), 0);
    a->se_have = false;  // a (re)START restarts every count
    a->se_vals.clear();
    std::string missing;
    for (int k = 0; k < n; ++k) {
      hsa_ven_amd_aqlprofile_block_name_t block;
      std::string bname;
      uint32_t event;
      if (!resolve(a->names[static_cast<size_t>(k)], block, bname, event)) {
        missing += (missing.empty() ? "" : ",") + a->names[static_cast<size_t>(k)];
        continue;
      }
      a->per_cu[static_cast<size_t>(k)] = bname == "TA" || bname == "TD" || bname == "TCP";
      a->per_se[static_cast<size_t>(k)] = bname == "SQ" || a->per_cu[static_cast<size_t>(k)];
      // one event per block instance (TA per CU, SQ per SE, GRBM per XCC ...)
      hsa_ven_amd_aqlprofile_profile_t q{};
      q.agent = a->agent;
      hsa_ven_amd_aqlprofile_id_query_t id{bname.c_str(), 0, 0};
      uint32_t inst = 1;
      const hsa_status_t qs = hsa_ven_amd_aqlprofile_get_info(&q, HSA_VEN_AMD_AQLPROFILE_INFO_BLOCK_ID, &id);
      if (qs == HSA_STATUS_SUCCESS && id.instance_count > 0) inst = id.instance_count;
      KGS_DBG("%s: block %s id=%u instances=%u (query status %d)\n", a->names[static_cast<size_t>(k)].c_str(),
              bname.c_str(), id.id, id.instance_count, static_cast<int>(qs));
      uint32_t valid = 0;
      for (uint32_t i = 0; i < inst; ++i) {
        hsa_ven_amd_aqlprofile_event_t ev{block, i, event};
        bool ok = false;
        if (hsa_ven_amd_aqlprofile_validate_event(a->agent, &ev, &ok) != HSA_STATUS_SUCCESS || !ok) continue;
        a->events.push_back(ev);
        a->ev_counter.push_back(k);
        ++valid;
      }
      KGS_DBG("%s: %u/%u instances valid\n", a->names[static_cast<size_t>(k)].c_str(), valid, inst);
    }
    if (a->events.empty()) {
      set_err(err, errlen, "no valid counter events (unresolved: " + missing + ")");
      return -1;
    }
    if (!a->queue) {
      // The READ queue carries PM4 packets only: no kernel ever needs scratch or LDS
      // on it.  KGS_AQL_QUEUE_SEGMENTS=max restores ROCr's defaults (measurement).
      const bool max_seg = std::getenv("KGS_AQL_QUEUE_SEGMENTS") && std::strcmp(std::getenv("KGS_AQL_QUEUE_SEGMENTS"), "max") == 0;
      const uint32_t seg = max_seg ? UINT32_MAX : 0;
      if (hsa_queue_create(a->agent, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, seg, seg, &a->queue) !=
          HSA_STATUS_SUCCESS) {
        set_err(err, errlen, "hsa_queue_create failed");
        return -1;
      }
      if (profile_ts()) hsa_amd_profiling_set_profiler_enabled(a->queue, 1);
    }
    if (!a->sig.handle && hsa_signal_create(1, 0, nullptr, &a->sig) != HSA_STATUS_SUCCESS) {  // kept across resets
      set_err(err, errlen, "hsa_signal_create failed");
      return -1;
    }
    // A re-open rebuilt a->events: the pipelined READ slots of the previous session
    // must point at the new array (same list: a hand-over / refresh re-START), or
    // be rebuilt by the next kgs_pmc_set_pipelined (another list).
    for (int k = 0; k < kMaxSlots; ++k)
      if (a->pcmd[k]) {
        a->pprof[k].events = a->events.data();
        a->pprof[k].event_count = static_cast<uint32_t>(a->events.size());
      }
    if (a->pcmd[0] && !same_events(a->pipe_events, a->events)) a->pipelined = false;
    if (!same_events(prev_events, a->events)) a->res_xcd_done = false;  // result layout changed: place XCDs again
    hsa_ven_amd_aqlprofile_profile_t& p = a->prof;
    p = hsa_ven_amd_aqlprofile_profile_t{};
    p.agent = a->agent;
    p.type = HSA_VEN_AMD_AQLPROFILE_EVENT_TYPE_PMC;
    p.events = a->events.data();
    p.event_count = static_cast<uint32_t>(a->events.size());
    uint32_t cmd_sz = 0, out_sz = 0;
    KGS_DBG("get_info sizes for %zu events\n", a->events.size());
    if (hsa_ven_amd_aqlprofile_get_info(&p, HSA_VEN_AMD_AQLPROFILE_INFO_COMMAND_BUFFER_SIZE, &cmd_sz) !=
            HSA_STATUS_SUCCESS ||
        hsa_ven_amd_aqlprofile_get_info(&p, HSA_VEN_AMD_AQLPROFILE_INFO_PMC_DATA_SIZE, &out_sz) != HSA_STATUS_SUCCESS) {
      set_err(err, errlen, "aqlprofile get_info: " + aql_error());
      return -1;
    }
    // The v1 size query does not grow with the event count on gfx950 (8 KiB
    // for 2 events and for 17: START then overruns it); both buffers are host
    // memory, so size them generously.
    cmd_sz = std::max<uint32_t>(cmd_sz, 256u << 10);
    out_sz = std::max<uint32_t>(out_sz, 64u << 10);
    // Re-open after kgs_pmc_close (the exporter handed the counters to another
    // profiler and takes them back): reuse the buffers when they are big enough.
    if (a->cmd && a->cmd_sz < cmd_sz) { hsa_amd_memory_pool_free(a->cmd); a->cmd = nullptr; }
    if (a->out && a->out_sz < out_sz) { hsa_amd_memory_pool_free(a->out); a->out = nullptr; }
    if (!a->cmd) a->cmd = host_alloc(a, cmd_sz);
    if (!a->out) a->out = host_alloc(a, out_sz);
    if (!a->cmd || !a->out) {
      set_err(err, errlen, "host buffer allocation failed");
      return -1;
    }
    std::memset(a->cmd, 0xAB, cmd_sz);  // dry mode measures how much START/READ/STOP wrote
    p.command_buffer = {a->cmd, cmd_sz};
    p.output_buffer = {a->out, out_sz};
    a->cmd_sz = cmd_sz;
    a->out_sz = out_sz;
    KGS_DBG("cmd=%u out=%u; building START/READ/STOP\n", cmd_sz, out_sz);
    if (hsa_ven_amd_aqlprofile_start(&p, &a->start_pkt) != HSA_STATUS_SUCCESS ||
        hsa_ven_amd_aqlprofile_read(&p, &a->read_pkt) != HSA_STATUS_SUCCESS ||
        hsa_ven_amd_aqlprofile_stop(&p, &a->stop_pkt) != HSA_STATUS_SUCCESS) {
      set_err(err, errlen, "aqlprofile packet build: " + aql_error());
      return -1;
    }
    if (lean_mode() > 0) {
      const int ch = lean_read_ib(a->read_pkt, lean_mode());
      KGS_DBG("lean READ mode %d: %d packets changed\n", lean_mode(), ch);
      a->lean_changed = ch;
    }
    if (std::getenv("KGS_AQL_DUMP")) {
      dump_packet("START", a->start_pkt);
      dump_packet("READ", a->read_pkt);
      dump_packet("STOP", a->stop_pkt);
    }
    if (std::getenv("KGS_AQL_DRY")) {  // packets built, nothing submitted (bring-up)
      const auto* c = static_cast<const uint8_t*>(a->cmd);
      uint32_t used = cmd_sz;
      while (used > 0 && c[used - 1] == 0xAB) --used;
      char b[200];
      std::snprintf(b, sizeof b, "dry: events=%zu cmd=%u cmd_used=%u out=%u", a->events.size(), cmd_sz, used,
                    out_sz);
      set_err(err, errlen, b);
      return -1;
    }
    a->inflight = -1;
    batch_reset(a);
    if (submit(a, a->start_pkt) != 0) {
      set_err(err, errlen, "START packet did not complete within " +
                               std::to_string(g_timeout_ns.load() / 1000000) + " ms");
      return -1;
    }
    a->started = true;
    if (read_values(a) != 0) {
      set_err(err, errlen, "initial READ failed");
      submit(a, a->stop_pkt);
      a->started = false;
      return -1;
    }
    if (!missing.empty()) {
      std::lock_guard<std::mutex> g(a->info_mu);
      a->err = "unresolved: " + missing;
    }
    snap_info(a);
    return static_cast<int>(h);
  }
  set_err(err, errlen, "no HSA GPU agent with kfd gpu_id " + std::to_string(kfd_gpu_id));
  return -1;
}

int kgs_pmc_sample(int handle, uint64_t* out, int n, uint32_t* read_ns) {
  return kgs_pmc_sample_ts(handle, out, n, read_ns, nullptr);
}

// Like kgs_pmc_sample, plus the CLOCK_MONOTONIC time (ns) the values were read
// by the CP.  In pipelined mode the values are those of the READ submitted on
// the previous call, so this time precedes the call; read_ns is the host time
// spent in the call (fold + submit), not the CP round trip.
int kgs_pmc_sample_ts(int handle, uint64_t* out, int n, uint32_t* read_ns, int64_t* sample_ns) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  if (!a->started) return -1;
  const int64_t t0 = mono_ns();
  int64_t ts = 0;
  int rc;
  if (a->pipelined && a->batch >= 2) {
    rc = read_batched(a, &ts);
  } else if (a->pipelined) {
    rc = read_pipelined(a, &ts);
    if (rc == 0) ++a->publishes;  // every unbatched READ writes the L2 back
  } else {
    rc = read_values(a);
    ts = t0 + half_rtt(a);
    if (rc == 0) ++a->publishes;
  }
  const int64_t t1 = mono_ns();
  a->host_ns.store(a->host_ns.load(std::memory_order_relaxed) + (t1 - t0), std::memory_order_relaxed);
  if (read_ns) *read_ns = static_cast<uint32_t>(t1 - t0);
  if (sample_ns) *sample_ns = ts;
  if (rc != 0) return rc;
  for (int k = 0; k < n && static_cast<size_t>(k) < a->vals.size(); ++k) out[k] = static_cast<uint64_t>(a->vals[static_cast<size_t>(k)]);
  return 0;
}

// Per-XCD values of reader counter `counter` from the last completed sample,
// cumulative like kgs_pmc_sample (max over the XCD's instances for max-reduced
// counters, sum otherwise).  Returns the number of XCDs written, 0..n-1 all
// present, or 0 when the results carry no XCD coordinate.  Call from the thread
// that samples the handle, after kgs_pmc_sample[_ts].
// 1 if the last sample returned by kgs_pmc_sample[_ts] read the per-SE counters
// (always, unless lite READs are on and it came from a non-publishing READ), 0 if
// it carries their last read values, -1 for a bad handle.  Same thread as sample.
int kgs_pmc_se_fresh(int handle) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  return g_agents[static_cast<size_t>(handle)]->last_se_fresh ? 1 : 0;
}

int kgs_pmc_sample_xcd(int handle, int counter, uint64_t* out, int max_xcd) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size() || !out) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  if (counter < 0 || static_cast<size_t>(counter) >= a->xcd_seen.size()) return -1;
  const uint32_t seen = a->xcd_seen[static_cast<size_t>(counter)];
  int n = 0;
  while (n < max_xcd && n < kMaxXcd && ((seen >> n) & 1u)) {
    out[n] = static_cast<uint64_t>(a->vals_xcd[static_cast<size_t>(counter) * kMaxXcd + static_cast<size_t>(n)]);
    ++n;
  }
  return (seen >> n) ? 0 : n;  // a gap (or more XCDs than the caller holds): do not guess
}

// Switch a handle between synchronous READs (submit + wait every sample) and
// pipelined READs (collect the previous one, submit the next).  0 = ok.
int kgs_pmc_set_pipelined(int handle, int on, char* err, int errlen) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  if (!a->started) return -1;
  if (a->inflight >= 0) {  // drain before changing mode (bounded; a READ still queued is re-armed before reuse)
    wait_done(a, a->psig[a->inflight]);
    a->inflight = -1;
  }
  batch_drain(a);
  if (on && (!a->pcmd[0] || !same_events(a->pipe_events, a->events) || a->batch != batch_size() ||
             a->pipe_lite != lite_on())) {
    std::string e;
    if (!setup_pipeline(a, a->cmd_sz, a->out_sz, e)) {
      set_err(err, errlen, e);
      return -1;
    }
  }
  a->pipelined = on != 0;
  snap_info(a);
  return 0;
}

// Publication counters for the exporter's self-metrics (any thread: atomics only):
// out[0] READs folded, out[1] READs that wrote the L2 back (every READ unless
// batched), out[2] batched READs dropped because a result was still unwritten
// when their half was folded (should stay near 0).  Returns the number of values
// written.
int kgs_pmc_stats(int handle, uint64_t* out, int n) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size() || !out) return -1;
  const Agent* a = g_agents[static_cast<size_t>(handle)];
  const uint64_t v[3] = {a->reads.load(), a->publishes.load(), a->land_timeouts.load()};
  const int m = std::min(n, 3);
  for (int i = 0; i < m; ++i) out[i] = v[i];
  return m;
}

int kgs_pmc_info(int handle, char* buf, int len) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  const uint64_t reads = a->reads.load();
  std::string o = "impl=aqlprofile;mode=cumulative;cu=" + std::to_string(a->cu_count) +
                  ";timeouts=" + std::to_string(a->timeouts.load()) +
                  ";enqueue_timeouts=" + std::to_string(a->enqueue_timeouts.load()) +
                  ";aborted=" + std::to_string(a->aborted.load()) + ";resets=" + std::to_string(a->resets.load()) +
                  ";stall_injected=" + std::to_string(a->stall_injected.load()) +
                  ";timeout_ms=" + std::to_string(g_timeout_ns.load() / 1000000) +
                  ";rtt_us=" + std::to_string(a->rtt_ns.load(std::memory_order_relaxed) / 1000) +
                  ";reads=" + std::to_string(reads) +
                  ";ready_on_poll=" + std::to_string(a->ready_on_poll.load(std::memory_order_relaxed)) +
                  ";waited_on_poll=" + std::to_string(a->waited_on_poll.load(std::memory_order_relaxed)) +
                  ";host_us_per_read=" +
                  std::to_string(reads ? a->host_ns.load(std::memory_order_relaxed) / 1000.0 / reads : 0.0) +
                  ";land_waits=" + std::to_string(a->land_waits.load()) +
                  ";land_timeouts=" + std::to_string(a->land_timeouts.load()) +
                  ";publishes=" + std::to_string(a->publishes.load()) +
                  ";lite=" + std::to_string(lite_on() ? 1 : 0) + ":" + std::to_string(a->lite_reads.load()) +
                  ";publish_us=" + std::to_string(g_publish_ns / 1000) + ";num_xcc=" + std::to_string(a->num_xcc) +
                  ";fence=" + std::to_string(read_fences().first) + "," + std::to_string(read_fences().second) +
                  ";signal=" + (poll_signals() ? "poll" : "interrupt");
  {
    std::lock_guard<std::mutex> g(a->info_mu);
    o += a->info_layout;
    if (!a->lite_why.empty()) o += ";lite_full_ib=" + a->lite_why;
    if (!a->err.empty()) o += ";" + a->err;
  }
  set_err(buf, len, o);
  return 0;
}

int kgs_pmc_mode(int handle) { return handle >= 0 && static_cast<size_t>(handle) < g_agents.size() ? 1 : -1; }

// STOP the session (bounded: a wedged CP costs at most two timeouts).
void kgs_pmc_close(int handle) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  if (a->started) {
    if (a->inflight >= 0) {
      wait_done(a, a->psig[a->inflight]);
      a->inflight = -1;
    }
    batch_drain(a);
    submit(a, a->stop_pkt);
    a->started = false;
  }
}

// Abort flag of one agent: while set, every wait and queue-slot reservation on it
// returns at once with an error (Sampler::stop() sets it so a sampler thread
// blocked on a wedged CP exits; start() clears it).  Any thread.
int kgs_pmc_abort(int handle, int on) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  g_agents[static_cast<size_t>(handle)]->abort.store(on ? 1 : 0);
  return 0;
}

// Circuit-breaker reset for a wedged command processor: forget the session and
// destroy the agent's READ queue (packets still on it never complete); the next
// kgs_pmc_open creates a fresh queue and re-STARTs.  The buffers, signals and
// pipelined READ slots are kept (signals are re-armed before every use).  Call
// only from the handle's thread, after kgs_pmc_close.
int kgs_pmc_reset(int handle) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  a->started = false;
  a->inflight = -1;
  batch_reset(a);
  if (a->queue) {
    hsa_queue_destroy(a->queue);
    a->queue = nullptr;
  }
  if (a->stall_sig.handle) {  // its barrier packet went with the queue
    hsa_signal_destroy(a->stall_sig);
    a->stall_sig = hsa_signal_t{};
  }
  a->stall_injected.store(0);
  a->resets.fetch_add(1, std::memory_order_relaxed);
  return 0;
}

// Test hook for the counter tier's fault boundary on hardware:
// wedge the agent's READ queue the way a stuck command processor would.  An AQL
// BARRIER_AND packet whose dependency signal is never signalled goes on the queue;
// the packet processor stops there, so every later READ, STOP or START on this
// queue never completes (the workload's own queues are untouched).  Only
// kgs_pmc_reset — hsa_queue_destroy — clears it.  Call from the handle's thread.
// 0 = injected, -1 = no queue / no slot / no signal.
int kgs_pmc_inject_stall(int handle) {
  if (handle < 0 || static_cast<size_t>(handle) >= g_agents.size()) return -1;
  Agent* a = g_agents[static_cast<size_t>(handle)];
  hsa_queue_t* q = a->queue;
  if (!q) return -1;
  if (!a->stall_sig.handle && hsa_signal_create(1, 0, nullptr, &a->stall_sig) != HSA_STATUS_SUCCESS) return -1;
  hsa_signal_store_relaxed(a->stall_sig, 1);
  uint64_t idx = 0;
  const kgs::SlotResult r = kgs::reserve_slot(
      q->size, mono_ns() + g_timeout_ns.load(std::memory_order_relaxed), &a->abort,
      [q] { return hsa_queue_load_read_index_scacquire(q); }, [q] { return hsa_queue_load_write_index_relaxed(q); },
      [q](uint64_t i) { hsa_queue_store_write_index_relaxed(q, i + 1); }, [] { return mono_ns(); },
      [] { sched_yield(); }, idx);
  if (r != kgs::SlotResult::kOk) return -1;
  auto* slot = reinterpret_cast<hsa_barrier_and_packet_t*>(q->base_address) + (idx & (q->size - 1));
  slot->reserved0 = 0;
  slot->reserved1 = 0;
  for (hsa_signal_t& d : slot->dep_signal) d = hsa_signal_t{};
  slot->dep_signal[0] = a->stall_sig;
  slot->reserved2 = 0;
  slot->completion_signal = hsa_signal_t{};
  const uint16_t header = static_cast<uint16_t>((HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                                                (1 << HSA_PACKET_HEADER_BARRIER));
  __atomic_store_n(&slot->header, header, __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
  a->stall_injected.store(1);
  return 0;
}

}  // extern "C"
