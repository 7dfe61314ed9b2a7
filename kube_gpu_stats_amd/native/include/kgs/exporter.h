// The node exporter: backend + counter source + sampler + attribution labels +
// Prometheus renderer + HTTP server (SURVEY.md §3.4 target call stack).
//
// Attribution (GPU → pod/namespace/container from the kubelet pod-resources
// API, PID → pod from cgroups) is computed by the Python control plane at 1 Hz
// and pushed in through set_device_owners()/set_pid_owners(); the scrape path
// only reads immutable snapshots of those tables.
#pragma once

#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "kgs/backend.h"
#include "kgs/pmc.h"
#include "kgs/sampler.h"

namespace kgs {

struct Owner {
  std::string pod, ns, container;
  // The GPU's busy integrals when this owner was first seen on it: the per-pod
  // counters (container_gpu_busy_seconds_total, ...) count from 0 at allocation.
  double base_busy_s = 0, base_mfma_s = 0, base_active_s = 0, base_energy_j = 0, base_cu_s = 0, base_util_s = 0;
  bool same(const Owner& o) const { return pod == o.pod && ns == o.ns && container == o.container; }
};
struct PidOwner {
  std::string pod, ns, container, pod_uid;
};

struct ExporterConfig {
  std::string backend = "amdsmi";   // "amdsmi" | "mock"
  std::string sysfs_root = "/sys";
  MockConfig mock;
  MockPmcConfig mock_pmc;
  SamplerConfig sampler;
  std::vector<std::string> bdfs;    // restrict sampling to these PCI addresses (empty = all)
  std::string pmc_source = "none";  // "none" | "rocprofiler" | "mock"
  std::string pmc_lib;              // path of libkgs_pmc.so
  bool pmc_pipeline = true;         // overlap counter READs with the tick sleep (aqlprofile reader)
  std::string pmc_set = "base";     // "base" (GRBM + MFMA busy) | "full" (+ TA busy: 10x the register reads)
  int pmc_lean = 2;                 // READ packet: 0 as aqlprofile builds it .. 2 no flushes/invalidations (default)
  int pmc_timeout_ms = 250;         // bound of every wait on the command processor (fault boundary)
  int pmc_batch = 8;                // counter READs per L2 writeback (aqlprofile reader; 1 = every READ)
  int pmc_publish_us = 1000;        // longest a batched READ waits for its L2 writeback (kgs/aql_batch.h)
  bool pmc_lite = true;             // a batch's non-publishing READs skip the per-SE counters (MFMA, TA)
  std::string listen_addr = "0.0.0.0";
  int port = 9400;                  // 0 = ephemeral, <0 = no HTTP server
  std::string node_name;
  std::string gpu_type_override;
  // Gauge averaging window.  Default = a typical Prometheus scrape interval, so
  // consecutive scrapes' gauges tile time instead of sampling 1 s of every 15;
  // the exact per-pod accounting uses the *_seconds_total counters anyway.
  double window_s = 15.0;
  // A device whose last good read (PMFW) or counter drain (PMC) is older than
  // this exports no window gauges: frozen values are worse than a gap.
  double stale_s = 5.0;
  // HBM bytes/s at 100 % UMC (memory-controller) activity: the PMFW activity is
  // linear in bandwidth, 11.89 %/(TB/s) on MI355X (profiles/umc_calib.md).
  double hbm_bytes_per_s_at_full_umc = 8.41e12;
  // Bytes per unit of the PMFW PCIe bandwidth accumulator.  amdsmi.h calls it
  // "accumulated bandwidth (GB/sec)"; measured on MI355X (Gen5 x16) it advances
  // by one unit per 102.65 B host→device and 108.74 B device→host, for 256 MiB
  // and 2 GiB copies alike, 108.3 B full-duplex (profiles/r2/pcie/): one factor is
  // good to ±3 %.
  double pcie_bytes_per_acc_unit = 105.7;
  // Bytes per unit of the PMFW per-link xGMI accumulators (xgmi_read/write_data_acc):
  // amdsmi.h documents KB.  Not yet pinned against traffic on hardware (a 1-GPU lease
  // has no peer); bench.py's N > 1 result carries the bytes its all-reduces imply
  // next to the measured rate, and their ratio is the correction.
  double xgmi_bytes_per_acc_unit = 1024.0;
  bool per_process = true;
  bool compat_series = true;        // container_gpu_sm_util (reference contract)
  bool compat_unallocated = false;  // also emit it for GPUs with no pod (pod_name="")
  // What container_gpu_sm_util / container_gpu_busy_seconds_total (and
  // amdgpu_gfx_busy_*) measure: "auto" (default) = the READ-immune integral
  // (Integrals::util_seconds: the counter tier's GRBM_SPI_BUSY while it runs, the
  // PMFW GFX busy otherwise); "pmfw" = the firmware's GFX busy alone (a dispatch in
  // flight; counts the counter tier's own READ packets as work,
  // profiles/r2/idle_busy/); "counters" = GRBM_SPI_BUSY alone (needs --pmc).
  std::string sm_util_source = "auto";
  bool control_http = false;        // serve /control/pause|resume (benchmarks only)
  // gzip level for /metrics when the client sends Accept-Encoding: gzip (0 = never).
  // Off by default: level 1 costs ≈0.6 ms per 8-GPU page (≈117 KB → 11 KB), about
  // eight times the render; worth it only where scrape bandwidth is scarce.
  int gzip_level = 0;
  // HTTP connection hygiene: a keep-alive connection idle this long is closed (a
  // scraper reconnects on its next scrape; 0 = never), and at most this many are
  // held at once — past it the least recently active one is closed, so a client
  // that opens connections and never reads cannot exhaust the exporter's fds.
  double http_idle_s = 300.0;
  int http_max_conns = 256;
  // Families on /metrics: comma-separated globs ('*', '?') over family names.  Empty
  // allow = every family; deny wins.  A histogram's _bucket/_sum/_count lines follow
  // their family.  Trims the per-node series count (≈150 per GPU with every tier on).
  std::string metric_allow;
  std::string metric_deny;
};

// The --metric-allow / --metric-deny decision for one family name.
class FamilyFilter {
 public:
  FamilyFilter() = default;
  FamilyFilter(const std::string& allow, const std::string& deny);
  bool active() const { return !allow_.empty() || !deny_.empty(); }
  bool allowed(const char* name) const;
  bool allowed(const std::string& name) const { return allowed(name.c_str()); }

 private:
  std::vector<std::string> allow_, deny_;
};

class HttpServer;

class Exporter {
 public:
  explicit Exporter(ExporterConfig cfg);
  ~Exporter();

  // Build the backend and counter source; returns false + error() on failure.
  bool init();
  void start();
  void stop();

  const std::string& error() const { return err_; }
  const std::string& pmc_error() const { return pmc_err_; }
  const ExporterConfig& config() const { return cfg_; }
  Backend* backend() const { return be_.get(); }
  Sampler* sampler() const { return sampler_.get(); }
  CounterSource* counters() const { return pmc_.get(); }
  int port() const;

  void set_device_owners(int dev, std::vector<Owner> owners);
  // Keyed by pid_key(gpu, pid): one process can hold several GPUs that belong
  // to different pods (or to none), and each line carries its own GPU's answer.
  void set_pid_owners(std::unordered_map<uint64_t, PidOwner> m);
  static uint64_t pid_key(int gpu, uint32_t pid) { return (static_cast<uint64_t>(static_cast<uint32_t>(gpu)) << 32) | pid; }
  void set_node_name(const std::string& n);
  // Pre-rendered exposition text from the control plane (attribution
  // self-metrics) appended to every /metrics body; swapped atomically.
  void set_extra_metrics(std::string text);

  // Prometheus text exposition of everything (the /metrics body).
  void render(std::string& out);
  std::string topology_json();
  std::string devices_json();
  std::string samples_json(int dev, int n);
  // Full-rate hardware-counter stream of one GPU, oldest first: the last `n`
  // drains, or (since > 0) every drain with seq > since still in the ring, so a
  // client polling with the last seq it saw receives the stream without gaps.
  // Each entry carries the cumulative counts and the rates over the interval
  // since the previous drain.
  std::string counters_json(int dev, int n, uint64_t since);
  bool healthy() const;
  // Stop / restart the sampler threads (HTTP and state stay up; integrals continue).
  void pause_sampling();
  void resume_sampling();
  bool sampling() const;
  // Hand the hardware counters to another profiler (false: the device's sampler
  // STOPs its counting session and skips the PMC tier) or take them back (true);
  // dev < 0 = every device.  Each device's own thread acts, so a hung GPU does
  // not delay the others.
  void set_pmc_enabled(bool on, int dev = -1, bool drop_queue = false);
  bool pmc_enabled() const;
  // Sampler tick rate (benchmarks switch tiers in place; integrals continue).
  // false if hz is outside (0, kMaxHz].
  bool set_sample_rate(double hz);
  double sample_rate() const;

  // self metrics
  std::atomic<uint64_t> scrapes{0};
  std::atomic<uint64_t> render_ns_total{0};
  std::atomic<uint64_t> render_ns_last{0};
  std::atomic<uint64_t> http_requests{0};
  std::atomic<uint64_t> http_conns_open{0};
  std::atomic<uint64_t> http_closed_idle{0};   // closed after http_idle_s without traffic
  std::atomic<uint64_t> http_closed_limit{0};  // evicted to admit a connection past http_max_conns
  std::atomic<size_t> last_render_bytes_{64 * 1024};  // sizes the next render's buffer
  std::atomic<bool> pmc_wanted_{true};

 private:
  void build_static_labels();
  std::shared_ptr<const std::map<int, std::vector<Owner>>> owners() const;
  std::shared_ptr<const std::unordered_map<uint64_t, PidOwner>> pid_owners() const;

  ExporterConfig cfg_;
  std::string err_, pmc_err_;
  std::unique_ptr<Backend> be_;
  std::unique_ptr<CounterSource> pmc_;
  std::unique_ptr<Sampler> sampler_;
  std::unique_ptr<HttpServer> http_;
  FamilyFilter filter_;                   // --metric-allow / --metric-deny
  std::vector<std::string> dev_labels_;   // pre-rendered `gpu="0",uuid=...,...`
  std::vector<TopoEdge> topo_;
  mutable std::mutex mu_;
  std::shared_ptr<const std::map<int, std::vector<Owner>>> owners_;
  std::shared_ptr<const std::unordered_map<uint64_t, PidOwner>> pid_owners_;
  std::string node_name_;
  std::shared_ptr<const std::string> extra_;
  // Render caches (guarded by mu_): the device-info + topology block changes only
  // with the node name; a device's xGMI link-info block only when the slow tier
  // publishes a new link table (compared by pointer; the held shared_ptr keeps
  // the address from being reused).
  std::shared_ptr<const std::string> static_block_;
  std::string static_block_node_;
  std::vector<std::pair<std::shared_ptr<const std::vector<LinkInfo>>, std::shared_ptr<const std::string>>> link_blocks_;
};

// Escape a Prometheus label value.
void append_label_value(std::string& out, const std::string& v);

}  // namespace kgs
