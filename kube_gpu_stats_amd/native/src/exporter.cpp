// Exporter lifecycle, attribution tables and JSON endpoints.  See exporter.h.
#include "kgs/exporter.h"

#include <cstring>

#include <unistd.h>

#include <cstdio>
#include <ctime>

#include "kgs/http.h"

namespace kgs {

namespace {
void jstr(std::string& o, const std::string& s) {
  o += '"';
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  o += '"';
}
void jnum(std::string& o, double v) {
  char b[40];
  std::snprintf(b, sizeof b, "%.17g", v);
  o += b;
}
}  // namespace

namespace {

// fnmatch-style: '*' any run, '?' one character.
bool glob_match(const char* p, const char* s) {
  const char* star = nullptr;
  const char* resume = nullptr;
  while (*s) {
    if (*p == '?' || *p == *s) {
      ++p;
      ++s;
    } else if (*p == '*') {
      star = p++;
      resume = s;
    } else if (star) {
      p = star + 1;
      s = ++resume;
    } else {
      return false;
    }
  }
  while (*p == '*') ++p;
  return *p == 0;
}

std::vector<std::string> split_globs(const std::string& csv) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= csv.size()) {
    size_t j = csv.find(',', i);
    if (j == std::string::npos) j = csv.size();
    std::string t = csv.substr(i, j - i);
    while (!t.empty() && t.front() == ' ') t.erase(t.begin());
    while (!t.empty() && t.back() == ' ') t.pop_back();
    if (!t.empty()) out.push_back(t);
    i = j + 1;
  }
  return out;
}

}  // namespace

FamilyFilter::FamilyFilter(const std::string& allow, const std::string& deny)
    : allow_(split_globs(allow)), deny_(split_globs(deny)) {}

bool FamilyFilter::allowed(const char* name) const {
  if (!active()) return true;
  // A histogram's series follow their family: kgs_x_bucket / _sum / _count → kgs_x.
  std::string base(name);
  for (const char* suf : {"_bucket", "_sum", "_count"}) {
    const size_t n = std::strlen(suf);
    if (base.size() > n && base.compare(base.size() - n, n, suf) == 0) {
      base.resize(base.size() - n);
      break;
    }
  }
  bool ok = allow_.empty();
  for (const std::string& g : allow_)
    if (glob_match(g.c_str(), base.c_str())) { ok = true; break; }
  if (!ok) return false;
  for (const std::string& g : deny_)
    if (glob_match(g.c_str(), base.c_str())) return false;
  return true;
}

Exporter::Exporter(ExporterConfig cfg) : cfg_(std::move(cfg)), filter_(cfg_.metric_allow, cfg_.metric_deny) {
  node_name_ = cfg_.node_name;
  if (node_name_.empty()) {
    char h[256] = {};
    if (gethostname(h, sizeof h - 1) == 0) node_name_ = h;
  }
}

Exporter::~Exporter() {
  stop();
  // A sampler thread stuck in a device call (abandoned by stop()) still points
  // into the sampler, the backend and the counter source: keep them alive.
  if (sampler_ && sampler_->abandoned_threads() > 0) {
    (void)sampler_.release();
    (void)pmc_.release();
    (void)be_.release();
  }
}

bool Exporter::init() {
  if (cfg_.sm_util_source != "auto" && cfg_.sm_util_source != "pmfw" && cfg_.sm_util_source != "counters") {
    err_ = "unknown sm_util_source '" + cfg_.sm_util_source + "' (auto | pmfw | counters)";
    return false;
  }
  if (cfg_.backend == "mock") {
    be_ = make_mock_backend(cfg_.mock);
  } else if (cfg_.backend == "amdsmi") {
    be_ = make_amdsmi_backend(err_, cfg_.sysfs_root);
    if (!be_) return false;
  } else {
    err_ = "unknown backend '" + cfg_.backend + "' (expected amdsmi or mock)";
    return false;
  }
  SamplerConfig sc = cfg_.sampler;
  for (const std::string& want : cfg_.bdfs) {
    int found = -1;
    for (int d = 0; d < be_->device_count(); ++d)
      if (be_->info(d).bdf == want) found = d;
    if (found < 0) {
      err_ = "no GPU with PCI address " + want;
      return false;
    }
    sc.devices.push_back(found);
  }
  std::vector<int> devs = sc.devices;
  if (devs.empty())
    for (int d = 0; d < be_->device_count(); ++d) devs.push_back(d);
  const uint32_t pmc_mask = pmc_set_mask(cfg_.pmc_set);
  if (pmc_mask == 0) {
    err_ = "unknown pmc_set '" + cfg_.pmc_set + "' (base | full | util)";
    return false;
  }
  if (cfg_.pmc_source == "mock") {
    MockPmcConfig mp = cfg_.mock_pmc;
    mp.mask = pmc_mask;
    pmc_ = make_mock_counter_source(*be_, cfg_.mock, mp);
  } else if (cfg_.pmc_source == "rocprofiler" || cfg_.pmc_source == "aqlprofile") {
    pmc_ = make_dl_counter_source(cfg_.pmc_source, cfg_.pmc_lib, *be_, devs, cfg_.pmc_pipeline, pmc_mask, cfg_.pmc_lean,
                                  pmc_err_, cfg_.pmc_timeout_ms, cfg_.pmc_batch,
                                  cfg_.pmc_publish_us, cfg_.pmc_lite);
  } else if (cfg_.pmc_source != "none" && !cfg_.pmc_source.empty()) {
    err_ = "unknown pmc_source '" + cfg_.pmc_source + "'";
    return false;
  }
  sc.pmc = pmc_ != nullptr;
  sampler_ = std::make_unique<Sampler>(be_.get(), pmc_.get(), sc);
  be_->topology(topo_);
  build_static_labels();
  return true;
}

void Exporter::build_static_labels() {
  dev_labels_.clear();
  for (int d = 0; d < be_->device_count(); ++d) {
    const DeviceInfo& in = be_->info(d);
    std::string lb;
    // Per-series identity is (gpu, uuid); bdf, type, serial, ... live once in
    // amdgpu_device_info (join on gpu/uuid) — keeps an 8-GPU scrape ≈30 % smaller.
    lb += "gpu=\"" + std::to_string(d) + "\"";
    lb += ",uuid=\"";
    append_label_value(lb, in.uuid);
    lb += '"';
    dev_labels_.push_back(std::move(lb));
  }
}

void Exporter::start() {
  if (!sampler_) return;
  sampler_->start();
  if (cfg_.port >= 0 && !http_) {
    http_ = std::make_unique<HttpServer>(this, cfg_.listen_addr, cfg_.port);
    if (!http_->start(err_)) http_.reset();
  }
}

void Exporter::stop() {
  if (http_) {
    http_->stop();
    http_.reset();
  }
  if (sampler_) sampler_->stop();
}

int Exporter::port() const { return http_ ? http_->port() : -1; }

void Exporter::pause_sampling() {
  if (sampler_) sampler_->stop();
}
void Exporter::resume_sampling() {
  if (sampler_) sampler_->start();
}
bool Exporter::sampling() const { return sampler_ && sampler_->running(); }
void Exporter::set_pmc_enabled(bool on, int dev, bool drop_queue) {
  if (dev < 0) pmc_wanted_.store(on);
  if (sampler_) sampler_->set_pmc_wanted(on, dev, drop_queue);
}
bool Exporter::pmc_enabled() const { return pmc_wanted_.load(); }

bool Exporter::set_sample_rate(double hz) { return sampler_ && sampler_->set_hz(hz); }
double Exporter::sample_rate() const { return sampler_ ? sampler_->hz() : 0.0; }

void Exporter::set_device_owners(int dev, std::vector<Owner> o) {
  Integrals I;
  if (sampler_ && dev >= 0 && dev < sampler_->device_count()) I = sampler_->state(dev).integrals();
  std::lock_guard<std::mutex> g(mu_);
  auto m = owners_ ? std::make_shared<std::map<int, std::vector<Owner>>>(*owners_)
                   : std::make_shared<std::map<int, std::vector<Owner>>>();
  const auto prev = m->find(dev);
  size_t kept_n = 0;
  for (Owner& x : o) {
    // An owner already on this GPU keeps its base; a new one starts counting now.
    const Owner* kept = nullptr;
    if (prev != m->end())
      for (const Owner& y : prev->second)
        if (y.same(x)) kept = &y;
    kept_n += kept != nullptr;
    x.base_busy_s = kept ? kept->base_busy_s : I.gfx_busy_seconds;
    x.base_mfma_s = kept ? kept->base_mfma_s : I.mfma_busy_seconds;
    x.base_active_s = kept ? kept->base_active_s : I.active_seconds;
    x.base_util_s = kept ? kept->base_util_s : I.util_seconds;
    x.base_energy_j = kept ? kept->base_energy_j : I.energy_joules;
    x.base_cu_s = kept ? kept->base_cu_s : (sampler_ ? sampler_->pod_cu_seconds(dev, x.ns + "/" + x.pod) : 0.0);
  }
  const size_t prev_n = prev != m->end() ? prev->second.size() : 0;
  const bool changed = kept_n != o.size() || kept_n != prev_n;
  if (o.empty()) m->erase(dev);
  else (*m)[dev] = std::move(o);
  owners_ = std::move(m);
  if (changed && sampler_) sampler_->drop_util_carry(dev);  // the old owner's carried busy is not the new one's
}

void Exporter::set_pid_owners(std::unordered_map<uint64_t, PidOwner> m) {
  if (sampler_) {  // (GPU, PID) → "namespace/pod": the slow tier's per-pod CU integrals
    auto pods = std::make_shared<std::unordered_map<uint64_t, std::string>>();
    for (const auto& [k, po] : m)
      if (!po.pod.empty()) (*pods)[k] = po.ns + "/" + po.pod;
    sampler_->set_pid_pods(std::move(pods));
  }
  auto p = std::make_shared<const std::unordered_map<uint64_t, PidOwner>>(std::move(m));
  std::lock_guard<std::mutex> g(mu_);
  pid_owners_ = std::move(p);
}

void Exporter::set_node_name(const std::string& n) {
  std::lock_guard<std::mutex> g(mu_);
  node_name_ = n;
}

void Exporter::set_extra_metrics(std::string text) {
  if (!text.empty() && text.back() != '\n') text += '\n';
  auto p = std::make_shared<const std::string>(std::move(text));
  std::lock_guard<std::mutex> g(mu_);
  extra_ = std::move(p);
}

std::shared_ptr<const std::map<int, std::vector<Owner>>> Exporter::owners() const {
  std::lock_guard<std::mutex> g(mu_);
  return owners_;
}
std::shared_ptr<const std::unordered_map<uint64_t, PidOwner>> Exporter::pid_owners() const {
  std::lock_guard<std::mutex> g(mu_);
  return pid_owners_;
}

bool Exporter::healthy() const {
  if (!sampler_) return false;
  for (int d = 0; d < sampler_->device_count(); ++d)
    if (sampler_->state(d).up.load()) return true;
  return false;
}

std::string Exporter::devices_json() {
  std::string o = "[";
  for (int d = 0; d < be_->device_count(); ++d) {
    const DeviceInfo& in = be_->info(d);
    if (d) o += ',';
    o += "{\"gpu\":" + std::to_string(d) + ",\"bdf\":";
    jstr(o, in.bdf);
    o += ",\"uuid\":";
    jstr(o, in.uuid);
    o += ",\"serial\":";
    jstr(o, in.serial);
    o += ",\"market_name\":";
    jstr(o, in.market_name);
    o += ",\"gpu_type\":";
    jstr(o, in.gpu_type);
    o += ",\"gfx_target\":";
    jstr(o, in.gfx_target);
    o += ",\"numa_node\":" + std::to_string(in.numa_node) + ",\"num_cu\":" + std::to_string(in.num_cu) +
         ",\"num_xcc\":" + std::to_string(in.num_xcc) + ",\"vram_total_bytes\":" + std::to_string(in.vram_total_bytes) +
         ",\"kfd_gpu_id\":" + std::to_string(in.kfd_gpu_id) + ",\"kfd_node\":" + std::to_string(in.kfd_node) +
         ",\"drm_card\":" + std::to_string(in.drm_card) + ",\"hip_id\":" + std::to_string(in.hip_id) +
         ",\"sysfs_dir\":";
    jstr(o, in.sysfs_dir);
    o += ",\"compute_partition\":";
    jstr(o, in.compute_partition);
    o += ",\"memory_partition\":";
    jstr(o, in.memory_partition);
    o += ",\"partition_id\":" + std::to_string(in.partition_id);
    o += ",\"cpu_pinned\":" + std::to_string(sampler_ ? sampler_->state(d).cpu_pinned.load() : -1);
    o += '}';
  }
  o += ']';
  return o;
}

std::string Exporter::topology_json() {
  std::string o = "{\"node\":";
  {
    std::lock_guard<std::mutex> g(mu_);
    jstr(o, node_name_);
  }
  o += ",\"devices\":" + devices_json() + ",\"edges\":[";
  for (size_t i = 0; i < topo_.size(); ++i) {
    const TopoEdge& e = topo_[i];
    if (i) o += ',';
    o += "{\"src\":" + std::to_string(e.src) + ",\"dst\":" + std::to_string(e.dst) +
         ",\"link_type\":" + std::to_string(e.link_type) + ",\"hops\":" + std::to_string(e.hops) +
         ",\"weight\":" + std::to_string(e.weight) + '}';
  }
  o += "],\"links\":[";
  bool first = true;
  for (int d = 0; sampler_ && d < sampler_->device_count(); ++d) {
    auto links = sampler_->state(d).get_links();
    if (!links) continue;
    for (const LinkInfo& l : *links) {
      if (!first) o += ',';
      first = false;
      o += "{\"gpu\":" + std::to_string(d) + ",\"link\":" + std::to_string(l.link) + ",\"peer_bdf\":";
      jstr(o, l.peer_bdf);
      o += ",\"link_type\":" + std::to_string(l.link_type) + ",\"bit_rate_gbps\":" + std::to_string(l.bit_rate_gbps) +
           ",\"max_bandwidth_gbps\":" + std::to_string(l.max_bw_gbps) + ",\"read_kb\":" + std::to_string(l.read_kb) +
           ",\"write_kb\":" + std::to_string(l.write_kb) + '}';
    }
  }
  o += "]}";
  return o;
}

std::string Exporter::samples_json(int dev, int n) {
  if (!sampler_ || dev < 0 || dev >= sampler_->device_count()) return "[]";
  if (n <= 0) n = 1;
  if (n > static_cast<int>(kRing) - 1) n = static_cast<int>(kRing) - 1;
  std::vector<GpuSample> buf(static_cast<size_t>(n));
  const size_t got = sampler_->state(dev).ring.recent(buf.data(), static_cast<size_t>(n));
  std::string o = "[";
  for (size_t i = got; i-- > 0;) {  // oldest first
    const GpuSample& s = buf[i];
    if (o.size() > 1) o += ',';
    o += "{\"seq\":" + std::to_string(s.seq) + ",\"fw_ts\":" + std::to_string(s.fw_ts) +
         ",\"wall_ns\":" + std::to_string(s.wall_ns) + ",\"gfx_busy_pct\":";
    jnum(o, s.gfx_busy_pct);
    o += ",\"gfx_busy_window_pct\":";
    jnum(o, s.gfx_busy_window_pct);
    o += ",\"umc_busy_window_pct\":";
    jnum(o, s.umc_busy_window_pct);
    o += ",\"dt_s\":";
    jnum(o, s.dt_s);
    o += ",\"power_w\":";
    jnum(o, s.power_w);
    o += ",\"temp_hotspot_c\":";
    jnum(o, s.temp_hotspot_c);
    o += ",\"vram_used_bytes\":" + std::to_string(s.vram_used_bytes) + ",\"read_ns\":" + std::to_string(s.read_ns) + '}';
  }
  o += ']';
  return o;
}

std::string Exporter::counters_json(int dev, int n, uint64_t since) {
  if (!sampler_ || dev < 0 || dev >= sampler_->device_count()) return "{\"samples\":[]}";
  const int cap = static_cast<int>(kPmcRing) - 2;
  if (n <= 0) n = 1;
  if (since > 0 || n > cap) n = cap;
  std::vector<PmcSample> buf;
  buf.reserve(static_cast<size_t>(n) + 1);
  // Newest first; one extra (older) entry gives the first returned sample its rates.
  // With lite READs only the publishing drains read the per-SE counters (se_fresh):
  // keep going, at most a batch further, until an older fresh drain is held too, so
  // the first fresh sample's MFMA / TA rates have their base.
  size_t extra_stale = 0;
  sampler_->state(dev).pmc_ring.visit_recent([&](const PmcSample& p) {
    buf.push_back(p);
    const bool enough = since > 0 ? p.seq <= since : buf.size() >= static_cast<size_t>(n) + 1;
    if (!enough) return true;
    return p.se_fresh == 0 && ++extra_stale < 64;
  });
  const int num_cu = be_->info(dev).num_cu;
  std::string o = "{\"gpu\":" + std::to_string(dev) + ",\"counters\":[";
  for (int i = 0; i < kPmcCount; ++i) {
    if (i) o += ',';
    jstr(o, pmc_counter_name(i));
  }
  o += "],\"samples\":[";
  bool first = true;
  const PmcSample* last_fresh = nullptr;  // newest fresh drain older than the sample being written
  for (size_t i = buf.size(); i-- > 0;) {  // oldest first
    const PmcSample& p = buf[i];
    // the newest n (or those after `since`) are returned; older ones are rate bases
    if (since > 0 ? p.seq <= since : i >= static_cast<size_t>(n)) {
      if (p.se_fresh) last_fresh = &p;
      continue;
    }
    if (!first) o += ',';
    first = false;
    o += "{\"seq\":" + std::to_string(p.seq) + ",\"mono_ns\":" + std::to_string(p.mono_ns) +
         ",\"se_fresh\":" + (p.se_fresh ? "1" : "0") + ",\"v\":[";
    for (int k = 0; k < kPmcCount; ++k) {
      if (k) o += ',';
      if (p.mask & (1u << k)) o += std::to_string(p.value[k]);
      else o += "null";
    }
    o += ']';
    if (i + 1 < buf.size()) {
      // Device-wide counters (GRBM, CPC) are read by every drain: rates over the last interval.
      const PmcRates r = pmc_rates(buf[i + 1], p, num_cu);
      o += ",\"dt_us\":";
      jnum(o, r.dt_s * 1e6);
      o += ",\"gpu_active_pct\":";
      jnum(o, r.gpu_active_pct);
      o += ",\"gpu_clock_mhz\":";
      jnum(o, r.gpu_clock_mhz);
      // Per-SE counters (MFMA, TA) only on a fresh drain, over the span since the
      // previous fresh one: a stale drain repeats the last values read.
      if (p.se_fresh && last_fresh) {
        const PmcRates f = pmc_rates(*last_fresh, p, num_cu);
        if (f.have_mfma && f.dt_s > 0) {
          o += ",\"mfma_util_pct\":";
          jnum(o, f.mfma_util_pct);
        }
        if (f.have_vmem && f.dt_s > 0) {
          o += ",\"vmem_busy_pct\":";
          jnum(o, f.vmem_busy_pct);
        }
        if (f.n_xcd > 0 && f.dt_s > 0) {
          o += ",\"xcd_mfma_util_pct\":[";
          for (int x = 0; x < f.n_xcd; ++x) {
            if (x) o += ',';
            jnum(o, f.xcd_mfma_util_pct[x]);
          }
          o += "]";
        }
      }
    }
    if (p.se_fresh) last_fresh = &p;
    o += '}';
  }
  o += "]}";
  return o;
}

}  // namespace kgs
