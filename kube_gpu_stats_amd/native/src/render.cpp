// Prometheus text-format (0.0.4) renderer for the node exporter.
//
// The reference's report consumes `container_gpu_sm_util` grouped by
// (kubernetes_io_hostname, nvidia_gpu_type, pod_name)
// (reference gpu_util_stats/gpu_util_stats.py:159); that series is emitted with
// exactly those label keys plus namespace/container/gpu/uuid, which the
// reference's `avg ... by` averages away.  Everything else is
// the amdgpu_* / kgs_* families documented in models/schema.py.
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>

#include "kgs/exporter.h"
#include "kgs/metric_help.h"

namespace kgs {

void append_label_value(std::string& out, const std::string& v) {
  // Label values almost never need escaping: append unescaped spans in bulk.
  const char* p = v.data();
  const char* const end = p + v.size();
  while (p < end) {
    const char* q = p;
    while (q < end && *q != '\\' && *q != '"' && *q != '\n') ++q;
    out.append(p, q);
    if (q == end) break;
    out += *q == '\n' ? "\\n" : (*q == '"' ? "\\\"" : "\\\\");
    p = q + 1;
  }
}

namespace {

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// Append-only writer over a raw buffer: one capacity check and memcpy per
// piece instead of std::string's per-append bookkeeping (the 8-GPU page is
// ≈950 lines / 100 KB).  Numbers go through std::to_chars (shortest round-trip
// form), so the hot path never touches locale-dependent printf.  finish()
// trims the string to what was written.
struct W {
  std::string& o;
  char* p = nullptr;
  char* end = nullptr;
  // --metric-allow / --metric-deny: one decision per run of lines of one family
  // (names are string literals, so consecutive lines share the pointer).
  const FamilyFilter* ff = nullptr;
  const char* last_name = nullptr;
  bool last_ok = true;
  bool ok(const char* name) {
    if (!ff) return true;
    if (name != last_name) {
      last_name = name;
      last_ok = ff->allowed(name);
    }
    return last_ok;
  }
  explicit W(std::string& s, size_t cap, const FamilyFilter* f = nullptr) : o(s), ff(f && f->active() ? f : nullptr) {
    o.resize(cap);
    p = &o[0];
    end = p + o.size();
  }
  void grow(size_t n) {
    const size_t used = static_cast<size_t>(p - o.data());
    o.resize(std::max(o.size() * 2, used + n + 4096));
    p = &o[0] + used;
    end = &o[0] + o.size();
  }
  void put(const char* s, size_t n) {
    if (static_cast<size_t>(end - p) < n) grow(n);
    std::memcpy(p, s, n);
    p += n;
  }
  void put(const std::string& s) { put(s.data(), s.size()); }
  void put(const char* s) { put(s, std::strlen(s)); }
  void put(char c) {
    if (p == end) grow(1);
    *p++ = c;
  }
  void finish() { o.resize(static_cast<size_t>(p - o.data())); }
  void num(double v) {
    if (std::isnan(v)) { put("NaN", 3); return; }
    if (std::isinf(v)) { put(v > 0 ? "+Inf" : "-Inf", 4); return; }
    if (end - p < 40) grow(40);
    p = std::to_chars(p, end, v).ptr;
  }
  void u64(uint64_t v) {
    if (end - p < 24) grow(24);
    p = std::to_chars(p, end, v).ptr;
  }
  // HELP and TYPE come from the metric catalogue (models/schema.py → kgs/metric_help.h),
  // in the text of the exporter's --sm-util-source mode; `doc` is resolved at compile
  // time (KGS_METRIC_DOC), so a family the catalogue lacks does not build.
  const char* mode = "";
  void head(size_t doc) {
    const MetricDoc& d = metric_doc_at(doc, mode);
    if (!ok(d.name)) return;
    put("# HELP ", 7); put(d.name); put(' '); put(d.help);
    put("\n# TYPE ", 8); put(d.name); put(' '); put(d.type); put('\n');
  }
  // name{base,extra} value
  void labels(const char* name, const std::string& base, const char* extra) {
    put(name); put('{'); put(base);
    if (extra && *extra) { put(','); put(extra); }
    put("} ", 2);
  }
  void line(const char* name, const std::string& base, const char* extra, double v) {
    if (!ok(name)) return;
    labels(name, base, extra); num(v); put('\n');
  }
  void line_u(const char* name, const std::string& base, const char* extra, uint64_t v) {
    if (!ok(name)) return;
    labels(name, base, extra); u64(v); put('\n');
  }
};

void kv(std::string& o, const char* k, const std::string& v, bool comma = true) {
  if (comma) o += ',';
  o += k; o += "=\""; append_label_value(o, v); o += '"';
}
// Integer-valued label without a std::to_string temporary.
void kvi(std::string& o, const char* k, int64_t v) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof b, v);
  o += ','; o += k; o += "=\""; o.append(b, r.ptr); o += '"';
}

// `le` labels of the read-latency histogram and `counter` labels of the PMC
// family never change: format them once.
const std::vector<std::string>& hist_le_labels() {
  static const std::vector<std::string> v = [] {
    std::vector<std::string> out;
    for (int b = 0; b <= kReadHistBuckets; ++b) {
      std::string e = "le=\"";
      if (b < kReadHistBuckets) {
        char nb[32];
        auto r = std::to_chars(nb, nb + sizeof nb, kReadHistBoundsUs[b] * 1e-6);
        e.append(nb, r.ptr);
      } else {
        e += "+Inf";
      }
      e += '"';
      out.push_back(std::move(e));
    }
    return out;
  }();
  return v;
}
const std::vector<std::string>& pmc_counter_labels() {
  static const std::vector<std::string> v = [] {
    std::vector<std::string> out;
    for (int i = 0; i < kPmcCount; ++i) out.push_back(std::string("counter=\"") + pmc_counter_name(i) + '"');
    return out;
  }();
  return v;
}
const char* const kXccLabels[kMaxXcc] = {"xcc=\"0\"", "xcc=\"1\"", "xcc=\"2\"", "xcc=\"3\"",
                                         "xcc=\"4\"", "xcc=\"5\"", "xcc=\"6\"", "xcc=\"7\""};
const char* const kLinkLabels[kMaxXgmi] = {"link=\"0\"", "link=\"1\"", "link=\"2\"", "link=\"3\"",
                                           "link=\"4\"", "link=\"5\"", "link=\"6\"", "link=\"7\""};
const char* const kThrottleLabels[kThrottleReasons] = {"reason=\"prochot\"", "reason=\"ppt\"",
                                                       "reason=\"socket_thermal\"", "reason=\"vr_thermal\"",
                                                       "reason=\"hbm_thermal\""};
const char* throttle_label(int r) { return kThrottleLabels[r]; }

}  // namespace

void Exporter::render(std::string& out) {
  const int64_t t0 = mono_ns();
  out.clear();
  W w(out, last_render_bytes_.load(std::memory_order_relaxed) + 8192, &filter_);
  w.mode = cfg_.sm_util_source == "auto" ? "" : cfg_.sm_util_source.c_str();
  Sampler& S = *sampler_;
  const int nd = S.device_count();
  const std::vector<int>& ids = S.sampled_devices();
  std::vector<char> sampled(static_cast<size_t>(nd), 0);
  for (int d : ids) sampled[static_cast<size_t>(d)] = 1;
  std::string node;
  std::shared_ptr<const std::string> extra;
  {
    std::lock_guard<std::mutex> g(mu_);
    node = node_name_;
    extra = extra_;
  }
  const auto own = owners();
  const auto pown = pid_owners();
  const int64_t now = mono_ns();

  // Snapshot all devices once.
  struct Snap {
    bool have = false, busy = false, pmc_have = false, pmc_rates = false;
    bool pmc_mfma = false;  // the counter set has MFMA busy (not `util`)
    GpuSample s;
    Integrals I;
    PmcSample p;
    PmcRates r;
    double g = 0, u = 0, util = 0;
    int n = 0;
    bool procs_fresh = false, links_fresh = false, health_fresh = false;
  };
  static thread_local std::vector<Snap> snaps;
  snaps.assign(static_cast<size_t>(nd), Snap{});
  const int64_t stale_ns = static_cast<int64_t>(cfg_.stale_s * 1e9);
  for (int d : ids) {
    Snap& x = snaps[static_cast<size_t>(d)];
    const DeviceState& st = S.state(d);
    x.have = st.latest.load(x.s);
    x.I = st.integrals();
    // Window gauges only from live data: a device that is down, or whose last
    // good read is older than stale_s (reads failing, sampling paused), exports
    // no busy gauges rather than its last value frozen; the counters stay.
    const int64_t ok_ns = st.last_ok_mono_ns.load(std::memory_order_relaxed);
    const bool pmfw_fresh = st.up.load(std::memory_order_relaxed) && ok_ns > 0 && now - ok_ns <= stale_ns;
    x.busy = x.have && pmfw_fresh && S.window_busy(d, cfg_.window_s, x.g, x.u, x.n, &x.util);
    // Slow tiers (per-device kgs-slow threads): a result older than stale_s — or
    // than three of its tier's periods, if longer — is not exported as current.
    auto fresh = [&](const std::atomic<int64_t>& ok, int64_t period) {
      const int64_t t = ok.load(std::memory_order_acquire);
      return t > 0 && now - t <= std::max(stale_ns, 3 * period);
    };
    x.procs_fresh = fresh(st.procs_ok_ns, S.proc_period_ns());
    x.links_fresh = fresh(st.links_ok_ns, S.link_period_ns());
    x.health_fresh = fresh(st.health_ok_ns, S.link_period_ns());
    x.pmc_have = st.pmc_latest.load(x.p);
    x.pmc_mfma = x.pmc_have && (x.p.mask & (1u << kPmcMfmaBusy));
    // Counter rates only while we hold the counters and drains keep arriving:
    // handed over (pmc_on = 0), stalled (a foreign profiler STOPped /
    // reprogrammed them) or stale → no rate gauges rather than wrong or frozen
    // ones; the raw totals and kgs_pmc_enabled / kgs_pmc_stalled stay.
    x.pmc_rates = x.pmc_have && st.pmc_on.load(std::memory_order_relaxed) &&
                  !st.pmc_stalled.load(std::memory_order_relaxed) && now - x.p.mono_ns <= stale_ns &&
                  S.window_pmc(d, cfg_.window_s, x.r);
  }

  // ---- reference-compatible series (F5) ---------------------------------
  if (cfg_.compat_series) {
    // Pod labels of every (GPU, owner) pair, built once for both per-pod families.
    static thread_local std::vector<std::pair<int, std::string>> pod_lines;
    pod_lines.clear();
    static thread_local std::vector<const Owner*> pod_owner;  // parallel to pod_lines (nullptr: unallocated)
    pod_owner.clear();
    for (int d : ids) {
      const Snap& x = snaps[static_cast<size_t>(d)];
      if (!x.have) continue;
      const DeviceInfo& in = be_->info(d);
      const std::string type = cfg_.gpu_type_override.empty() ? in.gpu_type : cfg_.gpu_type_override;
      auto emit = [&](const Owner* o) {
        std::string lb;
        lb.reserve(256);
        kv(lb, "kubernetes_io_hostname", node, false);
        kv(lb, "nvidia_gpu_type", type);
        kv(lb, "pod_name", o ? o->pod : std::string());
        kv(lb, "namespace", o ? o->ns : std::string());
        kv(lb, "container_name", o ? o->container : std::string());
        kv(lb, "gpu", std::to_string(d));
        kv(lb, "uuid", in.uuid);
        pod_lines.emplace_back(d, std::move(lb));
        pod_owner.push_back(o);
      };
      auto it = own ? own->find(d) : decltype(own->end()){};
      if (own && it != own->end() && !it->second.empty()) {
        for (const Owner& o : it->second) emit(&o);
      } else if (cfg_.compat_unallocated) {
        emit(nullptr);
      }
    }
    const bool from_counters = cfg_.sm_util_source == "counters";
    const bool from_auto = cfg_.sm_util_source == "auto";
    if (from_auto) {
      w.head(KGS_METRIC_DOC("container_gpu_sm_util"));
      for (const auto& [d, lb] : pod_lines)
        if (snaps[static_cast<size_t>(d)].busy)
          w.line("container_gpu_sm_util", lb, nullptr, std::clamp(snaps[static_cast<size_t>(d)].util, 0.0, 100.0));
    } else if (from_counters) {
      w.head(KGS_METRIC_DOC("container_gpu_sm_util"));
      for (const auto& [d, lb] : pod_lines) {
        const Snap& x = snaps[static_cast<size_t>(d)];
        if (x.pmc_rates) w.line("container_gpu_sm_util", lb, nullptr, x.r.gpu_active_pct);
      }
    } else {
      w.head(KGS_METRIC_DOC("container_gpu_sm_util"));
      for (const auto& [d, lb] : pod_lines)
        if (snaps[static_cast<size_t>(d)].busy) w.line("container_gpu_sm_util", lb, nullptr, snaps[static_cast<size_t>(d)].g);
    }
    // Exact per-pod accounting: the GPU's busy integral since the pod was given
    // it.  rate() / increase() over any range is the exact mean utilisation,
    // whatever the scrape interval — the gauge above only sees its window.
    w.head(KGS_METRIC_DOC("container_gpu_busy_seconds_total"));
    for (size_t i = 0; i < pod_lines.size(); ++i) {
      const Owner* o = pod_owner[i];
      const Snap& x = snaps[static_cast<size_t>(pod_lines[i].first)];
      if (from_counters && !x.pmc_have) continue;
      const double v = from_auto       ? x.I.util_seconds - (o ? o->base_util_s : 0.0)
                       : from_counters ? x.I.active_seconds - (o ? o->base_active_s : 0.0)
                                       : x.I.gfx_busy_seconds - (o ? o->base_busy_s : 0.0);
      w.line("container_gpu_busy_seconds_total", pod_lines[i].second, nullptr, v > 0 ? v : 0.0);
    }
    // Per-pod compute share: the CU-occupancy seconds of the pod's
    // own processes on this GPU (per-process tier, PID → pod from cgroups), kept
    // after they exit.  On a GPU shared by several pods each is billed its own
    // share, where container_gpu_busy_seconds_total bills each the whole GPU.
    bool any_cu = false;
    for (size_t i = 0; i < pod_lines.size() && !any_cu; ++i) any_cu = pod_owner[i] != nullptr && cfg_.per_process;
    if (any_cu) {
      w.head(KGS_METRIC_DOC("container_gpu_cu_seconds_total"));
      for (size_t i = 0; i < pod_lines.size(); ++i) {
        const Owner* o = pod_owner[i];
        if (!o) continue;
        const int d = pod_lines[i].first;
        auto pc = S.state(d).get_pod_cu();
        const std::string key = o->ns + "/" + o->pod;
        double v = 0;
        bool have = false;
        if (pc) {
          auto it = pc->find(key);
          if (it != pc->end()) {
            v = it->second;
            have = true;
          }
        }
        // A pod whose processes' CU occupancy could not be read has no CU-seconds yet:
        // its line is withheld rather than billed 0 (kgs_process_cu_unavailable says why).
        if (!have) {
          auto uk = S.state(d).get_pod_cu_unknown();
          if (uk && uk->count(key)) continue;
        }
        v -= o->base_cu_s;
        w.line("container_gpu_cu_seconds_total", pod_lines[i].second, nullptr, v > 0 ? v : 0.0);
      }
    }
    // Per-pod energy: the GPU's socket energy since the pod was given it (a GPU
    // shared by several pods counts in full for each: the pods hold it together;
    // a compute partition's energy is its share of the socket's, sampler.cpp).
    w.head(KGS_METRIC_DOC("container_gpu_energy_joules_total"));
    for (size_t i = 0; i < pod_lines.size(); ++i) {
      const Owner* o = pod_owner[i];
      const Snap& x = snaps[static_cast<size_t>(pod_lines[i].first)];
      const double v = x.I.energy_joules - (o ? o->base_energy_j : 0.0);
      w.line("container_gpu_energy_joules_total", pod_lines[i].second, nullptr, v > 0 ? v : 0.0);
    }
    bool any_pmc_int = false;
    for (const auto& pl : pod_lines) any_pmc_int |= snaps[static_cast<size_t>(pl.first)].pmc_mfma;
    if (any_pmc_int) {
      w.head(KGS_METRIC_DOC("container_gpu_mfma_busy_seconds_total"));
      for (size_t i = 0; i < pod_lines.size(); ++i) {
        const Snap& x = snaps[static_cast<size_t>(pod_lines[i].first)];
        if (!x.pmc_mfma) continue;
        const Owner* o = pod_owner[i];
        const double v = x.I.mfma_busy_seconds - (o ? o->base_mfma_s : 0.0);
        w.line("container_gpu_mfma_busy_seconds_total", pod_lines[i].second, nullptr, v > 0 ? v : 0.0);
      }
    }
    bool any_owner = false;
    for (const Owner* o : pod_owner) any_owner |= o != nullptr;
    if (any_owner) {
      w.head(KGS_METRIC_DOC("kgs_gpu_owner"));
      for (size_t i = 0; i < pod_lines.size(); ++i)
        if (pod_owner[i]) w.line("kgs_gpu_owner", pod_lines[i].second, nullptr, 1);
    }
    bool any_mfma = false;
    for (const auto& pl : pod_lines) any_mfma |= snaps[static_cast<size_t>(pl.first)].pmc_rates && snaps[static_cast<size_t>(pl.first)].r.have_mfma;
    if (any_mfma) {
      // Same labels, hardware-counter matrix-core busy: GFX busy counts a GPU busy
      // while any dispatch is in flight; this says how much of it was MFMA work.
      w.head(KGS_METRIC_DOC("container_gpu_mfma_util"));
      for (const auto& [d, lb] : pod_lines)
        if (snaps[static_cast<size_t>(d)].pmc_rates && snaps[static_cast<size_t>(d)].r.have_mfma)
          w.line("container_gpu_mfma_util", lb, nullptr, snaps[static_cast<size_t>(d)].r.mfma_util_pct);
    }
  }

  // ---- device info / topology (static: cached per node name) -------------
  std::string lb;  // scratch label buffer, reused (no per-line allocation)
  lb.reserve(512);
  std::shared_ptr<const std::string> sblock;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (static_block_ && static_block_node_ == node) sblock = static_block_;
  }
  if (!sblock) {
    std::string blk;
    W b(blk, 16384, &filter_);
    b.head(KGS_METRIC_DOC("amdgpu_device_info"));
    for (int d : ids) {
      const DeviceInfo& in = be_->info(d);
      lb.assign(dev_labels_[static_cast<size_t>(d)]);
      kv(lb, "bdf", in.bdf);
      kv(lb, "gpu_type", cfg_.gpu_type_override.empty() ? in.gpu_type : cfg_.gpu_type_override);
      kv(lb, "kubernetes_io_hostname", node);
      kv(lb, "serial", in.serial);
      kv(lb, "market_name", in.market_name);
      kv(lb, "gfx_target", in.gfx_target);
      kvi(lb, "numa_node", in.numa_node);
      kvi(lb, "num_cu", in.num_cu);
      kvi(lb, "num_xcc", in.num_xcc);
      kvi(lb, "kfd_gpu_id", in.kfd_gpu_id);
      kvi(lb, "hip_id", in.hip_id);
      kv(lb, "compute_partition", in.compute_partition);
      kv(lb, "memory_partition", in.memory_partition);
      kvi(lb, "partition_id", in.partition_id);
      b.line("amdgpu_device_info", lb, nullptr, 1);
    }
    if (!topo_.empty()) {
      b.head(KGS_METRIC_DOC("amdgpu_topology_link"));
      for (const TopoEdge& e : topo_) {
        if (!sampled[static_cast<size_t>(e.src)]) continue;
        lb.assign(dev_labels_[static_cast<size_t>(e.src)]);
        kvi(lb, "peer_gpu", e.dst);
        kv(lb, "peer_bdf", be_->info(e.dst).bdf);
        kv(lb, "link_type", e.link_type == 2 ? "xgmi" : (e.link_type == 1 ? "pcie" : "other"));
        kvi(lb, "hops", e.hops);
        kvi(lb, "weight", e.weight);
        b.line("amdgpu_topology_link", lb, nullptr, 1);
      }
    }
    b.finish();
    sblock = std::make_shared<const std::string>(std::move(blk));
    std::lock_guard<std::mutex> g(mu_);
    static_block_ = sblock;
    static_block_node_ = node;
  }
  w.put(*sblock);

  // ---- utilisation -------------------------------------------------------
  // amdgpu_gfx_busy_*: the same busy signal as container_gpu_sm_util (--sm-util-source;
  // default auto: READ-immune); amdgpu_pmfw_gfx_busy_* is always the firmware's own.
  const bool util_auto = cfg_.sm_util_source == "auto";
  w.head(KGS_METRIC_DOC("amdgpu_gfx_busy_percent"));
  for (int d : ids)
    if (snaps[d].busy)
      w.line("amdgpu_gfx_busy_percent", dev_labels_[d], nullptr, util_auto ? std::clamp(snaps[d].util, 0.0, 100.0) : snaps[d].g);
  w.head(KGS_METRIC_DOC("amdgpu_pmfw_gfx_busy_percent"));
  for (int d : ids) if (snaps[d].busy) w.line("amdgpu_pmfw_gfx_busy_percent", dev_labels_[d], nullptr, snaps[d].g);
  w.head(KGS_METRIC_DOC("amdgpu_gfx_busy_instant_percent"));
  for (int d : ids) if (snaps[d].have && (snaps[d].s.valid & kFGfxBusy)) w.line("amdgpu_gfx_busy_instant_percent", dev_labels_[d], nullptr, snaps[d].s.gfx_busy_pct);
  w.head(KGS_METRIC_DOC("amdgpu_gfx_busy_xcc_percent"));
  for (int d : ids) {
    const Snap& x = snaps[d];
    if (!x.have || !(x.s.valid & kFGfxBusyXcc)) continue;
    for (uint32_t c = 0; c < x.s.num_xcc && c < static_cast<uint32_t>(kMaxXcc); ++c) {
      w.line("amdgpu_gfx_busy_xcc_percent", dev_labels_[d], kXccLabels[c],
             x.s.dt_s > 0 ? x.s.gfx_busy_xcc_window[c] : x.s.gfx_busy_xcc[c]);
    }
  }
  w.head(KGS_METRIC_DOC("amdgpu_umc_busy_percent"));
  for (int d : ids) if (snaps[d].busy) w.line("amdgpu_umc_busy_percent", dev_labels_[d], nullptr, snaps[d].u);
  w.head(KGS_METRIC_DOC("amdgpu_gfx_busy_seconds_total"));
  for (int d : ids)
    if (snaps[d].have)
      w.line("amdgpu_gfx_busy_seconds_total", dev_labels_[d], nullptr, util_auto ? snaps[d].I.util_seconds : snaps[d].I.gfx_busy_seconds);
  w.head(KGS_METRIC_DOC("amdgpu_pmfw_gfx_busy_seconds_total"));
  for (int d : ids) if (snaps[d].have) w.line("amdgpu_pmfw_gfx_busy_seconds_total", dev_labels_[d], nullptr, snaps[d].I.gfx_busy_seconds);
  w.head(KGS_METRIC_DOC("kgs_util_source_seconds_total"));
  for (int d : ids) {
    if (!snaps[d].have) continue;
    w.line("kgs_util_source_seconds_total", dev_labels_[d], "source=\"counters\"", snaps[d].I.util_counter_seconds);
    w.line("kgs_util_source_seconds_total", dev_labels_[d], "source=\"pmfw\"",
           std::max(0.0, snaps[d].I.sampled_seconds - snaps[d].I.util_counter_seconds));
  }
  w.head(KGS_METRIC_DOC("kgs_util_carry_seconds"));
  for (int d : ids) if (snaps[d].have) w.line("kgs_util_carry_seconds", dev_labels_[d], nullptr, snaps[d].I.util_carry_seconds);
  w.head(KGS_METRIC_DOC("kgs_util_dropped_seconds_total"));
  for (int d : ids)
    if (snaps[d].have) w.line("kgs_util_dropped_seconds_total", dev_labels_[d], nullptr, snaps[d].I.util_dropped_seconds);
  w.head(KGS_METRIC_DOC("amdgpu_umc_busy_seconds_total"));
  for (int d : ids) if (snaps[d].have) w.line("amdgpu_umc_busy_seconds_total", dev_labels_[d], nullptr, snaps[d].I.umc_busy_seconds);
  const double full_bw = cfg_.hbm_bytes_per_s_at_full_umc;
  w.head(KGS_METRIC_DOC("amdgpu_hbm_bandwidth_bytes_per_second"));
  for (int d : ids) if (snaps[d].busy) w.line("amdgpu_hbm_bandwidth_bytes_per_second", dev_labels_[d], nullptr, snaps[d].u * 0.01 * full_bw);
  w.head(KGS_METRIC_DOC("amdgpu_hbm_bytes_total"));
  for (int d : ids) if (snaps[d].have) w.line("amdgpu_hbm_bytes_total", dev_labels_[d], nullptr, snaps[d].I.umc_busy_seconds * full_bw);

  // ---- memory ------------------------------------------------------------
  w.head(KGS_METRIC_DOC("amdgpu_hbm_used_bytes"));
  for (int d : ids) if (snaps[d].have && (snaps[d].s.valid & kFVram)) w.line_u("amdgpu_hbm_used_bytes", dev_labels_[d], nullptr, snaps[d].s.vram_used_bytes);
  w.head(KGS_METRIC_DOC("amdgpu_hbm_total_bytes"));
  for (int d : ids) w.line_u("amdgpu_hbm_total_bytes", dev_labels_[d], nullptr, be_->info(d).vram_total_bytes);

  // ---- thermals / power / clocks ----------------------------------------
  w.head(KGS_METRIC_DOC("amdgpu_temperature_celsius"));
  for (int d : ids) {
    const Snap& x = snaps[d];
    if (!x.have) continue;
    if (x.s.valid & kFTempHotspot) w.line("amdgpu_temperature_celsius", dev_labels_[d], "sensor=\"hotspot\"", x.s.temp_hotspot_c);
    if (x.s.valid & kFTempMem) w.line("amdgpu_temperature_celsius", dev_labels_[d], "sensor=\"hbm\"", x.s.temp_mem_c);
    if (x.s.valid & kFTempVrSoc) w.line("amdgpu_temperature_celsius", dev_labels_[d], "sensor=\"vrsoc\"", x.s.temp_vrsoc_c);
  }
  w.head(KGS_METRIC_DOC("amdgpu_power_watts"));
  for (int d : ids) if (snaps[d].have && (snaps[d].s.valid & kFPower)) w.line("amdgpu_power_watts", dev_labels_[d], nullptr, snaps[d].s.power_w);
  w.head(KGS_METRIC_DOC("amdgpu_energy_joules_total"));
  for (int d : ids) if (snaps[d].have) w.line("amdgpu_energy_joules_total", dev_labels_[d], nullptr, snaps[d].I.energy_joules);
  w.head(KGS_METRIC_DOC("amdgpu_clock_mhz"));
  for (int d : ids) {
    const Snap& x = snaps[d];
    if (!x.have) continue;
    if (x.s.valid & kFGfxClk) {
      double sum = 0;
      int n = 0;
      for (int c = 0; c < kMaxXcc; ++c)
        if (x.s.gfxclk_mhz[c]) { sum += x.s.gfxclk_mhz[c]; ++n; }
      if (n) w.line("amdgpu_clock_mhz", dev_labels_[d], "clock=\"gfx\"", sum / n);
    }
    if (x.s.valid & kFUclk) w.line("amdgpu_clock_mhz", dev_labels_[d], "clock=\"mem\"", x.s.uclk_mhz);
    if (x.s.valid & kFSocClk) w.line("amdgpu_clock_mhz", dev_labels_[d], "clock=\"soc\"", x.s.socclk_mhz);
  }
  w.head(KGS_METRIC_DOC("amdgpu_throttle_seconds_total"));
  for (int d : ids)
    if (snaps[d].have && (snaps[d].s.valid & kFThrottle))
      for (int r = 0; r < kThrottleReasons; ++r)
        w.line("amdgpu_throttle_seconds_total", dev_labels_[d], throttle_label(r), snaps[d].I.throttle_seconds[r]);

  // ---- interconnect ------------------------------------------------------
  w.head(KGS_METRIC_DOC("amdgpu_xgmi_read_bytes_total"));
  for (int d : ids) {
    const Snap& x = snaps[d];
    if (!x.have || !(x.s.valid & kFXgmi)) continue;
    for (int l = 0; l < kMaxXgmi; ++l) {
      if (x.s.xgmi_link_up[l] == 0xFFFF) continue;
      w.line("amdgpu_xgmi_read_bytes_total", dev_labels_[d], kLinkLabels[l],
             static_cast<double>(x.s.xgmi_read_kb[l]) * cfg_.xgmi_bytes_per_acc_unit);
    }
  }
  w.head(KGS_METRIC_DOC("amdgpu_xgmi_write_bytes_total"));
  for (int d : ids) {
    const Snap& x = snaps[d];
    if (!x.have || !(x.s.valid & kFXgmi)) continue;
    for (int l = 0; l < kMaxXgmi; ++l) {
      if (x.s.xgmi_link_up[l] == 0xFFFF) continue;
      w.line("amdgpu_xgmi_write_bytes_total", dev_labels_[d], kLinkLabels[l],
             static_cast<double>(x.s.xgmi_write_kb[l]) * cfg_.xgmi_bytes_per_acc_unit);
    }
  }
  w.head(KGS_METRIC_DOC("amdgpu_xgmi_link_up"));
  for (int d : ids) {
    const Snap& x = snaps[d];
    if (!x.have || !(x.s.valid & kFXgmi)) continue;
    for (int l = 0; l < kMaxXgmi; ++l) {
      if (x.s.xgmi_link_up[l] == 0xFFFF) continue;
      w.line("amdgpu_xgmi_link_up", dev_labels_[d], kLinkLabels[l], x.s.xgmi_link_up[l] ? 1 : 0);
    }
  }
  w.head(KGS_METRIC_DOC("amdgpu_xgmi_link_info"));
  for (int d : ids) {
    auto links = S.state(d).get_links();
    if (!links || !snaps[d].links_fresh) continue;
    std::shared_ptr<const std::string> lblock;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (link_blocks_.size() < static_cast<size_t>(nd)) link_blocks_.resize(static_cast<size_t>(nd));
      if (link_blocks_[d].first == links) lblock = link_blocks_[d].second;
    }
    if (!lblock) {  // the slow tier published a new link table: re-render this device's lines
      std::string blk;
      W b(blk, 4096, &filter_);
      for (const LinkInfo& li : *links) {
        lb.assign(dev_labels_[d]);
        kvi(lb, "link", li.link);
        kv(lb, "peer_bdf", li.peer_bdf);
        kv(lb, "link_type", li.link_type == 2 ? "xgmi" : (li.link_type == 1 ? "pcie" : "other"));
        kvi(lb, "bit_rate_gbps", li.bit_rate_gbps);
        kvi(lb, "max_bandwidth_gbps", li.max_bw_gbps);
        b.line("amdgpu_xgmi_link_info", lb, nullptr, 1);
      }
      b.finish();
      lblock = std::make_shared<const std::string>(std::move(blk));
      std::lock_guard<std::mutex> g(mu_);
      link_blocks_[d] = {links, lblock};
    }
    w.put(*lblock);
  }
  w.head(KGS_METRIC_DOC("amdgpu_ecc_errors_total"));
  for (int d : ids) {
    auto h = S.state(d).get_health();
    if (!h || !h->ecc_valid) continue;
    w.line_u("amdgpu_ecc_errors_total", dev_labels_[d], "type=\"correctable\"", h->ecc_correctable);
    w.line_u("amdgpu_ecc_errors_total", dev_labels_[d], "type=\"uncorrectable\"", h->ecc_uncorrectable);
    w.line_u("amdgpu_ecc_errors_total", dev_labels_[d], "type=\"deferred\"", h->ecc_deferred);
  }
  w.head(KGS_METRIC_DOC("amdgpu_ecc_block_errors_total"));
  for (int d : ids) {
    auto h = S.state(d).get_health();
    if (!h || !h->ecc_block_mask) continue;
    char lb[96];
    for (int b = 0; b < kEccBlocks; ++b) {
      if (!(h->ecc_block_mask & (1u << b))) continue;
      const uint64_t v[3] = {h->ecc_block_ce[b], h->ecc_block_ue[b], h->ecc_block_de[b]};
      const char* ty[3] = {"correctable", "uncorrectable", "deferred"};
      for (int k = 0; k < 3; ++k) {
        std::snprintf(lb, sizeof lb, "block=\"%s\",type=\"%s\"", kEccBlockNames[b], ty[k]);
        w.line_u("amdgpu_ecc_block_errors_total", dev_labels_[d], lb, v[k]);
      }
    }
  }
  w.head(KGS_METRIC_DOC("amdgpu_xgmi_error_status"));
  for (int d : ids) {
    auto h = S.state(d).get_health();
    if (h && h->xgmi_error_status >= 0 && snaps[d].health_fresh)
      w.line("amdgpu_xgmi_error_status", dev_labels_[d], nullptr, h->xgmi_error_status);
  }
  w.head(KGS_METRIC_DOC("amdgpu_pcie_bytes_total"));
  for (int d : ids)
    if (snaps[d].have && (snaps[d].s.valid & kFPcie))
      w.line("amdgpu_pcie_bytes_total", dev_labels_[d], nullptr,
             static_cast<double>(snaps[d].s.pcie_bw_acc_gb) * cfg_.pcie_bytes_per_acc_unit);
  w.head(KGS_METRIC_DOC("amdgpu_pcie_bandwidth_acc_total"));
  for (int d : ids) if (snaps[d].have && (snaps[d].s.valid & kFPcie)) w.line_u("amdgpu_pcie_bandwidth_acc_total", dev_labels_[d], nullptr, snaps[d].s.pcie_bw_acc_gb);

  // ---- hardware counters (PMC tier) ----------------------------------------
  bool any_pmc = false;
  for (int d : ids) any_pmc |= snaps[d].pmc_have;
  if (any_pmc) {
    w.head(KGS_METRIC_DOC("amdgpu_pmc_total"));
    for (int d : ids) {
      const Snap& x = snaps[d];
      if (!x.pmc_have) continue;
      for (int i = 0; i < kPmcCount; ++i)
        if (x.p.mask & (1u << i)) w.line_u("amdgpu_pmc_total", dev_labels_[d], pmc_counter_labels()[static_cast<size_t>(i)].c_str(), x.p.value[i]);
    }
    w.head(KGS_METRIC_DOC("amdgpu_gpu_active_seconds_total"));
    for (int d : ids) if (snaps[d].pmc_have) w.line("amdgpu_gpu_active_seconds_total", dev_labels_[d], nullptr, snaps[d].I.active_seconds);
    bool any_disp = false;
    for (int d : ids) any_disp |= snaps[d].pmc_have && snaps[d].I.dispatch_drains > 0;
    if (any_disp) {
      w.head(KGS_METRIC_DOC("amdgpu_dispatch_busy_seconds_total"));
      for (int d : ids)
        if (snaps[d].pmc_have && snaps[d].I.dispatch_drains > 0)
          w.line("amdgpu_dispatch_busy_seconds_total", dev_labels_[d], nullptr, snaps[d].I.dispatch_seconds);
      w.head(KGS_METRIC_DOC("kgs_pmc_read_cp_seconds"));
      for (int d : ids)
        if (snaps[d].pmc_have && snaps[d].I.dispatch_drains > 0)
          w.line("kgs_pmc_read_cp_seconds", dev_labels_[d], nullptr, snaps[d].I.cpc_read_us * 1e-6);
      w.head(KGS_METRIC_DOC("kgs_pmc_shader_clock_hz"));
      for (int d : ids) {
        if (!snaps[d].pmc_have || snaps[d].I.dispatch_drains == 0) continue;
        if (snaps[d].I.pmc_clk_idle_hz > 0)
          w.line("kgs_pmc_shader_clock_hz", dev_labels_[d], "kind=\"idle\"", snaps[d].I.pmc_clk_idle_hz);
        if (snaps[d].I.pmc_clk_busy_hz > 0)
          w.line("kgs_pmc_shader_clock_hz", dev_labels_[d], "kind=\"busy\"", snaps[d].I.pmc_clk_busy_hz);
      }
    }
    w.head(KGS_METRIC_DOC("amdgpu_mfma_busy_seconds_total"));
    for (int d : ids) if (snaps[d].pmc_mfma) w.line("amdgpu_mfma_busy_seconds_total", dev_labels_[d], nullptr, snaps[d].I.mfma_busy_seconds);
    w.head(KGS_METRIC_DOC("amdgpu_mfma_util_percent"));
    for (int d : ids) if (snaps[d].pmc_rates && snaps[d].r.have_mfma) w.line("amdgpu_mfma_util_percent", dev_labels_[d], nullptr, snaps[d].r.mfma_util_pct);
    w.head(KGS_METRIC_DOC("amdgpu_gpu_active_percent"));
    for (int d : ids) if (snaps[d].pmc_rates) w.line("amdgpu_gpu_active_percent", dev_labels_[d], nullptr, snaps[d].r.gpu_active_pct);
    w.head(KGS_METRIC_DOC("amdgpu_vmem_busy_percent"));
    for (int d : ids) if (snaps[d].pmc_rates && snaps[d].r.have_vmem) w.line("amdgpu_vmem_busy_percent", dev_labels_[d], nullptr, snaps[d].r.vmem_busy_pct);
    w.head(KGS_METRIC_DOC("amdgpu_gpu_clock_effective_mhz"));
    for (int d : ids) if (snaps[d].pmc_rates) w.line("amdgpu_gpu_clock_effective_mhz", dev_labels_[d], nullptr, snaps[d].r.gpu_clock_mhz);
    bool any_xcd = false;
    for (int d : ids) any_xcd |= snaps[d].pmc_rates && snaps[d].r.n_xcd > 0;
    if (any_xcd) {
      w.head(KGS_METRIC_DOC("amdgpu_mfma_util_xcc_percent"));
      for (int d : ids)
        if (snaps[d].pmc_rates)
          for (int x = 0; x < snaps[d].r.n_xcd; ++x)
            w.line("amdgpu_mfma_util_xcc_percent", dev_labels_[d], kXccLabels[x], snaps[d].r.xcd_mfma_util_pct[x]);
      bool any_xcd_vmem = false;
      for (int d : ids) any_xcd_vmem |= snaps[d].pmc_rates && snaps[d].r.n_xcd > 0 && snaps[d].r.have_xcd_vmem;
      if (any_xcd_vmem) {
        w.head(KGS_METRIC_DOC("amdgpu_vmem_busy_xcc_percent"));
        for (int d : ids)
          if (snaps[d].pmc_rates && snaps[d].r.have_xcd_vmem)
            for (int x = 0; x < snaps[d].r.n_xcd; ++x)
              w.line("amdgpu_vmem_busy_xcc_percent", dev_labels_[d], kXccLabels[x], snaps[d].r.xcd_vmem_busy_pct[x]);
      }
      w.head(KGS_METRIC_DOC("amdgpu_gpu_active_xcc_percent"));
      for (int d : ids)
        if (snaps[d].pmc_rates)
          for (int x = 0; x < snaps[d].r.n_xcd; ++x)
            w.line("amdgpu_gpu_active_xcc_percent", dev_labels_[d], kXccLabels[x], snaps[d].r.xcd_active_pct[x]);
    }
  }

  // ---- per-process attribution ------------------------------------------
  if (cfg_.per_process) {
    w.head(KGS_METRIC_DOC("amdgpu_process_hbm_bytes"));
    // Labels of every process line, built once per render and shared by the
    // five per-process families.
    std::vector<std::shared_ptr<const std::vector<ProcInfo>>> procs(static_cast<size_t>(nd));
    static thread_local std::vector<std::string> plabels;
    static thread_local std::vector<std::pair<int, const ProcInfo*>> plist;
    plist.clear();
    for (int d : ids) {
      if (!snaps[d].procs_fresh) continue;  // a stuck / failing process list: no lines, not old ones
      procs[d] = S.state(d).get_procs();
      if (procs[d]) for (const ProcInfo& p : *procs[d]) plist.emplace_back(d, &p);
    }
    if (plabels.size() < plist.size()) plabels.resize(plist.size());
    const std::string none;
    for (size_t i = 0; i < plist.size(); ++i) {
      const int d = plist[i].first;
      const ProcInfo& p = *plist[i].second;
      std::string& l = plabels[i];
      l.assign(dev_labels_[d]);
      kvi(l, "pid", p.pid);
      kv(l, "process", p.name);
      const PidOwner* po = nullptr;
      if (pown) {
        auto it = pown->find(pid_key(d, p.pid));
        if (it != pown->end()) po = &it->second;
      }
      kv(l, "pod", po ? po->pod : none);
      kv(l, "namespace", po ? po->ns : none);
      kv(l, "container", po ? po->container : none);
      kv(l, "pod_uid", po ? po->pod_uid : none);
    }
    for (size_t i = 0; i < plist.size(); ++i) w.line_u("amdgpu_process_hbm_bytes", plabels[i], nullptr, plist[i].second->vram_bytes);
    w.head(KGS_METRIC_DOC("amdgpu_process_gtt_bytes"));
    for (size_t i = 0; i < plist.size(); ++i) w.line_u("amdgpu_process_gtt_bytes", plabels[i], nullptr, plist[i].second->gtt_bytes);
    w.head(KGS_METRIC_DOC("amdgpu_process_cu_occupancy"));
    for (size_t i = 0; i < plist.size(); ++i)  // an unreadable occupancy is unknown: no line, not 0
      if (plist[i].second->cu_valid)
        w.line_u("amdgpu_process_cu_occupancy", plabels[i], nullptr, plist[i].second->cu_occupancy);
    w.head(KGS_METRIC_DOC("amdgpu_process_gfx_seconds_total"));
    for (size_t i = 0; i < plist.size(); ++i) w.line("amdgpu_process_gfx_seconds_total", plabels[i], nullptr, plist[i].second->gfx_ns * 1e-9);
    w.head(KGS_METRIC_DOC("amdgpu_process_cu_seconds_total"));
    for (size_t i = 0; i < plist.size(); ++i) w.line("amdgpu_process_cu_seconds_total", plabels[i], nullptr, plist[i].second->cu_seconds);
  }

  // ---- self metrics ------------------------------------------------------
  w.head(KGS_METRIC_DOC("kgs_up"));
  for (int d : ids) w.line("kgs_up", dev_labels_[d], nullptr, S.state(d).up.load());
  w.head(KGS_METRIC_DOC("kgs_last_sample_age_seconds"));
  for (int d : ids) {
    const int64_t t = S.state(d).last_ok_mono_ns.load();
    w.line("kgs_last_sample_age_seconds", dev_labels_[d], nullptr, t ? (now - t) * 1e-9 : -1.0);
  }
  w.head(KGS_METRIC_DOC("kgs_samples_total"));
  for (int d : ids) w.line_u("kgs_samples_total", dev_labels_[d], nullptr, snaps[d].I.distinct_samples);
  w.head(KGS_METRIC_DOC("kgs_reads_total"));
  for (int d : ids) w.line_u("kgs_reads_total", dev_labels_[d], nullptr, snaps[d].I.reads);
  w.head(KGS_METRIC_DOC("kgs_read_errors_total"));
  for (int d : ids) w.line_u("kgs_read_errors_total", dev_labels_[d], nullptr, snaps[d].I.read_errors);
  w.head(KGS_METRIC_DOC("kgs_sampler_overruns_total"));
  for (int d : ids) w.line_u("kgs_sampler_overruns_total", dev_labels_[d], nullptr, snaps[d].I.overruns);
  w.head(KGS_METRIC_DOC("kgs_device_recoveries_total"));
  for (int d : ids) w.line_u("kgs_device_recoveries_total", dev_labels_[d], nullptr, snaps[d].I.recoveries);
  w.head(KGS_METRIC_DOC("kgs_pmc_samples_total"));
  for (int d : ids) w.line_u("kgs_pmc_samples_total", dev_labels_[d], nullptr, snaps[d].I.pmc_samples);
  w.head(KGS_METRIC_DOC("kgs_pmc_read_seconds_total"));
  for (int d : ids) w.line("kgs_pmc_read_seconds_total", dev_labels_[d], nullptr, snaps[d].I.pmc_read_seconds);
  w.head(KGS_METRIC_DOC("kgs_pmc_errors_total"));
  for (int d : ids) w.line_u("kgs_pmc_errors_total", dev_labels_[d], nullptr, snaps[d].I.pmc_errors);
  if (cfg_.pmc_source != "none" && !cfg_.pmc_source.empty()) {
    w.head(KGS_METRIC_DOC("kgs_pmc_enabled"));
    for (int d : ids) w.line_u("kgs_pmc_enabled", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).pmc_on.load()));
    w.head(KGS_METRIC_DOC("kgs_pmc_releases_total"));
    for (int d : ids) w.line_u("kgs_pmc_releases_total", dev_labels_[d], nullptr, S.state(d).pmc_releases.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_stalled"));
    for (int d : ids) w.line_u("kgs_pmc_stalled", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).pmc_stalled.load()));
    w.head(KGS_METRIC_DOC("kgs_pmc_reclaims_total"));
    for (int d : ids) w.line_u("kgs_pmc_reclaims_total", dev_labels_[d], nullptr, S.state(d).pmc_reclaims.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_refreshes_total"));
    for (int d : ids) w.line_u("kgs_pmc_refreshes_total", dev_labels_[d], nullptr, S.state(d).pmc_refreshes.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_quiet"));
    for (int d : ids) w.line_u("kgs_pmc_quiet", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).pmc_quiet.load()));
    w.head(KGS_METRIC_DOC("kgs_pmc_quiet_skips_total"));
    for (int d : ids) w.line_u("kgs_pmc_quiet_skips_total", dev_labels_[d], nullptr, S.state(d).pmc_quiet_skips.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_dispatch_bound"));
    for (int d : ids)
      w.line_u("kgs_pmc_dispatch_bound", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).pmc_dbound.load()));
    w.head(KGS_METRIC_DOC("kgs_pmc_parked"));
    for (int d : ids) w.line_u("kgs_pmc_parked", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).pmc_parked.load()));
    w.head(KGS_METRIC_DOC("kgs_pmc_parks_total"));
    for (int d : ids) w.line_u("kgs_pmc_parks_total", dev_labels_[d], nullptr, S.state(d).pmc_parks.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_parked_seconds_total"));
    for (int d : ids) {
      DeviceState::ParkTime pt;  // never written: never parked
      S.state(d).park_time.load(pt);
      const int64_t cur = pt.since_ns > 0 ? std::max<int64_t>(0, mono_ns() - pt.since_ns) : 0;
      w.line("kgs_pmc_parked_seconds_total", dev_labels_[d], nullptr, (pt.ended_ns + cur) * 1e-9);
    }
    w.head(KGS_METRIC_DOC("kgs_pmc_dispatch_skips_total"));
    for (int d : ids) w.line_u("kgs_pmc_dispatch_skips_total", dev_labels_[d], nullptr, S.state(d).pmc_dbound_skips.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_failed"));
    for (int d : ids) w.line_u("kgs_pmc_failed", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).pmc_failed.load()));
    w.head(KGS_METRIC_DOC("kgs_pmc_breaker_trips_total"));
    for (int d : ids) w.line_u("kgs_pmc_breaker_trips_total", dev_labels_[d], nullptr, S.state(d).pmc_breaker_trips.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_retries_total"));
    for (int d : ids) w.line_u("kgs_pmc_retries_total", dev_labels_[d], nullptr, S.state(d).pmc_retries.load());
    w.head(KGS_METRIC_DOC("kgs_pmc_reordered_total"));
    for (int d : ids) w.line_u("kgs_pmc_reordered_total", dev_labels_[d], nullptr, S.state(d).pmc_reordered.load());
    w.head(KGS_METRIC_DOC("kgs_sampler_wake_lateness_seconds"));
    for (int d : ids) {
      const DeviceState& st = S.state(d);
      uint64_t cum = 0;
      for (int b = 0; b <= kReadHistBuckets; ++b) {
        cum += st.wake_hist[b].load(std::memory_order_relaxed);
        w.line_u("kgs_sampler_wake_lateness_seconds_bucket", dev_labels_[d], hist_le_labels()[static_cast<size_t>(b)].c_str(), cum);
      }
      w.line("kgs_sampler_wake_lateness_seconds_sum", dev_labels_[d], nullptr, st.wake_late_ns.load(std::memory_order_relaxed) * 1e-9);
      w.line_u("kgs_sampler_wake_lateness_seconds_count", dev_labels_[d], nullptr, cum);
    }
    if (pmc_) {
      std::vector<std::pair<int, CounterSource::PublishStats>> ps;
      for (int d : ids) {
        CounterSource::PublishStats p;
        if (pmc_->publish_stats(d, p)) ps.emplace_back(d, p);
      }
      if (!ps.empty()) {
        w.head(KGS_METRIC_DOC("kgs_pmc_publishes_total"));
        for (const auto& [d, p] : ps) w.line_u("kgs_pmc_publishes_total", dev_labels_[d], nullptr, p.publishes);
        w.head(KGS_METRIC_DOC("kgs_pmc_unlanded_total"));
        for (const auto& [d, p] : ps) w.line_u("kgs_pmc_unlanded_total", dev_labels_[d], nullptr, p.unlanded);
      }
    }
  }
  w.head(KGS_METRIC_DOC("kgs_sampler_thread_hung"));
  for (int d : ids) w.line_u("kgs_sampler_thread_hung", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).thread_hung.load()));
  w.head(KGS_METRIC_DOC("kgs_slow_reads_total"));
  for (int d : ids) {
    const DeviceState& st = S.state(d);
    w.line_u("kgs_slow_reads_total", dev_labels_[d], "tier=\"procs\"", st.proc_reads.load(std::memory_order_relaxed));
    w.line_u("kgs_slow_reads_total", dev_labels_[d], "tier=\"links\"", st.link_reads.load(std::memory_order_relaxed));
  }
  w.head(KGS_METRIC_DOC("kgs_slow_read_seconds_total"));
  for (int d : ids) w.line("kgs_slow_read_seconds_total", dev_labels_[d], nullptr, S.state(d).slow_ns_total.load(std::memory_order_relaxed) * 1e-9);
  w.head(KGS_METRIC_DOC("kgs_slow_errors_total"));
  for (int d : ids) {
    const DeviceState& st = S.state(d);
    w.line_u("kgs_slow_errors_total", dev_labels_[d], "tier=\"procs\"", st.proc_errors.load(std::memory_order_relaxed));
    w.line_u("kgs_slow_errors_total", dev_labels_[d], "tier=\"links\"", st.link_errors.load(std::memory_order_relaxed));
    w.line_u("kgs_slow_errors_total", dev_labels_[d], "tier=\"health\"", st.health_errors.load(std::memory_order_relaxed));
  }
  if (cfg_.per_process) {
    w.head(KGS_METRIC_DOC("kgs_process_cu_unavailable"));
    for (int d : ids)
      w.line_u("kgs_process_cu_unavailable", dev_labels_[d], nullptr,
               static_cast<uint64_t>(S.state(d).procs_cu_unavailable.load(std::memory_order_relaxed)));
  }
  w.head(KGS_METRIC_DOC("kgs_slow_last_ok_age_seconds"));
  for (int d : ids) {
    const DeviceState& st = S.state(d);
    const std::atomic<int64_t>* oks[3] = {&st.procs_ok_ns, &st.links_ok_ns, &st.health_ok_ns};
    const int64_t per[3] = {S.proc_period_ns(), S.link_period_ns(), S.link_period_ns()};
    for (int t = 0; t < 3; ++t) {
      if (per[t] <= 0) continue;
      const int64_t ok = oks[t]->load(std::memory_order_acquire);
      char tl[24];
      std::snprintf(tl, sizeof tl, "tier=\"%s\"", slow_tier_name(t));
      w.line("kgs_slow_last_ok_age_seconds", dev_labels_[d], tl, ok > 0 ? (now - ok) * 1e-9 : -1.0);
    }
  }
  w.head(KGS_METRIC_DOC("kgs_slow_call_seconds"));
  for (int d : ids) {
    const int64_t t = S.state(d).slow_call_ns.load(std::memory_order_acquire);
    w.line("kgs_slow_call_seconds", dev_labels_[d], nullptr, t > 0 && now > t ? (now - t) * 1e-9 : 0.0);
  }
  w.head(KGS_METRIC_DOC("kgs_slow_thread_hung"));
  for (int d : ids) w.line_u("kgs_slow_thread_hung", dev_labels_[d], nullptr, static_cast<uint64_t>(S.state(d).slow_hung.load()));
  w.head(KGS_METRIC_DOC("kgs_sampled_seconds_total"));
  for (int d : ids) w.line("kgs_sampled_seconds_total", dev_labels_[d], nullptr, snaps[d].I.sampled_seconds);
  w.head(KGS_METRIC_DOC("kgs_sample_read_seconds"));
  for (int d : ids) {
    const DeviceState& st = S.state(d);
    uint64_t cum = 0;
    for (int b = 0; b <= kReadHistBuckets; ++b) {
      cum += st.read_hist[b].load(std::memory_order_relaxed);
      w.line_u("kgs_sample_read_seconds_bucket", dev_labels_[d], hist_le_labels()[static_cast<size_t>(b)].c_str(), cum);
    }
    w.line("kgs_sample_read_seconds_sum", dev_labels_[d], nullptr, snaps[d].I.read_seconds);
    w.line_u("kgs_sample_read_seconds_count", dev_labels_[d], nullptr, cum);
  }
  std::string nl;
  kv(nl, "kubernetes_io_hostname", node, false);
  w.head(KGS_METRIC_DOC("kgs_scrapes_total"));
  w.line_u("kgs_scrapes_total", nl, nullptr, scrapes.load() + 1);
  w.head(KGS_METRIC_DOC("kgs_scrape_render_seconds_total"));
  w.line("kgs_scrape_render_seconds_total", nl, nullptr, render_ns_total.load() * 1e-9);
  w.head(KGS_METRIC_DOC("kgs_scrape_render_last_seconds"));
  w.line("kgs_scrape_render_last_seconds", nl, nullptr, render_ns_last.load() * 1e-9);
  w.head(KGS_METRIC_DOC("kgs_http_connections"));
  w.line_u("kgs_http_connections", nl, nullptr, http_conns_open.load());
  w.head(KGS_METRIC_DOC("kgs_http_connections_closed_total"));
  w.line_u("kgs_http_connections_closed_total", nl, "reason=\"idle\"", http_closed_idle.load());
  w.line_u("kgs_http_connections_closed_total", nl, "reason=\"limit\"", http_closed_limit.load());
  w.head(KGS_METRIC_DOC("kgs_build_info"));
  {
    std::string lb = nl;
    kv(lb, "version", "0.1.0");
    kv(lb, "backend", be_->name());
    kv(lb, "pmc_source", pmc_ ? pmc_->name() : std::string("none"));
    kv(lb, "sample_hz", std::to_string(S.hz()));
    w.line("kgs_build_info", lb, nullptr, 1);
  }
  if (extra && !filter_.active()) {
    w.put(*extra);
  } else if (extra) {  // the control plane's text block: filter it line by line
    const std::string& x = *extra;
    size_t i = 0;
    while (i < x.size()) {
      size_t e = x.find('\n', i);
      if (e == std::string::npos) e = x.size();
      size_t s = i;
      if (x.compare(i, 7, "# HELP ") == 0 || x.compare(i, 7, "# TYPE ") == 0) s = i + 7;
      size_t n = s;
      while (n < e && x[n] != '{' && x[n] != ' ') ++n;
      if (filter_.allowed(x.substr(s, n - s))) {
        w.put(x.data() + i, e - i);
        w.put('\n');
      }
      i = e + 1;
    }
  }
  w.finish();
  last_render_bytes_.store(out.size(), std::memory_order_relaxed);

  const int64_t dt = mono_ns() - t0;
  scrapes.fetch_add(1);
  render_ns_total.fetch_add(static_cast<uint64_t>(dt));
  render_ns_last.store(static_cast<uint64_t>(dt));
}

}  // namespace kgs
