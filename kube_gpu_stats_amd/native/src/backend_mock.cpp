// Deterministic N-GPU mock provider (tests + BASELINE.json config 1).
//
// Every quantity is a closed-form function of *firmware time* (time quantised
// to the PMFW cadence, 20 ms by default as measured on MI355X), so tests can
// check the exporter's integrals against analytic values.  Fault injection
// covers the failure modes of SURVEY.md §5.3: read errors, stalls, a device
// that disappears, accumulator wrap.
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <ctime>
#include <mutex>
#include <thread>

#include <algorithm>
#include <array>
#include <memory>

#include "kgs/backend.h"
#include "kgs/gpu_metrics.h"

namespace kgs {
namespace {

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}
int64_t wall_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

constexpr double kTwoPi = 6.283185307179586;

double clamp100(double u) { return u < 0 ? 0 : (u > 100 ? 100 : u); }

int parts_of(const MockConfig& c) {
  const uint32_t n = partitions_of_mode(c.compute_partition.c_str());
  return n == 0 ? 1 : static_cast<int>(n);
}

// Curve k: busy percent at t, and its integral from 0 (percent·s).
double curve_util(const MockConfig& c, int k, double t) {
  if (c.square_duty > 0) {
    const double ph = t / c.util_period_s - std::floor(t / c.util_period_s);
    return ph < c.square_duty ? clamp100(c.util_base + c.util_amp) : clamp100(c.util_base - c.util_amp);
  }
  return clamp100(c.util_base + c.util_amp * std::sin(kTwoPi * t / c.util_period_s + 0.7 * k));
}
double curve_integral(const MockConfig& c, int k, double t) {
  if (c.square_duty > 0) {
    const double T = c.util_period_s, on = c.square_duty * T;
    const double hi = clamp100(c.util_base + c.util_amp), lo = clamp100(c.util_base - c.util_amp);
    const double n = std::floor(t / T), r = t - n * T;
    return n * (on * hi + (T - on) * lo) + std::min(r, on) * hi + std::max(0.0, r - on) * lo;
  }
  // closed form (clamping ignored when base ± amp stays inside [0, 100])
  const double w = kTwoPi / c.util_period_s, ph = 0.7 * k;
  return c.util_base * t + c.util_amp / w * (std::cos(ph) - std::cos(w * t + ph));
}

// XCC x of physical GPU g runs curve g·8 + x when partitioned; an SPX device d runs curve d.
int xcc_curve(const MockConfig& c, int gpu, int x) { return gpu * kMaxXcc + x; }

void sleep_s(double s) {
  if (s > 0) std::this_thread::sleep_for(std::chrono::duration<double>(s));
}

// The load as the PMFW GFX busy sees it (MockConfig::pmfw_busy_floor): a square
// wave's low level lifted to the floor.
MockConfig pmfw_view(const MockConfig& c) {
  MockConfig f = c;
  if (c.pmfw_busy_floor > 0 && c.square_duty > 0) {
    const double hi = std::max(clamp100(c.util_base + c.util_amp), c.pmfw_busy_floor);
    const double lo = std::max(clamp100(c.util_base - c.util_amp), c.pmfw_busy_floor);
    f.util_base = 0.5 * (hi + lo);
    f.util_amp = 0.5 * (hi - lo);
  }
  return f;
}

class MockBackend final : public Backend {
 public:
  explicit MockBackend(const MockConfig& c) : cfg_(c), pmfw_(pmfw_view(c)), t0_(mono_ns()), parts_(parts_of(c)) {
    const int xcc_per = kMaxXcc / parts_;
    for (int g = 0; g < cfg_.n_gpus; ++g) {
      for (int p = 0; p < parts_; ++p) {
        const int d = g * parts_ + p;
        DeviceInfo in;
        in.index = d;
        char bdf[32];
        std::snprintf(bdf, sizeof bdf, "0000:%02x:00.0", 0x11 + 0x10 * g);
        in.bdf = bdf;  // every partition of a GPU shares its PCI function
        char uuid[64];
        std::snprintf(uuid, sizeof uuid, "mock-75a3-0000-1000-80b8-%012d", d);
        in.uuid = uuid;
        in.serial = "MOCK" + std::to_string(g);
        in.market_name = "AMD Instinct MI355 OAM";
        in.gpu_type = gpu_type_from_market_name(in.market_name);
        in.gfx_target = "gfx950";
        in.numa_node = g < cfg_.n_gpus / 2 ? 0 : 1;
        in.num_cu = 256 / parts_;
        in.num_xcc = static_cast<uint32_t>(xcc_per);
        in.xcc_first = static_cast<uint32_t>(p * xcc_per);
        in.vram_total_bytes = cfg_.vram_total_bytes;
        in.kfd_gpu_id = 40000 + d;
        in.kfd_node = 2 + d;
        in.drm_card = 8 * g + p;
        in.hip_id = d;
        in.compute_partition = cfg_.compute_partition;
        in.memory_partition = "NPS1";
        in.partition_id = p;
        infos_.push_back(in);
        rng_.push_back(cfg_.seed * 0x9E3779B97F4A7C15ull + static_cast<uint64_t>(d) + 1);
      }
    }
    rng_mu_ = std::vector<std::mutex>(infos_.size());
    for (int g = 0; g < cfg_.n_gpus; ++g) inj_.push_back(std::make_unique<LinkInj>());
  }

  // Port l (1 .. n_gpus-1) of GPU g faces the l-th other GPU in index order
  // (port 0 is the disabled self port, as on MI355X); read_links reports the same.
  int link_of(int g, int peer) const { return peer < g ? peer + 1 : peer; }

  int inject_xgmi(int src, int dst, uint64_t bytes) override {
    const int gs = src / parts_, gd = dst / parts_;
    if (src < 0 || dst < 0 || src >= device_count() || dst >= device_count() || gs == gd) return -1;
    const uint64_t kb = bytes / 1024;
    inj_[static_cast<size_t>(gs)]->wr[static_cast<size_t>(link_of(gs, gd))].fetch_add(kb);
    inj_[static_cast<size_t>(gd)]->rd[static_cast<size_t>(link_of(gd, gs))].fetch_add(kb);
    return 0;
  }

  std::string name() const override { return "mock"; }
  int device_count() const override { return static_cast<int>(infos_.size()); }
  const DeviceInfo& info(int d) const override { return infos_[d]; }

  double util(int d, double t) const { return mock_device_util(cfg_, d, t); }
  double util_integral(int d, double t) const { return mock_device_util_integral(cfg_, d, t); }
  // What the PMFW GFX busy reads (the floor of MockConfig::pmfw_busy_floor applied).
  double pmfw_util(int d, double t) const {
    return std::max(mock_device_util(pmfw_, d, t), cfg_.pmfw_busy_floor);
  }
  double pmfw_util_integral(int d, double t) const { return mock_device_util_integral(pmfw_, d, t); }

  // A vanished device stays gone for vanish_for_s, then needs recover(): like a
  // GPU reset, the firmware restarts with its accumulators at zero.
  bool gone(int d, double t) const {
    if (cfg_.vanish_dev != d || t < cfg_.vanish_after_s) return false;
    if (cfg_.vanish_for_s < 0 || t < cfg_.vanish_after_s + cfg_.vanish_for_s) return true;
    return reset_ns_.load(std::memory_order_acquire) == 0;
  }

  int recover(int d) override {
    const int64_t now = mono_ns();
    if (cfg_.vanish_dev != d || cfg_.vanish_for_s < 0) return gone(d, (now - t0_) * 1e-9) ? -1 : 0;
    if ((now - t0_) * 1e-9 < cfg_.vanish_after_s + cfg_.vanish_for_s) return -1;
    int64_t expect = 0;
    reset_ns_.compare_exchange_strong(expect, now, std::memory_order_acq_rel);
    return 0;
  }

  int read_metrics(int d, GpuSample& s) override {
    const int64_t now = mono_ns();
    double t = (now - t0_) * 1e-9;
    sleep_s(cfg_.metrics_latency_s);
    if (cfg_.stall_s > 0) std::this_thread::sleep_for(std::chrono::duration<double>(cfg_.stall_s));
    if (gone(d, t)) return -2;
    if (cfg_.fail_rate > 0 && next_uniform(d) < cfg_.fail_rate) return -1;
    const int64_t rs = reset_ns_.load(std::memory_order_acquire);
    if (d == cfg_.vanish_dev && rs != 0) t = (now - rs) * 1e-9;  // firmware clock restarted

    // Firmware time: quantised to the PMFW cadence.
    const double tf = std::floor(t / cfg_.fw_period_s) * cfg_.fw_period_s;
    // The PMFW table is per physical GPU: every XCC's busy and accumulator, the
    // chip-wide mean, then (partitions) the device's own XCCs.
    const int g = d / parts_;
    const double u = parts_ > 1 ? chip_util(g, tf) : pmfw_util(d, tf);
    const double ui = parts_ > 1 ? chip_util_integral(g, tf) : pmfw_util_integral(d, tf);
    s.fw_ts = static_cast<uint64_t>(tf * 1e8) + 1000;  // 10 ns units, never 0
    s.gfx_busy_pct = static_cast<float>(u);
    s.umc_busy_pct = static_cast<float>(u * 0.5);
    s.num_xcc = 8;
    // Accumulators in PMFW units: accumulation_counter ticks once per ms,
    // gfx_activity_acc adds the busy percent every tick.
    const double ms = tf * 1000.0;
    s.accumulation_counter = static_cast<uint64_t>(std::llround(ms));
    s.gfx_activity_acc = static_cast<uint64_t>(std::llround(ui * 1000.0));
    s.mem_activity_acc = static_cast<uint64_t>(std::llround(ui * 500.0));
    s.throttle_res_acc[1] = static_cast<uint64_t>(std::llround(ms * cfg_.ppt_frac));  // ppt
    s.ppt_residency_acc = s.throttle_res_acc[1];
    s.valid |= kFThrottle;
    for (int x = 0; x < kMaxXcc; ++x) {
      if (parts_ > 1) {
        s.gfx_busy_xcc[x] = static_cast<float>(curve_util(cfg_, xcc_curve(cfg_, g, x), tf));
        s.gfx_busy_acc_xcc[x] = static_cast<uint64_t>(std::llround(curve_integral(cfg_, xcc_curve(cfg_, g, x), tf) * 1000.0));
      } else {
        s.gfx_busy_xcc[x] = static_cast<float>(u);
        s.gfx_busy_acc_xcc[x] = s.gfx_activity_acc;
      }
    }
    s.valid |= kFXccAcc;
    s.temp_hotspot_c = static_cast<float>(40 + 0.4 * u);
    s.temp_mem_c = static_cast<float>(35 + 0.2 * u);
    s.temp_vrsoc_c = static_cast<float>(38 + 0.1 * u);
    s.power_w = static_cast<float>(200 + 8 * u);
    // energy: ∫ (200 + 8u) dt in 2^-16 J units — of the socket: partitions of one
    // GPU read the same accumulator, as on hardware
    double ej = 200 * tf + 8 * ui;
    uint64_t e = static_cast<uint64_t>(ej * 65536.0);
    if (cfg_.energy_wrap_at) e %= cfg_.energy_wrap_at;
    s.energy_acc = e;
    for (int x = 0; x < kMaxXcc; ++x) s.gfxclk_mhz[x] = static_cast<uint32_t>(2400 - 4 * u);
    s.uclk_mhz = 2000;
    s.socclk_mhz = 1200;
    for (int l = 0; l < kMaxXgmi; ++l) {
      const bool up = l >= 1 && l < cfg_.n_gpus;
      // 1 GB/s per link at 100 % utilisation, link 0 is the unused self-port.
      const uint64_t kb = up && cfg_.xgmi_bg ? static_cast<uint64_t>(util_integral(d, tf) * 1e4) : 0;
      const LinkInj& in = *inj_[static_cast<size_t>(g)];
      s.xgmi_read_kb[l] = kb + in.rd[static_cast<size_t>(l)].load();
      s.xgmi_write_kb[l] = kb / 2 + in.wr[static_cast<size_t>(l)].load();
      s.xgmi_link_up[l] = up ? 1 : 0xFFFF;
    }
    s.xgmi_link_speed_gbps = 38;
    s.xgmi_link_width = 16;
    s.pcie_link_width = 16;
    s.pcie_link_speed_01gts = 320;
    s.pcie_bw_acc_gb = static_cast<uint64_t>(tf * 3);
    s.vram_total_bytes = cfg_.vram_total_bytes;
    s.vram_used_bytes = (1ull << 30) + static_cast<uint64_t>(u * 1e9);
    s.valid |= kFGfxBusy | kFUmcBusy | kFGfxBusyXcc | kFTempHotspot | kFTempMem | kFTempVrSoc | kFPower |
               kFEnergy | kFGfxClk | kFUclk | kFSocClk | kFXgmi | kFPcie | kFVram | kFAcc | kFFwTs;
    if (parts_ > 1) restrict_to_xccs(s, infos_[d].xcc_first, infos_[d].num_xcc);
    s.mono_ns = mono_ns();
    s.wall_ns = wall_ns();
    return 0;
  }

  // Chip-wide mean over the 8 XCC curves of physical GPU g (partitioned mock).
  double chip_util(int g, double t) const {
    double u = 0;
    for (int x = 0; x < kMaxXcc; ++x) u += curve_util(cfg_, xcc_curve(cfg_, g, x), t);
    return u / kMaxXcc;
  }
  double chip_util_integral(int g, double t) const {
    double u = 0;
    for (int x = 0; x < kMaxXcc; ++x) u += curve_integral(cfg_, xcc_curve(cfg_, g, x), t);
    return u / kMaxXcc;
  }

  // Slow-tier fault injection (MockConfig::slow_fault_*): 0 = no fault, -1 = the
  // call fails.  A hang blocks here, before the management-library lock.
  int slow_fault(int d, const char* tier) {
    if (d != cfg_.slow_fault_dev || cfg_.slow_fault_tier != tier) return 0;
    if ((mono_ns() - t0_) * 1e-9 < cfg_.slow_fault_after_s) return 0;
    if (cfg_.slow_fault_kind == "error") return -1;
    const int64_t end = cfg_.slow_hang_s < 0 ? INT64_MAX : mono_ns() + static_cast<int64_t>(cfg_.slow_hang_s * 1e9);
    while (mono_ns() < end) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    return 0;
  }

  int read_procs(int d, std::vector<ProcInfo>& out) override {
    if (slow_fault(d, "procs") != 0) return -1;
    std::lock_guard<std::mutex> lk(smi_mu_);
    sleep_s(cfg_.proc_latency_s);
    out.clear();
    const double t = (mono_ns() - t0_) * 1e-9;
    if (gone(d, t)) return -2;
    const bool shares = !cfg_.proc_cu_share.empty();
    const int n = shares ? static_cast<int>(cfg_.proc_cu_share.size()) : 1 + (d % 2);
    for (int k = 0; k < n; ++k) {
      ProcInfo p;
      p.pid = static_cast<uint32_t>(100000 + d * 10 + k);
      p.name = "python3";
      p.vram_bytes = (1ull << 30) * static_cast<uint64_t>(k + 1);
      p.gfx_ns = static_cast<uint64_t>(util_integral(d, t) * 1e7 / n);
      p.cu_occupancy = shares ? static_cast<uint32_t>(std::lround(cfg_.proc_cu_share[static_cast<size_t>(k)] *
                                                                  infos_[static_cast<size_t>(d)].num_cu))
                              : 128;
      if (k == cfg_.proc_cu_fail) {  // its KFD stats unreadable (a process tearing down)
        p.cu_valid = false;
        p.cu_occupancy = 0;
      }
      out.push_back(p);
    }
    return 0;
  }

  int read_links(int d, std::vector<LinkInfo>& out) override {
    if (slow_fault(d, "links") != 0) return -1;
    std::lock_guard<std::mutex> lk(smi_mu_);
    sleep_s(cfg_.link_latency_s);
    out.clear();
    const double t = (mono_ns() - t0_) * 1e-9;
    int l = 0;
    const int g = d / parts_;
    for (int p = 0; p < cfg_.n_gpus; ++p) {
      if (p == g) continue;
      LinkInfo li;
      li.link = ++l;  // port 0 is the disabled self port, as on MI355X
      li.peer_bdf = infos_[static_cast<size_t>(p * parts_)].bdf;
      li.link_type = 2;
      li.bit_rate_gbps = 38;
      li.max_bw_gbps = 608;
      const uint64_t bg = cfg_.xgmi_bg ? static_cast<uint64_t>(util_integral(d, t) * 1e4) : 0;
      li.read_kb = bg + inj_[static_cast<size_t>(g)]->rd[static_cast<size_t>(li.link)].load();
      li.write_kb = bg / 2 + inj_[static_cast<size_t>(g)]->wr[static_cast<size_t>(li.link)].load();
      out.push_back(li);
    }
    if (g == cfg_.xgmi_swap_dev && out.size() >= 2) std::swap(out[0].peer_bdf, out[1].peer_bdf);
    return 0;
  }

  int read_health(int d, HealthInfo& out) override {
    if (slow_fault(d, "health") != 0) return -1;
    std::lock_guard<std::mutex> lk(smi_mu_);
    sleep_s(cfg_.health_latency_s);
    const double t = (mono_ns() - t0_) * 1e-9;
    out.ecc_valid = true;
    out.ecc_correctable = static_cast<uint64_t>(t * static_cast<double>(cfg_.ecc_correctable_per_s));
    out.ecc_uncorrectable = 0;
    out.ecc_deferred = 0;
    // UMC (HBM) carries the correctable errors; GFX and xGMI are enabled and clean.
    out.ecc_block_mask = (1u << 0) | (1u << 2) | (1u << 7);
    out.ecc_block_ce[0] = out.ecc_correctable;
    out.xgmi_error_status = 0;
    return 0;
  }

  int topology(std::vector<TopoEdge>& out) override {
    out.clear();
    const int n = device_count();
    for (int a = 0; a < n; ++a)
      for (int b = 0; b < n; ++b) {
        if (a == b) continue;
        // partitions of one GPU share the die fabric: 0 hops; other GPUs: one xGMI hop
        if (a / parts_ == b / parts_) out.push_back(TopoEdge{a, b, 2, 0, 0});
        else out.push_back(TopoEdge{a, b, 2, 1, 15});
      }
    return 0;
  }

 private:
  double next_uniform(int d) {
    std::lock_guard<std::mutex> g(rng_mu_[static_cast<size_t>(d)]);
    uint64_t& x = rng_[static_cast<size_t>(d)];
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return (x >> 11) * (1.0 / 9007199254740992.0);
  }

  struct LinkInj {  // injected peer-copy KB per port of one physical GPU
    std::array<std::atomic<uint64_t>, kMaxXgmi> rd{}, wr{};
  };

  MockConfig cfg_;
  MockConfig pmfw_;        // cfg_ as the PMFW busy sees it (pmfw_busy_floor)
  int64_t t0_;
  int parts_;              // devices per physical GPU (compute partitions)
  std::vector<std::unique_ptr<LinkInj>> inj_;
  std::mutex smi_mu_;      // the management library's process-wide lock (latency model)
  std::atomic<int64_t> reset_ns_{0};
  std::vector<DeviceInfo> infos_;
  std::vector<uint64_t> rng_;
  std::vector<std::mutex> rng_mu_;
};

}  // namespace

std::unique_ptr<Backend> make_mock_backend(const MockConfig& cfg) { return std::make_unique<MockBackend>(cfg); }

double mock_device_util(const MockConfig& cfg, int dev, double t) {
  const int parts = parts_of(cfg);
  if (parts == 1) return curve_util(cfg, dev, t);
  const int g = dev / parts, p = dev % parts, per = kMaxXcc / parts;
  double u = 0;
  for (int x = p * per; x < (p + 1) * per; ++x) u += curve_util(cfg, xcc_curve(cfg, g, x), t);
  return u / per;
}

double mock_device_util_integral(const MockConfig& cfg, int dev, double t) {
  const int parts = parts_of(cfg);
  if (parts == 1) return curve_integral(cfg, dev, t);
  const int g = dev / parts, p = dev % parts, per = kMaxXcc / parts;
  double u = 0;
  for (int x = p * per; x < (p + 1) * per; ++x) u += curve_integral(cfg, xcc_curve(cfg, g, x), t);
  return u / per;
}

}  // namespace kgs
