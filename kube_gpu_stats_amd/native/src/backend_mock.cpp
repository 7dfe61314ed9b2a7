// Deterministic N-GPU mock provider (tests + BASELINE.json config 1).
//
// Every quantity is a closed-form function of *firmware time* (time quantised
// to the PMFW cadence, 20 ms by default as measured on MI355X), so tests can
// check the exporter's integrals against analytic values.  Fault injection
// covers the failure modes of SURVEY.md §5.3: read errors, stalls, a device
// that disappears, accumulator wrap.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <ctime>
#include <mutex>
#include <thread>

#include "kgs/backend.h"

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

class MockBackend final : public Backend {
 public:
  explicit MockBackend(const MockConfig& c) : cfg_(c), t0_(mono_ns()) {
    for (int d = 0; d < cfg_.n_gpus; ++d) {
      DeviceInfo in;
      in.index = d;
      char bdf[32];
      std::snprintf(bdf, sizeof bdf, "0000:%02x:00.0", 0x11 + 0x10 * d);
      in.bdf = bdf;
      char uuid[64];
      std::snprintf(uuid, sizeof uuid, "mock-75a3-0000-1000-80b8-%012d", d);
      in.uuid = uuid;
      in.serial = "MOCK" + std::to_string(d);
      in.market_name = "AMD Instinct MI355 OAM";
      in.gpu_type = gpu_type_from_market_name(in.market_name);
      in.gfx_target = "gfx950";
      in.numa_node = d < cfg_.n_gpus / 2 ? 0 : 1;
      in.num_cu = 256;
      in.num_xcc = 8;
      in.vram_total_bytes = cfg_.vram_total_bytes;
      in.kfd_gpu_id = 40000 + d;
      in.kfd_node = 2 + d;
      in.drm_card = 8 * d;
      in.hip_id = d;
      in.compute_partition = "SPX";
      in.memory_partition = "NPS1";
      in.partition_id = 0;
      infos_.push_back(in);
      rng_.push_back(cfg_.seed * 0x9E3779B97F4A7C15ull + static_cast<uint64_t>(d) + 1);
    }
    rng_mu_ = std::vector<std::mutex>(static_cast<size_t>(cfg_.n_gpus));
  }

  std::string name() const override { return "mock"; }
  int device_count() const override { return cfg_.n_gpus; }
  const DeviceInfo& info(int d) const override { return infos_[d]; }

  // Utilisation in percent at firmware time t (seconds).
  double util(int d, double t) const {
    const double u = cfg_.util_base + cfg_.util_amp * std::sin(kTwoPi * t / cfg_.util_period_s + 0.7 * d);
    return u < 0 ? 0 : (u > 100 ? 100 : u);
  }
  // ∫_0^t util dt (percent·seconds), closed form (clamping ignored when base±amp ∈ [0,100]).
  double util_integral(int d, double t) const {
    const double w = kTwoPi / cfg_.util_period_s, ph = 0.7 * d;
    return cfg_.util_base * t + cfg_.util_amp / w * (std::cos(ph) - std::cos(w * t + ph));
  }

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
    if (cfg_.stall_s > 0) std::this_thread::sleep_for(std::chrono::duration<double>(cfg_.stall_s));
    if (gone(d, t)) return -2;
    if (cfg_.fail_rate > 0 && next_uniform(d) < cfg_.fail_rate) return -1;
    const int64_t rs = reset_ns_.load(std::memory_order_acquire);
    if (d == cfg_.vanish_dev && rs != 0) t = (now - rs) * 1e-9;  // firmware clock restarted

    // Firmware time: quantised to the PMFW cadence.
    const double tf = std::floor(t / cfg_.fw_period_s) * cfg_.fw_period_s;
    const double u = util(d, tf);
    s.fw_ts = static_cast<uint64_t>(tf * 1e8) + 1000;  // 10 ns units, never 0
    s.gfx_busy_pct = static_cast<float>(u);
    s.umc_busy_pct = static_cast<float>(u * 0.5);
    s.num_xcc = 8;
    for (int x = 0; x < kMaxXcc; ++x) s.gfx_busy_xcc[x] = static_cast<float>(u);
    // Accumulators in PMFW units: accumulation_counter ticks once per ms,
    // gfx_activity_acc adds the busy percent every tick.
    const double ms = tf * 1000.0;
    s.accumulation_counter = static_cast<uint64_t>(std::llround(ms));
    s.gfx_activity_acc = static_cast<uint64_t>(std::llround(util_integral(d, tf) * 1000.0));
    s.mem_activity_acc = static_cast<uint64_t>(std::llround(util_integral(d, tf) * 500.0));
    for (int x = 0; x < kMaxXcc; ++x) s.gfx_busy_acc_xcc[x] = s.gfx_activity_acc;
    s.valid |= kFXccAcc;
    s.temp_hotspot_c = static_cast<float>(40 + 0.4 * u);
    s.temp_mem_c = static_cast<float>(35 + 0.2 * u);
    s.temp_vrsoc_c = static_cast<float>(38 + 0.1 * u);
    s.power_w = static_cast<float>(200 + 8 * u);
    // energy: ∫ (200 + 8u) dt in 2^-16 J units
    double ej = 200 * tf + 8 * util_integral(d, tf);
    uint64_t e = static_cast<uint64_t>(ej * 65536.0);
    if (cfg_.energy_wrap_at) e %= cfg_.energy_wrap_at;
    s.energy_acc = e;
    for (int x = 0; x < kMaxXcc; ++x) s.gfxclk_mhz[x] = static_cast<uint32_t>(2400 - 4 * u);
    s.uclk_mhz = 2000;
    s.socclk_mhz = 1200;
    for (int l = 0; l < kMaxXgmi; ++l) {
      const bool up = l >= 1 && l < cfg_.n_gpus;
      // 1 GB/s per link at 100 % utilisation, link 0 is the unused self-port.
      const uint64_t kb = up ? static_cast<uint64_t>(util_integral(d, tf) * 1e4) : 0;
      s.xgmi_read_kb[l] = kb;
      s.xgmi_write_kb[l] = kb / 2;
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
    s.mono_ns = mono_ns();
    s.wall_ns = wall_ns();
    return 0;
  }

  int read_procs(int d, std::vector<ProcInfo>& out) override {
    out.clear();
    const double t = (mono_ns() - t0_) * 1e-9;
    if (gone(d, t)) return -2;
    for (int k = 0; k < 1 + (d % 2); ++k) {
      ProcInfo p;
      p.pid = static_cast<uint32_t>(100000 + d * 10 + k);
      p.name = "python3";
      p.vram_bytes = (1ull << 30) * static_cast<uint64_t>(k + 1);
      p.gfx_ns = static_cast<uint64_t>(util_integral(d, t) * 1e7 / (1 + (d % 2)));
      p.cu_occupancy = 128;
      out.push_back(p);
    }
    return 0;
  }

  int read_links(int d, std::vector<LinkInfo>& out) override {
    out.clear();
    const double t = (mono_ns() - t0_) * 1e-9;
    int l = 0;
    for (int p = 0; p < cfg_.n_gpus; ++p) {
      if (p == d) continue;
      LinkInfo li;
      li.link = ++l;
      li.peer_bdf = infos_[p].bdf;
      li.link_type = 2;
      li.bit_rate_gbps = 38;
      li.max_bw_gbps = 608;
      li.read_kb = static_cast<uint64_t>(util_integral(d, t) * 1e4);
      li.write_kb = li.read_kb / 2;
      out.push_back(li);
    }
    return 0;
  }

  int read_health(int d, HealthInfo& out) override {
    const double t = (mono_ns() - t0_) * 1e-9;
    out.ecc_valid = true;
    out.ecc_correctable = static_cast<uint64_t>(t * static_cast<double>(cfg_.ecc_correctable_per_s));
    out.ecc_uncorrectable = 0;
    out.ecc_deferred = 0;
    out.xgmi_error_status = 0;
    return 0;
  }

  int topology(std::vector<TopoEdge>& out) override {
    out.clear();
    for (int a = 0; a < cfg_.n_gpus; ++a)
      for (int b = 0; b < cfg_.n_gpus; ++b)
        if (a != b) out.push_back(TopoEdge{a, b, 2, 1, 15});
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

  MockConfig cfg_;
  int64_t t0_;
  std::atomic<int64_t> reset_ns_{0};
  std::vector<DeviceInfo> infos_;
  std::vector<uint64_t> rng_;
  std::vector<std::mutex> rng_mu_;
};

}  // namespace

std::unique_ptr<Backend> make_mock_backend(const MockConfig& cfg) { return std::make_unique<MockBackend>(cfg); }

}  // namespace kgs
