// Counter-source plumbing: counter catalogue, derived rates, the mock source and
// the dlopen bridge to the counter readers (libkgs_pmc_aql.so, the direct CP
// reader; libkgs_pmc.so, rocprofiler-sdk device counting, tests only).
#include "kgs/pmc.h"

#include <deque>
#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <thread>
#include <ctime>
#include <mutex>

namespace kgs {

namespace {
const char* const kNames[kPmcCount] = {
    "GRBM_COUNT", "GRBM_SPI_BUSY", "SQ_VALU_MFMA_BUSY_CYCLES", "TA_TA_BUSY", "CPC_CPC_STAT_BUSY",
};
const int kReduce[kPmcCount] = {kReduceMax, kReduceMax, kReduceSum, kReduceAvg, kReduceMax};

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}
}  // namespace

const char* pmc_counter_name(int idx) { return (idx >= 0 && idx < kPmcCount) ? kNames[idx] : "?"; }
int pmc_counter_reduce(int idx) { return (idx >= 0 && idx < kPmcCount) ? kReduce[idx] : kReduceSum; }

uint32_t pmc_set_mask(const std::string& name) {
  if (name == "base" || name.empty()) return kPmcSetBase;
  if (name == "full") return kPmcSetFull;
  if (name == "util") return kPmcSetUtil;
  return 0;
}

PmcRates pmc_rates(const PmcSample& a, const PmcSample& b, int num_cu) {
  PmcRates r;
  const double dt = (b.mono_ns - a.mono_ns) * 1e-9;
  if (dt <= 0) return r;
  r.dt_s = dt;
  auto d = [&](int i) {
    return b.value[i] >= a.value[i] ? static_cast<double>(b.value[i] - a.value[i]) : 0.0;
  };
  const double cnt = d(kPmcGrbmCount), act = d(kPmcGrbmActive);
  const double cu = num_cu > 0 ? num_cu : 256;
  if (cnt > 0) r.gpu_active_pct = 100.0 * act / cnt;
  r.have_vmem = (a.mask & b.mask & (1u << kPmcTaBusy)) != 0;
  r.have_mfma = (a.mask & b.mask & (1u << kPmcMfmaBusy)) != 0;
  if (act > 0) {
    // Shares of the active (SPI-busy) cycles, capped: over a single ~125 µs drain a
    // kernel's tail can leave MFMA / TA cycles in an interval whose SPI-busy count
    // is a few hundred clocks.
    if (r.have_mfma) r.mfma_util_pct = std::min(100.0, 100.0 * d(kPmcMfmaBusy) / (act * cu * 4.0));
    if (r.have_vmem) r.vmem_busy_pct = std::min(100.0, 100.0 * d(kPmcTaBusy) / act);
  }
  r.gpu_clock_mhz = cnt / dt * 1e-6;
  const uint32_t nx = std::min(a.n_xcd, b.n_xcd);
  if (nx > 0 && nx <= static_cast<uint32_t>(kMaxXcc) && a.n_xcd == b.n_xcd) {
    r.n_xcd = static_cast<int>(nx);
    const double simds = cu / nx * 4.0;
    for (uint32_t x = 0; x < nx; ++x) {
      const double ax = b.xcd_active[x] >= a.xcd_active[x] ? static_cast<double>(b.xcd_active[x] - a.xcd_active[x]) : 0.0;
      const double mx = b.xcd_mfma[x] >= a.xcd_mfma[x] ? static_cast<double>(b.xcd_mfma[x] - a.xcd_mfma[x]) : 0.0;
      if (cnt > 0) r.xcd_active_pct[x] = 100.0 * ax / cnt;
      if (ax > 0) r.xcd_mfma_util_pct[x] = std::min(100.0, 100.0 * mx / (ax * simds));
    }
    r.have_xcd_vmem = r.have_vmem;
    if (r.have_xcd_vmem)
      for (uint32_t x = 0; x < nx; ++x) {
        const double ax = b.xcd_active[x] >= a.xcd_active[x] ? static_cast<double>(b.xcd_active[x] - a.xcd_active[x]) : 0.0;
        const double tx = b.xcd_ta[x] >= a.xcd_ta[x] ? static_cast<double>(b.xcd_ta[x] - a.xcd_ta[x]) : 0.0;
        if (ax > 0) r.xcd_vmem_busy_pct[x] = std::min(100.0, 100.0 * tx / (cu / nx) / ax);
      }
  }
  return r;
}

namespace {

class MockCounterSource final : public CounterSource {
 public:
  MockCounterSource(const MockConfig& b, const MockPmcConfig& c, int n_dev)
      : b_(b), c_(c), t0_(mono_ns()), restart_(static_cast<size_t>(std::max(n_dev, 1)), 0),
        restart_reads_(static_cast<size_t>(std::max(n_dev, 1)), 0),
        delayed_(static_cast<size_t>(std::max(n_dev, 1))),
        se_last_(static_cast<size_t>(std::max(n_dev, 1))),
        se_n_(static_cast<size_t>(std::max(n_dev, 1)), 0) {
    for (int d = 0; d < std::max(n_dev, 1); ++d) fault_.push_back(std::make_unique<Fault>());
  }
  std::string name() const override { return "mock"; }
  int release(int) override { return 0; }
  int acquire(int dev) override {  // like a re-START: the counts restart at 0
    if (dev < 0 || static_cast<size_t>(dev) >= restart_.size()) return -1;
    if (dev == c_.acquire_fail_dev && hung(dev)) return -1;
    if (fault_[static_cast<size_t>(dev)]->stalled.load()) return -1;  // START waits behind the stall too
    restart_[static_cast<size_t>(dev)] = mono_ns();
    restart_reads_[static_cast<size_t>(dev)] = fault_[static_cast<size_t>(dev)]->samples.load();
    delayed_[static_cast<size_t>(dev)].clear();
    se_n_[static_cast<size_t>(dev)] = 0;
    se_last_[static_cast<size_t>(dev)] = PmcSample{};
    return 0;
  }
  int reset(int dev) override {
    if (dev < 0 || static_cast<size_t>(dev) >= fault_.size()) return -1;
    Fault& f = *fault_[static_cast<size_t>(dev)];
    f.resets.fetch_add(1);
    if (c_.hang_heals_on_reset && dev == c_.hang_dev) f.healed.store(1);
    f.stalled.store(0);  // a fresh queue: the injected stall is gone with the old one
    return 0;
  }
  int inject_stall(int dev) override {
    if (dev < 0 || static_cast<size_t>(dev) >= fault_.size()) return -1;
    fault_[static_cast<size_t>(dev)]->stalled.store(1);
    return 0;
  }
  void cancel(int dev, bool on) override {
    if (dev < 0 || static_cast<size_t>(dev) >= fault_.size()) return;
    fault_[static_cast<size_t>(dev)]->cancelled.store(on ? 1 : 0);
  }
  uint64_t resets(int dev) const override {
    return dev >= 0 && static_cast<size_t>(dev) < fault_.size() ? fault_[static_cast<size_t>(dev)]->resets.load() : 0;
  }
  bool publish_stats(int dev, PublishStats& out) const override {  // one writeback per `batch` READs
    if (dev < 0 || static_cast<size_t>(dev) >= fault_.size()) return false;
    out.reads = fault_[static_cast<size_t>(dev)]->samples.load();
    out.publishes = out.reads / static_cast<uint64_t>(std::max(c_.batch, 1));
    out.unlanded = 0;
    return true;
  }
  int sample(int dev, PmcSample& s) override {
    if (dev >= 0 && static_cast<size_t>(dev) < fault_.size()) {
      Fault& f = *fault_[static_cast<size_t>(dev)];
      if (dev == c_.slow_dev && c_.slow_s > 0 && wait_cancel(f, c_.slow_s)) return -3;
      if (f.stalled.load()) return wait_cancel(f, c_.hang_timeout_s) ? -3 : -2;  // the reader's deadline
      const uint64_t n = f.samples.fetch_add(1) + 1;
      if (dev == c_.hang_dev && !f.healed.load() && n > c_.hang_after) {
        if (c_.hang_timeout_s < 0)
          for (;;) pause();  // stuck for good, cancel or not: only abandoning the thread helps
        return wait_cancel(f, c_.hang_timeout_s) ? -3 : -2;  // aborted / deadline passed
      }
    }
    const int64_t now = mono_ns();
    const int64_t r = dev >= 0 && static_cast<size_t>(dev) < restart_.size() ? restart_[static_cast<size_t>(dev)] : 0;
    int64_t t = now;
    if (c_.freeze_after_s > 0) t = std::min(now, (r > 0 ? r : t0_) + static_cast<int64_t>(c_.freeze_after_s * 1e9));
    const uint64_t nreads = dev >= 0 && static_cast<size_t>(dev) < fault_.size() ? fault_[static_cast<size_t>(dev)]->samples.load() : 0;
    fill(dev, t, s, nreads);
    if (r > 0) {
      PmcSample z;
      fill(dev, r, z, restart_reads_[static_cast<size_t>(dev)]);
      for (int i = 0; i < kPmcCount; ++i) s.value[i] -= std::min(s.value[i], z.value[i]);
      for (uint32_t x = 0; x < s.n_xcd; ++x) {
        s.xcd_active[x] -= std::min(s.xcd_active[x], z.xcd_active[x]);
        s.xcd_mfma[x] -= std::min(s.xcd_mfma[x], z.xcd_mfma[x]);
        s.xcd_ta[x] -= std::min(s.xcd_ta[x], z.xcd_ta[x]);
      }
    }
    s.mono_ns = now;
    s.read_ns = 1000;
    s.se_fresh = 1;
    if (c_.lite_every > 1 && dev >= 0 && static_cast<size_t>(dev) < se_last_.size()) {
      // lite READs: only every lite_every-th one reads the per-SE counters
      PmcSample& last = se_last_[static_cast<size_t>(dev)];
      if (se_n_[static_cast<size_t>(dev)]++ % static_cast<uint64_t>(c_.lite_every) != 0) {
        s.value[kPmcMfmaBusy] = last.value[kPmcMfmaBusy];
        s.value[kPmcTaBusy] = last.value[kPmcTaBusy];
        std::copy(last.xcd_mfma, last.xcd_mfma + kMaxXcc, s.xcd_mfma);
        std::copy(last.xcd_ta, last.xcd_ta + kMaxXcc, s.xcd_ta);
        s.se_fresh = 0;
      } else {
        last = s;
      }
    }
    if (c_.batch > 1 && dev >= 0 && static_cast<size_t>(dev) < delayed_.size()) {
      std::deque<PmcSample>& q = delayed_[static_cast<size_t>(dev)];  // this device's sampler thread only
      q.push_back(s);
      if (q.size() <= static_cast<size_t>(c_.batch)) return kPmcPending;
      s = q.front();
      q.pop_front();
    }
    return 0;
  }

 private:
  // Cumulative counts since the source opened, at time `now`.
  void fill(int dev, int64_t now, PmcSample& s, uint64_t reads) const {
    const double t = (now - t0_) * 1e-9;
    // ∫ util/100 dt (fraction-seconds): the mock backend's load curve for this device
    const double busy_s = mock_device_util_integral(b_, dev, t) / 100.0;
    const double clk = c_.clock_mhz * 1e6;
    s.n = kPmcCount;
    s.value[kPmcGrbmCount] = static_cast<uint64_t>(clk * t);
    const double wave_s = busy_s * std::clamp(c_.wave_frac, 0.0, 1.0);  // waves present
    s.value[kPmcGrbmActive] = static_cast<uint64_t>(clk * wave_s);
    s.value[kPmcMfmaBusy] = static_cast<uint64_t>(clk * wave_s * c_.mfma_frac * 1024.0);
    s.value[kPmcTaBusy] = static_cast<uint64_t>(clk * wave_s * c_.vmem_frac);
    // The CP is busy while the load runs, plus cpc_read_us for each READ so far.
    s.value[kPmcCpcBusy] = static_cast<uint64_t>(clk * (busy_s + c_.cpc_read_us * 1e-6 * static_cast<double>(reads)));
    s.mask = c_.mask;
    for (int i = 0; i < kPmcCount; ++i)
      if (!(s.mask & (1u << i))) s.value[i] = 0;
    // XCD x is busy (1 - skew·x) of the time XCD 0 is (the active counter reduces by max
    // over XCDs, so XCD 0 carries the device value); MFMA cycles split likewise.
    // the real reader has a per-XCD fold only with the MFMA counter in the set
    s.n_xcd = (s.mask & (1u << kPmcMfmaBusy)) ? static_cast<uint32_t>(std::clamp(c_.n_xcd, 0, kMaxXcc)) : 0;
    double wsum = 0;
    for (uint32_t x = 0; x < s.n_xcd; ++x) wsum += 1.0 - c_.xcd_skew * x;
    for (uint32_t x = 0; x < s.n_xcd; ++x) {
      const double w = 1.0 - c_.xcd_skew * x;
      s.xcd_active[x] = static_cast<uint64_t>(clk * wave_s * w);
      s.xcd_mfma[x] = wsum > 0 ? static_cast<uint64_t>(s.value[kPmcMfmaBusy] * (w / wsum)) : 0;
      // TA: vmem_frac of the XCD's active cycles on each of its 32 CUs (256-CU mock)
      s.xcd_ta[x] = (s.mask & (1u << kPmcTaBusy)) ? static_cast<uint64_t>(clk * wave_s * w * c_.vmem_frac * 32.0) : 0;
    }
  }

  struct Fault {
    std::atomic<uint64_t> samples{0}, resets{0};
    std::atomic<int> healed{0};
    std::atomic<int> cancelled{0};
    std::atomic<int> stalled{0};  // inject_stall: every sample times out until reset()
  };
  bool hung(int dev) const {
    const Fault& f = *fault_[static_cast<size_t>(dev)];
    return dev == c_.hang_dev && !f.healed.load() && f.samples.load() > c_.hang_after;
  }
  // Sleep up to `s` seconds in 1 ms steps (a condition variable's timed wait is
  // not intercepted by GCC 11's TSAN); true if cancel() cut it short.
  static bool wait_cancel(Fault& f, double s) {
    const int64_t end = mono_ns() + static_cast<int64_t>(s * 1e9);
    while (mono_ns() < end) {
      if (f.cancelled.load()) return true;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return f.cancelled.load() != 0;
  }

  MockConfig b_;
  MockPmcConfig c_;
  int64_t t0_;
  std::vector<int64_t> restart_;  // per device: time of the last acquire (0 = never released)
  std::vector<uint64_t> restart_reads_;  // per device: samples taken at the last acquire
  std::vector<std::deque<PmcSample>> delayed_;  // per device: samples held back (MockPmcConfig::batch)
  std::vector<PmcSample> se_last_;              // per device: the last sample that read the per-SE counters
  std::vector<uint64_t> se_n_;                  // per device: samples since the last (re)START (lite_every)
  std::vector<std::unique_ptr<Fault>> fault_;
};

// --- dlopen bridge -------------------------------------------------------
using init_fn = int (*)(char*, int);
using open_fn = int (*)(uint64_t, const char* const*, const int*, int, char*, int);
using sample_fn = int (*)(int, uint64_t*, int, uint32_t*);
using sample_ts_fn = int (*)(int, uint64_t*, int, uint32_t*, int64_t*);
using sample_xcd_fn = int (*)(int, int, uint64_t*, int);
using pipelined_fn = int (*)(int, int, char*, int);
using configure_fn = int (*)(const char*, int);
using se_fresh_fn = int (*)(int);
using close_fn = void (*)(int);
using info_fn = int (*)(int, char*, int);
using abort_fn = int (*)(int, int);
using reset_fn = int (*)(int);
using stats_fn = int (*)(int, uint64_t*, int);
using stall_fn = int (*)(int);

class DlCounterSource final : public CounterSource {
 public:
  explicit DlCounterSource(std::string name) : name_(std::move(name)) {}
  ~DlCounterSource() override {
    if (close_)
      for (int h : handles_)
        if (h >= 0) close_(h);
    // The library stays loaded: HSA/rocprofiler must not be unloaded mid-process.
  }

  bool load(const std::string& path, const Backend& be, const std::vector<int>& devices, bool pipelined,
            uint32_t mask, int lean, int timeout_ms, int batch, int publish_us, bool lite, std::string& err) {
    lib_ = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!lib_) {
      err = std::string("dlopen failed: ") + dlerror();
      return false;
    }
    auto init = reinterpret_cast<init_fn>(dlsym(lib_, "kgs_pmc_init"));
    open_ = reinterpret_cast<open_fn>(dlsym(lib_, "kgs_pmc_open"));
    sample_ = reinterpret_cast<sample_fn>(dlsym(lib_, "kgs_pmc_sample"));
    close_ = reinterpret_cast<close_fn>(dlsym(lib_, "kgs_pmc_close"));
    info_ = reinterpret_cast<info_fn>(dlsym(lib_, "kgs_pmc_info"));
    sample_ts_ = reinterpret_cast<sample_ts_fn>(dlsym(lib_, "kgs_pmc_sample_ts"));    // optional
    auto set_pipe = reinterpret_cast<pipelined_fn>(dlsym(lib_, "kgs_pmc_set_pipelined"));  // optional
    if (!init || !open_ || !sample_ || !close_) {
      err = path + ": missing kgs_pmc_* symbols";
      return false;
    }
    auto configure = reinterpret_cast<configure_fn>(dlsym(lib_, "kgs_pmc_configure"));  // optional
    if (configure && lean >= 0) configure("lean", lean);
    if (configure && timeout_ms > 0) configure("timeout_ms", timeout_ms);
    if (configure && batch > 1 && configure("batch", batch) != 0) err += "reader ignores batch=" + std::to_string(batch) + "; ";
    if (configure && batch > 1 && publish_us >= 0) configure("publish_us", publish_us);
    // explicit either way: the setting is process-wide in the reader library
    if (configure && configure("lite", lite ? 1 : 0) != 0 && lite) err += "reader ignores lite; ";
    se_fresh_ = reinterpret_cast<se_fresh_fn>(dlsym(lib_, "kgs_pmc_se_fresh"));  // optional
    abort_ = reinterpret_cast<abort_fn>(dlsym(lib_, "kgs_pmc_abort"));  // optional (aqlprofile reader)
    reset_ = reinterpret_cast<reset_fn>(dlsym(lib_, "kgs_pmc_reset"));  // optional
    stats_ = reinterpret_cast<stats_fn>(dlsym(lib_, "kgs_pmc_stats"));  // optional
    stall_ = reinterpret_cast<stall_fn>(dlsym(lib_, "kgs_pmc_inject_stall"));  // optional (test hook)
    char ebuf[512] = {};
    if (init(ebuf, sizeof ebuf) != 0) {
      err = std::string("kgs_pmc_init: ") + ebuf;
      return false;
    }
    const char* names[kPmcCount];
    int is_max[kPmcCount];
    nsel_ = 0;
    for (int i = 0; i < kPmcCount; ++i) {
      reader_idx_[i] = -1;
      if (!(mask & (1u << i))) continue;
      names[nsel_] = kNames[i];
      is_max[nsel_] = kReduce[i];
      reader_idx_[i] = nsel_;
      sel_[nsel_++] = i;
    }
    sample_xcd_ = reinterpret_cast<sample_xcd_fn>(dlsym(lib_, "kgs_pmc_sample_xcd"));  // optional
    mask_ = mask;
    for (int k = 0; k < nsel_; ++k) {
      names_[k] = names[k];
      is_max_[k] = is_max[k];
    }
    set_pipe_ = set_pipe;
    pipelined_ = pipelined;
    int opened = 0;
    handles_ = std::vector<std::atomic<int>>(static_cast<size_t>(be.device_count()));
    for (auto& h : handles_) h.store(-1);
    agent_ = std::vector<std::atomic<int>>(static_cast<size_t>(be.device_count()));
    for (auto& h : agent_) h.store(-1);
    resets_ = std::vector<std::atomic<uint64_t>>(static_cast<size_t>(be.device_count()));
    kfd_ids_.assign(static_cast<size_t>(be.device_count()), 0);
    for (int d : devices) {
      kfd_ids_[static_cast<size_t>(d)] = be.info(d).kfd_gpu_id;
      std::string e;
      if (open_dev(d, e) == 0) ++opened;
      else err += "dev" + std::to_string(d) + ": " + e + "; ";
      if (!e.empty() && handles_[static_cast<size_t>(d)] >= 0) err += "dev" + std::to_string(d) + " " + e + "; ";
    }
    return opened > 0;
  }

  // Open the device's counting session (START), pipelined if asked.  A failed
  // switch to pipelined reads leaves a usable synchronous session (note in err).
  int open_dev(int d, std::string& err) {
    char ebuf[512] = {};
    const int h = open_(kfd_ids_[static_cast<size_t>(d)], names_, is_max_, nsel_, ebuf, sizeof ebuf);
    handles_[static_cast<size_t>(d)] = h;
    if (h >= 0) agent_[static_cast<size_t>(d)] = h;  // the reader's handle is its agent index: stable
    if (h < 0) {
      err = ebuf;
      return -1;
    }
    if (pipelined_ && set_pipe_) {
      ebuf[0] = 0;
      if (set_pipe_(h, 1, ebuf, sizeof ebuf) != 0) err = std::string("pipelined reads unavailable: ") + ebuf;
    }
    return 0;
  }

  int release(int dev) override {
    if (dev < 0 || dev >= static_cast<int>(handles_.size()) || handles_[static_cast<size_t>(dev)] < 0) return -1;
    close_(handles_[static_cast<size_t>(dev)]);
    handles_[static_cast<size_t>(dev)] = -1;
    return 0;
  }
  int acquire(int dev) override {
    if (dev < 0 || dev >= static_cast<int>(handles_.size())) return -1;
    if (handles_[static_cast<size_t>(dev)] >= 0) return 0;
    std::string e;
    return open_dev(dev, e);
  }
  int reset(int dev) override {
    if (dev < 0 || dev >= static_cast<int>(handles_.size())) return -1;
    if (handles_[static_cast<size_t>(dev)] >= 0) release(dev);
    const int a = agent_[static_cast<size_t>(dev)];
    if (!reset_ || a < 0) return -1;
    resets_[static_cast<size_t>(dev)].fetch_add(1);
    return reset_(a);
  }
  void cancel(int dev, bool on) override {
    if (!abort_ || dev < 0 || dev >= static_cast<int>(agent_.size())) return;
    const int a = agent_[static_cast<size_t>(dev)];
    if (a >= 0) abort_(a, on ? 1 : 0);
  }
  uint64_t resets(int dev) const override {
    return dev >= 0 && dev < static_cast<int>(resets_.size()) ? resets_[static_cast<size_t>(dev)].load() : 0;
  }
  int inject_stall(int dev) override {
    if (!stall_ || dev < 0 || dev >= static_cast<int>(handles_.size())) return -1;
    const int h = handles_[static_cast<size_t>(dev)];
    return h >= 0 ? stall_(h) : -1;
  }
  // By agent, not by session handle: the totals survive hand-overs and resets.
  bool publish_stats(int dev, PublishStats& out) const override {
    if (!stats_ || dev < 0 || dev >= static_cast<int>(agent_.size())) return false;
    const int a = agent_[static_cast<size_t>(dev)];
    uint64_t v[3] = {};
    if (a < 0 || stats_(a, v, 3) != 3) return false;
    out.reads = v[0];
    out.publishes = v[1];
    out.unlanded = v[2];
    return true;
  }
  void set_fresh(int dev, bool fresh) override {
    if (!pipelined_ || !set_pipe_ || dev < 0 || dev >= static_cast<int>(handles_.size())) return;
    const int h = handles_[static_cast<size_t>(dev)];
    char ebuf[256] = {};
    if (h >= 0) set_pipe_(h, fresh ? 0 : 1, ebuf, sizeof ebuf);  // a failed switch keeps the current mode
  }

  std::string name() const override { return name_; }

  std::string info(int dev) const override {
    if (!info_ || dev < 0 || dev >= static_cast<int>(handles_.size()) || handles_[dev] < 0) return "closed";
    char buf[1024] = {};
    info_(handles_[dev], buf, sizeof buf);
    return buf;
  }

  int sample(int dev, PmcSample& s) override {
    if (dev < 0 || dev >= static_cast<int>(handles_.size()) || handles_[dev] < 0) return -1;
    uint32_t rns = 0;
    int64_t ts = 0;
    uint64_t v[kPmcCount] = {};
    const int rc = sample_ts_ ? sample_ts_(handles_[dev], v, nsel_, &rns, &ts)
                              : sample_(handles_[dev], v, nsel_, &rns);
    if (rc != 0) return rc;
    for (int k = 0; k < nsel_; ++k) s.value[sel_[k]] = v[k];  // reader order → PmcIndex
    s.mask = mask_;
    s.n = kPmcCount;
    s.read_ns = rns;
    s.n_xcd = 0;
    if (sample_xcd_ && reader_idx_[kPmcGrbmActive] >= 0 && reader_idx_[kPmcMfmaBusy] >= 0) {
      const int na = sample_xcd_(handles_[dev], reader_idx_[kPmcGrbmActive], s.xcd_active, kMaxXcc);
      const int nm = sample_xcd_(handles_[dev], reader_idx_[kPmcMfmaBusy], s.xcd_mfma, kMaxXcc);
      if (na > 0 && na == nm) s.n_xcd = static_cast<uint32_t>(na);
      if (s.n_xcd > 0 && reader_idx_[kPmcTaBusy] >= 0 &&
          sample_xcd_(handles_[dev], reader_idx_[kPmcTaBusy], s.xcd_ta, kMaxXcc) != static_cast<int>(s.n_xcd))
        std::fill(s.xcd_ta, s.xcd_ta + kMaxXcc, 0);
    }
    s.se_fresh = se_fresh_ ? (se_fresh_(handles_[dev]) != 0 ? 1u : 0u) : 1u;
    s.mono_ns = ts > 0 ? ts : mono_ns();  // when the CP read the counters (pipelined: previous call)
    return 0;
  }

 private:
  void* lib_ = nullptr;
  open_fn open_ = nullptr;
  sample_fn sample_ = nullptr;
  sample_ts_fn sample_ts_ = nullptr;
  sample_xcd_fn sample_xcd_ = nullptr;
  se_fresh_fn se_fresh_ = nullptr;
  pipelined_fn set_pipe_ = nullptr;
  bool pipelined_ = false;
  const char* names_[kPmcCount] = {};
  int is_max_[kPmcCount] = {};
  std::vector<uint64_t> kfd_ids_;
  int sel_[kPmcCount] = {};  // reader's counter k is PmcIndex sel_[k]
  int reader_idx_[kPmcCount] = {};  // inverse: PmcIndex → reader counter, -1 not read
  int nsel_ = 0;
  uint32_t mask_ = 0;
  close_fn close_ = nullptr;
  info_fn info_ = nullptr;
  abort_fn abort_ = nullptr;
  reset_fn reset_ = nullptr;
  stats_fn stats_ = nullptr;
  stall_fn stall_ = nullptr;
  std::vector<std::atomic<int>> agent_;  // per device: reader agent index once opened (-1 never)
  std::vector<std::atomic<uint64_t>> resets_;
  // Written by the device's sampler thread (release / acquire), read by info()
  // from the HTTP / control threads.
  std::vector<std::atomic<int>> handles_;
  std::string name_;
};

}  // namespace

std::unique_ptr<CounterSource> make_mock_counter_source(const Backend& be, const MockConfig& bcfg,
                                                        const MockPmcConfig& cfg) {
  return std::make_unique<MockCounterSource>(bcfg, cfg, be.device_count());
}

std::unique_ptr<CounterSource> make_dl_counter_source(const std::string& name, const std::string& lib_path,
                                                      const Backend& be, const std::vector<int>& devices,
                                                      bool pipelined, uint32_t mask, int lean, std::string& err,
                                                      int timeout_ms, int batch, int publish_us, bool lite) {
  auto s = std::make_unique<DlCounterSource>(name);
  if (!s->load(lib_path, be, devices, pipelined, mask, lean, timeout_ms, batch, publish_us, lite, err)) return nullptr;
  return s;
}

}  // namespace kgs
