// Per-GPU sampler threads.  See sampler.h.
#include "kgs/sampler.h"
#include "kgs/unpark.h"

#include <poll.h>
#include <pthread.h>
#include <sys/prctl.h>
#include <sched.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <algorithm>
#include <climits>

namespace kgs {

const double kReadHistBoundsUs[kReadHistBuckets] = {10, 25, 50, 100, 250, 500, 1000, 2500, 5000, 10000, 25000, 100000};

namespace {

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// Delta of a PMFW accumulator that the v1.8 table stores in 32 bits.
bool acc_delta(uint64_t prev, uint64_t cur, uint64_t& d) {
  if (cur >= prev) {
    d = cur - prev;
    return true;
  }
  if (prev <= 0xFFFFFFFFull && cur <= 0xFFFFFFFFull) {
    d = cur + 0x100000000ull - prev;
    return true;
  }
  return false;  // counter reset
}

enum WorkerKind : int { kPmfw = 0, kPmc = 1, kSlow = 2 };

}  // namespace

// One sampler thread.  Shared with the thread itself, so a thread that stop()
// abandons still has a live `done` / `abandoned` pair to look at when (if) its
// stuck call returns — and then exits without touching the sampler.
struct Sampler::Worker {
  int dev = -1;
  int kind = kPmfw;
  std::thread t;
  std::atomic<bool> done{false};
  std::atomic<bool> abandoned{false};
};

EstimatorParams estimator_params(const SamplerConfig& cfg, int num_cu) {
  EstimatorParams p;
  p.quiet_active_frac = kQuietActiveFrac;
  p.cpc_full_frac = kCpcFullFrac;
  p.clock_split_ns = kClockSplitNs;
  p.read_overlap_ns = kReadOverlapNs;
  p.read_only_bills_zero = kReadOnlyBillsZero;
  p.time_split_ns = kTimeSplitNs;
  p.time_split_weight = kTimeSplitWeight;
  p.gap_clock_fresh_ns = kGapClockFreshNs;
  p.quiet_hold_ns = kQuietHoldNs;
  p.cp_only_min = cfg.pmc_cp_only_min;
  p.dbound_hold_ns = static_cast<int64_t>(cfg.pmc_dispatch_hold_s * 1e9);
  p.plausible_mhz_lo = kPlausibleMhzLo;
  p.plausible_mhz_hi = kPlausibleMhzHi;
  p.num_simds = (num_cu > 0 ? num_cu : 256) * 4.0;
  return p;
}

std::vector<int> numa_cpus(int node) {
  std::vector<int> cpus;
  if (node < 0) return cpus;
  char path[128];
  std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = std::fopen(path, "r");
  if (!f) return cpus;
  char buf[4096];
  size_t n = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[n] = 0;
  char* p = buf;
  while (*p) {
    char* end;
    long a = std::strtol(p, &end, 10);
    if (end == p) break;
    long b = a;
    p = end;
    if (*p == '-') {
      b = std::strtol(p + 1, &end, 10);
      p = end;
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) cpus.push_back(static_cast<int>(c));
    while (*p == ',' || *p == '\n' || *p == ' ') ++p;
  }
  return cpus;
}

Sampler::Sampler(Backend* be, CounterSource* pmc, SamplerConfig cfg) : be_(be), pmc_(pmc), cfg_(std::move(cfg)) {
  const int n = be_->device_count();
  for (int d = 0; d < n; ++d) states_.push_back(std::make_unique<DeviceState>());
  if (cfg_.devices.empty()) {
    for (int d = 0; d < n; ++d) dev_ids_.push_back(d);
  } else {
    for (int d : cfg_.devices)
      if (d >= 0 && d < n) dev_ids_.push_back(d);
  }
  if (!(cfg_.hz > 0)) cfg_.hz = 1;
  if (cfg_.hz > kMaxHz) cfg_.hz = kMaxHz;
  hz_.store(cfg_.hz);
  if (cfg_.pmc_breaker_k < 1) cfg_.pmc_breaker_k = 1;
  if (!(cfg_.pmc_retry_s > 0)) cfg_.pmc_retry_s = 1.0;
  if (cfg_.pmc_retry_max_s < cfg_.pmc_retry_s) cfg_.pmc_retry_max_s = cfg_.pmc_retry_s;
  const double ih = cfg_.pmc_idle_hz;
  pmc_idle_hz_.store(!(ih > 0) ? 0.0 : std::clamp(ih, kMinIdleHz, kMaxHz));
  if (!set_pmc_dispatch_hz(cfg_.pmc_dispatch_hz)) set_pmc_dispatch_hz(500.0);
  if (!set_pmc_quiet_release_s(cfg_.pmc_quiet_release_s)) set_pmc_quiet_release_s(0.0);
  if (!(cfg_.pmc_cp_only_min >= 0 && cfg_.pmc_cp_only_min <= 1)) cfg_.pmc_cp_only_min = 0.0;
  if (!(cfg_.pmc_dispatch_hold_s >= 0)) cfg_.pmc_dispatch_hold_s = 0.0;
  for (int d : dev_ids_) {
    DeviceState& st = *states_[static_cast<size_t>(d)];
    st.pmc_on.store(cfg_.pmc && pmc_ ? 1 : 0);
    st.pmc_backoff_s = cfg_.pmc_retry_s;
  }
  cu_seconds_.resize(static_cast<size_t>(n));
  pod_cu_.resize(static_cast<size_t>(n));
  last_proc_ns_.assign(static_cast<size_t>(n), 0);
  util_bill_.resize(static_cast<size_t>(n));
  stop_fd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
}

bool Sampler::inject_pmc_stall(int dev) {
  if (std::find(dev_ids_.begin(), dev_ids_.end(), dev) == dev_ids_.end() || !pmc_) return false;
  states_[static_cast<size_t>(dev)]->pmc_stall_req.store(1);
  return true;
}

int64_t Sampler::proc_period_ns() const {
  const int64_t tick_ns = static_cast<int64_t>(1e9 / hz_.load());
  return cfg_.proc_period_s > 0 ? static_cast<int64_t>(cfg_.proc_period_s * 1e9)
         : cfg_.proc_every > 0  ? tick_ns * cfg_.proc_every
                                : 0;
}

int64_t Sampler::link_period_ns() const {
  const int64_t tick_ns = static_cast<int64_t>(1e9 / hz_.load());
  return cfg_.link_period_s > 0 ? static_cast<int64_t>(cfg_.link_period_s * 1e9)
         : cfg_.link_every > 0  ? tick_ns * cfg_.link_every
                                : 0;
}

bool Sampler::set_hz(double hz) {
  if (!(hz > 0 && hz <= kMaxHz)) return false;
  std::lock_guard<std::mutex> lk(life_mu_);
  const bool was = running_.load();
  stop_locked();
  hz_.store(hz);
  if (was) start_locked();
  return true;
}

bool Sampler::set_pmc_idle_hz(double hz) {
  if (!(hz == 0 || (hz >= kMinIdleHz && hz <= kMaxHz))) return false;
  pmc_idle_hz_.store(hz, std::memory_order_relaxed);
  return true;
}

bool Sampler::set_pmc_dispatch_hz(double hz) {
  if (!(hz > 0 && hz <= kMaxHz)) return false;
  pmc_dispatch_hz_.store(hz, std::memory_order_relaxed);
  return true;
}

bool Sampler::set_pmc_quiet_release_s(double v) {
  if (!(v >= 0 && v <= 86400)) return false;
  pmc_quiet_release_s_.store(v, std::memory_order_relaxed);
  return true;
}

void Sampler::set_pmc_wanted(bool on, int dev, bool drop_queue) {
  for (int d : dev_ids_)
    if (dev < 0 || d == dev) {
      DeviceState& st = *states_[static_cast<size_t>(d)];
      if (!on && drop_queue) st.pmc_drop_queue.store(1);
      if (on) st.pmc_unpark_req.store(1);  // an explicit acquire also ends a quiet release
      st.pmc_want.store(on ? 1 : 0);
    }
}

void Sampler::drop_util_carry(int dev) {
  if (dev >= 0 && dev < device_count()) states_[static_cast<size_t>(dev)]->util_carry_drop.store(1);
}

void Sampler::set_pid_pods(std::shared_ptr<const std::unordered_map<uint64_t, std::string>> m) {
  std::lock_guard<std::mutex> g(pid_pods_mu_);
  pid_pods_ = std::move(m);
}

double Sampler::pod_cu_seconds(int dev, const std::string& ns_pod) const {
  if (dev < 0 || dev >= device_count()) return 0.0;
  auto m = states_[static_cast<size_t>(dev)]->get_pod_cu();
  if (!m) return 0.0;
  auto it = m->find(ns_pod);
  return it == m->end() ? 0.0 : it->second;
}

Sampler::~Sampler() {
  stop();
  // An abandoned thread may still be inside a backend / counter-source call; it
  // exits without touching `this`, but its stop flag lives here: leave the fd.
  if (stop_fd_ >= 0 && abandoned_total_.load() == 0) close(stop_fd_);
}

void Sampler::start() {
  std::lock_guard<std::mutex> lk(life_mu_);
  start_locked();
}

void Sampler::stop() {
  std::lock_guard<std::mutex> lk(life_mu_);
  stop_locked();
}

void Sampler::spawn(int dev, int kind) {
  auto w = std::make_shared<Worker>();
  w->dev = dev;
  w->kind = kind;
  w->t = std::thread([this, w] {
    if (w->kind == kPmfw) run_pmfw(*w);
    else if (w->kind == kPmc) run_pmc(*w);
    else run_slow(*w);
    w->done.store(true, std::memory_order_release);
  });
  workers_.push_back(std::move(w));
}

void Sampler::start_locked() {
  if (running_.exchange(true)) return;
  stop_.store(false);
  uint64_t drain;
  while (read(stop_fd_, &drain, sizeof drain) > 0) {
  }
  // A (device, tier) whose abandoned thread is still stuck gets no second thread:
  // two threads on one device's reader would break its one-thread-per-handle rule.
  auto stuck = [&](int dev, int kind) {
    for (const auto& w : abandoned_)
      if (w->dev == dev && w->kind == kind && !w->done.load(std::memory_order_acquire)) return true;
    return false;
  };
  abandoned_.erase(std::remove_if(abandoned_.begin(), abandoned_.end(),
                                  [](const std::shared_ptr<Worker>& w) { return w->done.load(); }),
                   abandoned_.end());
  const bool pmc = cfg_.pmc && pmc_;
  for (int d : dev_ids_) {
    DeviceState& st = *states_[static_cast<size_t>(d)];
    bool hung = false;
    if (!stuck(d, kPmfw)) spawn(d, kPmfw);
    else hung = true;
    if (pmc) {
      if (!stuck(d, kPmc)) {
        pmc_->cancel(d, false);
        spawn(d, kPmc);
      } else {
        hung = true;
      }
    }
    st.thread_hung.store(hung ? 1 : 0);
    // One slow thread per device (sampler.h): a management-library call stuck on
    // one GPU leaves the others' per-process / link / RAS tiers running.
    if (proc_period_ns() > 0 || link_period_ns() > 0) {
      const bool slow_stuck = stuck(d, kSlow);
      if (!slow_stuck) spawn(d, kSlow);
      st.slow_hung.store(slow_stuck ? 1 : 0);
    }
  }
}

void Sampler::stop_locked() {
  if (!running_.load()) return;
  stop_.store(true);
  const uint64_t one = 1;
  if (write(stop_fd_, &one, sizeof one) < 0) {
  }
  // Calls blocked on a device's counters (a wedged CP) return at once.
  if (cfg_.pmc && pmc_)
    for (int d : dev_ids_) pmc_->cancel(d, true);
  const int64_t deadline = mono_ns() + static_cast<int64_t>(cfg_.stop_timeout_s * 1e9);
  for (;;) {
    bool all = true;
    for (const auto& w : workers_) all = all && w->done.load(std::memory_order_acquire);
    if (all || mono_ns() >= deadline) break;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  for (auto& w : workers_) {
    if (w->done.load(std::memory_order_acquire)) {
      w->t.join();
      continue;
    }
    // Stuck inside a device call: detach.  The thread checks `abandoned` after
    // every such call and exits without touching this sampler.
    w->abandoned.store(true, std::memory_order_release);
    w->t.detach();
    if (w->dev >= 0) (w->kind == kSlow ? states_[static_cast<size_t>(w->dev)]->slow_hung
                                       : states_[static_cast<size_t>(w->dev)]->thread_hung).store(1);
    abandoned_total_.fetch_add(1);
    abandoned_.push_back(w);
  }
  workers_.clear();
  running_.store(false);
}

void Sampler::pin(int dev, const char* fmt) {
  DeviceState& st = *states_[static_cast<size_t>(dev)];
  if (cfg_.pin_numa) {
    const std::vector<int> cpus = numa_cpus(be_->info(dev).numa_node);
    if (!cpus.empty()) {
      cpu_set_t set;
      CPU_ZERO(&set);
      for (int c : cpus) CPU_SET(c, &set);
      if (pthread_setaffinity_np(pthread_self(), sizeof set, &set) == 0) st.cpu_pinned.store(static_cast<int>(cpus.size()));
    }
  }
  char tname[16];
  std::snprintf(tname, sizeof tname, fmt, dev);
  pthread_setname_np(pthread_self(), tname);
  // The default 50 µs timer slack is 40 % of an 8 kHz period: wake on time.
  // (KGS_TIMERSLACK_NS overrides, for interference experiments.)
  const char* slack = std::getenv("KGS_TIMERSLACK_NS");
  prctl(PR_SET_TIMERSLACK, slack ? std::strtoul(slack, nullptr, 10) : 1000UL, 0, 0, 0);
}

void Sampler::integrate(int dev, const GpuSample* prev, GpuSample& cur, Integrals& I) {
  (void)dev;
  if (!prev) return;
  double dt;
  if ((cur.valid & kFFwTs) && (prev->valid & kFFwTs) && cur.fw_ts > prev->fw_ts)
    dt = static_cast<double>(cur.fw_ts - prev->fw_ts) * 1e-8;
  else
    dt = static_cast<double>(cur.mono_ns - prev->mono_ns) * 1e-9;
  if (dt <= 0 || dt > 3600) return;
  cur.dt_s = static_cast<float>(dt);

  double g = cur.gfx_busy_pct, u = cur.umc_busy_pct;
  uint64_t dc, dg, du;
  if ((cur.valid & kFAcc) && (prev->valid & kFAcc) &&
      acc_delta(prev->accumulation_counter, cur.accumulation_counter, dc) && dc > 0 &&
      acc_delta(prev->gfx_activity_acc, cur.gfx_activity_acc, dg) &&
      acc_delta(prev->mem_activity_acc, cur.mem_activity_acc, du)) {
    g = static_cast<double>(dg) / static_cast<double>(dc);
    u = static_cast<double>(du) / static_cast<double>(dc);
  }
  g = g < 0 ? 0 : (g > 100 ? 100 : g);
  u = u < 0 ? 0 : (u > 100 ? 100 : u);
  // Per-XCC (XCD) window means from the per-partition accumulators.  PMFW counts
  // an XCC busy while a dispatch is in flight on it, so a chip-wide kernel keeps
  // all 8 near 100 % even when waves run on a few (profiles/r1/xcd/README.md);
  // the counter tier's per-XCD MFMA split shows where they run.
  for (uint32_t x = 0; x < cur.num_xcc && x < static_cast<uint32_t>(kMaxXcc); ++x) {
    double v = cur.gfx_busy_xcc[x];
    uint64_t dx;
    if ((cur.valid & kFXccAcc) && (prev->valid & kFXccAcc) && (cur.valid & kFAcc) && (prev->valid & kFAcc) &&
        acc_delta(prev->accumulation_counter, cur.accumulation_counter, dc) && dc > 0 &&
        cur.gfx_busy_acc_xcc[x] >= prev->gfx_busy_acc_xcc[x]) {
      dx = cur.gfx_busy_acc_xcc[x] - prev->gfx_busy_acc_xcc[x];
      v = static_cast<double>(dx) / static_cast<double>(dc);
    }
    cur.gfx_busy_xcc_window[x] = static_cast<float>(v < 0 ? 0 : (v > 100 ? 100 : v));
  }
  cur.gfx_busy_window_pct = static_cast<float>(g);
  cur.umc_busy_window_pct = static_cast<float>(u);
  I.gfx_busy_seconds += g * 0.01 * dt;
  I.umc_busy_seconds += u * 0.01 * dt;
  I.sampled_seconds += dt;
  if ((cur.valid & kFEnergy) && (prev->valid & kFEnergy) && cur.energy_acc >= prev->energy_acc) {
    double e = energy_units_to_joules(cur.energy_acc - prev->energy_acc);
    // Compute partitions (DPX/QPX/CPX) read one socket's energy accumulator: each
    // takes its XCCs' share of the chip's GFX busy over the interval (an equal
    // share while the chip is idle), so the partitions' counters add up to the
    // socket's energy instead of counting it once per partition.
    if (cur.energy_parts > 1) {
      double share = 1.0 / cur.energy_parts;
      if ((cur.valid & kFXccAcc) && (prev->valid & kFXccAcc) && cur.xcc_acc_chip > prev->xcc_acc_chip &&
          cur.xcc_acc_own >= prev->xcc_acc_own)
        share = static_cast<double>(cur.xcc_acc_own - prev->xcc_acc_own) /
                static_cast<double>(cur.xcc_acc_chip - prev->xcc_acc_chip);
      e *= std::clamp(share, 0.0, 1.0);
    }
    I.energy_joules += e;
  }
  // Throttler residencies: the fraction of accumulation cycles each controller was
  // active (amdsmi.h PVIOL / TVIOL), times the interval.
  if ((cur.valid & kFThrottle) && (prev->valid & kFThrottle) && (cur.valid & kFAcc) && (prev->valid & kFAcc) &&
      acc_delta(prev->accumulation_counter, cur.accumulation_counter, dc) && dc > 0)
    for (int r = 0; r < kThrottleReasons; ++r) {
      uint64_t dr;
      if (!acc_delta(prev->throttle_res_acc[r], cur.throttle_res_acc[r], dr)) continue;
      const double f = static_cast<double>(dr) / static_cast<double>(dc);
      I.throttle_seconds[r] += (f > 1.0 ? 1.0 : f) * dt;
    }
}

// ---- READ-immune busy integral (--sm-util-source auto) ------------------------
// Per distinct PMFW interval (dt of firmware time, dgfx_s of PMFW GFX busy in it):
// while the device's counter tier ran through the interval — same epoch as at the
// previous PMFW sample, counters held and not stalled, a drain no older than three
// of its slowest READ periods — the interval is billed from the counter tier's
// busy integral (Δdispatch_seconds: CP busy less the exporter's own READ packets,
// floored at SPI busy — a dispatch in flight, the PMFW busy's meaning; Δactive_seconds,
// waves in a shader engine, for a counter set without CPC busy), else the PMFW GFX
// busy (a dispatch in flight, but counting each READ as ≈80 µs of work,
// profiles/r2/idle_busy/).  Drains land on host time and intervals are firmware time,
// so an interval can receive more than dt of counter busy (two drains) and the next
// none: UtilBiller (util_estimator.h) carries the excess forward instead of dropping
// it (at 10 Hz dropping it billed a saturated GPU 75 %).
void Sampler::run_pmfw_util(int dev, int64_t now, double dgfx_s, double dt_s, Integrals& I, GpuSample& s) {
  DeviceState& st = *states_[static_cast<size_t>(dev)];
  Integrals pc;
  st.pmc_integ.load(pc);
  double slow_hz = hz_.load(std::memory_order_relaxed);
  const double idle = pmc_idle_hz_.load(std::memory_order_relaxed);
  if (idle > 0) slow_hz = std::min(slow_hz, idle);
  if (cfg_.pmc_cp_only_min > 0 && idle > 0)
    slow_hz = std::min(slow_hz, pmc_dispatch_hz_.load(std::memory_order_relaxed));
  const int64_t fresh_ns = static_cast<int64_t>(3e9 / slow_hz) + 50000000LL;
  CounterCover c;
  c.ok = st.pmc_on.load(std::memory_order_relaxed) && !st.pmc_stalled.load(std::memory_order_relaxed) &&
         !st.pmc_failed.load(std::memory_order_relaxed) && pc.pmc_last_ns > 0 && now - pc.pmc_last_ns <= fresh_ns;
  c.epoch = pc.pmc_epoch;
  // The counter tier's busy integral: dispatch in flight (CP busy less our READs)
  // when the counter set has CPC busy, else waves in a shader engine (SPI busy).
  c.dispatch = pc.dispatch_drains > 0;
  c.busy_s = c.dispatch ? pc.dispatch_seconds : pc.active_seconds;
  c.share = pc.pmc_last_share;
  c.since_s = (now - pc.pmc_last_ns) * 1e-9;
  c.drains = pc.pmc_samples;
  // Carry (and run the last drain on) at most one freshness window, and never more
  // than kMaxUtilCarryS: the drain-vs-interval jitter, never a backlog.
  if (st.util_carry_drop.exchange(0, std::memory_order_relaxed)) util_bill_[static_cast<size_t>(dev)].drop_carry();
  const UtilBiller::Bill b =
      util_bill_[static_cast<size_t>(dev)].bill(dt_s, dgfx_s, c, std::min(fresh_ns * 1e-9, kMaxUtilCarryS));
  I.util_seconds += b.billed_s;
  if (b.from_counters) I.util_counter_seconds += dt_s;
  I.util_carry_seconds = util_bill_[static_cast<size_t>(dev)].carry_s();
  I.util_dropped_seconds = util_bill_[static_cast<size_t>(dev)].dropped_s();
  s.cum_util_s = I.util_seconds;
  s.util_window_pct = dt_s > 0 ? static_cast<float>(100.0 * b.billed_s / dt_s) : -1.0f;
}

// ---- PMFW tier: the firmware metrics table + HBM occupancy --------------------
// At min(hz, pmfw_hz): the table refreshes every ≈20 ms, so reading it faster
// only re-reads the same table.  A failing device backs off; every 4th failure
// of a streak asks the backend to re-open / re-initialise it.
void Sampler::run_pmfw(Worker& w) {
  const int dev = w.dev;
  DeviceState& st = *states_[static_cast<size_t>(dev)];
  Backend* const be = be_;
  pin(dev, "kgs-pmfw%d");
  const double hz = hz_.load();
  const double rate = cfg_.pmfw_hz > 0 && cfg_.pmfw_hz < hz ? cfg_.pmfw_hz : hz;
  const int64_t period_ns = static_cast<int64_t>(1e9 / rate);
  Integrals I;
  GpuSample& prev = st.pmfw_prev;
  bool& have_prev = st.have_pmfw_prev;
  uint64_t seq = 0;
  {  // resume after a pause: integrals and sequence numbers continue
    st.integ.load(I);
    GpuSample last;
    if (st.latest.load(last)) seq = last.seq;
  }
  int64_t next = mono_ns();
  while (!stop_.load(std::memory_order_relaxed)) {
    int backoff_shift = 0;
    GpuSample s;
    const int64_t t0 = mono_ns();
    const int rc = be->read_metrics(dev, s);
    const int64_t t1 = mono_ns();
    if (w.abandoned.load(std::memory_order_acquire)) return;  // stop() gave up on us while we were in the call
    const double us = (t1 - t0) * 1e-3;
    int b = 0;
    while (b < kReadHistBuckets && us > kReadHistBoundsUs[b]) ++b;
    st.read_hist[b].fetch_add(1, std::memory_order_relaxed);
    ++I.reads;
    I.read_seconds += (t1 - t0) * 1e-9;
    if (rc == 0) {
      s.read_ns = static_cast<uint32_t>(t1 - t0);
      if (s.mono_ns == 0) s.mono_ns = t1;
      st.up.store(1, std::memory_order_relaxed);
      st.consecutive_errors.store(0, std::memory_order_relaxed);
      st.last_ok_mono_ns.store(t1, std::memory_order_relaxed);
      const bool distinct = !have_prev || !(s.valid & kFFwTs) || s.fw_ts != prev.fw_ts;
      // Firmware clock went backwards: the SMU restarted (GPU reset), so every
      // accumulator restarted too — re-baseline instead of reading a wrap.
      const bool reset = have_prev && (s.valid & kFFwTs) && (prev.valid & kFFwTs) && s.fw_ts < prev.fw_ts;
      if (distinct) {
        const double g0 = I.gfx_busy_seconds, d0 = I.sampled_seconds;
        integrate(dev, have_prev && !reset ? &prev : nullptr, s, I);
        run_pmfw_util(dev, t1, I.gfx_busy_seconds - g0, I.sampled_seconds - d0, I, s);
        s.cum_gfx_s = I.gfx_busy_seconds;
        s.cum_umc_s = I.umc_busy_seconds;
        s.cum_dt_s = I.sampled_seconds;
        s.seq = ++seq;
        ++I.distinct_samples;
        st.ring.push(s);
        st.latest.store(s);
        prev = s;
        have_prev = true;
      } else {
        // Same PMFW table: refresh host-side fields only (HBM occupancy).
        prev.vram_used_bytes = s.vram_used_bytes;
        prev.mono_ns = s.mono_ns;
        prev.wall_ns = s.wall_ns;
        st.latest.store(prev);
      }
    } else {
      ++I.read_errors;
      const uint64_t ce = st.consecutive_errors.fetch_add(1, std::memory_order_relaxed) + 1;
      if (ce >= 3) st.up.store(0, std::memory_order_relaxed);
      backoff_shift = ce > 10 ? 10 : static_cast<int>(ce);
      // Every 4th failure of a streak (≈ every 4·max_backoff once backed off):
      // let the backend reopen / re-initialise the device.
      if (ce % 4 == 0) {
        ++I.recover_attempts;
        const int rr = be->recover(dev);
        if (w.abandoned.load(std::memory_order_acquire)) return;
        if (rr == 0) {
          ++I.recoveries;
          have_prev = false;
        }
      }
    }

    int64_t step = period_ns;
    if (backoff_shift > 0) {
      step = period_ns << backoff_shift;
      const int64_t cap = static_cast<int64_t>(cfg_.max_backoff_ms) * 1000000LL;
      if (step > cap) step = cap > period_ns ? cap : period_ns;
    }
    next += step;
    const int64_t now = mono_ns();
    if (next <= now) {
      ++I.overruns;
      // Late by a few periods (a long read, a descheduled thread): keep the
      // absolute schedule, the missed ticks run at once and the rate holds.
      // Further behind: re-anchor and sleep a quarter period instead of bursting.
      if (backoff_shift) next = now + step;
      else if (now - next > kCatchUpPeriods * step) next = now + period_ns / 4;
    }
    st.integ.store(I);
    const int64_t wait = next - now;
    timespec ts{static_cast<time_t>(wait / 1000000000LL), static_cast<long>(wait % 1000000000LL)};
    pollfd pfd{stop_fd_, POLLIN, 0};
    ppoll(&pfd, 1, &ts, nullptr);
  }
  st.integ.store(I);
}

// ---- counter tier: one hardware-counter drain per tick ------------------------
void Sampler::run_pmc(Worker& w) {
  const int dev = w.dev;
  DeviceState& st = *states_[static_cast<size_t>(dev)];
  CounterSource* const src = pmc_;
  const DeviceInfo& info = be_->info(dev);
  pin(dev, "kgs-gpu%d");
  const double hz = hz_.load();
  const int64_t period_ns = static_cast<int64_t>(1e9 / hz);
  // A PMFW tier silent this long wakes a parked device: three of its periods, ≥ 1 s.
  const double pmfw_rate = cfg_.pmfw_hz > 0 && cfg_.pmfw_hz < hz ? cfg_.pmfw_hz : hz;
  const int64_t pmfw_silent_ns = std::max<int64_t>(1000000000LL, static_cast<int64_t>(3e9 / pmfw_rate));
  auto gone = [&w] { return w.abandoned.load(std::memory_order_acquire); };
  Integrals P;
  uint64_t pmc_seq = 0;
  int64_t last_slow_ns = 0;
  {  // resume after a pause: counters and sequence numbers continue
    st.pmc_integ.load(P);
    PmcSample lp;
    if (st.pmc_latest.load(lp)) pmc_seq = lp.seq;
  }
  // A thread that stopped (pause, rate change) while its device was quiet left
  // the reader in synchronous mode: start pipelined, not quiet.
  if (st.pmc_on.load()) {
    src->set_fresh(dev, false);
    if (gone()) return;
  }
  st.pmc_quiet.store(0, std::memory_order_relaxed);
  st.pmc_dbound.store(0, std::memory_order_relaxed);
  // Everything learned from the counts (READ cost, clocks, rate hysteresis, stall
  // watch) lives in the estimator (util_estimator.h); this thread schedules the
  // READs and publishes.
  EstimatorParams ep = estimator_params(cfg_, info.num_cu);
  DispatchEstimator est;
  est.invalidate(mono_ns());
  int64_t grid = mono_ns();  // the fixed tick grid; next = grid + the dithered offset
  int64_t next = grid;
  TickDither dither(0x9E3779B97F4A7C15ull ^ (static_cast<uint64_t>(dev) << 32) ^ static_cast<uint64_t>(grid));
  PmcSample& pmc_base = st.pmc_base;
  bool fresh_mode = false;           // reader switched to synchronous READs (quiet at the idle rate)
  int64_t last_pmc_ns = 0;
  int64_t last_start_ns = mono_ns();  // last (re)START of the counter session
  int64_t quiet_run_ns = 0;          // start of the current run of quiet drains (quiet release)
  int64_t park_ns = 0;               // when the session was last released for quiet
  int64_t unpark_retry_at_ns = 0;    // after a failed re-acquire of a parked device
  UnparkDetector unpark(kUnparkTablePct, kUnparkBusyPct, kUnparkWindowS);  // kgs/unpark.h
  // A fresh START restarts every count at 0: the interval from START to the first
  // READ is then counted exactly (acquire → first READ was dropped).
  auto started_at = [&](int64_t t) {
    est.restart(t);
    fresh_mode = false;  // a (re)opened session reads pipelined
    last_start_ns = t;
  };
  // Totals of the published stream become the base of the next session's counts.
  auto carry_base = [&] {
    PmcSample last;
    if (st.pmc_latest.load(last)) pmc_base = last;
  };
  // A park ended: its time joins the total (kgs_pmc_parked_seconds_total).
  DeviceState::ParkTime pt;  // this thread's copy of st.park_time (carried over a pause / resume)
  st.park_time.load(pt);
  auto end_park = [&] {
    if (pt.since_ns > 0) {
      pt.ended_ns += mono_ns() - pt.since_ns;
      pt.since_ns = 0;
      st.park_time.store(pt);
    }
  };
  // Open the breaker: stop READing this device, retry after the backoff.
  auto trip = [&](int64_t now) {
    ++P.pmc_epoch;  // the counter integral stops here: the READ-immune util falls back to PMFW
    st.pmc_failed.store(1);
    st.pmc_breaker_trips.fetch_add(1, std::memory_order_relaxed);
    carry_base();
    src->release(dev);  // bounded by the source's deadline
    st.pmc_on.store(0);
    st.pmc_stalled.store(0);
    st.pmc_quiet.store(0, std::memory_order_relaxed);
    st.pmc_dbound.store(0, std::memory_order_relaxed);
    st.pmc_fail_streak = 0;
    st.pmc_retry_at_ns = now + static_cast<int64_t>(st.pmc_backoff_s * 1e9);
    st.pmc_backoff_s = std::min(st.pmc_backoff_s * 2, cfg_.pmc_retry_max_s);
    est.invalidate(now);
  };

  while (!stop_.load(std::memory_order_relaxed)) {
    const int want = st.pmc_want.load(std::memory_order_relaxed);
    // ---- hand-over: release on request ----------------------------------------
    if (st.pmc_stall_req.exchange(0, std::memory_order_relaxed) && st.pmc_on.load(std::memory_order_relaxed)) {
      if (src->inject_stall(dev) == 0) st.pmc_stalls_injected.fetch_add(1, std::memory_order_relaxed);
      if (gone()) return;
    }
    if (!want && st.pmc_on.load(std::memory_order_relaxed)) {
      ++P.pmc_epoch;
      src->release(dev);  // a failed STOP still ends our READs
      if (gone()) return;
      st.pmc_on.store(0);
      st.pmc_stalled.store(0);
      st.pmc_releases.fetch_add(1, std::memory_order_relaxed);
      // The next START restarts the counts at 0: carry the published totals
      // as a base so the exported counters stay monotonic.
      carry_base();
    }
    if (!want && st.pmc_parked.load(std::memory_order_relaxed)) {
      end_park();
      st.pmc_parked.store(0);  // handed over while parked: nothing is held, the hand-over stands
      st.pmc_releases.fetch_add(1, std::memory_order_relaxed);
    }
    if (!want && st.pmc_drop_queue.exchange(0)) {  // "released": no queue left mapped either
      src->reset(dev);
      if (gone()) return;
    }
    // ---- quiet release ended: PMFW busy again, or the control plane asked -----
    if (want && st.pmc_parked.load(std::memory_order_relaxed) && mono_ns() >= unpark_retry_at_ns) {
      // ... or parking is off now: the quiet release set to 0, or profiling mode (every
      // tick READ) switched on while parked.
      bool wake = st.pmc_unpark_req.exchange(0, std::memory_order_relaxed) != 0 ||
                  !(pmc_quiet_release_s_.load(std::memory_order_relaxed) > 0) ||
                  !(pmc_idle_hz_.load(std::memory_order_relaxed) > 0);
      // ... or the PMFW shows work again, or has gone silent for three of its periods
      // (≥ 1 s: nothing would bill the GPU while parked) — kgs/unpark.h.
      int64_t busy_ns = 0;
      GpuSample g;
      const bool have_g = st.latest.load(g);
      if (!wake) wake = unpark.poll(mono_ns(), have_g ? &g : nullptr, pmfw_silent_ns, &busy_ns);
      if (wake) {
        const int rc = src->acquire(dev);
        if (gone()) return;
        const int64_t now_c = mono_ns();
        if (rc == 0) {
          ++P.pmc_epoch;
          st.pmc_on.store(1);
          end_park();
          st.pmc_parked.store(0);
          started_at(now_c);
          src->set_fresh(dev, false);  // the released session was READ synchronously (quiet)
          if (gone()) return;
          quiet_run_ns = 0;
          if (busy_ns) st.pmc_unpark_lag_ns.store(now_c - busy_ns, std::memory_order_relaxed);
        } else {
          ++P.pmc_errors;
          unpark_retry_at_ns = now_c + 1000000000LL;  // stays parked (PMFW billing); retry ≤ 1/s
        }
      }
    }
    st.pmc_unpark_req.store(0, std::memory_order_relaxed);  // only meaningful while parked
    // ---- (re)acquire: after a hand-over, or a retry of an open breaker --------
    if (want && !st.pmc_on.load(std::memory_order_relaxed) && !st.pmc_parked.load(std::memory_order_relaxed) &&
        mono_ns() >= st.pmc_retry_at_ns) {
      const bool failed = st.pmc_failed.load() != 0;
      if (failed) {  // wedged before: drop the old queue, then START on a fresh one
        st.pmc_retries.fetch_add(1, std::memory_order_relaxed);
        src->reset(dev);
        if (gone()) return;
      }
      const int rc = src->acquire(dev);
      if (gone()) return;
      const int64_t now_c = mono_ns();
      if (rc == 0) {
        ++P.pmc_epoch;
        st.pmc_on.store(1);
        started_at(now_c);  // the breaker closes on the first good drain
      } else {
        ++P.pmc_errors;
        if (failed) {
          st.pmc_retry_at_ns = now_c + static_cast<int64_t>(st.pmc_backoff_s * 1e9);
          st.pmc_backoff_s = std::min(st.pmc_backoff_s * 2, cfg_.pmc_retry_max_s);
        } else {
          st.pmc_retry_at_ns = now_c + 1000000000LL;  // after a failed START: ≤ 1 retry/s
        }
      }
    }
    bool pmc_now = st.pmc_on.load(std::memory_order_relaxed) != 0;
    if (pmc_now && (est.quiet() || est.dbound())) {
      // Quiet (no waves) READs at the idle rate, a dispatch-bound stream at the
      // dispatch rate; profiling mode (idle rate 0) READs every tick.
      const double idle_hz = pmc_idle_hz_.load(std::memory_order_relaxed);
      const double slow_hz = est.quiet() ? idle_hz : pmc_dispatch_hz_.load(std::memory_order_relaxed);
      if (idle_hz > 0 && slow_hz < hz && mono_ns() - last_pmc_ns < static_cast<int64_t>(1e9 / slow_hz)) {
        pmc_now = false;
        (est.quiet() ? st.pmc_quiet_skips : st.pmc_dbound_skips).fetch_add(1, std::memory_order_relaxed);
      }
    }
    if (pmc_now) {
      PmcSample ps;
      const int64_t p0 = mono_ns();
      last_pmc_ns = p0;
      const int prc = src->sample(dev, ps);
      if (gone()) return;
      P.pmc_read_seconds += (mono_ns() - p0) * 1e-9;
      if (prc == 0 && est.have_prev() && ps.mono_ns < est.prev_ns()) {
        // A drain stamped before the previous one: folding it would
        // run the published totals and integrals backwards.  The counts are
        // cumulative, so the next drain covers the interval; drop this one.
        st.pmc_reordered.fetch_add(1, std::memory_order_relaxed);
      } else if (prc == 0) {
        st.pmc_fail_streak = 0;
        if (st.pmc_failed.load(std::memory_order_relaxed)) {  // a retry worked: close the breaker
          st.pmc_failed.store(0);
          st.pmc_backoff_s = cfg_.pmc_retry_s;
        }
        Drain dr;
        dr.mono_ns = ps.mono_ns;
        dr.mask = ps.mask;
        dr.count = ps.value[kPmcGrbmCount];
        dr.spi = ps.value[kPmcGrbmActive];
        dr.mfma = ps.value[kPmcMfmaBusy];
        dr.cpc = ps.value[kPmcCpcBusy];
        dr.se_fresh = ps.se_fresh != 0;
        dr.fresh_mode = fresh_mode;
        const DrainStep r = est.feed(dr, ep);
        P.mfma_busy_seconds += r.mfma_s;
        P.active_seconds += r.active_s;
        if (r.have_dispatch) {
          P.dispatch_seconds += r.dispatch_s;
          ++P.dispatch_drains;
        }
        if (r.span_s > 0) P.pmc_last_share = (r.have_dispatch ? r.dispatch_s : r.active_s) / r.span_s;
        if (r.learned && dr.se_fresh) P.cpc_read_us = est.cpc_read_us();
        P.pmc_clk_idle_hz = est.clk_idle_hz();
        P.pmc_clk_busy_hz = est.clk_busy_hz();
        st.pmc_quiet.store(r.quiet ? 1 : 0, std::memory_order_relaxed);
        st.pmc_dbound.store(r.dbound ? 1 : 0, std::memory_order_relaxed);
        {  // quiet release: how long the device has been quiet, READ at the idle rate
          const double qr = pmc_quiet_release_s_.load(std::memory_order_relaxed);
          if (r.quiet && qr > 0 && pmc_idle_hz_.load(std::memory_order_relaxed) > 0) {
            if (quiet_run_ns == 0) quiet_run_ns = ps.mono_ns;
          } else {
            quiet_run_ns = 0;
          }
        }
        {
          const double idle_hz = pmc_idle_hz_.load(std::memory_order_relaxed);
          const bool slow = r.quiet && idle_hz > 0 && idle_hz < hz;
          if (slow != fresh_mode) {
            src->set_fresh(dev, slow);
            if (gone()) return;
            fresh_mode = slow;
          }
        }
        const int64_t stall = ps.mono_ns - est.last_plausible_ns();
        st.pmc_stalled.store(stall >= kPmcStallNs ? 1 : 0, std::memory_order_relaxed);
        for (int i = 0; i < kPmcCount; ++i) ps.value[i] += pmc_base.value[i];
        if (pmc_base.n_xcd == ps.n_xcd)
          for (uint32_t x = 0; x < ps.n_xcd && x < static_cast<uint32_t>(kMaxXcc); ++x) {
            ps.xcd_active[x] += pmc_base.xcd_active[x];
            ps.xcd_mfma[x] += pmc_base.xcd_mfma[x];
            ps.xcd_ta[x] += pmc_base.xcd_ta[x];
          }
        ps.seq = ++pmc_seq;
        st.pmc_ring.push(ps);
        if (ps.se_fresh && ps.mono_ns - last_slow_ns >= kPmcSlowNs) {  // window gauges: fresh MFMA / TA
          st.pmc_slow_ring.push(ps);
          last_slow_ns = ps.mono_ns;
        }
        st.pmc_latest.store(ps);
        ++P.pmc_samples;
        P.pmc_last_ns = ps.mono_ns;
        const bool reclaim = cfg_.pmc_reclaim_s > 0 && stall >= static_cast<int64_t>(cfg_.pmc_reclaim_s * 1e9);
        const bool refresh = cfg_.pmc_refresh_s > 0 &&
                             ps.mono_ns - last_start_ns >= static_cast<int64_t>(cfg_.pmc_refresh_s * 1e9);
        if ((reclaim || refresh) && st.pmc_want.load(std::memory_order_relaxed)) {
          // STOP + START our session (selects reprogrammed, counts from 0); totals
          // carry over like a hand-over.
          pmc_base = ps;
          src->release(dev);
          if (gone()) return;
          const int arc = src->acquire(dev);
          if (gone()) return;
          const int64_t t = mono_ns();
          if (arc == 0) {
            (reclaim ? st.pmc_reclaims : st.pmc_refreshes).fetch_add(1, std::memory_order_relaxed);
            started_at(t);
          } else {
            ++P.pmc_epoch;
            st.pmc_on.store(0);
            st.pmc_retry_at_ns = t + 1000000000LL;
            ++P.pmc_errors;
            est.invalidate(t);
            last_start_ns = t;
          }
        }
        const double qr = pmc_quiet_release_s_.load(std::memory_order_relaxed);
        if (quiet_run_ns && qr > 0 && st.pmc_on.load(std::memory_order_relaxed) &&
            st.pmc_want.load(std::memory_order_relaxed) && ps.mono_ns - quiet_run_ns >= static_cast<int64_t>(qr * 1e9)) {
          // Park: STOP the session and destroy the READ queue (nothing of the counter
          // tier left on the GPU); totals carry over like a hand-over, and the billing
          // falls back to the PMFW at the epoch change.
          ++P.pmc_epoch;
          carry_base();
          src->release(dev);
          if (gone()) return;
          src->reset(dev);
          if (gone()) return;
          park_ns = mono_ns();
          unpark.parked(park_ns);
          st.pmc_on.store(0);
          pt.since_ns = park_ns;
          st.park_time.store(pt);
          st.pmc_parked.store(1);
          st.pmc_parks.fetch_add(1, std::memory_order_relaxed);
          st.pmc_quiet.store(0, std::memory_order_relaxed);
          st.pmc_dbound.store(0, std::memory_order_relaxed);
          st.pmc_unpark_req.store(0, std::memory_order_relaxed);
          quiet_run_ns = 0;
          fresh_mode = false;
          est.invalidate(park_ns);
        }
      } else if (prc == kPmcPending) {
        // A batched reader's first READs are not published yet: nothing to fold.
      } else if (stop_.load(std::memory_order_relaxed)) {
        break;  // stop() aborted the wait: not a device failure
      } else {
        ++P.pmc_errors;
        if (++st.pmc_fail_streak >= cfg_.pmc_breaker_k) {
          trip(mono_ns());
          if (gone()) return;
        }
      }
    }

    // ---- schedule --------------------------------------------------------
    int64_t step = period_ns;
    // Nothing to READ (handed over / breaker open): poll the hand-over flag and the
    // retry deadline at ≤ 100 Hz instead of every tick.
    if (!st.pmc_on.load(std::memory_order_relaxed)) step = std::max<int64_t>(period_ns, 10000000LL);
    grid += step;
    next = grid + static_cast<int64_t>(dither.step(period_ns, cfg_.tick_dither));
    const int64_t now = mono_ns();
    if (next <= now) {
      ++P.overruns;
      // Late by a few periods (a slow drain, a descheduled thread): keep the
      // absolute schedule, so the missed ticks run at once and the delivered rate
      // stays the configured one.  Further behind, the rate is beyond the work (or
      // the host stalled): re-anchor and sleep a quarter period instead of bursting.
      if (now - next > kCatchUpPeriods * step) {
        grid = next = now + period_ns / 4;
        dither.reset();
      }
    }
    st.pmc_integ.store(P);
    // Sleep until the absolute deadline or until stop() signals the eventfd.
    const int64_t wait = next - now;
    if (wait > 0) {
      timespec ts{static_cast<time_t>(wait / 1000000000LL), static_cast<long>(wait % 1000000000LL)};
      pollfd pfd{stop_fd_, POLLIN, 0};
      ppoll(&pfd, 1, &ts, nullptr);
    }
    {  // wake-up lateness (kgs_sampler_wake_lateness_seconds)
      const int64_t late = mono_ns() - next;
      if (late > 0) st.wake_late_ns.fetch_add(static_cast<uint64_t>(late), std::memory_order_relaxed);
      const double us = late * 1e-3;
      int b = 0;
      while (b < kReadHistBuckets && us > kReadHistBoundsUs[b]) ++b;
      st.wake_hist[b].fetch_add(1, std::memory_order_relaxed);
    }
  }
  st.pmc_integ.store(P);
}

// Management-library tiers of one device (see sampler.h): its per-process list
// and its link table + RAS health, on its own "kgs-slow<N>" thread.  A call that
// never returns stalls this device's slow tiers only; their results go stale
// (the renderer drops them after stale_after) and stop() abandons the thread.
void Sampler::run_slow(Worker& w) {
  const int dev = w.dev;
  DeviceState& st = *states_[static_cast<size_t>(dev)];
  char tname[16];
  std::snprintf(tname, sizeof tname, "kgs-slow%d", dev);
  pthread_setname_np(pthread_self(), tname);
  const int64_t proc_ns = proc_period_ns(), link_ns = link_period_ns();
  Backend* const be = be_;
  auto gone = [&w] { return w.abandoned.load(std::memory_order_acquire); };
  // Bracket one management-library call: kgs_slow_call_seconds shows it while in flight.
  auto begin = [&](int tier) {
    st.slow_call_tier.store(tier, std::memory_order_relaxed);
    st.slow_call_ns.store(mono_ns(), std::memory_order_release);
  };
  auto end = [&] { st.slow_call_ns.store(0, std::memory_order_release); };
  // Stagger the devices' first passes over one period: with AMD SMI serialising
  // callers, N threads waking together would queue behind each other every pass.
  const int n_dev = std::max<int>(1, static_cast<int>(dev_ids_.size()));
  const int pos = static_cast<int>(std::find(dev_ids_.begin(), dev_ids_.end(), dev) - dev_ids_.begin());
  int64_t next_proc = mono_ns() + (proc_ns > 0 ? proc_ns / n_dev * pos : 0);
  int64_t next_link = mono_ns() + (link_ns > 0 ? link_ns / n_dev * pos : 0);
  std::vector<ProcInfo> procs;
  std::vector<LinkInfo> links;
  while (!stop_.load(std::memory_order_relaxed)) {
    const int64_t t0 = mono_ns();
    if (proc_ns > 0 && t0 >= next_proc) {
      std::shared_ptr<const std::unordered_map<uint64_t, std::string>> pid_pods;
      {
        std::lock_guard<std::mutex> g(pid_pods_mu_);
        pid_pods = pid_pods_;
      }
      const int64_t a = mono_ns();
      begin(kSlowProcs);
      const int rc = be->read_procs(dev, procs);
      end();
      if (gone()) return;
      if (rc == 0) {
        const int64_t now_p = mono_ns();
        int64_t& last = last_proc_ns_[static_cast<size_t>(dev)];
        const double dt = last ? (now_p - last) * 1e-9 : 0.0;
        const int cu = be->info(dev).num_cu;
        const double ncu = cu > 0 ? cu : 256.0;
        auto& cs = cu_seconds_[static_cast<size_t>(dev)];  // (pid, ∫ occupancy share dt), sorted by pid
        auto& pods = pod_cu_[static_cast<size_t>(dev)];
        bool pods_changed = false;
        std::vector<std::pair<uint32_t, double>> next_cs;
        next_cs.reserve(procs.size());
        int unavailable = 0;
        std::set<std::string> unknown_pods;
        for (ProcInfo& p : procs) {
          auto it = std::lower_bound(cs.begin(), cs.end(), std::make_pair(p.pid, -1.0));
          const bool known = it != cs.end() && it->first == p.pid;
          // An unreadable CU occupancy adds nothing, not 0 % of the interval: the
          // process's integral stands still, and its pod is flagged.
          const double inc = known && p.cu_valid ? p.cu_occupancy / ncu * dt : 0.0;
          unavailable += !p.cu_valid;
          p.cu_seconds = known ? it->second + inc : 0.0;
          next_cs.emplace_back(p.pid, p.cu_seconds);
          // The pod's integral keeps what its processes ran after they exit: the
          // per-pod compute share a shared GPU is billed by.
          if (pid_pods) {
            auto po = pid_pods->find((static_cast<uint64_t>(static_cast<uint32_t>(dev)) << 32) | p.pid);
            if (po != pid_pods->end()) {
              if (!p.cu_valid) {
                unknown_pods.insert(po->second);
              } else {
                auto [pv, fresh] = pods.try_emplace(po->second, 0.0);
                if (inc > 0 || fresh) pods_changed = true;
                pv->second += inc;
              }
            }
          }
        }
        std::sort(next_cs.begin(), next_cs.end());
        cs.swap(next_cs);  // processes that exited drop out
        last = now_p;
        auto sp = std::make_shared<const std::vector<ProcInfo>>(procs);
        std::shared_ptr<const std::map<std::string, double>> pc;
        if (pods_changed) pc = std::make_shared<const std::map<std::string, double>>(pods);
        auto uk = std::make_shared<const std::set<std::string>>(std::move(unknown_pods));
        {
          std::lock_guard<std::mutex> g(st.slow_mu);
          st.procs = std::move(sp);
          st.procs_mono_ns = now_p;
          if (pc) st.pod_cu = std::move(pc);
          st.pod_cu_unknown = std::move(uk);
        }
        st.procs_cu_unavailable.store(unavailable, std::memory_order_relaxed);
        st.procs_ok_ns.store(now_p, std::memory_order_release);
        st.proc_reads.fetch_add(1, std::memory_order_relaxed);
      } else {
        st.proc_errors.fetch_add(1, std::memory_order_relaxed);
      }
      st.slow_ns_total.fetch_add(static_cast<uint64_t>(mono_ns() - a), std::memory_order_relaxed);
      next_proc += proc_ns;
      if (next_proc <= mono_ns()) next_proc = mono_ns() + proc_ns;  // a pass overran: skip, do not burst
    }
    if (link_ns > 0 && mono_ns() >= next_link && !stop_.load(std::memory_order_relaxed)) {
      const int64_t a = mono_ns();
      begin(kSlowLinks);
      const int lrc = be->read_links(dev, links);
      end();
      if (gone()) return;
      if (lrc == 0) {
        auto l = std::make_shared<const std::vector<LinkInfo>>(links);
        {
          std::lock_guard<std::mutex> g(st.slow_mu);
          st.links = std::move(l);
        }
        st.links_ok_ns.store(mono_ns(), std::memory_order_release);
      } else {
        st.link_errors.fetch_add(1, std::memory_order_relaxed);
      }
      HealthInfo h;
      begin(kSlowHealth);
      const int hrc = be->read_health(dev, h);
      end();
      if (gone()) return;
      if (hrc == 0) {
        auto hp = std::make_shared<const HealthInfo>(h);
        {
          std::lock_guard<std::mutex> g(st.slow_mu);
          st.health = std::move(hp);
        }
        st.health_ok_ns.store(mono_ns(), std::memory_order_release);
      } else {
        st.health_errors.fetch_add(1, std::memory_order_relaxed);
      }
      st.link_reads.fetch_add(1, std::memory_order_relaxed);
      st.slow_ns_total.fetch_add(static_cast<uint64_t>(mono_ns() - a), std::memory_order_relaxed);
      next_link += link_ns;
      if (next_link <= mono_ns()) next_link = mono_ns() + link_ns;
    }
    slow_passes_.fetch_add(1, std::memory_order_relaxed);
    int64_t next = INT64_MAX;
    if (proc_ns > 0) next = next_proc;
    if (link_ns > 0 && next_link < next) next = next_link;
    const int64_t wait = next - mono_ns();
    if (wait > 0) {
      timespec ts{static_cast<time_t>(wait / 1000000000LL), static_cast<long>(wait % 1000000000LL)};
      pollfd pfd{stop_fd_, POLLIN, 0};
      ppoll(&pfd, 1, &ts, nullptr);
    }
  }
}

bool Sampler::window_busy(int dev, double window_s, double& gfx, double& umc, int& n, double* util) const {
  const DeviceState& st = *states_[dev];
  n = 0;
  GpuSample b, a, e;
  const uint64_t h = st.ring.head();  // one view of the ring for the whole search
  if (st.ring.at_from(h, 0, b) && b.cum_dt_s > 0) {
    // Newest ring entry with at least window_s of firmware time after it: the
    // window mean is the difference of the two running sums (O(log ring) loads).
    const double want = b.cum_dt_s - window_s;
    size_t lo = 1, hi = std::min<uint64_t>(h, kRing - 1);
    bool have = false;
    while (lo < hi) {
      const size_t mid = lo + (hi - lo) / 2;
      if (!st.ring.at_from(h, mid, e)) {  // torn / lapped under us: treat as too new
        lo = mid + 1;
        continue;
      }
      if (e.cum_dt_s <= want) {
        a = e;
        have = true;
        hi = mid;
      } else {
        lo = mid + 1;
      }
    }
    if (!have) {  // window longer than the history held: use the oldest entry
      const size_t m = std::min<uint64_t>(h, kRing - 1);
      have = m > 1 && st.ring.at_from(h, m - 1, a);
    }
    if (have && b.cum_dt_s > a.cum_dt_s) {
      const double dt = b.cum_dt_s - a.cum_dt_s;
      gfx = 100.0 * (b.cum_gfx_s - a.cum_gfx_s) / dt;
      umc = 100.0 * (b.cum_umc_s - a.cum_umc_s) / dt;
      if (util) *util = 100.0 * (b.cum_util_s - a.cum_util_s) / dt;
      n = static_cast<int>(b.seq - a.seq);
      return true;
    }
  }
  GpuSample s;
  if (!st.latest.load(s)) return false;
  gfx = s.gfx_busy_pct;
  umc = s.umc_busy_pct;
  if (util) *util = s.util_window_pct >= 0 ? s.util_window_pct : s.gfx_busy_pct;
  n = 1;
  return true;
}

bool Sampler::window_pmc(int dev, double window_s, PmcRates& out) const {
  const DeviceState& st = *states_[dev];
  PmcSample b;
  if (!st.pmc_latest.load(b)) return false;
  // Binary search the decimated ring (time-ordered, newest first) for the newest
  // entry at least window_s older than `b`; fall back to the oldest one held.
  const int64_t want = b.mono_ns - static_cast<int64_t>(window_s * 1e9);
  const uint64_t h = st.pmc_slow_ring.head();
  size_t lo = 0, hi = std::min<uint64_t>(h, kPmcSlowRing - 1);
  if (hi == 0) return false;
  PmcSample a, e;
  bool have_a = false;
  while (lo < hi) {
    const size_t mid = lo + (hi - lo) / 2;
    if (!st.pmc_slow_ring.at_from(h, mid, e)) {  // torn / lapped under us: treat as too new
      lo = mid + 1;
      continue;
    }
    if (e.mono_ns <= want) {
      a = e;
      have_a = true;
      hi = mid;
    } else {
      lo = mid + 1;
    }
  }
  if (!have_a) {  // window longer than the history: use the oldest entry
    const size_t n = std::min<uint64_t>(h, kPmcSlowRing - 1);
    if (n == 0 || !st.pmc_slow_ring.at_from(h, n - 1, a)) return false;
  }
  if (a.mono_ns >= b.mono_ns) return false;
  out = pmc_rates(a, b, be_->info(dev).num_cu);
  return out.dt_s > 0;
}

}  // namespace kgs
