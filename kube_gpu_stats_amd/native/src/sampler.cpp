// Per-GPU sampler threads.  See sampler.h.
#include "kgs/sampler.h"

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

}  // namespace

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
  if (cfg_.hz <= 0) cfg_.hz = 1;
  pmc_idle_hz_.store(cfg_.pmc_idle_hz < 0 ? 0 : cfg_.pmc_idle_hz);
  for (int d : dev_ids_) states_[static_cast<size_t>(d)]->pmc_on.store(cfg_.pmc && pmc_ ? 1 : 0);
  cu_seconds_.resize(static_cast<size_t>(n));
  last_proc_ns_.assign(static_cast<size_t>(n), 0);
  stop_fd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
}

void Sampler::set_hz(double hz) {
  if (hz <= 0) return;
  const bool was = running_.load();
  stop();
  cfg_.hz = hz;
  if (was) start();
}

void Sampler::set_pmc_wanted(bool on) {
  for (int d : dev_ids_) states_[static_cast<size_t>(d)]->pmc_want.store(on ? 1 : 0);
}

Sampler::~Sampler() {
  stop();
  if (stop_fd_ >= 0) close(stop_fd_);
}

void Sampler::start() {
  if (running_.exchange(true)) return;
  stop_.store(false);
  uint64_t drain;
  while (read(stop_fd_, &drain, sizeof drain) > 0) {
  }
  for (int d : dev_ids_) threads_.emplace_back([this, d] { run(d); });
  if (cfg_.proc_every > 0 || cfg_.link_every > 0 || cfg_.proc_period_s > 0 || cfg_.link_period_s > 0)
    slow_thread_ = std::thread([this] { run_slow(); });
}

void Sampler::stop() {
  if (!running_.load()) return;
  stop_.store(true);
  const uint64_t one = 1;
  if (write(stop_fd_, &one, sizeof one) < 0) {
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  if (slow_thread_.joinable()) slow_thread_.join();
  running_.store(false);
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
  if ((cur.valid & kFEnergy) && (prev->valid & kFEnergy) && cur.energy_acc >= prev->energy_acc)
    I.energy_joules += energy_units_to_joules(cur.energy_acc - prev->energy_acc);
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

void Sampler::run(int dev) {
  DeviceState& st = *states_[dev];
  const DeviceInfo& info = be_->info(dev);
  if (cfg_.pin_numa) {
    const std::vector<int> cpus = numa_cpus(info.numa_node);
    if (!cpus.empty()) {
      cpu_set_t set;
      CPU_ZERO(&set);
      for (int c : cpus) CPU_SET(c, &set);
      if (pthread_setaffinity_np(pthread_self(), sizeof set, &set) == 0) st.cpu_pinned.store(static_cast<int>(cpus.size()));
    }
  }
  char tname[16];
  std::snprintf(tname, sizeof tname, "kgs-gpu%d", dev);
  pthread_setname_np(pthread_self(), tname);
  // The default 50 µs timer slack is 40 % of an 8 kHz period: wake on time.
  // (KGS_TIMERSLACK_NS overrides, for interference experiments.)
  const char* slack = std::getenv("KGS_TIMERSLACK_NS");
  prctl(PR_SET_TIMERSLACK, slack ? std::strtoul(slack, nullptr, 10) : 1000UL, 0, 0, 0);

  const int64_t period_ns = static_cast<int64_t>(1e9 / cfg_.hz);
  const uint64_t pmfw_every = cfg_.pmfw_hz > 0 && cfg_.pmfw_hz < cfg_.hz
                                  ? static_cast<uint64_t>(cfg_.hz / cfg_.pmfw_hz + 0.5)
                                  : 1;
  Integrals I;
  GpuSample& prev = st.pmfw_prev;
  bool& have_prev = st.have_pmfw_prev;
  uint64_t seq = 0, pmc_seq = 0, tick = 0;
  int64_t last_slow_ns = 0;
  {  // resume after a pause: counters and sequence numbers continue
    st.integ.load(I);
    GpuSample last;
    if (st.latest.load(last)) seq = last.seq;
    PmcSample lp;
    if (st.pmc_latest.load(lp)) pmc_seq = lp.seq;
  }
  // A thread that stopped (pause, rate change) while its device was quiet left
  // the reader in synchronous mode: start pipelined, not quiet.
  if (cfg_.pmc && pmc_ && st.pmc_on.load()) pmc_->set_fresh(dev, false);
  st.pmc_quiet.store(0, std::memory_order_relaxed);
  int64_t next = mono_ns();
  int late_streak = 0;  // consecutive overrun ticks
  PmcSample& pmc_base = st.pmc_base;
  int64_t last_acquire_fail_ns = 0;
  bool have_prev_ps = false;         // stall detection: previous raw GRBM_COUNT and its time
  uint64_t prev_ps_count = 0, prev_ps_mfma = 0, prev_ps_active = 0;
  bool quiet = false;                // adaptive READ rate (SamplerConfig::pmc_idle_hz)
  int64_t quiet_since_ns = 0;        // start of the current run of quiet READ intervals (0 = none)
  bool fresh_mode = false;           // reader switched to synchronous READs (quiet at the idle rate)
  int64_t last_pmc_ns = 0;
  int64_t prev_ps_ns = 0;
  int64_t last_plausible_ns = mono_ns();
  int64_t last_start_ns = mono_ns();  // last (re)START of the counter session

  while (!stop_.load(std::memory_order_relaxed)) {
    // ---- fast tier: the PMFW table (refreshed by firmware every ≈20 ms) is
    // read every `pmfw_every` ticks, i.e. at ≤ pmfw_hz however fast the
    // counter tier runs.  A failing device backs off on this tier. ----------
    int backoff_shift = 0;
    if (tick % pmfw_every == 0 || st.consecutive_errors.load(std::memory_order_relaxed) > 0) {
      GpuSample s;
      const int64_t t0 = mono_ns();
      const int rc = be_->read_metrics(dev, s);
      const int64_t t1 = mono_ns();
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
          integrate(dev, have_prev && !reset ? &prev : nullptr, s, I);
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
          if (be_->recover(dev) == 0) {
            ++I.recoveries;
            have_prev = false;
          }
        }
      }
    }

    // ---- PMC tier ------------------------------------------------------
    bool pmc_now = false;
    if (cfg_.pmc && pmc_) {
      const int want = st.pmc_want.load(std::memory_order_relaxed);
      if (want != st.pmc_on.load(std::memory_order_relaxed)) {
        const int64_t now_c = mono_ns();
        if (!want) {
          pmc_->release(dev);  // a failed STOP still ends our READs
          st.pmc_on.store(0);
          st.pmc_stalled.store(0);
          st.pmc_releases.fetch_add(1, std::memory_order_relaxed);
          // The next START restarts the counts at 0: carry the published totals
          // as a base so the exported counters stay monotonic.
          PmcSample last;
          if (st.pmc_latest.load(last)) pmc_base = last;
        } else if (now_c - last_acquire_fail_ns >= 1000000000LL) {  // after a failed START: ≤ 1 retry/s
          if (pmc_->acquire(dev) == 0) {
            st.pmc_on.store(1);
            have_prev_ps = false;
            quiet = false;
            quiet_since_ns = 0;
            fresh_mode = false;  // a (re)opened session reads pipelined
            last_plausible_ns = now_c;
            last_start_ns = now_c;
          } else {
            last_acquire_fail_ns = now_c;
            ++I.pmc_errors;
          }
        }
      }
      pmc_now = st.pmc_on.load(std::memory_order_relaxed) != 0;
    }
    if (pmc_now && quiet) {
      const double idle_hz = pmc_idle_hz_.load(std::memory_order_relaxed);
      if (idle_hz > 0 && idle_hz < cfg_.hz && mono_ns() - last_pmc_ns < static_cast<int64_t>(1e9 / idle_hz)) {
        pmc_now = false;
        st.pmc_quiet_skips.fetch_add(1, std::memory_order_relaxed);
      }
    }
    if (pmc_now) {
      PmcSample ps;
      const int64_t p0 = mono_ns();
      last_pmc_ns = p0;
      const int prc = pmc_->sample(dev, ps);
      I.pmc_read_seconds += (mono_ns() - p0) * 1e-9;
      if (prc == 0) {
        // Stall detection: GRBM_COUNT free-runs at the shader clock while our
        // session is programmed; frozen or foreign counts give no plausible clock.
        if (have_prev_ps && ps.mono_ns > prev_ps_ns) {
          const uint64_t raw = ps.value[kPmcGrbmCount];
          const double mhz = raw >= prev_ps_count ? (raw - prev_ps_count) * 1e3 / (ps.mono_ns - prev_ps_ns) : 0.0;
          if (mhz >= kPlausibleMhzLo && mhz <= kPlausibleMhzHi) last_plausible_ns = ps.mono_ns;
        }
        if (have_prev_ps && ps.mono_ns > prev_ps_ns && (ps.mask & (1u << kPmcMfmaBusy)) &&
            ps.value[kPmcGrbmCount] > prev_ps_count && ps.value[kPmcMfmaBusy] >= prev_ps_mfma) {
          // MFMA-busy share of all SIMD-cycles in the interval, times its length.
          const double simds = (info.num_cu > 0 ? info.num_cu : 256) * 4.0;
          const double frac = static_cast<double>(ps.value[kPmcMfmaBusy] - prev_ps_mfma) /
                              (simds * static_cast<double>(ps.value[kPmcGrbmCount] - prev_ps_count));
          I.mfma_busy_seconds += (frac > 1.0 ? 1.0 : frac) * (ps.mono_ns - prev_ps_ns) * 1e-9;
        }
        if (have_prev_ps && ps.mono_ns > prev_ps_ns && (ps.mask & (1u << kPmcGrbmActive)) &&
            ps.value[kPmcGrbmCount] > prev_ps_count && ps.value[kPmcGrbmActive] >= prev_ps_active) {
          const double frac = static_cast<double>(ps.value[kPmcGrbmActive] - prev_ps_active) /
                              static_cast<double>(ps.value[kPmcGrbmCount] - prev_ps_count);
          I.active_seconds += (frac > 1.0 ? 1.0 : frac) * (ps.mono_ns - prev_ps_ns) * 1e-9;
        }
        // Quiet = a shader engine had waves for < kQuietActiveFrac of the clocks
        // since the previous READ, and no MFMA cycle ran.  Both counters are
        // (nearly) blind to our own READs: SPI busy reads 0.65 % with nothing but
        // 8 kHz of READs on the GPU (profiles/r2/immunity/).
        // Without the activity counter in the set a device is never quiet.
        bool quiet_interval = false;
        if (have_prev_ps && (ps.mask & (1u << kPmcGrbmActive)) && ps.value[kPmcGrbmCount] > prev_ps_count) {
          const double act = static_cast<double>(ps.value[kPmcGrbmActive] - std::min(ps.value[kPmcGrbmActive], prev_ps_active));
          const double clk = static_cast<double>(ps.value[kPmcGrbmCount] - prev_ps_count);
          quiet_interval = act < kQuietActiveFrac * clk && ps.value[kPmcMfmaBusy] == prev_ps_mfma;
        }
        if (!quiet_interval) {
          quiet_since_ns = 0;
        } else if (quiet_since_ns == 0) {
          quiet_since_ns = prev_ps_ns;  // the interval began at the previous READ
        }
        quiet = quiet_interval && ps.mono_ns - quiet_since_ns >= kQuietHoldNs;
        st.pmc_quiet.store(quiet ? 1 : 0, std::memory_order_relaxed);
        {
          const double idle_hz = pmc_idle_hz_.load(std::memory_order_relaxed);
          const bool slow = quiet && idle_hz > 0 && idle_hz < cfg_.hz;
          if (slow != fresh_mode) {
            pmc_->set_fresh(dev, slow);
            fresh_mode = slow;
          }
        }
        prev_ps_count = ps.value[kPmcGrbmCount];
        prev_ps_mfma = ps.value[kPmcMfmaBusy];
        prev_ps_active = ps.value[kPmcGrbmActive];
        prev_ps_ns = ps.mono_ns;
        have_prev_ps = true;
        const int64_t stall = ps.mono_ns - last_plausible_ns;
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
        if (ps.mono_ns - last_slow_ns >= kPmcSlowNs) {
          st.pmc_slow_ring.push(ps);
          last_slow_ns = ps.mono_ns;
        }
        st.pmc_latest.store(ps);
        ++I.pmc_samples;
        const bool reclaim = cfg_.pmc_reclaim_s > 0 && stall >= static_cast<int64_t>(cfg_.pmc_reclaim_s * 1e9);
        const bool refresh = cfg_.pmc_refresh_s > 0 &&
                             ps.mono_ns - last_start_ns >= static_cast<int64_t>(cfg_.pmc_refresh_s * 1e9);
        if ((reclaim || refresh) && st.pmc_want.load(std::memory_order_relaxed)) {
          // STOP + START our session (selects reprogrammed, counts from 0); totals
          // carry over like a hand-over.
          pmc_base = ps;
          pmc_->release(dev);
          last_start_ns = ps.mono_ns;
          if (pmc_->acquire(dev) == 0) {
            (reclaim ? st.pmc_reclaims : st.pmc_refreshes).fetch_add(1, std::memory_order_relaxed);
          } else {
            st.pmc_on.store(0);
            last_acquire_fail_ns = ps.mono_ns;
            ++I.pmc_errors;
          }
          have_prev_ps = false;
          quiet = false;
          quiet_since_ns = 0;
          fresh_mode = false;
          last_plausible_ns = mono_ns();  // a full reclaim period before the next one
        }
      } else {
        ++I.pmc_errors;
      }
    }

    ++tick;

    // ---- schedule --------------------------------------------------------
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
      // A tick that ran long (the PMFW table read is ≈50–130 µs, longer than a
      // kHz period) is followed by one immediate tick, so the counter tier keeps
      // its rate; a second overrun in a row means the rate is beyond the work,
      // and then the thread sleeps a quarter period instead of spinning.
      next = now + (backoff_shift ? step : 0);
      if (next <= now && ++late_streak > 1) next = now + period_ns / 4;
    } else {
      late_streak = 0;
    }
    st.integ.store(I);
    // Sleep until the absolute deadline or until stop() signals the eventfd.
    const int64_t wait = next - now;
    timespec ts{static_cast<time_t>(wait / 1000000000LL), static_cast<long>(wait % 1000000000LL)};
    pollfd pfd{stop_fd_, POLLIN, 0};
    ppoll(&pfd, 1, &ts, nullptr);
  }
  st.integ.store(I);
}

// Node-wide management-library tiers (see sampler.h).  Each due device is read
// in turn; the per-GPU threads never wait on these calls.
void Sampler::run_slow() {
  pthread_setname_np(pthread_self(), "kgs-slow");
  const int64_t tick_ns = static_cast<int64_t>(1e9 / cfg_.hz);
  const int64_t proc_ns = cfg_.proc_period_s > 0 ? static_cast<int64_t>(cfg_.proc_period_s * 1e9)
                        : cfg_.proc_every > 0   ? tick_ns * cfg_.proc_every
                                                : 0;
  const int64_t link_ns = cfg_.link_period_s > 0 ? static_cast<int64_t>(cfg_.link_period_s * 1e9)
                        : cfg_.link_every > 0   ? tick_ns * cfg_.link_every
                                                : 0;
  int64_t next_proc = mono_ns(), next_link = next_proc;
  std::vector<ProcInfo> procs;
  std::vector<LinkInfo> links;
  while (!stop_.load(std::memory_order_relaxed)) {
    const int64_t t0 = mono_ns();
    if (proc_ns > 0 && t0 >= next_proc) {
      for (int dev : dev_ids_) {
        if (stop_.load(std::memory_order_relaxed)) break;
        DeviceState& st = *states_[static_cast<size_t>(dev)];
        const int64_t a = mono_ns();
        if (be_->read_procs(dev, procs) == 0) {
          const int64_t now_p = mono_ns();
          int64_t& last = last_proc_ns_[static_cast<size_t>(dev)];
          const double dt = last ? (now_p - last) * 1e-9 : 0.0;
          const int cu = be_->info(dev).num_cu;
          const double ncu = cu > 0 ? cu : 256.0;
          auto& cs = cu_seconds_[static_cast<size_t>(dev)];  // (pid, ∫ occupancy share dt), sorted by pid
          std::vector<std::pair<uint32_t, double>> next_cs;
          next_cs.reserve(procs.size());
          for (ProcInfo& p : procs) {
            auto it = std::lower_bound(cs.begin(), cs.end(), std::make_pair(p.pid, -1.0));
            const bool known = it != cs.end() && it->first == p.pid;
            p.cu_seconds = known ? it->second + p.cu_occupancy / ncu * dt : 0.0;
            next_cs.emplace_back(p.pid, p.cu_seconds);
          }
          std::sort(next_cs.begin(), next_cs.end());
          cs.swap(next_cs);  // processes that exited drop out
          last = now_p;
          auto sp = std::make_shared<const std::vector<ProcInfo>>(procs);
          {
            std::lock_guard<std::mutex> g(st.slow_mu);
            st.procs = std::move(sp);
            st.procs_mono_ns = now_p;
          }
          st.proc_reads.fetch_add(1, std::memory_order_relaxed);
        } else {
          st.proc_errors.fetch_add(1, std::memory_order_relaxed);
        }
        st.slow_ns_total.fetch_add(static_cast<uint64_t>(mono_ns() - a), std::memory_order_relaxed);
      }
      next_proc += proc_ns;
      if (next_proc <= mono_ns()) next_proc = mono_ns() + proc_ns;  // a pass overran: skip, do not burst
    }
    if (link_ns > 0 && mono_ns() >= next_link) {
      for (int dev : dev_ids_) {
        if (stop_.load(std::memory_order_relaxed)) break;
        DeviceState& st = *states_[static_cast<size_t>(dev)];
        const int64_t a = mono_ns();
        if (be_->read_links(dev, links) == 0) {
          auto l = std::make_shared<const std::vector<LinkInfo>>(links);
          std::lock_guard<std::mutex> g(st.slow_mu);
          st.links = std::move(l);
        }
        HealthInfo h;
        if (be_->read_health(dev, h) == 0) {
          auto hp = std::make_shared<const HealthInfo>(h);
          std::lock_guard<std::mutex> g(st.slow_mu);
          st.health = std::move(hp);
        }
        st.link_reads.fetch_add(1, std::memory_order_relaxed);
        st.slow_ns_total.fetch_add(static_cast<uint64_t>(mono_ns() - a), std::memory_order_relaxed);
      }
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

bool Sampler::window_busy(int dev, double window_s, double& gfx, double& umc, int& n) const {
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
      n = static_cast<int>(b.seq - a.seq);
      return true;
    }
  }
  GpuSample s;
  if (!st.latest.load(s)) return false;
  gfx = s.gfx_busy_pct;
  umc = s.umc_busy_pct;
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
