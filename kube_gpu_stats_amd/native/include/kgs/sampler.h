// Per-GPU sampler threads (SURVEY.md §3.4 "HOT LOOP", §2.3 device fan-out).
//
// One std::thread per device, pinned to the CPUs of the GPU's NUMA node, wakes
// on an absolute CLOCK_MONOTONIC deadline and every tick reads the PMFW table +
// HBM occupancy (fast tier, capped at pmfw_hz) and, if enabled, drains the
// hardware counters (PMC tier).  Those two are per-device files / queues: the
// per-GPU thread never takes a node-wide lock.
//
// The management-library tiers — per-process list (mid tier, every proc_every
// ticks' worth of time), xGMI link table + RAS health (slow tier, every
// link_every ticks' worth) — go through AMD SMI, which serialises callers on one
// process-wide mutex and takes milliseconds per call.  They run on ONE node-wide
// "kgs-slow" thread that walks the devices in turn, so a slow
// amdsmi_get_gpu_process_list on GPU 3 can never delay GPU 5's 8 kHz counter
// drain (profiles/r2/mock_scaling.md).
// A sample counts as *distinct* only when the firmware timestamp moved
// (BASELINE.md measurement rule).  Results are published through seqlocks; the
// scrape path never calls into the driver.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kgs/backend.h"
#include "kgs/pmc.h"
#include "kgs/sample.h"
#include "kgs/seqlock.h"

namespace kgs {

struct SamplerConfig {
  double hz = 10.0;            // tick rate: counter (PMC) tier runs every tick
  double pmfw_hz = 100.0;      // PMFW-table tier rate cap (table refreshes every ≈20 ms; 0 = every tick)
  int proc_every = 10;         // mid tier period = proc_every / hz seconds (0 disables)
  int link_every = 100;        // slow tier period = link_every / hz seconds (0 disables)
  // Absolute periods (seconds) for the two tiers; > 0 overrides the *_every
  // ticks, so a tick-rate change (set_hz) leaves them alone.
  double proc_period_s = 0, link_period_s = 0;
  bool pin_numa = true;
  bool pmc = false;            // drain hardware counters every tick
  // A foreign profiler (rocprofv3 --pmc) that STOPs or reprograms the perfmon
  // block leaves the exporter reading frozen or foreign counts (run r44).  The
  // counters are "stalled" when GRBM_COUNT has not advanced at a plausible clock
  // for kPmcStallNs; after pmc_reclaim_s of stall the sampler re-STARTs its
  // session (0 = never).  While handed over (SIGUSR1) nothing is reclaimed.
  double pmc_reclaim_s = 10.0;
  // A profiler that reprograms the counter selects can leave GRBM_COUNT counting
  // something clock-like (no stall) while our MFMA slot counts its event (run
  // r45: MFMA util 0 under load).  Nothing in the READ shows that, so the session
  // is also re-STARTed (selects reprogrammed) every pmc_refresh_s (0 = never).
  double pmc_refresh_s = 60.0;
  // Adaptive READ rate.  Every counter READ is a packet on the command processor
  // that GUI-active and the PMFW GFX busy (container_gpu_sm_util's source) count
  // as ≈190 / ≈80 µs of work: at 8 kHz an idle GPU reads ~99 % busy
  // (profiles/r2/idle_busy/).  While the last READ interval had waves for less
  // than kQuietActiveFrac of its clocks and no MFMA cycle (GRBM_SPI_BUSY and
  // MFMA busy, both blind to READs), the device is "quiet" and READs drop to
  // pmc_idle_hz; the first READ that sees work puts it back on every tick.
  // Cumulative counters keep every integral exact; only the time resolution of
  // idle stretches drops.  0 = READ every tick (profiling mode: full resolution,
  // and the PMFW GFX busy reads the READs as work).
  double pmc_idle_hz = 100.0;
  int max_backoff_ms = 1000;   // while a device keeps failing
  std::vector<int> devices;    // subset to sample (empty = all)
};

constexpr size_t kRing = 1024;          // ≥10 s of history at 100 Hz
// Counter samples decimated to one per kPmcSlowNs feed the window gauges, so a
// 1 s window is covered at any tick rate (the full-rate ring holds 85 ms at 12 kHz).
constexpr size_t kPmcSlowRing = 2048;
constexpr size_t kPmcRing = 8192;       // raw counter stream: ≥1 s at 8 kHz (/counters)
constexpr int64_t kPmcSlowNs = 5000000;  // 5 ms → ≥10 s of history
constexpr int kReadHistBuckets = 12;    // backend read latency histogram
constexpr int64_t kPmcStallNs = 500000000;  // GRBM_COUNT without a plausible clock this long = stalled
constexpr double kPlausibleMhzLo = 100.0, kPlausibleMhzHi = 4000.0;
// Adaptive READ rate: an interval whose SPI-busy share is below this is quiet.
constexpr double kQuietActiveFrac = 0.02;
// ... and the device counts as quiet only after this long of quiet intervals in a
// row: a host sync between kernels leaves the GPU idle for tens of µs, which is not
// worth a drop to the idle READ rate (the first READ after it would come up to one
// idle period late, and every tick in between is a lost sample).
constexpr int64_t kQuietHoldNs = 5000000;
extern const double kReadHistBoundsUs[kReadHistBuckets];

struct DeviceState {
  Seqlock<GpuSample> latest;
  SampleRing<GpuSample, kRing> ring;
  Seqlock<Integrals> integ;
  Seqlock<PmcSample> pmc_latest;
  SampleRing<PmcSample, kPmcRing> pmc_ring;         // every counter drain
  SampleRing<PmcSample, kPmcSlowRing> pmc_slow_ring;  // ≥ kPmcSlowNs apart (window gauges)

  mutable std::mutex slow_mu;  // guards the two shared_ptrs below
  std::shared_ptr<const std::vector<ProcInfo>> procs;
  std::shared_ptr<const std::vector<LinkInfo>> links;
  std::shared_ptr<const HealthInfo> health;
  int64_t procs_mono_ns = 0;

  std::atomic<int> up{0};
  std::atomic<int64_t> last_ok_mono_ns{0};
  std::atomic<uint64_t> consecutive_errors{0};
  std::atomic<uint64_t> read_hist[kReadHistBuckets + 1] = {};
  std::atomic<int> cpu_pinned{-1};
  // Counter hand-over (`kgs exporter` SIGUSR1 / SIGUSR2, /control/pmc/*): the
  // control plane sets pmc_want; the sampler thread releases / re-acquires the
  // counters itself and reports the state in pmc_on.
  std::atomic<int> pmc_want{1};
  std::atomic<int> pmc_on{0};
  std::atomic<uint64_t> pmc_releases{0};
  std::atomic<int> pmc_stalled{0};          // counters frozen / implausible for ≥ kPmcStallNs
  std::atomic<uint64_t> pmc_reclaims{0};    // automatic re-STARTs after a stall
  std::atomic<uint64_t> pmc_refreshes{0};   // periodic re-STARTs (pmc_refresh_s)
  std::atomic<int> pmc_quiet{0};            // last READ interval had no wave: READs at pmc_idle_hz
  std::atomic<uint64_t> pmc_quiet_skips{0};  // ticks that skipped their READ while quiet
  PmcSample pmc_base;  // totals carried over hand-overs (sampler thread only; survives pause/resume)
  // Last distinct PMFW sample (sampler thread only).  Kept across pause/resume:
  // the firmware accumulators keep counting while the thread is stopped, so the
  // first sample after a resume integrates the paused interval exactly.
  GpuSample pmfw_prev;
  bool have_pmfw_prev = false;
  // Slow-thread self metrics: completed passes and their latency per tier.
  std::atomic<uint64_t> proc_reads{0}, proc_errors{0}, link_reads{0};
  std::atomic<uint64_t> slow_ns_total{0};

  std::shared_ptr<const std::vector<ProcInfo>> get_procs() const {
    std::lock_guard<std::mutex> g(slow_mu);
    return procs;
  }
  std::shared_ptr<const std::vector<LinkInfo>> get_links() const {
    std::lock_guard<std::mutex> g(slow_mu);
    return links;
  }
  std::shared_ptr<const HealthInfo> get_health() const {
    std::lock_guard<std::mutex> g(slow_mu);
    return health;
  }
};

class Sampler {
 public:
  Sampler(Backend* be, CounterSource* pmc, SamplerConfig cfg);
  ~Sampler();
  void start();
  void stop();
  bool running() const { return running_.load(); }

  int device_count() const { return static_cast<int>(states_.size()); }
  const DeviceState& state(int dev) const { return *states_[dev]; }
  const SamplerConfig& config() const { return cfg_; }
  const std::vector<int>& sampled_devices() const { return dev_ids_; }
  Backend* backend() const { return be_; }

  // Mean of gfx/umc busy over the trailing `window_s` of firmware time
  // (time-weighted by each sample's dt).  Returns false if no data.
  bool window_busy(int dev, double window_s, double& gfx_pct, double& umc_pct, int& n) const;
  // Counter-derived rates over the trailing window.
  bool window_pmc(int dev, double window_s, PmcRates& out) const;
  // Ask every sampled device's thread to hand its counters to another profiler
  // (false) or to take them back (true).  Takes effect within one tick.
  void set_pmc_wanted(bool on);
  // Change the tick rate (stops and restarts the threads; integrals continue).
  void set_hz(double hz);
  // Quiet-GPU counter READ rate (SamplerConfig::pmc_idle_hz), in place.
  void set_pmc_idle_hz(double hz) { pmc_idle_hz_.store(hz < 0 ? 0 : hz, std::memory_order_relaxed); }
  double pmc_idle_hz() const { return pmc_idle_hz_.load(std::memory_order_relaxed); }
  // Node-wide slow thread: passes completed and whether it is running.
  uint64_t slow_passes() const { return slow_passes_.load(); }

 private:
  void run(int dev);
  void run_slow();
  void integrate(int dev, const GpuSample* prev, GpuSample& cur, Integrals& I);

  Backend* be_;
  CounterSource* pmc_;
  SamplerConfig cfg_;
  std::vector<std::unique_ptr<DeviceState>> states_;
  std::vector<int> dev_ids_;
  std::vector<std::thread> threads_;
  std::thread slow_thread_;
  std::atomic<uint64_t> slow_passes_{0};
  std::atomic<double> pmc_idle_hz_{0.0};
  // Per-device process CU-occupancy integrals (slow thread only; survive pause/resume).
  std::vector<std::vector<std::pair<uint32_t, double>>> cu_seconds_;
  std::vector<int64_t> last_proc_ns_;
  std::atomic<bool> running_{false};
  std::atomic<bool> stop_{false};
  int stop_fd_ = -1;  // eventfd: readable once stop() was called; sampler threads ppoll() on it
};

// CPU list of a NUMA node ("0-31,64-95" parsed); empty if unknown.
std::vector<int> numa_cpus(int node);

}  // namespace kgs
