// Per-GPU sampler threads (SURVEY.md §3.4 "HOT LOOP", §2.3 device fan-out).
//
// Two std::threads per device, both pinned to the CPUs of the GPU's NUMA node and
// woken on absolute CLOCK_MONOTONIC deadlines:
//   * "kgs-pmfw<N>" reads the PMFW table + HBM occupancy (fast tier, at
//     min(hz, pmfw_hz)) — power, temperature, clocks, GFX/UMC busy;
//   * "kgs-gpu<N>" drains the hardware counters every tick (PMC tier, at hz).
// They share nothing but the device's publication slots, so a counter READ that
// blocks on a wedged command processor never silences the same GPU's power /
// temperature / utilisation, and the ≈110 µs PMFW pread never makes an 8 kHz
// counter tick overrun.  Neither takes a node-wide lock.
//
// Fault boundary of the counter tier: every CounterSource call is bounded by the
// source's deadline; after pmc_breaker_k consecutive failures the breaker opens
// (kgs_pmc_failed = 1): the session is released, and after pmc_retry_s (doubling
// to pmc_retry_max_s) the source is reset (fresh AQL queue) and re-acquired.
// stop() raises the source's cancel flag, waits at most stop_timeout_s for every
// thread, and abandons (detaches) any thread still stuck in a call — a DaemonSet
// pod then still exits on SIGTERM during the GPU hang it is reporting.
//
// The management-library tiers — per-process list (mid tier, every proc_every
// ticks' worth of time), xGMI link table + RAS health (slow tier, every
// link_every ticks' worth) — go through AMD SMI, which serialises callers on one
// process-wide mutex and takes milliseconds per call.  They run on a third thread
// per device, "kgs-slow<N>", so an amdsmi_get_gpu_process_list on GPU 3 can never
// delay GPU 5's 8 kHz counter drain, and a call that hangs
// on GPU 3 leaves GPU 5's per-process list, link table and per-pod CU-seconds
// fresh.  Every slow-tier result carries the time of its last
// good read; the renderer drops a device's per-process, link and RAS-status
// lines once they are older than the exporter's stale_after, and exports each
// tier's age (kgs_slow_last_ok_age_seconds) and any call in flight for longer
// (kgs_slow_call_seconds).  A hang inside AMD SMI's own process-wide lock stalls
// every device's slow thread alike — those tiers then all go stale, while the
// PMFW and counter tiers (no AMD SMI call) keep sampling.
// A sample counts as *distinct* only when the firmware timestamp moved
// (BASELINE.md measurement rule).  Results are published through seqlocks; the
// scrape path never calls into the driver.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "kgs/backend.h"
#include "kgs/pmc.h"
#include "kgs/sample.h"
#include "kgs/seqlock.h"
#include "kgs/util_estimator.h"

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
  // Dispatch-bound READ rate (needs CPC busy in the counter set).  A GPU that
  // runs nothing but µs kernels back to back keeps the command processor busy
  // while its shader engines hold waves only part of the time (a HIP graph of
  // 1.7 µs copies: CPC busy ≈100 %, SPI busy ≈41 %; long MFMA, GEMM or HBM
  // kernels: the two within ≈8 points, profiles/r4/).  That stream is exactly the
  // one each READ packet slows (+3.8 … 4.2 % at 8 kHz, +0.5 % at 1 kHz,
  // +0.05 % at 100 Hz; profiles/r4/ r4c, r4d).  While the
  // READ intervals of the last pmc_dispatch_hold_s had the CP dispatching with no
  // wave in flight for at least pmc_cp_only_min of their clocks, READs drop to
  // pmc_dispatch_hz; the first interval below restores every tick.  The hold keeps a
  // few ms of small kernels inside a training step at full rate (the bench step's
  // 2000-kernel graph runs 3.5 ms, and past 4 ms on a slow host, r4j).  0 = off;
  // off in profiling mode.  Integrals stay exact (cumulative counters); only the
  // time resolution of those stretches drops.  (Round 5's SPI-keyed "dispatch gap"
  // rate is gone: a saturated MFMA stream's SPI share wanders 89-95 % from box to
  // box, so no fixed SPI threshold separates it from a gapped stream; the CP-only
  // share does, and this rate already covers the µs-kernel case.)
  double pmc_cp_only_min = 0.3;
  double pmc_dispatch_hold_s = 0.010;
  double pmc_dispatch_hz = 500.0;
  // Quiet release ("parking").  A programmed perfmon session and a mapped READ queue
  // keep an idle MI355X out of its low-power state: ≈291 W against ≈258 W, +32 … +35 W
  // per idle GPU with the session and its 100 Hz quiet READs against the session
  // released (bench phase P, r6h / r6i; the level drops ≈5 s after the last GPU work).
  // After the device has been quiet (no wave, no MFMA cycle) for this long, its counter
  // thread STOPs the session and destroys the READ queue; it re-acquires when the PMFW
  // table shows GFX busy again (kUnparkTablePct in one interval, or kUnparkBusyPct over
  // kUnparkWindowS of table time), on a control-plane acquire, when parking is
  // switched off (this set to 0, or profiling mode), or when no PMFW table has come for
  // 1 s (nothing else would bill the GPU).  In between the READ-immune
  // utilisation is billed from the PMFW GFX busy — which no READ inflates while parked.
  // 0 = never (profiling mode never parks either).
  double pmc_quiet_release_s = 0.0;
  int max_backoff_ms = 1000;   // while a device keeps failing
  std::vector<int> devices;    // subset to sample (empty = all)
  // Counter-tier circuit breaker: consecutive failed drains that open it, and the
  // retry backoff (seconds, doubling per failed retry up to the max).
  int pmc_breaker_k = 3;
  double pmc_retry_s = 1.0, pmc_retry_max_s = 60.0;
  // stop() waits this long for the sampler threads, then abandons the stuck ones.
  double stop_timeout_s = 1.0;
  // Counter-tick dither: each tick's deadline sits off the fixed grid by an offset
  // that random-walks (± tick_dither of a period per tick, reflected at ± half a
  // period), so the READ phase does not lock onto a periodic workload (a kernel
  // every 1 ms against a 125 µs tick keeps one phase for seconds, and the per-interval
  // rules then err the same way on every kernel).  The grid keeps the long-run rate
  // exact.  0 = a fixed grid.
  double tick_dither = 0.25;
};

constexpr double kMaxHz = 100000.0;     // tick-rate ceiling accepted at run time (set_hz)
constexpr double kMinIdleHz = 0.01;     // pmc_idle_hz: 0 (off) or at least this
// UtilBiller's carry (and run-on guess) never exceeds this, whatever the freshness
// window: at --pmc-idle-hz 0.01 that window is 300 s, and busy carried that long would
// be billed into a later idle stretch — or a later pod.
constexpr double kMaxUtilCarryS = 1.0;
// A parked counter tier (SamplerConfig::pmc_quiet_release_s) re-acquires once one
// distinct PMFW interval shows kUnparkTablePct GFX busy (a load starting: ≥ 2 ms of
// kernels in a 20 ms table), or the busy over kUnparkWindowS of table time since the
// park settled reaches kUnparkBusyPct (a trickle of work: an idle MI355X with nothing
// READing it shows 0.07 %, r6b phase U 10 Hz idle row; 1 ms of kernels in 100 ms shows
// 1 %).  Round 6's first rule, one interval ≥ 1 %, woke on stray blips (a 0.2 ms packet
// in a 20 ms table): r6g phase P un- and re-parked in 2 of 6 parked blocks.  Whatever
// runs meanwhile is billed from the PMFW busy, which nothing inflates while no READ runs.
constexpr double kUnparkTablePct = 10.0;
constexpr double kUnparkBusyPct = 1.0;
constexpr double kUnparkWindowS = 0.1;

// The counter tick's dithered offset from its fixed grid (SamplerConfig::tick_dither): a
// random walk of at most `dither` of a period per tick, reflected into ± half a period.
class TickDither {
 public:
  explicit TickDither(uint64_t seed) : rng_(seed ? seed : 0x9E3779B97F4A7C15ull) {}
  // The next tick's offset (ns) for a grid period of period_ns.
  double step(int64_t period_ns, double dither) {
    if (!(dither > 0)) return off_ = 0;
    const double half = 0.5 * static_cast<double>(period_ns);
    off_ += uniform() * std::min(dither, 0.5) * static_cast<double>(period_ns);
    if (off_ > half) off_ = 2 * half - off_;
    if (off_ < -half) off_ = -2 * half - off_;
    return off_;
  }
  void reset() { off_ = 0; }
  double offset() const { return off_; }

 private:
  double uniform() {  // xorshift64*: [-1, 1)
    rng_ ^= rng_ >> 12;
    rng_ ^= rng_ << 25;
    rng_ ^= rng_ >> 27;
    return static_cast<double>((rng_ * 0x2545F4914F6CDD1Dull) >> 11) * (2.0 / 9007199254740992.0) - 1.0;
  }
  uint64_t rng_;
  double off_ = 0;
};

constexpr size_t kRing = 1024;          // ≥10 s of history at 100 Hz
// Counter samples decimated to one per kPmcSlowNs feed the window gauges, so a
// 1 s window is covered at any tick rate (the full-rate ring holds 85 ms at 12 kHz).
constexpr size_t kPmcSlowRing = 2048;
constexpr size_t kPmcRing = 8192;       // raw counter stream: ≥1 s at 8 kHz (/counters)
constexpr int64_t kPmcSlowNs = 5000000;  // 5 ms → ≥10 s of history
constexpr int kReadHistBuckets = 12;    // backend read latency histogram
// A tick late by at most this many periods keeps the absolute schedule (the missed
// ticks run back to back); later than that the schedule re-anchors.
constexpr int64_t kCatchUpPeriods = 4;
constexpr int64_t kPmcStallNs = 500000000;  // GRBM_COUNT without a plausible clock this long = stalled
constexpr double kPlausibleMhzLo = 100.0, kPlausibleMhzHi = 4000.0;
// Adaptive READ rate: an interval whose SPI-busy share is below this is quiet.
constexpr double kQuietActiveFrac = 0.02;
// ... and the device counts as quiet only after this long of quiet intervals in a
// row: a host sync between kernels leaves the GPU idle for tens of µs, which is not
// worth a drop to the idle READ rate (the first READ after it would come up to one
// idle period late, and every tick in between is a lost sample).
constexpr int64_t kQuietHoldNs = 5000000;
// Dispatch-busy integral: a READ interval whose CPC busy share is at least this is a
// dispatch in flight throughout (the READ's own CP time hides under the workload's;
// the CPC idles a few % of each 125 µs interval under a long kernel at 8 kHz, r4f).
constexpr double kCpcFullFrac = 0.90;
// ... and a READ interval at least this long that mixes a kernel with idle is split by
// the learned busy / idle shader clocks (at 8 kHz the edge intervals are short and the
// split over-read 0.2 ms bursts in replay, tools/util_estimator_sim.py; at 1 kHz it
// closes most of a 1 ms-burst train's −1.3 … −2.3 points).
constexpr int64_t kClockSplitNs = 400000;
// ... and counts the READ packet's own CP time once where it overlaps dispatch busy:
// busy = (CPC − r) / (1 − r/clk), a READ landing at a uniformly random point of the
// interval.  Subtracting r whole under-read the 1 kHz burst trains of r4f's raw READs
// by 0.3 / 0.8 points (a READ during a kernel adds no CP busy).  At 8 kHz the rule
// over-reads 0.2 ms / 1 ms trains on MI355X (r6a: +1.39 points with it at every
// interval length, though the r4f / r5l dumps replay it at +0.04 / +0.53), so it stays
// with the long intervals.
constexpr int64_t kReadOverlapNs = 400000;
// ... and is split in time rather than cycles: idle time = its cycles at the learned
// idle clock, busy time = the rest.  A cycle share under-weights power-capped kernels
// (1 ms MFMA bursts at ≈2.1 GHz between ≈2.4 GHz gaps), and a low READ rate may never
// see the fully busy interval the clock-ratio split needs: in the r5b raw READs (the
// exporter's READ mode) the 1 ms / 5 ms train read −2.2 / −2.7 / −2.6 points at 1 kHz /
// 100 Hz / 10 Hz with the clock-ratio split, −0.5 / +1.4 / +1.5 with this.
constexpr int64_t kTimeSplitNs = 400000;
// ... and blended with the cycle share: the gaps between kernels clock between the
// kernels' clock (the cycle share's assumption) and the learned idle clock (the time
// split's), so the truth lies between the two.  Replayed on the r4f, r5b and r5l raw
// READs (1 kHz / 100 Hz / 10 Hz, 1 ms / 5 ms and 0.2 ms / 1 ms trains), the worst error
// is 2.7 points with the cycle share, 2.0 with the time split alone, 1.5 / 1.4 / 1.3 /
// 1.5 at weights 0.5 / 0.6 / 0.7 / 0.8 (1.07 at 0.6 with kGapClockFreshNs below).
// Round 6 refit it on those dumps plus the exporter's own live 10 Hz drains
// under seeded random 5 µs - 20 ms MFMA kernels with random gaps (r6e,
// profiles/r6/r6e/gpu_tests/irregular_raw_10hz.json): long gaps clock nearer the idle
// clock than a periodic train's short ones, and at 0.6 that load read −1.53 (live −1.4 …
// −1.8 on four boxes).  Minimax over trains and live capture: 1.53 / 1.30 / 1.42 / 1.54 at
// 0.6 / 0.7 / 0.75 / 0.8 → 0.7 (trains ≤ 1.3, live −0.99); the held-out r6c dump, never
// used for the choice, replays every irregular load within 1.1 at 10 Hz - 8 kHz with it.
// Then phase U on six more boxes read the 10 Hz random load at −1.02 … −1.61 with 0.7
// (r6f, r6j, r6n, r6p, r6x): the exporter's own drains put the truth nearer the time split
// (0.885 of the way on r6e's capture) than the probe's dumps do (0.7 on r6c).  0.75 takes
// the worst reading over everything to ≈ 1.42 (r5l's 0.2 ms / 1 ms train at 1 kHz in
// replay; r6x's −1.61 moves to ≈ −1.3 at the slope r6e's capture shows; r6c ≤ 1.22).
constexpr double kTimeSplitWeight = 0.75;
// ... unless READ-only intervals taught the idle clock within this long before the
// interval: READ-only intervals among the kernels (a 1 ms train at 1 kHz: 3-4 of every 5
// intervals) measure the gaps' own clock, and the time split alone is right there (the
// three dumps' 1 kHz 1 ms trains: −0.55 / −1.41 / −0.17 points blended, +0.02 / −0.90 /
// +0.02 with this; at 100 Hz and 10 Hz no READ-only interval falls inside a train).
constexpr int64_t kGapClockFreshNs = 10000000;
// A READ-only interval (no waves, no MFMA cycle, the CP mostly idle: the intervals that
// teach the READ cost) bills no dispatch.  Its CP busy less the learned mean READ cost
// is that READ's scatter, and keeping the positive half (max 0) billed an idle GPU 0.1-
// 0.2 % at 8 kHz and a 1 ms / 5 ms train +0.6 points (r5l dump: its full intervals alone
// sum to the kernels' duty; r6a on MI355X: the 8 kHz 1 ms train +0.53 → +0.04 points).
constexpr bool kReadOnlyBillsZero = true;
extern const double kReadHistBoundsUs[kReadHistBuckets];
// Slow tiers (DeviceState::slow_call_tier, kgs_slow_* labels).
enum SlowTier : int { kSlowProcs = 0, kSlowLinks = 1, kSlowHealth = 2 };
inline const char* slow_tier_name(int t) { return t == kSlowProcs ? "procs" : t == kSlowLinks ? "links" : "health"; }

struct DeviceState {
  Seqlock<GpuSample> latest;
  SampleRing<GpuSample, kRing> ring;
  Seqlock<Integrals> integ;      // PMFW-tier fields (writer: kgs-pmfw<N>)
  Seqlock<Integrals> pmc_integ;  // counter-tier fields (writer: kgs-gpu<N>)
  Seqlock<PmcSample> pmc_latest;
  SampleRing<PmcSample, kPmcRing> pmc_ring;         // every counter drain
  SampleRing<PmcSample, kPmcSlowRing> pmc_slow_ring;  // ≥ kPmcSlowNs apart (window gauges)

  mutable std::mutex slow_mu;  // guards the two shared_ptrs below
  std::shared_ptr<const std::vector<ProcInfo>> procs;
  std::shared_ptr<const std::vector<LinkInfo>> links;
  std::shared_ptr<const HealthInfo> health;
  // Per-pod CU-occupancy seconds on this GPU ("namespace/pod" → ∫ Σ share dt of the
  // pod's processes), processes that exited included (slow tier).
  std::shared_ptr<const std::map<std::string, double>> pod_cu;
  // Pods ("namespace/pod") with a process whose CU occupancy could not be read in the
  // last per-process pass (ProcInfo::cu_valid false): their CU-seconds are unknown.
  std::shared_ptr<const std::set<std::string>> pod_cu_unknown;
  int64_t procs_mono_ns = 0;

  std::atomic<int> up{0};
  std::atomic<int64_t> last_ok_mono_ns{0};
  std::atomic<uint64_t> consecutive_errors{0};
  std::atomic<uint64_t> read_hist[kReadHistBuckets + 1] = {};
  // Counter thread: how late each wake-up was against its absolute deadline (same
  // buckets as read_hist) — the CPU contention / idle-state cost behind overruns.
  std::atomic<uint64_t> wake_hist[kReadHistBuckets + 1] = {};
  std::atomic<uint64_t> wake_late_ns{0};              // sum of the positive lateness
  std::atomic<int> cpu_pinned{-1};
  // Counter hand-over (`kgs exporter` SIGUSR1 / SIGUSR2, /control/pmc/*): the
  // control plane sets pmc_want; the sampler thread releases / re-acquires the
  // counters itself and reports the state in pmc_on.
  std::atomic<int> pmc_want{1};
  std::atomic<int> pmc_drop_queue{0};       // with a release: destroy the READ queue too
  std::atomic<int> pmc_on{0};
  std::atomic<uint64_t> pmc_releases{0};
  std::atomic<int> pmc_stalled{0};          // counters frozen / implausible for ≥ kPmcStallNs
  std::atomic<uint64_t> pmc_reclaims{0};    // automatic re-STARTs after a stall
  std::atomic<uint64_t> pmc_refreshes{0};   // periodic re-STARTs (pmc_refresh_s)
  std::atomic<int> pmc_quiet{0};            // last READ interval had no wave: READs at pmc_idle_hz
  std::atomic<uint64_t> pmc_quiet_skips{0};  // ticks that skipped their READ while quiet
  std::atomic<int> pmc_dbound{0};            // dispatch-bound (pmc_cp_only_min): READs at pmc_dispatch_hz
  std::atomic<int> pmc_parked{0};            // session released after pmc_quiet_release_s of quiet
  std::atomic<uint64_t> pmc_parks{0};        // quiet releases
  // Parked time (kgs_pmc_parked_seconds_total): the parks that ended, and the start of
  // the current one (0: not parked) — one seqlocked pair, so a scrape never sees a park
  // counted twice or not at all while it ends (writer: kgs-gpu<N>).
  struct ParkTime {
    int64_t ended_ns = 0;
    int64_t since_ns = 0;
  };
  Seqlock<ParkTime> park_time;
  std::atomic<int> pmc_unpark_req{0};        // control plane: re-acquire a parked device now
  std::atomic<int64_t> pmc_unpark_lag_ns{-1};  // last re-acquire: mono time since the PMFW sample that showed busy
  std::atomic<uint64_t> pmc_dbound_skips{0};  // ticks that skipped their READ while dispatch-bound
  // Counter-tier fault boundary (sampler.h header comment).
  std::atomic<int> pmc_failed{0};            // breaker open: no READs until a retry succeeds
  std::atomic<uint64_t> pmc_breaker_trips{0};
  std::atomic<uint64_t> pmc_retries{0};      // reset + acquire attempts while the breaker is open
  std::atomic<int> thread_hung{0};           // a sampler thread of this device was abandoned by stop()
  std::atomic<uint64_t> pmc_reordered{0};    // drains dropped: CP time earlier than the previous drain's
  std::atomic<int> util_carry_drop{0};       // owners changed: the PMFW thread drops the billing carry
  // Test hook (Sampler::inject_pmc_stall, /control/pmc/stall with --control-http):
  // the device's own counter thread asks the source to wedge its READ queue.
  std::atomic<int> pmc_stall_req{0};
  std::atomic<uint64_t> pmc_stalls_injected{0};
  // Slow tiers (kgs-slow<N>): CLOCK_MONOTONIC of each tier's last good read (0 =
  // never), and the start of the management-library call in flight (0 = none).
  std::atomic<int64_t> procs_ok_ns{0}, links_ok_ns{0}, health_ok_ns{0};
  std::atomic<int64_t> slow_call_ns{0};
  std::atomic<int> slow_call_tier{-1};       // kSlowProcs | kSlowLinks | kSlowHealth while in a call
  std::atomic<int> slow_hung{0};             // the slow thread was abandoned by stop() (stuck in a call)
  std::atomic<uint64_t> link_errors{0}, health_errors{0};
  PmcSample pmc_base;  // totals carried over hand-overs (sampler thread only; survives pause/resume)
  int pmc_fail_streak = 0;                   // counter thread only (survive pause/resume)
  int64_t pmc_retry_at_ns = 0;
  double pmc_backoff_s = 0;
  // Last distinct PMFW sample (sampler thread only).  Kept across pause/resume:
  // the firmware accumulators keep counting while the thread is stopped, so the
  // first sample after a resume integrates the paused interval exactly.
  GpuSample pmfw_prev;
  bool have_pmfw_prev = false;
  // Slow-thread self metrics: completed passes and their latency per tier.
  std::atomic<uint64_t> proc_reads{0}, proc_errors{0}, link_reads{0};
  std::atomic<int> procs_cu_unavailable{0};  // processes of the last pass whose CU occupancy was unreadable
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
  std::shared_ptr<const std::map<std::string, double>> get_pod_cu() const {
    std::lock_guard<std::mutex> g(slow_mu);
    return pod_cu;
  }
  std::shared_ptr<const std::set<std::string>> get_pod_cu_unknown() const {
    std::lock_guard<std::mutex> g(slow_mu);
    return pod_cu_unknown;
  }
  // Both tiers' integrals in one view (overruns: both threads').
  Integrals integrals() const {
    Integrals a, b;
    integ.load(a);
    pmc_integ.load(b);
    a.overruns += b.overruns;
    a.pmc_samples = b.pmc_samples;
    a.pmc_errors = b.pmc_errors;
    a.pmc_read_seconds = b.pmc_read_seconds;
    a.mfma_busy_seconds = b.mfma_busy_seconds;
    a.active_seconds = b.active_seconds;
    a.pmc_epoch = b.pmc_epoch;
    a.pmc_last_ns = b.pmc_last_ns;
    a.dispatch_seconds = b.dispatch_seconds;
    a.dispatch_drains = b.dispatch_drains;
    a.pmc_last_share = b.pmc_last_share;
    a.cpc_read_us = b.cpc_read_us;
    a.pmc_clk_idle_hz = b.pmc_clk_idle_hz;
    a.pmc_clk_busy_hz = b.pmc_clk_busy_hz;
    return a;
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
  // util_pct (optional): the READ-immune busy mean (GpuSample::cum_util_s) over the same window.
  bool window_busy(int dev, double window_s, double& gfx_pct, double& umc_pct, int& n, double* util_pct = nullptr) const;
  // Counter-derived rates over the trailing window.
  bool window_pmc(int dev, double window_s, PmcRates& out) const;
  // Ask a device's counter thread (dev < 0: every sampled device's) to hand its
  // counters to another profiler (false) or to take them back (true).  Takes
  // effect within one tick of that device's own thread: a hung device never
  // delays the others.
  // drop_queue (release only): also destroy the reader's READ queue
  // (CounterSource::reset), so nothing of the counter tier stays mapped on the GPU
  // until the next acquire — the benchmark's "released" condition.
  void set_pmc_wanted(bool on, int dev = -1, bool drop_queue = false);
  // Change the tick rate (stops and restarts the threads; integrals continue).
  // false (nothing changed) unless 0 < hz <= kMaxHz.
  bool set_hz(double hz);
  double hz() const { return hz_.load(std::memory_order_relaxed); }
  // Quiet-GPU counter READ rate (SamplerConfig::pmc_idle_hz), in place; false
  // (unchanged) unless hz == 0 or kMinIdleHz <= hz <= kMaxHz.
  bool set_pmc_idle_hz(double hz);
  double pmc_idle_hz() const { return pmc_idle_hz_.load(std::memory_order_relaxed); }
  // Dispatch-bound READ rate (SamplerConfig::pmc_dispatch_hz), in place; false
  // (unchanged) unless 0 < hz <= kMaxHz.
  bool set_pmc_dispatch_hz(double hz);
  double pmc_dispatch_hz() const { return pmc_dispatch_hz_.load(std::memory_order_relaxed); }
  // Quiet-release delay (SamplerConfig::pmc_quiet_release_s), in place; 0 = never park.
  // false (unchanged) unless 0 <= s <= 86400.
  bool set_pmc_quiet_release_s(double s);
  double pmc_quiet_release_s() const { return pmc_quiet_release_s_.load(std::memory_order_relaxed); }
  // Slow-tier passes completed (all devices).
  uint64_t slow_passes() const { return slow_passes_.load(); }
  // Test hook: the device's counter thread wedges its reader's queue
  // (CounterSource::inject_stall) on its next tick.  false if dev is not sampled.
  bool inject_pmc_stall(int dev);
  // Slow-tier periods in force (ns; 0 = tier off): freshness checks size their
  // deadline on these.
  int64_t proc_period_ns() const;
  int64_t link_period_ns() const;
  // Threads stop() gave up on (stuck in a device call); they are detached and
  // exit on their own if the call ever returns.  The owner must then keep the
  // backend, counter source and this sampler alive (Exporter leaks them).
  uint64_t abandoned_threads() const { return abandoned_total_.load(); }
  // (GPU, PID) → "namespace/pod" of the processes' pods, for the per-pod CU
  // integrals (slow tier; the exporter pushes it with its PID → pod table).
  void set_pid_pods(std::shared_ptr<const std::unordered_map<uint64_t, std::string>> m);
  // The GPU's owner set changed: its PMFW thread drops the billing carry at its next
  // distinct sample (UtilBiller::drop_carry).
  void drop_util_carry(int dev);
  // ∫ CU-occupancy share dt of the pod `ns_pod` ("namespace/pod") on `dev`, 0 if none.
  double pod_cu_seconds(int dev, const std::string& ns_pod) const;

 private:
  struct Worker;
  void start_locked();
  void stop_locked();
  void spawn(int dev, int kind);
  void run_pmfw(Worker& w);
  void run_pmc(Worker& w);
  void run_slow(Worker& w);
  void run_pmfw_util(int dev, int64_t now, double dgfx_s, double dt_s, Integrals& I, GpuSample& s);
  void pin(int dev, const char* fmt);
  void integrate(int dev, const GpuSample* prev, GpuSample& cur, Integrals& I);

  Backend* be_;
  CounterSource* pmc_;
  SamplerConfig cfg_;
  std::vector<std::unique_ptr<DeviceState>> states_;
  std::vector<int> dev_ids_;
  std::mutex life_mu_;  // start / stop / set_hz (HTTP control thread vs Python pause / resume)
  std::vector<std::shared_ptr<Worker>> workers_;    // running threads (guarded by life_mu_)
  std::vector<std::shared_ptr<Worker>> abandoned_;  // detached, maybe still stuck (guarded by life_mu_)
  std::atomic<uint64_t> abandoned_total_{0};
  std::atomic<double> hz_{10.0};
  std::atomic<uint64_t> slow_passes_{0};
  std::atomic<double> pmc_idle_hz_{0.0};
  std::atomic<double> pmc_dispatch_hz_{500.0};
  std::atomic<double> pmc_quiet_release_s_{0.0};
  mutable std::mutex pid_pods_mu_;
  std::shared_ptr<const std::unordered_map<uint64_t, std::string>> pid_pods_;
  std::vector<std::map<std::string, double>> pod_cu_;  // device's slow thread only
  // Per-device process CU-occupancy integrals (device's slow thread only; survive pause/resume).
  std::vector<std::vector<std::pair<uint32_t, double>>> cu_seconds_;
  std::vector<int64_t> last_proc_ns_;
  // READ-immune util integral: the billing state carried between distinct PMFW
  // samples (each device's PMFW thread only; survives pause/resume).
  std::vector<UtilBiller> util_bill_;
  std::atomic<bool> running_{false};
  std::atomic<bool> stop_{false};
  int stop_fd_ = -1;  // eventfd: readable once stop() was called; sampler threads ppoll() on it
};

// The estimator parameters a sampler with this config runs its counter tier with (the
// offline replay binds the same function: _kgs_native.sampler_estimator_params).
EstimatorParams estimator_params(const SamplerConfig& cfg, int num_cu);

// CPU list of a NUMA node ("0-31,64-95" parsed); empty if unknown.
std::vector<int> numa_cpus(int node);

}  // namespace kgs
