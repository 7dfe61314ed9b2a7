// The utilisation estimators behind container_gpu_sm_util / container_gpu_busy_seconds_total
// (reference gpu_util_stats/gpu_util_stats.py:159 reads the series, :62-94 bills each
// pod its mean) as pure, replayable units: no threads, no clocks, no device calls.
//
//  * DispatchEstimator — one hardware-counter drain in, the interval's integrals out.
//    It owns everything the counter tier learns from the cumulative counts: the READ
//    packet's own CP cost (learned on intervals without waves, per READ mode and per
//    full / lite READ), the busy / idle shader clocks and the clock split of partial
//    intervals, the full-interval rule, the stall (plausible-clock) watch, and the
//    two READ-rate hysteresis machines (quiet, dispatch-bound).
//    Sampler::run_pmc feeds it every drain and only schedules and publishes.
//  * UtilBiller — one distinct PMFW interval in, the seconds billed out.  While the
//    counter tier covers the interval the counter integral's increment is billed;
//    what exceeds the interval (drains land on host time, intervals are firmware
//    time, and at 10 Hz one interval can hold two drains and the next none) is
//    carried to the next intervals instead of being dropped — so the billed integral
//    equals the counter integral over any window longer than a drain, at every rate.
//
// The pybind11 module binds both (bindings.cpp: DispatchEstimator, UtilBiller), so
// the offline replay (tools/util_estimator_sim.py, tests/test_estimator_replay.py)
// runs this very code on raw READ dumps recorded on MI355X.
#pragma once

#include <algorithm>
#include <cstdint>

#include "kgs/pmc.h"

namespace kgs {

struct EstimatorParams {
  // An interval whose SPI-busy share is below this (and with no MFMA cycle) has no
  // waves: quiet, and its CP busy is the READ's own (sampler.h kQuietActiveFrac).
  double quiet_active_frac = 0.02;
  // A drain interval the CP was busy for at least this share counts whole.
  double cpc_full_frac = 0.90;
  // Partial intervals at least this long are split by the learned busy / idle clocks.
  int64_t clock_split_ns = 400000;
  double clock_ratio_lo = 0.9, clock_ratio_hi = 1.1;
  // Partial intervals at least this long count the READ's own CP time once where it
  // overlaps dispatch busy (0 = every interval, < 0 = never).
  int64_t read_overlap_ns = -1;
  // Partial intervals at least this long are split in time, not cycles: idle time =
  // idle cycles / the learned idle clock, busy time = the rest of the span — no busy
  // clock needed, which a low READ rate may never see in a fully busy interval
  // (0 = never; the clock-ratio split above applies instead).
  int64_t time_split_ns = 0;
  double time_split_ratio_hi = 1.5;   // ... within f_idle / f_busy ≤ this (busy clock ≥ 0.67 × idle)
  // ... and taken this far from the cycle share: the cycle share assumes the gaps ran
  // at the kernels' clock, the time split that they ran at the learned idle clock; the
  // truth lies between (1 = the time split alone).
  double time_split_weight = 1.0;
  // ... unless the idle clock was learned this recently before the interval (0 = never):
  // READ-only intervals among the kernels measure the clock of the gaps themselves
  // (1 ms bursts every 5 ms at 1 kHz), and the time split alone is then right.
  int64_t gap_clock_fresh_ns = 0;
  // A READ-only interval (the READ-cost learning rule's) bills no dispatch (false: its CP
  // busy less the learned READ cost, floored at 0).
  bool read_only_bills_zero = false;
  double ewma = 0.05;                 // weight of a new sample in every learned EWMA
  int64_t quiet_hold_ns = 5000000;    // quiet intervals in a row before the device counts as quiet
  double cp_only_min = 0.0;           // dispatch-bound: CP busy with no wave ≥ this share (0 = off)
  int64_t dbound_hold_ns = 10000000;
  double plausible_mhz_lo = 100.0, plausible_mhz_hi = 4000.0;
  double num_simds = 1024.0;          // CUs × 4 (MFMA share of all SIMD cycles)
};

// One drain: cumulative counts since the session's START (mask bit i: value i read).
struct Drain {
  int64_t mono_ns = 0;
  uint32_t mask = 0;
  uint64_t count = 0, spi = 0, mfma = 0, cpc = 0;
  bool se_fresh = true;   // the per-SE counters (MFMA) were read by this drain
  bool fresh_mode = false;  // taken as a synchronous READ (quiet device), not pipelined
};

// What one drain adds, and the rate states after it.
struct DrainStep {
  bool interval = false;      // a previous drain existed: the increments below are real
  double span_s = 0;
  double active_s = 0;        // ∫ SPI-busy share dt
  double mfma_s = 0;          // ∫ MFMA share of all SIMD cycles dt (fresh drains only)
  bool have_dispatch = false;
  double dispatch_s = 0;      // ∫ dispatch-in-flight share dt
  double cp_only_share = 0;   // CP busy with no wave in flight, share of the clocks
  bool learned = false;       // this interval taught the READ cost
  bool quiet_interval = false, dbound_interval = false;
  bool quiet = false, dbound = false;  // hysteresis states after this drain
};

class DispatchEstimator {
 public:
  // A (re)START: every count restarts at 0 at time t, the rate states reset.
  void restart(int64_t t) {
    have_prev_ = have_se_ = true;
    prev_count_ = prev_mfma_ = prev_spi_ = prev_cpc_ = 0;
    prev_ns_ = se_ns_ = t;
    se_count_ = se_mfma_ = 0;
    quiet_ = dbound_ = false;
    quiet_since_ = dbound_since_ = 0;
    last_plausible_ns_ = t;
  }
  // A break with no new baseline (breaker trip, failed re-START): the next drain
  // only re-baselines.
  void invalidate(int64_t t) {
    have_prev_ = have_se_ = false;
    last_plausible_ns_ = t;
  }
  bool have_prev() const { return have_prev_; }
  int64_t prev_ns() const { return prev_ns_; }
  int64_t last_plausible_ns() const { return last_plausible_ns_; }
  // The READ packet's own CP time, as last learned on a full (se_fresh) READ (µs).
  double cpc_read_us() const { return cpc_read_us_; }
  double read_cycles(bool fresh_mode, bool full) const { return read_cyc_[fresh_mode][full]; }
  double read_spi_cycles(bool fresh_mode, bool full) const { return read_spi_[fresh_mode][full]; }
  uint64_t read_learned(bool fresh_mode, bool full) const { return read_n_[fresh_mode][full]; }
  double clk_busy_hz() const { return clk_busy_hz_; }
  double clk_idle_hz() const { return clk_idle_hz_; }
  bool quiet() const { return quiet_; }
  bool dbound() const { return dbound_; }

  DrainStep feed(const Drain& d, const EstimatorParams& p) {
    DrainStep r;
    const bool prev = have_prev_ && d.mono_ns > prev_ns_;
    // Stall watch: GRBM_COUNT free-runs at the shader clock while our session is
    // programmed; frozen or foreign counts give no plausible clock.
    if (prev) {
      const double mhz = d.count >= prev_count_ ? (d.count - prev_count_) * 1e3 / (d.mono_ns - prev_ns_) : 0.0;
      if (mhz >= p.plausible_mhz_lo && mhz <= p.plausible_mhz_hi) last_plausible_ns_ = d.mono_ns;
    }
    // MFMA-busy share of all SIMD cycles since the previous drain that read the
    // per-SE counters (every drain, unless lite READs are on), times that span.
    if (d.se_fresh && have_se_ && d.mono_ns > se_ns_ && (d.mask & (1u << kPmcMfmaBusy)) && d.count > se_count_ &&
        d.mfma >= se_mfma_) {
      const double frac = static_cast<double>(d.mfma - se_mfma_) / (p.num_simds * static_cast<double>(d.count - se_count_));
      r.mfma_s = std::min(frac, 1.0) * (d.mono_ns - se_ns_) * 1e-9;
    }
    if (d.se_fresh) {
      have_se_ = true;
      se_count_ = d.count;
      se_mfma_ = d.mfma;
      se_ns_ = d.mono_ns;
    }
    const bool have_act = (d.mask & (1u << kPmcGrbmActive)) != 0;
    if (prev) {
      r.interval = true;
      r.span_s = (d.mono_ns - prev_ns_) * 1e-9;
    }
    if (prev && have_act && d.count > prev_count_ && d.spi >= prev_spi_) {
      const double frac = static_cast<double>(d.spi - prev_spi_) / static_cast<double>(d.count - prev_count_);
      r.active_s = std::min(frac, 1.0) * r.span_s;
    }
    // Dispatch in flight: the CP busy share of the interval, less the READ packet's own
    // CP time, never below the SPI share.
    if (prev && (d.mask & (1u << kPmcCpcBusy)) && d.count > prev_count_ && d.cpc >= prev_cpc_) {
      const double clk = static_cast<double>(d.count - prev_count_);
      const double cpc = std::min(clk, static_cast<double>(d.cpc - prev_cpc_));
      const double act = have_act && d.spi >= prev_spi_ ? static_cast<double>(d.spi - prev_spi_) : 0.0;
      const int m = d.fresh_mode ? 1 : 0;
      const int f = d.se_fresh ? 1 : 0;
      const int64_t span_ns = d.mono_ns - prev_ns_;
      const double hz_now = clk / (span_ns * 1e-9);
      // No wave, no MFMA cycle and the CP mostly idle: the CP busy here is our READ's,
      // and so is the SPI blip (≈0.9 µs per READ: 0.7 % of the clocks at 8 kHz, so the
      // test is the quiet threshold, not "no SPI at all" — r4f: a 0.5 % test kept 2 %
      // of the 8 kHz READ-only intervals, the cheap ones, and learned 13 µs for 15.5).
      const bool read_only_shape = act < p.quiet_active_frac * clk && d.mfma == prev_mfma_ && cpc < 0.5 * clk;
      // ... and, once this READ kind's cost is known, CP busy within 2 × that cost: the
      // shape alone also fits CP-only work (a stream of wave-less dispatches at 30-50 % of
      // the clocks), which must neither teach the READ cost nor bill zero.
      const double known = read_n_[m][f] ? read_cyc_[m][f] : 0.0;
      const bool read_only = read_only_shape && (known <= 0 || cpc <= 2.0 * known);
      if (read_only) {
        const bool first = read_n_[m][f] == 0;
        read_cyc_[m][f] = first ? cpc : (1 - p.ewma) * read_cyc_[m][f] + p.ewma * cpc;
        read_spi_[m][f] = first ? act : (1 - p.ewma) * read_spi_[m][f] + p.ewma * act;
        ++read_n_[m][f];
        r.learned = true;
        if (f) cpc_read_us_ = read_cyc_[m][f] / (hz_now * 1e-6);
        // the idle clock between kernels, not a quiet GPU's (its clock drops: r4r)
        if (!d.fresh_mode) {
          clk_idle_hz_ = clk_idle_hz_ > 0 ? (1 - p.ewma) * clk_idle_hz_ + p.ewma * hz_now : hz_now;
          idle_learned_ns_ = d.mono_ns;
        }
      }
      // This READ's learned cost, or the other kind's before it has its own.
      const int k = read_n_[m][f] ? f : 1 - f;
      const double rcyc = read_cyc_[m][k];
      // Waves of the workload: SPI busy less the READ's own blip.
      const double wav = std::max(0.0, act - read_spi_[m][k]);
      // An interval the CP was busy for ≥ cpc_full_frac counts whole: under a kernel the
      // CPC idles a few % of each 125 µs interval at 8 kHz (r4f: MFMA and GEMM intervals
      // 0.95-1.0), and subtracting a READ-only cost there under-read a GEMM stream by 4
      // points.  Partial intervals count the READ's CP time once where it overlaps
      // dispatch busy, (cpc − read) / (1 − read/clk) (sampler.h kReadOverlapNs).
      const bool full = cpc >= p.cpc_full_frac * clk;
      const double net = p.read_overlap_ns >= 0 && span_ns >= p.read_overlap_ns && rcyc < 0.5 * clk
                             ? (cpc - rcyc) / (1.0 - rcyc / clk)
                             : cpc - rcyc;
      // A READ-only interval (the learning rule's: no waves, no MFMA cycle, the CP mostly
      // idle) bills nothing: its CP busy less the learned mean READ cost is that READ's
      // own scatter, and keeping the positive half of it (max 0) billed ≈2 µs per READ-only
      // interval — 0.6 points on a 1 ms / 5 ms train at 8 kHz, whose gaps are all READ-only
      // intervals (r5l dump: full intervals alone sum to the kernels' duty).
      const double busy = full ? clk : (read_only && p.read_only_bills_zero) ? 0.0 : std::max(wav, std::max(0.0, net));
      double share = std::min(1.0, busy / clk);
      if (full) {
        clk_busy_hz_ = clk_busy_hz_ > 0 ? (1 - p.ewma) * clk_busy_hz_ + p.ewma * hz_now : hz_now;
      } else if (p.time_split_ns > 0 && span_ns >= p.time_split_ns && share > 0 && clk_idle_hz_ > 0) {
        // A long interval at a low READ rate: many kernels and gaps, each part at its
        // own clock (MFMA bursts power-capped at ≈2.1 GHz, gaps up to ≈2.4).  With the
        // gaps at the learned idle clock, the idle part's time is its cycles at that
        // clock and the busy part is the rest; bounded to busy clocks between f_idle /
        // time_split_ratio_hi and f_idle / clock_ratio_lo, so an idle stretch that
        // clocked below the learned idle clock (a GPU left quiet long enough to drop its
        // clock) must not read as busy.  But gaps between kernels clock between the two
        // (r5b, r5l dumps: 1 ms / 5 ms trains clock 2.28-2.32 GHz on average, 0.2 ms /
        // 1 ms trains 2.34-2.37, against 2.41 idle), so the cycle share reads low and the
        // time split high, by up to 2.2 and 2.0 points: time_split_weight blends them —
        // unless READ-only intervals among these kernels taught the idle clock just now
        // (gap_clock_fresh_ns): then it is the gaps' own clock.
        const double idle_s = std::max(0.0, clk - busy) / clk_idle_hz_;
        const double t = 1.0 - idle_s / (span_ns * 1e-9);
        auto time_share = [share](double ratio) { return share * ratio / (1.0 - share + share * ratio); };
        const double ts = std::clamp(t, time_share(p.clock_ratio_lo), time_share(p.time_split_ratio_hi));
        const bool gap_clock = p.gap_clock_fresh_ns > 0 && idle_learned_ns_ > 0 && prev_ns_ >= idle_learned_ns_ &&
                               prev_ns_ - idle_learned_ns_ <= p.gap_clock_fresh_ns;
        share += (gap_clock ? 1.0 : p.time_split_weight) * (ts - share);
      } else if (span_ns >= p.clock_split_ns && share > 0 && clk_busy_hz_ > 0 && clk_idle_hz_ > 0) {
        // A cycle share under-weights a kernel that ran at a lower clock than the idle
        // rest of the interval (MFMA under the power cap: ≈2.1 GHz against ≈2.4 idle):
        // the time share is s·r / (1 − s + s·r), r = f_idle / f_busy.  f_busy comes from
        // the last fully busy intervals, whose kernels need not clock like this one (a
        // 0.2 ms burst is not power-capped like a 1 ms one): r is kept within ±10 %
        // (r4q: ±25 % over-read a 0.2 ms train by 2 points).
        const double rr = std::clamp(clk_idle_hz_ / clk_busy_hz_, p.clock_ratio_lo, p.clock_ratio_hi);
        share = share * rr / (1.0 - share + share * rr);
      }
      r.have_dispatch = true;
      r.dispatch_s = share * span_ns * 1e-9;
      r.cp_only_share = std::max(0.0, busy - wav) / clk;
      // Dispatch-bound: the CP dispatching with no wave in flight for a large share.
      r.dbound_interval = p.cp_only_min > 0 && busy - wav >= p.cp_only_min * clk;
    }
    // Quiet = a shader engine had waves for < quiet_active_frac of the clocks since the
    // previous READ, and no MFMA cycle ran.  Both counters are (nearly) blind to our own
    // READs: SPI busy reads 0.65 % with nothing but 8 kHz of READs on the GPU
    // (profiles/r2/immunity/).  Without the activity counter a device is never quiet.
    if (have_prev_ && have_act && d.count > prev_count_) {
      const double act = static_cast<double>(d.spi - std::min(d.spi, prev_spi_));
      const double clk = static_cast<double>(d.count - prev_count_);
      r.quiet_interval = act < p.quiet_active_frac * clk && d.mfma == prev_mfma_;
    }
    quiet_ = hold(r.quiet_interval, quiet_since_, d.mono_ns, p.quiet_hold_ns);
    dbound_ = hold(r.dbound_interval, dbound_since_, d.mono_ns, p.dbound_hold_ns) && !quiet_;
    r.quiet = quiet_;
    r.dbound = dbound_;
    prev_count_ = d.count;
    prev_mfma_ = d.mfma;
    prev_spi_ = d.spi;
    prev_cpc_ = d.cpc;
    prev_ns_ = d.mono_ns;
    have_prev_ = true;
    return r;
  }

 private:
  // A run of qualifying intervals that began at the previous READ; true once it is
  // at least hold_ns long.
  bool hold(bool qualifies, int64_t& since, int64_t now, int64_t hold_ns) const {
    if (!qualifies) {
      since = 0;
      return false;
    }
    if (since == 0) since = prev_ns_;
    return now - since >= hold_ns;
  }

  bool have_prev_ = false, have_se_ = false;
  uint64_t prev_count_ = 0, prev_mfma_ = 0, prev_spi_ = 0, prev_cpc_ = 0;
  int64_t prev_ns_ = 0;
  uint64_t se_count_ = 0, se_mfma_ = 0;
  int64_t se_ns_ = 0;
  // READ cost [synchronous?][full READ?]: CPC cycles, SPI-blip cycles (EWMA), samples.
  double read_cyc_[2][2] = {};
  double read_spi_[2][2] = {};
  uint64_t read_n_[2][2] = {};
  double cpc_read_us_ = 0;
  double clk_busy_hz_ = 0, clk_idle_hz_ = 0;
  int64_t idle_learned_ns_ = 0;  // the drain that last taught clk_idle_hz_
  bool quiet_ = false, dbound_ = false;
  int64_t quiet_since_ = 0, dbound_since_ = 0;
  int64_t last_plausible_ns_ = 0;
};

// The counter tier as the PMFW thread sees it at one distinct PMFW sample.
struct CounterCover {
  bool ok = false;        // on, not stalled or failed, last drain fresh
  uint64_t epoch = 0;     // bumped on every break of the counter integral
  bool dispatch = false;  // busy_s is the dispatch integral (else SPI active)
  double busy_s = 0;      // the counter tier's cumulative busy integral at its last drain
  double share = 0;       // busy share of the last drain interval
  double since_s = 0;     // host time from the last drain to this PMFW sample
  uint64_t drains = 0;    // drains folded so far (a new one restarts the run-on guess)
};

class UtilBiller {
 public:
  struct Bill {
    double billed_s = 0;
    bool from_counters = false;
  };
  // One distinct PMFW interval: dt_s of firmware time, dgfx_s of PMFW GFX busy in it.
  //
  // While the counter tier held one epoch since the previous PMFW sample, the
  // interval is billed from the counter integral: its value at the last drain, run
  // on to this sample (at 10 Hz the last drain can be 100 ms old; the next drain
  // corrects the guess), plus what earlier intervals could not take, at most dt_s.
  // The run-on guesses each PMFW interval after the drain at the last drain's share,
  // never above the PMFW GFX busy share of that interval: a guess past the end of a
  // load cannot be taken back from a counter, and the PMFW — whatever else it counts
  // (our READs: ≈80 µs each) — sees the GPU stop at once (r5j: 10 Hz, a saturated
  // 3 s load billed 0.042 s past its end without this bound).  The rest carries on
  // to the next intervals (negative: billed ahead of the drains, paid back first) —
  // capped at ±max_carry_s, so a firmware clock slower than the host's cannot bank
  // busy time that a saturated GPU then bills into a following idle stretch.  Else
  // the PMFW busy, and the carry is dropped (its time lies in the intervals PMFW billed).
  Bill bill(double dt_s, double dgfx_s, const CounterCover& c, double max_carry_s) {
    Bill b;
    const double share = std::clamp(c.share, 0.0, 1.0);
    const double since = std::clamp(c.since_s, 0.0, max_carry_s);
    const double rate = dt_s > 0 ? std::min(share, std::clamp(dgfx_s / dt_s, 0.0, 1.0)) : 0.0;
    if (c.drains != drains_ || !have_) guess_s_ = rate * std::min(since, std::max(dt_s, 0.0));
    else guess_s_ = std::min(guess_s_ + rate * std::max(dt_s, 0.0), share * since);
    drains_ = c.drains;
    const double v = c.busy_s + guess_s_;
    const bool cont = c.ok && have_ && epoch_ == c.epoch && dispatch_ == c.dispatch && c.busy_s >= last_s_;
    if (cont) carry_s_ += v - last_v_;
    else carry_s_ = 0;
    if (dt_s > 0) {
      if (cont) {
        b.billed_s = std::clamp(carry_s_, 0.0, dt_s);
        carry_s_ -= b.billed_s;
        if (carry_s_ > max_carry_s) {
          dropped_s_ += carry_s_ - max_carry_s;
          carry_s_ = max_carry_s;
        }
        carry_s_ = std::max(carry_s_, -max_carry_s);
        b.from_counters = true;
      } else {
        b.billed_s = std::clamp(dgfx_s, 0.0, dt_s);
      }
    }
    have_ = c.ok;
    epoch_ = c.epoch;
    dispatch_ = c.dispatch;
    last_s_ = c.busy_s;
    last_v_ = v;
    return b;
  }
  double carry_s() const { return carry_s_; }
  // The GPU changed hands (a pod's allocation ended or began): busy still carried is the
  // previous owner's, and container_gpu_busy_seconds_total counts per allocation — drop
  // it (into dropped_s) rather than bill it to the next pod.
  void drop_carry() {
    dropped_s_ += std::max(carry_s_, 0.0);
    carry_s_ = 0;
  }
  // Counter busy beyond max_carry_s, never billed (a firmware / host clock skew, or a
  // counter integral running ahead of firmware time).
  double dropped_s() const { return dropped_s_; }

 private:
  bool have_ = false, dispatch_ = false;
  uint64_t epoch_ = 0, drains_ = 0;
  double last_s_ = 0, last_v_ = 0, carry_s_ = 0, dropped_s_ = 0, guess_s_ = 0;
};

}  // namespace kgs
