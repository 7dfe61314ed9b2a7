// When a parked counter tier (SamplerConfig::pmc_quiet_release_s) takes the GPU back,
// from the PMFW samples alone: a pure class, fed one PMFW sample per poll of the
// parked device's counter thread, unit-tested without threads (native/tests/test_core.cpp).
//
// Wakes on (sampler.h kUnparkTablePct / kUnparkBusyPct / kUnparkWindowS):
//  * one PMFW interval ≥ kUnparkTablePct GFX busy — a load starting;
//  * ≥ kUnparkBusyPct over a tumbling window of kUnparkWindowS of table time — a trickle
//    (one interval ≥ 1 % woke on stray 0.2 ms blips: r6g phase P);
//  * no PMFW table for `silent_ns` — nothing else would bill the GPU while parked.
// Tables read in the first kSettleNs after the park are skipped: the STOP and the READ
// queue's teardown are CP work of their own.
#pragma once

#include <cstdint>

#include "kgs/sample.h"

namespace kgs {

class UnparkDetector {
 public:
  static constexpr int64_t kSettleNs = 50000000;  // 50 ms

  UnparkDetector(double table_pct, double window_pct, double window_s)
      : table_pct_(table_pct), window_pct_(window_pct), window_s_(window_s) {}

  void parked(int64_t park_ns) {
    park_ns_ = park_ns;
    base_dt_ = -1;
  }

  // One poll at `now_ns`; `g` is the latest PMFW sample (nullptr: none yet).  True to
  // wake; `busy_ns` then holds the sample that showed the work (0 for silence).
  bool poll(int64_t now_ns, const GpuSample* g, int64_t silent_ns, int64_t* busy_ns) {
    *busy_ns = 0;
    if (now_ns - park_ns_ > silent_ns && (!g || now_ns - g->mono_ns > silent_ns)) return true;
    if (!g || g->mono_ns <= park_ns_ + kSettleNs || !(g->cum_dt_s > 0)) return false;
    if (g->gfx_busy_window_pct >= table_pct_) {
      *busy_ns = g->mono_ns;
      return true;
    }
    if (base_dt_ < 0 || g->cum_dt_s < base_dt_) {  // first settled table, or the device re-opened
      base_dt_ = g->cum_dt_s;
      base_gfx_ = g->cum_gfx_s;
      return false;
    }
    if (g->cum_dt_s - base_dt_ < window_s_) return false;
    const double pct = 100.0 * (g->cum_gfx_s - base_gfx_) / (g->cum_dt_s - base_dt_);
    base_dt_ = g->cum_dt_s;
    base_gfx_ = g->cum_gfx_s;
    if (pct < window_pct_) return false;
    *busy_ns = g->mono_ns;
    return true;
  }

 private:
  double table_pct_, window_pct_, window_s_;
  int64_t park_ns_ = 0;
  double base_dt_ = -1, base_gfx_ = 0;
};

}  // namespace kgs
