// Hardware performance-counter sources for the high-rate tier (BASELINE.json
// config 4: MFMA-busy + HBM-BW + xGMI at 100 Hz).
//
// The real source is the rocprofiler-sdk *device counting service* driven from
// our own HSA client (native/counters/pmc_rocprofiler.cpp, built as a separate
// shared object `libkgs_pmc.so` and dlopen'd only when counters are enabled, so
// the exporter never pulls HSA into a process that does not want it).  Reads
// are agent-wide: every wave on the GPU is counted regardless of which process
// launched it, and no kernel is dispatched by the reader.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "kgs/backend.h"
#include "kgs/sample.h"

namespace kgs {

// Index of each base counter inside PmcSample::value.
enum PmcIndex : int {
  kPmcGrbmCount = 0,      // GRBM_COUNT (max over XCC): free-running GPU clocks
  kPmcGrbmGuiActive = 1,  // GRBM_GUI_ACTIVE (max over XCC): clocks the GPU had work
  kPmcMfmaBusy = 2,       // SQ_VALU_MFMA_BUSY_CYCLES (sum over SIMDs)
  kPmcSqBusyCu = 3,       // SQ_BUSY_CU_CYCLES (sum, quad-cycles)
  kPmcTccRdReq = 4,       // TCC_EA0_RDREQ (sum)
  kPmcTccBubble = 5,      // TCC_BUBBLE (sum): 128-byte read requests
  kPmcTccWrReq = 6,       // TCC_EA0_WRREQ (sum)
  kPmcTccWrReq64 = 7,     // TCC_EA0_WRREQ_64B (sum)
  kPmcCount = 8,
};
static_assert(kPmcCount <= kMaxPmc, "PmcSample too small");

const char* pmc_counter_name(int idx);
bool pmc_counter_is_max(int idx);  // reduce over dimensions with max (GRBM) vs sum

// Derived quantities over an interval between two cumulative samples.
struct PmcRates {
  double gpu_active_pct = 0;     // 100 * ΔGUI_ACTIVE / ΔGRBM_COUNT
  double mfma_util_pct = 0;      // 100 * ΔMFMA_BUSY / (ΔGUI_ACTIVE * SIMD_NUM)
  double cu_busy_pct = 0;        // 100 * 4*ΔSQ_BUSY_CU / (ΔGUI_ACTIVE * CU_NUM)
  double hbm_read_Bps = 0;       // bytes/s from TCC→EA read requests
  double hbm_write_Bps = 0;
  double gpu_clock_mhz = 0;      // ΔGRBM_COUNT / Δt
  double dt_s = 0;
};
PmcRates pmc_rates(const PmcSample& a, const PmcSample& b, int num_cu);
// Cumulative HBM bytes implied by one sample's request counts.
double pmc_read_bytes(const PmcSample& s);
double pmc_write_bytes(const PmcSample& s);

class CounterSource {
 public:
  virtual ~CounterSource() = default;
  virtual std::string name() const = 0;
  // Fill `out.value[0..kPmcCount)` with cumulative counts for device `dev`.
  virtual int sample(int dev, PmcSample& out) = 0;
  // Human-readable diagnostics (mode, per-counter instance counts, missing counters).
  virtual std::string info(int dev) const { return name(); }
};

struct MockPmcConfig {
  double clock_mhz = 2100;
  double mfma_frac = 0.6;       // fraction of active time the MFMA pipes are busy
  double read_Bps = 2e12, write_Bps = 1e12;
};
// Mock counters consistent with the mock backend's utilisation curve.
std::unique_ptr<CounterSource> make_mock_counter_source(const Backend& be, const MockConfig& bcfg,
                                                        const MockPmcConfig& cfg);
// dlopen `lib_path` (libkgs_pmc.so) and open one device-counting context per
// device.  nullptr + err on failure (no permission, no HSA, ...).
std::unique_ptr<CounterSource> make_rocprofiler_counter_source(const std::string& lib_path, const Backend& be,
                                                               const std::vector<int>& devices, std::string& err);

}  // namespace kgs
