// Hardware performance-counter sources for the high-rate tier (BASELINE.json
// config 4: MFMA-busy + memory-pipe busy at 100 Hz and beyond).
//
// The product source is the direct command-processor reader
// (native/counters/pmc_aqlprofile.cpp → libkgs_pmc_aql.so): one private AQL queue
// per GPU carrying aqlprofile-built PM4 START / READ packets, no profiler
// framework in between.  It is a separate shared object, dlopen'd only when
// counters are enabled, so the exporter never pulls HSA into a process that does
// not want it.  Reads are agent-wide: every wave on the GPU is counted whichever
// process launched it, and the reader dispatches no kernel.
// (native/counters/pmc_rocprofiler.cpp, the rocprofiler-sdk device-counting
// reader with the same C ABI, is kept for tests and cross-checks only: its HSA
// event thread burns a core, profiles/r1/pmc_helper_thread.md.)
//
// Counter set — chosen by measurement on MI355X / ROCm 7.2 (profiles/aql_probe.md,
// profiles/pmc_probe.md): device-wide, GRBM, SQ_VALU_MFMA_BUSY_CYCLES, TA and TD
// count; the other SQ counters and every TCC counter read (near) zero, so HBM
// bandwidth comes from the PMFW UMC-activity accumulators instead.  GRBM has 2
// slots.
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
  kPmcGrbmActive = 1,     // GRBM_SPI_BUSY (max over XCC): clocks a shader engine had waves to run
  kPmcMfmaBusy = 2,       // SQ_VALU_MFMA_BUSY_CYCLES (sum over SIMDs)
  kPmcTaBusy = 3,         // TA_TA_BUSY (mean over TA instances): vector-memory address unit busy cycles
  // CPC_CPC_STAT_BUSY (max over XCC): clocks the compute command processor was busy —
  // ≈100 % whenever a dispatch is in flight, µs kernels back to back included, plus a
  // short fixed time per counter READ packet (Sampler's dispatch-busy integral removes it).
  kPmcCpcBusy = 4,
  kPmcCount = 5,
  // TD_TD_BUSY tracks TA_TA_BUSY on every load tried and doubles the drain cost
  // (288 more instances, ≈+110 µs per read), so it is not in the default set.
};
static_assert(kPmcCount <= kMaxPmc, "PmcSample too small");

// How a counter's dimension instances (XCC × SE × unit) reduce to one value.
enum PmcReduce : int { kReduceSum = 0, kReduceMax = 1, kReduceAvg = 2 };

const char* pmc_counter_name(int idx);
int pmc_counter_reduce(int idx);

// Counter sets (bits of PmcSample::mask).  Every READ costs the command
// processor time that a dispatch-bound workload on the same GPU feels
// (profiles/launch_overhead.md): the TA block alone is 512 instance reads of
// the 568 in `full`, so the default `base` set drops it and keeps the READ to
// 56 register reads (GRBM count + SPI busy × 8 XCC, MFMA busy × 32 SE, CPC busy × 8).
//
// Activity is GRBM_SPI_BUSY, not GRBM_GUI_ACTIVE.  GUI-active — like the PMFW
// GFX-activity accumulator behind amdgpu_gfx_busy_percent — counts the graphics
// pipe busy while ANY packet is in flight, our own READs included: on an idle
// MI355X every READ reads as ≈190 µs of GUI-active and ≈80 µs of PMFW GFX busy,
// whatever the packet holds (even an IB of NOPs), so an idle GPU sampled at
// 8 kHz reads ~99 % active (profiles/r2/idle_busy/).  SPI busy needs waves: it
// reads 0.65 % under 8 kHz of READs alone and 95 % under an MFMA load, for
// queues created before or after the counters started.  (SQ_BUSY_CYCLES /
// SQ_WAVES read 0 for other processes' kernels in device mode, and the SPI
// block's own wave counter misses queues that predate the session;
// profiles/r2/immunity/.)  GRBM has two counter slots per XCC, so SPI busy
// takes GUI-active's.  It is also the sampler's READ-immune activity test for
// the adaptive READ rate (SamplerConfig::pmc_idle_hz).
constexpr uint32_t kPmcSetBase =
    (1u << kPmcGrbmCount) | (1u << kPmcGrbmActive) | (1u << kPmcMfmaBusy) | (1u << kPmcCpcBusy);
constexpr uint32_t kPmcSetFull = kPmcSetBase | (1u << kPmcTaBusy);
// `util`: only what the reference-contract utilisation needs — the dispatch
// integral (GRBM count, SPI busy, CPC busy): 24 register reads.  A READ's cost to a
// dispatch-bound stream grows with its register reads (≈0.09 µs of a µs-kernel
// stream's time per read, profiles/launch_overhead.md; 56 reads ≈ 5.3 µs per READ,
// profiles/r4/ r4d), so a node that needs no MFMA or per-XCD gauges pays less.
constexpr uint32_t kPmcSetUtil = (1u << kPmcGrbmCount) | (1u << kPmcGrbmActive) | (1u << kPmcCpcBusy);
// "base" | "full" | "util" → mask; 0 for an unknown name.
uint32_t pmc_set_mask(const std::string& name);

// Derived quantities over an interval between two cumulative samples.
struct PmcRates {
  bool have_vmem = false;        // TA counter in the set
  bool have_mfma = false;        // MFMA busy in the set (not in `util`)
  double gpu_active_pct = 0;     // 100 * ΔSPI_BUSY / ΔGRBM_COUNT (READ-immune)
  // 100 * ΔMFMA_BUSY / (ΔSPI_BUSY * SIMD_NUM): MFMA share of the SIMD cycles while a
  // shader engine had waves.  Not rocprofv3's MfmaUtil (that divides by
  // GRBM_GUI_ACTIVE, which counts our own READ packets as busy); the wall-clock
  // figure is amdgpu_mfma_busy_seconds_total (Integrals::mfma_busy_seconds).
  double mfma_util_pct = 0;
  double vmem_busy_pct = 0;      // 100 * ΔTA_BUSY(avg) / ΔSPI_BUSY
  double gpu_clock_mhz = 0;      // ΔGRBM_COUNT / Δt
  double dt_s = 0;
  // Per XCD (both samples carry the breakdown): active % of clocks, and MFMA
  // busy % of that XCD's active SIMD cycles (num_cu / n_xcd CUs × 4 SIMDs).
  // An imbalance here is a workgroup→XCD mapping problem, invisible in the
  // device-wide numbers.
  int n_xcd = 0;
  double xcd_active_pct[kMaxXcc] = {};
  double xcd_mfma_util_pct[kMaxXcc] = {};
  bool have_xcd_vmem = false;    // TA read per XCD (full set)
  double xcd_vmem_busy_pct[kMaxXcc] = {};  // TA busy, mean over the XCD's CUs, % of its active cycles
};
PmcRates pmc_rates(const PmcSample& a, const PmcSample& b, int num_cu);

constexpr int kPmcPending = 1;

class CounterSource {
 public:
  virtual ~CounterSource() = default;
  virtual std::string name() const = 0;
  // Fill `out.value[0..kPmcCount)` with cumulative counts for device `dev`.  0 =
  // a sample, kPmcPending = no new sample yet (a batched reader's first READs are
  // still unpublished; not a failure), < 0 = failed.
  virtual int sample(int dev, PmcSample& out) = 0;
  // Human-readable diagnostics (mode, per-counter instance counts, missing counters).
  virtual std::string info(int dev) const { return name(); }
  // Hand the device's counters back (STOP: another profiler wants the perfmon
  // block, as with `rocprofv3 --pmc`) / program them again (START; counts restart
  // at 0).  Called only from the device's sampler thread.  0 = ok, <0 = failed or
  // unsupported.
  virtual int release(int dev) { return -1; }
  virtual int acquire(int dev) { return -1; }
  // Quiet device (adaptive READ rate): return values read by this very call
  // (synchronous READ) instead of those of the READ submitted on the previous
  // one — at an idle rate of 100 Hz a pipelined sample would be 10 ms old, which
  // doubles the time to notice that work started.  Sampler thread only.
  virtual void set_fresh(int dev, bool fresh) {}
  // Fault boundary.  Every call above is bounded by the source's
  // own deadline (a wedged command processor costs one timeout, never a hang).
  // reset(): after release(), drop whatever the device's session ran on (the
  // reader's AQL queue) so the next acquire() starts from scratch — the circuit
  // breaker's recovery step.  Sampler thread only.  0 = ok.
  virtual int reset(int dev) { return -1; }
  // cancel(dev, true): calls blocked on the device (and new ones) return an error
  // at once, until cancel(dev, false).  Any thread (Sampler::stop()).
  virtual void cancel(int dev, bool on) {}
  // Counters of the fault boundary (for kgs_pmc_* self-metrics): resets done.
  virtual uint64_t resets(int dev) const { return 0; }
  // Test hook (the fault-boundary test on hardware): wedge the
  // device's counter path the way a stuck command processor would — the aqlprofile
  // reader puts a barrier packet that waits on a never-signalled signal at the head
  // of its READ queue, so every later READ, STOP and START on that queue stalls —
  // until reset() drops the queue.  Sampler thread only.  0 = ok.
  virtual int inject_stall(int dev) { return -1; }
  // Publication of READ results (batched reader, include/kgs/aql_batch.h): READs
  // folded, READs that wrote the GPU's L2 back, and results that had not reached
  // host memory when folded.  Any thread.  false = the source does not say.
  struct PublishStats {
    uint64_t reads = 0, publishes = 0, unlanded = 0;
  };
  virtual bool publish_stats(int dev, PublishStats& out) const { return false; }
};

struct MockPmcConfig {
  double clock_mhz = 2100;
  double mfma_frac = 0.6;       // fraction of active time the MFMA pipes are busy
  double vmem_frac = 0.3;       // fraction of active time the TA units are busy
  double cpc_read_us = 2.0;     // CPC_CPC_STAT_BUSY time each READ adds (the real reader's own packet)
  double wave_frac = 1.0;       // share of the CP-busy time with waves in a shader engine (< 1: µs-kernel stream)
  uint32_t mask = kPmcSetFull;  // counters the mock "reads"
  int n_xcd = 8;                // per-XCD breakdown (0 = none)
  double xcd_skew = 0.0;        // XCD x is active (1 - skew·x) of XCD 0's cycles
  double freeze_after_s = 0.0;  // counts stop this long after each (re)START, as after a foreign STOP (0 = never)
  // Fault injection for the counter tier's fault boundary (tests):
  int slow_dev = -1;            // every sample on this device takes slow_s, then succeeds
  double slow_s = 0.0;
  int hang_dev = -1;            // after hang_after samples, samples on this device stop completing:
  uint64_t hang_after = 0;
  // ... each blocks hang_timeout_s and fails (a reader's deadline; cancel() ends it
  // early); < 0: never returns at all, cancel() or not (a call stuck in the driver).
  double hang_timeout_s = 0.25;
  bool hang_heals_on_reset = false;  // reset() clears the hang (the recreated queue works)
  int acquire_fail_dev = -1;    // acquire() fails on this device while its hang is active
  // Batched publication like the aqlprofile reader's (kgs_pmc_configure("batch")):
  // after each acquire the first `batch` samples return kPmcPending, then every
  // sample is the one taken `batch` calls earlier (1 = off).
  int batch = 1;
  // Lite READs (--pmc-lite): only every lite_every-th sample reads the per-SE
  // counters (MFMA, TA); the others carry the last values with se_fresh = 0 (0 = off).
  int lite_every = 0;
};
// Mock counters consistent with the mock backend's utilisation curve.
std::unique_ptr<CounterSource> make_mock_counter_source(const Backend& be, const MockConfig& bcfg,
                                                        const MockPmcConfig& cfg);
// dlopen `lib_path` — libkgs_pmc_aql.so (direct aqlprofile reader, "aqlprofile")
// or libkgs_pmc.so (rocprofiler-sdk device counting, "rocprofiler"); both export
// the kgs_pmc_* C ABI — and open one counting session per device.  nullptr +
// err on failure (no permission, no HSA, ...).  `pipelined` asks a reader that
// exports kgs_pmc_set_pipelined (aqlprofile) to overlap each READ's CP round
// trip with the sampler's sleep: a sample returns the READ submitted on the
// previous tick, stamped with the time the CP executed it.  `lean` (aqlprofile
// reader: 0-3, -1 = reader default) strips the per-dispatch-profiling flushes and
// cache invalidations from the READ packet (native/counters/pmc_aqlprofile.cpp).
std::unique_ptr<CounterSource> make_dl_counter_source(const std::string& name, const std::string& lib_path,
                                                      const Backend& be, const std::vector<int>& devices,
                                                      bool pipelined, uint32_t mask, int lean, std::string& err,
                                                      int timeout_ms = 250, int batch = 1, int publish_us = 1000,
                                                      bool lite = false);

}  // namespace kgs
