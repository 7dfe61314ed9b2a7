// Fixed-size sample records produced by the per-GPU sampler threads.
//
// The reference consumes exactly one GPU series, `container_gpu_sm_util`
// (reference gpu_util_stats/gpu_util_stats.py:159), produced by an exporter that
// lives outside that repository.  These records are the MI355X-native source of
// that series and of the wider amdgpu_* families.
//
// Everything here is trivially copyable so it can travel through the seqlock
// slots in seqlock.h without locks or allocation on the hot path.
#pragma once

#include <cstdint>
#include <cstring>
#include <type_traits>

namespace kgs {

constexpr int kMaxXcc = 8;       // MI355X: 8 XCDs, one XCC each (SPX mode)
constexpr int kMaxXgmi = 8;      // gpu_metrics v1.8 NUM_XGMI_LINKS
constexpr int kMaxPmc = 8;       // hardware counters drained per tick

// Bits of GpuSample::valid.  A field whose bit is clear is "N/A" on this
// device / driver (PMFW reports 0xFFFF / 0xFFFFFFFF for those).
enum SampleField : uint64_t {
  kFGfxBusy = 1ull << 0,
  kFUmcBusy = 1ull << 1,
  kFGfxBusyXcc = 1ull << 2,
  kFTempHotspot = 1ull << 3,
  kFTempMem = 1ull << 4,
  kFTempVrSoc = 1ull << 5,
  kFPower = 1ull << 6,
  kFEnergy = 1ull << 7,
  kFGfxClk = 1ull << 8,
  kFUclk = 1ull << 9,
  kFSocClk = 1ull << 10,
  kFXgmi = 1ull << 11,
  kFPcie = 1ull << 12,
  kFVram = 1ull << 13,
  kFAcc = 1ull << 14,        // gfx/mem activity accumulators present
  kFThrottle = 1ull << 15,
  kFFwTs = 1ull << 16,
  kFXccAcc = 1ull << 17,     // per-XCC busy accumulators present
};

// One hardware reading of one GPU (the PMFW metrics table + HBM occupancy).
struct GpuSample {
  uint64_t seq = 0;            // per-device sequence number of distinct samples
  int64_t mono_ns = 0;         // host CLOCK_MONOTONIC when the read completed
  int64_t wall_ns = 0;         // host CLOCK_REALTIME (for /samples consumers)
  uint64_t fw_ts = 0;          // PMFW timestamp, 10 ns units (distinctness key)
  uint64_t valid = 0;          // SampleField bits
  uint32_t read_ns = 0;        // duration of the backend read
  uint32_t num_xcc = 0;

  float gfx_busy_pct = 0;      // instantaneous, average over XCCs
  float umc_busy_pct = 0;      // memory-controller (HBM) activity
  float gfx_busy_xcc[kMaxXcc] = {};
  float gfx_busy_xcc_window[kMaxXcc] = {};  // per-XCC exact mean since the previous distinct sample
  uint64_t gfx_busy_acc_xcc[kMaxXcc] = {};  // PMFW per-XCC busy accumulators
  // Exact means over the interval since the previous distinct sample, derived
  // from the PMFW activity accumulators (no aliasing: every PMFW tick counts).
  float gfx_busy_window_pct = -1;
  float umc_busy_window_pct = -1;
  float dt_s = 0;              // firmware time since the previous distinct sample
  // Running sums of the sampler's integrals at this sample (Integrals::
  // gfx_busy_seconds / umc_busy_seconds / sampled_seconds): the mean over any
  // window is a difference of two samples, found by binary search of the ring.
  double cum_gfx_s = 0, cum_umc_s = 0, cum_dt_s = 0;
  // Running READ-immune busy integral (Integrals::util_seconds) at this sample.
  double cum_util_s = 0;
  float util_window_pct = -1;  // its mean since the previous distinct sample

  float temp_hotspot_c = 0, temp_mem_c = 0, temp_vrsoc_c = 0;
  float power_w = 0;
  uint32_t gfxclk_mhz[kMaxXcc] = {};
  uint32_t uclk_mhz = 0, socclk_mhz = 0;

  uint64_t energy_acc = 0;             // raw, 15.259 uJ units (2^-16 J)
  uint64_t gfx_activity_acc = 0;       // PMFW accumulators
  uint64_t mem_activity_acc = 0;
  uint64_t accumulation_counter = 0;
  uint64_t ppt_residency_acc = 0, thm_residency_acc = 0;
  // Throttler residency accumulators, kThrottleReasons order (each incremented
  // every accumulation cycle its controller is active; amdsmi.h PVIOL/TVIOL).
  uint64_t throttle_res_acc[5] = {};
  uint64_t xgmi_read_kb[kMaxXgmi] = {};
  uint64_t xgmi_write_kb[kMaxXgmi] = {};
  uint16_t xgmi_link_up[kMaxXgmi] = {};
  uint32_t xgmi_link_speed_gbps = 0, xgmi_link_width = 0;
  uint64_t pcie_bw_acc_gb = 0, pcie_bw_inst_gbps = 0;
  uint64_t pcie_replay_acc = 0;
  uint32_t pcie_link_width = 0, pcie_link_speed_01gts = 0;

  uint64_t vram_used_bytes = 0;
  uint64_t vram_total_bytes = 0;

  // Compute partitions (gpu_metrics.h restrict_to_xccs): the socket's energy
  // accumulator is shared by energy_parts devices; each is billed its XCCs' share
  // of the chip's GFX busy (Σ own / Σ all per-XCC busy accumulators).
  uint32_t energy_parts = 1;
  uint64_t xcc_acc_own = 0, xcc_acc_chip = 0;
};
static_assert(std::is_trivially_copyable<GpuSample>::value, "seqlock payload");

// One drain of the hardware performance counters (the counter tier's reader,
// pmc.h).  Values are cumulative since the counter source opened.
struct PmcSample {
  uint64_t seq = 0;
  int64_t mono_ns = 0;
  uint32_t read_ns = 0;
  uint32_t n = 0;
  uint32_t mask = 0;           // bit i set: value[i] was read (PmcIndex)
  uint64_t value[kMaxPmc] = {};
  // Per-XCD breakdown (MI355X: 8 XCDs, each with its own GRBM and 4 SEs of SQs;
  // workgroups are dispatched round-robin over them).  n_xcd = 0 when the
  // reader could not place its results on XCDs.  Cumulative like value[].
  uint32_t n_xcd = 0;
  uint64_t xcd_active[kMaxXcc] = {};  // GRBM_SPI_BUSY of each XCD
  uint64_t xcd_mfma[kMaxXcc] = {};    // SQ_VALU_MFMA_BUSY_CYCLES summed over each XCD's SEs
  uint64_t xcd_ta[kMaxXcc] = {};      // TA_TA_BUSY summed over each XCD's TA instances (full set; 0 otherwise)
  // The per-SE counters (MFMA busy, TA) were read by this drain.  With lite READs
  // (--pmc-lite) only the publishing READs read them; the others carry the last
  // values read, and every integral of a per-SE counter spans fresh drains only.
  uint32_t se_fresh = 1;
};
static_assert(std::is_trivially_copyable<PmcSample>::value, "seqlock payload");

// Running integrals maintained by the sampler so that Prometheus `rate()` over
// any window gives exact averages regardless of scrape interval.
// Throttlers the PMFW table accounts residency for (gpu_metrics v1.8).
constexpr int kThrottleReasons = 5;
inline const char* throttle_reason_name(int i) {
  static const char* const n[kThrottleReasons] = {"prochot", "ppt", "socket_thermal", "vr_thermal", "hbm_thermal"};
  return i >= 0 && i < kThrottleReasons ? n[i] : "?";
}

struct Integrals {
  double gfx_busy_seconds = 0;   // ∫ gfx busy fraction dt
  double umc_busy_seconds = 0;
  double energy_joules = 0;      // wrap-safe accumulation of energy_acc deltas
  double sampled_seconds = 0;    // ∫ dt over distinct samples (firmware time)
  uint64_t distinct_samples = 0; // samples with a new firmware timestamp
  uint64_t reads = 0;            // backend reads attempted
  uint64_t read_errors = 0;
  uint64_t overruns = 0;         // ticks where the read exceeded the period
  uint64_t pmc_samples = 0;
  uint64_t pmc_errors = 0;
  double read_seconds = 0;       // total time spent in backend reads
  double pmc_read_seconds = 0;   // total time spent in counter drains
  uint64_t recoveries = 0;       // successful Backend::recover() after a failure streak
  uint64_t recover_attempts = 0;
  // ∫ MFMA-busy fraction of wall time dt from the counter stream: per drain,
  // ΔMFMA_BUSY / (SIMDs · ΔGRBM_COUNT) · Δt (all SIMDs busy with MFMA for 1 s = 1).
  double mfma_busy_seconds = 0;
  // ∫ GPU-active (GRBM_SPI_BUSY share of clocks) dt from the counter stream: the
  // READ-immune busy integral (--sm-util-source counters).
  double active_seconds = 0;
  // Counter-tier continuity, published with the counter integrals: bumped on every
  // break (release, breaker trip, failed re-START), and the CLOCK_MONOTONIC time of
  // the last folded drain.  The PMFW thread uses a Δactive_seconds only across an
  // interval with one epoch and a fresh drain (Sampler::run_pmfw).
  uint64_t pmc_epoch = 0;
  int64_t pmc_last_ns = 0;
  // ∫ dispatch-in-flight fraction dt from the counter stream: per drain, the compute
  // command processor's busy share of the clocks (CPC_CPC_STAT_BUSY) minus the time
  // the exporter's own READ packet kept it busy (learned on intervals with no waves),
  // never below the SPI-busy share; an interval the CP was busy for (nearly) all of
  // counts whole.  dispatch_drains > 0 once the counter set carries CPC busy.
  double dispatch_seconds = 0;
  uint64_t dispatch_drains = 0;
  double pmc_last_share = 0;    // busy share (dispatch, else SPI) of the last drain interval
  double cpc_read_us = 0;       // the READ's own CP busy time as last learned (µs)
  // The shader clocks the estimator learned (DispatchEstimator): on READ-only intervals
  // (idle) and on fully busy ones (busy); 0 until seen.  The time split of long partial
  // intervals prices idle cycles at the idle clock.
  double pmc_clk_idle_hz = 0;
  double pmc_clk_busy_hz = 0;
  // ∫ busy dt that does not count the exporter's own counter READs (the default
  // --sm-util-source auto behind container_gpu_sm_util / container_gpu_busy_seconds_total):
  // per PMFW interval, the counter tier's dispatch integral (dispatch_seconds; SPI
  // active_seconds for a set without CPC busy) while that tier covered the interval,
  // the excess over an interval carried to the next (UtilBiller), else the PMFW GFX
  // busy.  util_counter_seconds: the firmware time billed from the counters;
  // util_carry_seconds: counter busy received but not yet billed;
  // util_dropped_seconds: counter busy beyond the carry cap, never billed.
  double util_seconds = 0;
  double util_counter_seconds = 0;
  double util_carry_seconds = 0;
  double util_dropped_seconds = 0;
  // ∫ throttled fraction dt per reason (Δresidency / Δaccumulation_counter per
  // distinct PMFW table): seconds the GPU ran held back by each controller.
  double throttle_seconds[kThrottleReasons] = {};
};
static_assert(std::is_trivially_copyable<Integrals>::value, "seqlock payload");

inline double energy_units_to_joules(uint64_t units) {
  return static_cast<double>(units) * (1.0 / 65536.0);  // 15.259 uJ = 2^-16 J
}

}  // namespace kgs
