// Device backends.  Exactly one real provider exists — AMD SMI + the PMFW
// metrics table on sysfs (backend_amdsmi.cpp) — plus a deterministic mock used
// by tests and the CPU-only plumbing config (BASELINE.json config 1).  There is
// no NVML/DCGM path and no runtime multi-vendor dispatch.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "kgs/sample.h"

namespace kgs {

struct DeviceInfo {
  int index = 0;               // exporter-local index (label gpu="N")
  std::string bdf;             // 0000:72:00.0
  std::string uuid;            // amdsmi UUID
  std::string serial;
  std::string market_name;     // "AMD Instinct MI355 OAM"
  std::string gpu_type;        // short label value, e.g. "MI355X"
  std::string gfx_target;      // "gfx950"
  int numa_node = -1;
  int num_cu = 0;
  uint32_t num_xcc = 0;
  uint64_t vram_total_bytes = 0;
  uint64_t kfd_gpu_id = 0;     // KFD gpu_id (matches rocprofiler agent gpu_id)
  int kfd_node = -1;
  int drm_card = -1;
  int hip_id = -1;
  std::string sysfs_dir;       // /sys/class/drm/cardN/device
  // MI355X partitioning: compute SPX (all 8 XCDs one device) … CPX (one XCD per
  // device), memory NPS1 / NPS2; each compute partition is its own device with a
  // partition id.  "" / -1 where the driver does not report it.
  std::string compute_partition;
  std::string memory_partition;
  int partition_id = -1;
  // XCCs of the physical GPU's PMFW table this device owns: [xcc_first,
  // xcc_first + num_xcc).  SPX: 0 and all of them (gpu_metrics.h restrict_to_xccs).
  uint32_t xcc_first = 0;
};

struct ProcInfo {
  uint32_t pid = 0;
  std::string name;
  uint64_t vram_bytes = 0, gtt_bytes = 0, cpu_bytes = 0;
  uint64_t gfx_ns = 0;         // cumulative engine time (if the driver reports it)
  uint32_t cu_occupancy = 0;   // CUs in use by the process' waves
  // cu_occupancy was read (false: its KFD stats are unreadable — a process tearing down;
  // the sampler neither integrates nor exports it, kgs_process_cu_unavailable counts it)
  bool cu_valid = true;
  uint32_t evicted_ms = 0;
  // ∫ cu_occupancy / num_cu dt, integrated by the sampler across reads: ROCm compute
  // runs on user-mode queues the driver does not time (gfx_ns reads 0 on MI355X), so
  // CU-occupancy-seconds is the per-process compute-share counter.
  double cu_seconds = 0;
};

struct LinkInfo {
  int link = 0;
  std::string peer_bdf;
  int link_type = 0;            // amdsmi_link_type_t (2 = xGMI)
  uint32_t bit_rate_gbps = 0;
  uint32_t max_bw_gbps = 0;
  uint64_t read_kb = 0, write_kb = 0;
};

// RAS / link health (slow tier).
// RAS blocks in amdsmi_gpu_block_t bit order (bit i = 1 << i): UMC (HBM), SDMA, GFX, ...
constexpr int kEccBlocks = 19;
extern const char* const kEccBlockNames[kEccBlocks];

struct HealthInfo {
  uint64_t ecc_correctable = 0, ecc_uncorrectable = 0, ecc_deferred = 0;
  int xgmi_error_status = -1;   // amdsmi_xgmi_status_t: 0 ok, 1 error, 2 multiple; -1 unknown
  bool ecc_valid = false;
  // Per-block counts for the blocks with ECC enabled whose counts could be read
  // (bit i of ecc_block_mask = block i valid).
  uint32_t ecc_block_mask = 0;
  uint64_t ecc_block_ce[kEccBlocks] = {}, ecc_block_ue[kEccBlocks] = {}, ecc_block_de[kEccBlocks] = {};
};

struct TopoEdge {
  int src = 0, dst = 0;
  int link_type = 0;            // 2 = xGMI, 1 = PCIe
  uint64_t hops = 0;
  uint64_t weight = 0;
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  virtual int device_count() const = 0;
  virtual const DeviceInfo& info(int dev) const = 0;
  // Fast tier: fill everything the PMFW table + HBM occupancy give.  Must be
  // callable concurrently for *different* devices.  0 on success.
  virtual int read_metrics(int dev, GpuSample& out) = 0;
  // Mid tier: per-process compute/HBM.  0 on success.
  virtual int read_procs(int dev, std::vector<ProcInfo>& out) = 0;
  // Slow tier: per-link xGMI metrics with peer BDFs.
  virtual int read_links(int dev, std::vector<LinkInfo>& out) = 0;
  // Pairwise topology among the visible devices.
  virtual int topology(std::vector<TopoEdge>& out) = 0;
  // Slow tier: ECC totals and xGMI error status.
  virtual int read_health(int dev, HealthInfo& out) { return -1; }
  // Called by the sampler after repeated read failures (GPU reset, driver
  // reload): reopen file handles, re-resolve the device and, if needed,
  // re-initialise the management library.  0 when the device reads again;
  // the sampler then drops its accumulator baseline (counters restart).
  virtual int recover(int dev) { return -1; }
  // Mock provider only (bench.py --mock phase X, tests): account a peer copy of
  // `bytes` from device src to device dst on the xGMI link between them, as the
  // PMFW per-link accumulators would.  -1 where unsupported.
  virtual int inject_xgmi(int src, int dst, uint64_t bytes) { return -1; }
};

// Mock provider configuration (tests, plumbing benchmark).
struct MockConfig {
  int n_gpus = 8;               // physical GPUs
  double fw_period_s = 0.020;   // PMFW cadence measured on MI355X (≈20 ms)
  // Load curve per GPU (per XCC when partitioned): a sine base ± amp, or, with
  // square_duty > 0, a square wave at base + amp for the first square_duty of
  // every period and base − amp for the rest (bursty jobs between scrapes).
  double util_base = 50, util_amp = 40, util_period_s = 10;
  double square_duty = 0;
  // The PMFW GFX busy (gfx_busy, its accumulator, per-XCC) never reads below this
  // percent, as on MI355X when the counter tier READs every tick (≈80 µs of PMFW
  // busy per READ: 99.7 % on an idle GPU at 8 kHz, profiles/r2/idle_busy/).  The mock
  // counter source still sees the true load.  Exact for square-wave loads (the
  // floor lifts the low level); a sine load only has its instantaneous value floored.
  double pmfw_busy_floor = 0;
  double ppt_frac = 0;          // share of accumulation cycles the package-power throttler is active
  // "SPX" | "DPX" | "QPX" | "CPX": each GPU shows up as this many devices, all
  // with the GPU's BDF, one partition_id each, XCC curve g·8 + x per XCC.
  std::string compute_partition = "SPX";
  // AMD SMI latency model: the management-library calls take this long and hold
  // one process-wide lock while they do (amdsmi serialises callers); the PMFW
  // table read is a per-device sysfs pread (no lock).  0 = instantaneous.
  double proc_latency_s = 0, link_latency_s = 0, health_latency_s = 0, metrics_latency_s = 0;
  uint64_t vram_total_bytes = 309220868096ull;  // 288 GiB HBM3E as reported by sysfs
  double fail_rate = 0;         // probability a read returns an error
  double stall_s = 0;           // extra latency injected into every read
  int vanish_dev = -1;          // device that starts failing after vanish_after_s
  double vanish_after_s = 0;
  double vanish_for_s = -1;     // >=0: the device is back after this long, but only
                                // once recover() ran (models a GPU reset that needs a reopen)
  uint64_t energy_wrap_at = 0;  // if >0 the energy accumulator wraps at this value
  uint64_t ecc_correctable_per_s = 0;  // injected correctable ECC error rate
  // Per-process load: process k of every device holds proc_cu_share[k] of its CUs
  // (empty: 1 + dev % 2 processes at half the CUs each).  Two tenants sharing one
  // GPU with shares {0.6, 0.0} is the shared-GPU billing test.
  std::vector<double> proc_cu_share;
  // Process k of every device whose CU occupancy cannot be read (ProcInfo::cu_valid
  // false), as for a process tearing down; -1 = none.
  int proc_cu_fail = -1;
  // Background xGMI traffic on every link, following the util curve (1 GB/s per
  // link at 100 %); off, only inject_xgmi() moves the link accumulators.
  bool xgmi_bg = true;
  // A wrong link map (phase X's self-check): this GPU's link table reports the peers
  // of its first two xGMI ports swapped, while its bytes still land on the true ports.
  int xgmi_swap_dev = -1;
  // Slow-tier fault injection (per-device isolation test): after
  // slow_fault_after_s, calls of tier slow_fault_tier ("procs" | "links" |
  // "health") on device slow_fault_dev either hang (kind "hang": block for
  // slow_hang_s, < 0 = until the process exits, outside the management-library
  // lock — a call stuck in one device's driver path) or fail (kind "error").
  int slow_fault_dev = -1;
  std::string slow_fault_tier = "procs";
  std::string slow_fault_kind = "hang";
  double slow_fault_after_s = 0;
  double slow_hang_s = -1;
  uint64_t seed = 1;
  std::string hostname_seed;    // reserved
};

std::unique_ptr<Backend> make_mock_backend(const MockConfig& cfg);
// The mock's closed-form load: busy percent of exporter device `dev` at mock time
// t (s since the backend started), and ∫_0^t of it (percent·s).  Partition
// devices average their XCCs' curves.  Shared with the mock counter source.
double mock_device_util(const MockConfig& cfg, int dev, double t);
double mock_device_util_integral(const MockConfig& cfg, int dev, double t);
// Returns nullptr and fills `err` if AMD SMI cannot be initialised.
std::unique_ptr<Backend> make_amdsmi_backend(std::string& err, const std::string& sysfs_root = "/sys");

// Shorten an amdsmi market name to a gpu_type label ("AMD Instinct MI355 OAM" → "MI355X").
std::string gpu_type_from_market_name(const std::string& market);

}  // namespace kgs
