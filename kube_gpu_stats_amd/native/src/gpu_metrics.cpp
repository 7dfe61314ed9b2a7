// PMFW gpu_metrics v1.8 parser (MI355X / gfx950).  See gpu_metrics.h.
#include "kgs/gpu_metrics.h"

#include <cstring>
#include <string>

namespace kgs {

namespace {

template <class T>
inline T rd(const uint8_t* b, size_t off) {
  T v;
  std::memcpy(&v, b + off, sizeof(T));
  return v;
}

// Offsets inside struct gpu_metrics_v1_8 (naturally aligned, little endian).
enum : size_t {
  kHdrSize = 0,          // u16 structure_size, u8 format, u8 content
  kTempHotspot = 4,      // u16 °C
  kTempMem = 6,
  kTempVrSoc = 8,
  kSocketPower = 10,     // u16 W
  kAvgGfxAct = 12,       // u16 %
  kAvgUmcAct = 14,
  kMemMaxBw = 16,        // u64 GB/s
  kEnergyAcc = 24,       // u64, 15.259 uJ
  kSysClock = 32,        // u64 ns (driver)
  kAccumCounter = 40,    // u32
  kProchotRes = 44,
  kPptRes = 48,
  kSocketThmRes = 52,
  kVrThmRes = 56,
  kHbmThmRes = 60,
  kGfxclkLock = 64,      // u32
  kPcieWidth = 68,       // u16
  kPcieSpeed = 70,       // u16, 0.1 GT/s
  kXgmiWidth = 72,
  kXgmiSpeed = 74,
  kGfxActAcc = 76,       // u32
  kMemActAcc = 80,       // u32
  kPcieBwAcc = 88,       // u64
  kPcieBwInst = 96,
  kPcieL0Recov = 104,
  kPcieReplay = 112,
  kPcieReplayRover = 120,
  kNakSent = 128,        // u32
  kNakRcvd = 132,
  kXgmiRead = 136,       // u64[8] KB
  kXgmiWrite = 200,      // u64[8] KB
  kXgmiStatus = 264,     // u16[8]
  kFwTs = 288,           // u64, 10 ns
  kCurGfxclk = 296,      // u16[8]
  kCurSocclk = 312,      // u16[4]
  kCurVclk0 = 320,       // u16[4]
  kCurDclk0 = 328,       // u16[4]
  kCurUclk = 336,        // u16
  kNumPartition = 338,   // u16
  kXcpBase = 344,        // struct amdgpu_xcp_metrics_v1_2[8], 440 B each
  kXcpStride = 440,
  kXcpGfxBusyInst = 0,   // u32[8] %
  kXcpGfxBusyAcc = 120,  // u64[8] accumulated % (same units as gfx_activity_acc)
};

inline bool na16(uint16_t v) { return v == 0xFFFF; }
inline bool na32(uint32_t v) { return v == 0xFFFFFFFFu; }
inline bool na64(uint64_t v) { return v == ~0ull; }

}  // namespace

int gpu_metrics_revision(const uint8_t* buf, size_t len) {
  if (len < 4) return -1;
  return (static_cast<int>(buf[2]) << 8) | buf[3];
}

int parse_gpu_metrics_v1_8(const uint8_t* b, size_t len, GpuSample& s) {
  if (len < kGpuMetricsV18Size) return -1;
  if (rd<uint16_t>(b, kHdrSize) != kGpuMetricsV18Size || b[2] != 1 || b[3] != 8) return -1;

  uint64_t valid = 0;
  const uint16_t th = rd<uint16_t>(b, kTempHotspot), tm = rd<uint16_t>(b, kTempMem),
                 tv = rd<uint16_t>(b, kTempVrSoc), pw = rd<uint16_t>(b, kSocketPower),
                 ga = rd<uint16_t>(b, kAvgGfxAct), ua = rd<uint16_t>(b, kAvgUmcAct);
  if (!na16(th)) { s.temp_hotspot_c = th; valid |= kFTempHotspot; }
  if (!na16(tm)) { s.temp_mem_c = tm; valid |= kFTempMem; }
  if (!na16(tv)) { s.temp_vrsoc_c = tv; valid |= kFTempVrSoc; }
  if (!na16(pw)) { s.power_w = pw; valid |= kFPower; }
  if (!na16(ga)) { s.gfx_busy_pct = ga; valid |= kFGfxBusy; }
  if (!na16(ua)) { s.umc_busy_pct = ua; valid |= kFUmcBusy; }

  const uint64_t e = rd<uint64_t>(b, kEnergyAcc);
  if (!na64(e)) { s.energy_acc = e; valid |= kFEnergy; }

  const uint32_t acc = rd<uint32_t>(b, kAccumCounter), gacc = rd<uint32_t>(b, kGfxActAcc),
                 macc = rd<uint32_t>(b, kMemActAcc);
  if (!na32(acc) && !na32(gacc) && !na32(macc)) {
    s.accumulation_counter = acc;
    s.gfx_activity_acc = gacc;
    s.mem_activity_acc = macc;
    valid |= kFAcc;
  }
  const uint32_t ppt = rd<uint32_t>(b, kPptRes), thm = rd<uint32_t>(b, kSocketThmRes);
  if (!na32(ppt)) { s.ppt_residency_acc = ppt; valid |= kFThrottle; }
  if (!na32(thm)) s.thm_residency_acc = thm;
  const size_t res_off[kThrottleReasons] = {kProchotRes, kPptRes, kSocketThmRes, kVrThmRes, kHbmThmRes};
  for (int r = 0; r < kThrottleReasons; ++r) {
    const uint32_t v = rd<uint32_t>(b, res_off[r]);
    s.throttle_res_acc[r] = na32(v) ? 0 : v;
  }

  const uint16_t pwid = rd<uint16_t>(b, kPcieWidth), psp = rd<uint16_t>(b, kPcieSpeed);
  const uint64_t pbw = rd<uint64_t>(b, kPcieBwAcc), pbi = rd<uint64_t>(b, kPcieBwInst),
                 prp = rd<uint64_t>(b, kPcieReplay);
  if (!na16(pwid)) s.pcie_link_width = pwid;
  if (!na16(psp)) s.pcie_link_speed_01gts = psp;
  if (!na64(pbw)) { s.pcie_bw_acc_gb = pbw; valid |= kFPcie; }
  if (!na64(pbi)) s.pcie_bw_inst_gbps = pbi;
  if (!na64(prp)) s.pcie_replay_acc = prp;

  const uint16_t xw = rd<uint16_t>(b, kXgmiWidth), xs = rd<uint16_t>(b, kXgmiSpeed);
  if (!na16(xw)) s.xgmi_link_width = xw;
  if (!na16(xs)) s.xgmi_link_speed_gbps = xs;
  bool any_xgmi = false;
  for (int l = 0; l < kMaxXgmi; ++l) {
    const uint64_t r = rd<uint64_t>(b, kXgmiRead + 8 * l), w = rd<uint64_t>(b, kXgmiWrite + 8 * l);
    const uint16_t st = rd<uint16_t>(b, kXgmiStatus + 2 * l);
    s.xgmi_read_kb[l] = na64(r) ? 0 : r;
    s.xgmi_write_kb[l] = na64(w) ? 0 : w;
    s.xgmi_link_up[l] = na16(st) ? 0xFFFF : st;
    any_xgmi |= !na64(r);
  }
  if (any_xgmi) valid |= kFXgmi;

  const uint64_t fw = rd<uint64_t>(b, kFwTs);
  if (!na64(fw)) { s.fw_ts = fw; valid |= kFFwTs; }

  uint32_t nclk = 0;
  for (int x = 0; x < kMaxXcc; ++x) {
    const uint16_t c = rd<uint16_t>(b, kCurGfxclk + 2 * x);
    s.gfxclk_mhz[x] = na16(c) ? 0 : c;
    nclk += !na16(c);
  }
  if (nclk) valid |= kFGfxClk;
  const uint16_t uclk = rd<uint16_t>(b, kCurUclk), soc = rd<uint16_t>(b, kCurSocclk);
  if (!na16(uclk)) { s.uclk_mhz = uclk; valid |= kFUclk; }
  if (!na16(soc)) { s.socclk_mhz = soc; valid |= kFSocClk; }

  // Per-XCC instantaneous busy from partition 0 .. num_partition-1 (SPX: one
  // partition holding all 8 XCCs; CPX: 8 partitions of one XCC each).
  uint16_t nparts = rd<uint16_t>(b, kNumPartition);
  if (na16(nparts) || nparts == 0) nparts = 1;
  if (nparts > kV18NumXcp) nparts = kV18NumXcp;
  uint32_t nxcc = 0;
  bool xcc_acc = true;
  for (int p = 0; p < nparts && nxcc < static_cast<uint32_t>(kMaxXcc); ++p) {
    const size_t base = kXcpBase + static_cast<size_t>(p) * kXcpStride;
    for (int x = 0; x < kMaxXcc && nxcc < static_cast<uint32_t>(kMaxXcc); ++x) {
      const uint32_t v = rd<uint32_t>(b, base + kXcpGfxBusyInst + 4 * x);
      if (na32(v)) continue;
      const uint64_t acc = rd<uint64_t>(b, base + kXcpGfxBusyAcc + 8 * x);
      xcc_acc &= !na64(acc);
      s.gfx_busy_acc_xcc[nxcc] = na64(acc) ? 0 : acc;
      s.gfx_busy_xcc[nxcc++] = static_cast<float>(v);
    }
  }
  if (nxcc) { s.num_xcc = nxcc; valid |= kFGfxBusyXcc; }
  if (nxcc && xcc_acc) valid |= kFXccAcc;

  s.valid |= valid;
  return 0;
}

void restrict_to_xccs(GpuSample& s, uint32_t first, uint32_t count) {
  if (count == 0 || first + count > s.num_xcc || (first == 0 && count == s.num_xcc)) return;
  s.energy_parts = s.num_xcc / count;
  s.xcc_acc_own = s.xcc_acc_chip = 0;
  for (uint32_t x = 0; x < s.num_xcc && x < static_cast<uint32_t>(kMaxXcc); ++x) {
    s.xcc_acc_chip += s.gfx_busy_acc_xcc[x];
    if (x >= first && x < first + count) s.xcc_acc_own += s.gfx_busy_acc_xcc[x];
  }
  double inst = 0, acc = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const uint32_t x = first + k;
    s.gfx_busy_xcc[k] = s.gfx_busy_xcc[x];
    s.gfx_busy_acc_xcc[k] = s.gfx_busy_acc_xcc[x];
    s.gfxclk_mhz[k] = s.gfxclk_mhz[x];
    inst += s.gfx_busy_xcc[x];
    acc += static_cast<double>(s.gfx_busy_acc_xcc[k]);
  }
  for (uint32_t k = count; k < static_cast<uint32_t>(kMaxXcc); ++k) {
    s.gfx_busy_xcc[k] = 0;
    s.gfx_busy_acc_xcc[k] = 0;
    s.gfxclk_mhz[k] = 0;
  }
  s.num_xcc = count;
  s.gfx_busy_pct = static_cast<float>(inst / count);
  // Per-XCC accumulators share gfx_activity_acc's units (accumulated percent per
  // accumulation_counter tick), so their mean is the partition's activity
  // accumulator and Sampler::integrate needs no partition logic.
  if (s.valid & kFXccAcc) s.gfx_activity_acc = static_cast<uint64_t>(acc / count + 0.5);
}

uint32_t partitions_of_mode(const char* mode) {
  if (!mode) return 1;
  const std::string m(mode);
  if (m == "DPX") return 2;
  if (m == "QPX") return 4;
  if (m == "CPX") return 8;
  return 1;
}

}  // namespace kgs
