// The real MI355X provider: AMD SMI for enumeration / processes / links /
// topology, plus a direct pread of the PMFW metrics table and of the HBM
// occupancy file for the fast tier.
#include <amd_smi/amdsmi.h>
#include <fcntl.h>
#include <limits.h>
#include <stdlib.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>
#include <vector>

#include "kgs/backend.h"
#include "kgs/gpu_metrics.h"
#include "kgs/kfd_procs.h"

namespace kgs {

namespace {

std::string fmt_bdf(const amdsmi_bdf_t& b) {
  char buf[32];
  std::snprintf(buf, sizeof buf, "%04llx:%02x:%02x.%x",
                static_cast<unsigned long long>(b.domain_number), static_cast<unsigned>(b.bus_number),
                static_cast<unsigned>(b.device_number), static_cast<unsigned>(b.function_number));
  return buf;
}

int64_t now_ns(clockid_t c) {
  timespec ts;
  clock_gettime(c, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

bool read_small_file(const std::string& p, std::string& out) {
  FILE* f = std::fopen(p.c_str(), "r");
  if (!f) return false;
  char buf[256];
  size_t n = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[n] = 0;
  out.assign(buf);
  while (!out.empty() && std::isspace(static_cast<unsigned char>(out.back()))) out.pop_back();
  return true;
}

struct Dev {
  amdsmi_processor_handle h = nullptr;
  DeviceInfo info;
  int fd_metrics = -1;
  int fd_vram_used = -1;
  bool partitioned = false;  // a DPX/QPX/CPX partition: restrict the table to its XCCs
  uint64_t ecc_mask = 0;     // blocks with ECC enabled (read once, slow thread only)
  bool ecc_mask_read = false;
  DrmFdCache fd_cache;       // per-process DRM fds (slow thread only)
  alignas(64) uint8_t buf[4096];
};

// /proc/<pid>/comm without the trailing newline ("" if unreadable).
std::string proc_comm(uint32_t pid) {
  char path[64];
  std::snprintf(path, sizeof path, "/proc/%u/comm", pid);
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return {};
  char buf[64];
  const ssize_t n = read(fd, buf, sizeof buf);
  close(fd);
  if (n <= 0) return {};
  size_t len = static_cast<size_t>(n);
  while (len > 0 && (buf[len - 1] == '\n' || buf[len - 1] == 0)) --len;
  return std::string(buf, len);
}

class AmdSmiBackend final : public Backend {
 public:
  ~AmdSmiBackend() override {
    for (auto& d : devs_) {
      if (d->fd_metrics >= 0) close(d->fd_metrics);
      if (d->fd_vram_used >= 0) close(d->fd_vram_used);
    }
    if (inited_) amdsmi_shut_down();
  }

  bool init(std::string& err, const std::string& sysfs_root) {
    sysfs_root_ = sysfs_root;
    amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) {
      err = "amdsmi_init failed: status " + std::to_string(static_cast<int>(st));
      return false;
    }
    inited_ = true;
    uint32_t nsock = 0;
    if (amdsmi_get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS || nsock == 0) {
      err = "no AMD GPU sockets";
      return false;
    }
    std::vector<amdsmi_socket_handle> socks(nsock);
    amdsmi_get_socket_handles(&nsock, socks.data());
    for (auto s : socks) {
      uint32_t np = 0;
      if (amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> hs(np);
      amdsmi_get_processor_handles(s, &np, hs.data());
      for (auto h : hs) {
        processor_type_t pt;
        if (amdsmi_get_processor_type(h, &pt) == AMDSMI_STATUS_SUCCESS && pt != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
        add_device(h, sysfs_root);
      }
    }
    if (devs_.empty()) {
      err = "amdsmi found no GPU processors";
      return false;
    }
    return true;
  }

  std::string name() const override { return "amdsmi"; }
  int device_count() const override { return static_cast<int>(devs_.size()); }
  const DeviceInfo& info(int d) const override { return devs_[d]->info; }

  int read_metrics(int d, GpuSample& s) override {
    Dev& dv = *devs_[d];
    int rc = -1;
    if (dv.fd_metrics >= 0) {
      ssize_t n = pread(dv.fd_metrics, dv.buf, sizeof dv.buf, 0);
      if (n <= 0) {
        // The driver can invalidate an open sysfs file (GPU reset / hot unplug): reopen once.
        close(dv.fd_metrics);
        dv.fd_metrics = open((dv.info.sysfs_dir + "/gpu_metrics").c_str(), O_RDONLY | O_CLOEXEC);
        n = dv.fd_metrics >= 0 ? pread(dv.fd_metrics, dv.buf, sizeof dv.buf, 0) : -1;
      }
      if (n > 0 && gpu_metrics_revision(dv.buf, static_cast<size_t>(n)) == 0x0108)
        rc = parse_gpu_metrics_v1_8(dv.buf, static_cast<size_t>(n), s);
    }
    if (rc != 0) {
      std::lock_guard<std::mutex> g(smi_mu_);
      rc = read_metrics_amdsmi_locked(dv, s);
    }
    if (rc != 0) return rc;
    if (dv.partitioned) restrict_to_xccs(s, dv.info.xcc_first, dv.info.num_xcc);
    read_vram(dv, s);
    s.mono_ns = now_ns(CLOCK_MONOTONIC);
    s.wall_ns = now_ns(CLOCK_REALTIME);
    return 0;
  }

  int read_procs(int d, std::vector<ProcInfo>& out) override {
    out.clear();
    // The KFD's own per-process files first: no queue walk, no stdout message, no AMD
    // SMI lock, and a per-process flag when the CU occupancy cannot be read
    // (kgs/kfd_procs.h).  AMD SMI only where the KFD sysfs cannot be listed.
    const DeviceInfo& in = devs_[d]->info;
    if (in.kfd_gpu_id &&
        read_kfd_procs(kKfdProcRoot, "/proc", in.kfd_gpu_id, in.bdf, out, &devs_[d]->fd_cache, now_ns(CLOCK_MONOTONIC)) == 0)
      return 0;
    std::vector<amdsmi_proc_info_t> list;
    uint32_t cap = 0;
    {
      std::lock_guard<std::mutex> g(smi_mu_);
      uint32_t n = 0;
      amdsmi_status_t st = amdsmi_get_gpu_process_list(devs_[d]->h, &n, nullptr);
      if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return -static_cast<int>(st);
      if (n == 0) return 0;
      list.resize(n + 8);
      cap = static_cast<uint32_t>(list.size());
      st = amdsmi_get_gpu_process_list(devs_[d]->h, &cap, list.data());
      if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return -static_cast<int>(st);
    }
    for (uint32_t i = 0; i < cap && i < list.size(); ++i) {
      const auto& p = list[i];
      ProcInfo pi;
      pi.pid = p.pid;
      pi.name.assign(p.name, strnlen(p.name, sizeof p.name));
      // AMD SMI leaves the name empty where it cannot read it (seen on the gpurun box);
      // with hostPID (the DaemonSet) the host's /proc has it.
      if (pi.name.empty()) pi.name = proc_comm(p.pid);
      pi.vram_bytes = p.memory_usage.vram_mem;
      pi.gtt_bytes = p.memory_usage.gtt_mem;
      pi.cpu_bytes = p.memory_usage.cpu_mem;
      pi.gfx_ns = p.engine_usage.gfx;
      pi.cu_occupancy = p.cu_occupancy;
      {  // AMD SMI reads a process's CU occupancy through its KFD queues directory and
         // reports 0 when that is gone: unknown, not idle
        char qp[96];
        std::snprintf(qp, sizeof qp, "%s/%u/queues", kKfdProcRoot, p.pid);
        pi.cu_valid = access(qp, R_OK | X_OK) == 0;
        if (!pi.cu_valid) pi.cu_occupancy = 0;
      }
      pi.evicted_ms = p.evicted_time;
      out.push_back(std::move(pi));
    }
    return 0;
  }

  int read_links(int d, std::vector<LinkInfo>& out) override {
    std::lock_guard<std::mutex> g(smi_mu_);
    out.clear();
    amdsmi_link_metrics_t lm;
    std::memset(&lm, 0, sizeof lm);
    amdsmi_status_t st = amdsmi_get_link_metrics(devs_[d]->h, &lm);
    if (st != AMDSMI_STATUS_SUCCESS) return -static_cast<int>(st);
    // `num_links` counts the *connected* ports, but the array is indexed by
    // physical port (the PMFW xgmi_*_data_acc index): on MI355X port 0 is the
    // disabled self port (BDF all ones) and the 7 peers sit on ports 1..7, so
    // num_links = 7 while the last peer is links[7] (measured,
    // profiles/r2/xgmi/).  Walk every port slot the PMFW table has and keep the
    // ones that name a peer.
    uint32_t found = 0;
    for (uint32_t i = 0; i < AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK && found < lm.num_links; ++i) {
      const auto& e = lm.links[i];
      const bool disabled = e.bdf.domain_number == 0xFFFFFFFFFFFFull || e.bdf.as_uint == ~0ull;
      const bool empty = e.bdf.as_uint == 0 && e.link_type == 0 && e.bit_rate == 0;
      if (disabled || empty) continue;
      ++found;
      LinkInfo li;
      li.link = static_cast<int>(i);
      li.peer_bdf = fmt_bdf(e.bdf);
      li.link_type = static_cast<int>(lm.links[i].link_type);
      li.bit_rate_gbps = lm.links[i].bit_rate;
      li.max_bw_gbps = lm.links[i].max_bandwidth;
      li.read_kb = lm.links[i].read;
      li.write_kb = lm.links[i].write;
      out.push_back(std::move(li));
    }
    return 0;
  }

  int read_health(int d, HealthInfo& out) override {
    std::lock_guard<std::mutex> g(smi_mu_);
    amdsmi_error_count_t ec;
    std::memset(&ec, 0, sizeof ec);
    out.ecc_valid = amdsmi_get_gpu_total_ecc_count(devs_[d]->h, &ec) == AMDSMI_STATUS_SUCCESS;
    if (out.ecc_valid) {
      out.ecc_correctable = ec.correctable_count;
      out.ecc_uncorrectable = ec.uncorrectable_count;
      out.ecc_deferred = ec.deferred_count;
    }
    // Per-block counts: the enabled mask is fixed by the VBIOS / driver, so it is kept
    // once read (a failed read is retried on the next RAS pass), then one sysfs-backed
    // count per enabled block.
    if (!devs_[d]->ecc_mask_read) {
      uint64_t en = 0;
      if (amdsmi_get_gpu_ecc_enabled(devs_[d]->h, &en) == AMDSMI_STATUS_SUCCESS) {
        devs_[d]->ecc_mask = en;
        devs_[d]->ecc_mask_read = true;
      }
    }
    out.ecc_block_mask = 0;
    for (int b = 0; b < kEccBlocks; ++b) {
      if (!(devs_[d]->ecc_mask & (1ULL << b))) continue;
      amdsmi_error_count_t bc;
      std::memset(&bc, 0, sizeof bc);
      if (amdsmi_get_gpu_ecc_count(devs_[d]->h, static_cast<amdsmi_gpu_block_t>(1ULL << b), &bc) != AMDSMI_STATUS_SUCCESS)
        continue;
      out.ecc_block_mask |= 1u << b;
      out.ecc_block_ce[b] = bc.correctable_count;
      out.ecc_block_ue[b] = bc.uncorrectable_count;
      out.ecc_block_de[b] = bc.deferred_count;
    }
    amdsmi_xgmi_status_t xs;
    out.xgmi_error_status =
        amdsmi_gpu_xgmi_error_status(devs_[d]->h, &xs) == AMDSMI_STATUS_SUCCESS ? static_cast<int>(xs) : -1;
    return out.ecc_valid || out.xgmi_error_status >= 0 ? 0 : -1;
  }

  int topology(std::vector<TopoEdge>& out) override {
    std::lock_guard<std::mutex> g(smi_mu_);
    out.clear();
    for (size_t a = 0; a < devs_.size(); ++a) {
      for (size_t b = 0; b < devs_.size(); ++b) {
        if (a == b) continue;
        TopoEdge e;
        e.src = static_cast<int>(a);
        e.dst = static_cast<int>(b);
        amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
        uint64_t hops = 0, w = 0;
        if (amdsmi_topo_get_link_type(devs_[a]->h, devs_[b]->h, &hops, &t) == AMDSMI_STATUS_SUCCESS) {
          e.link_type = static_cast<int>(t);
          e.hops = hops;
        }
        if (amdsmi_topo_get_link_weight(devs_[a]->h, devs_[b]->h, &w) == AMDSMI_STATUS_SUCCESS) e.weight = w;
        out.push_back(e);
      }
    }
    return 0;
  }

  // After a GPU reset or driver reload: (1) reopen the sysfs files, re-resolving
  // the DRM card by PCI address (card numbers can change on reload); (2) if the
  // table still does not read, re-initialise AMD SMI (stale handles) at most
  // once per 10 s for all devices and remap every handle by BDF.
  int recover(int d) override {
    std::lock_guard<std::mutex> g(smi_mu_);
    Dev& dv = *devs_[d];
    const std::string dir = find_sysfs_dir(sysfs_root_, -1, dv.info.bdf);
    if (!dir.empty() && dir != dv.info.sysfs_dir) dv.info.sysfs_dir = dir;
    open_files(dv);
    GpuSample s;
    if (dv.fd_metrics >= 0) {
      const ssize_t n = pread(dv.fd_metrics, dv.buf, sizeof dv.buf, 0);
      if (n > 0 && parse_gpu_metrics_v1_8(dv.buf, static_cast<size_t>(n), s) == 0) return 0;
    }
    const int64_t now = now_ns(CLOCK_MONOTONIC);
    if (now - last_reinit_ns_ < 10000000000LL) return -1;
    last_reinit_ns_ = now;
    ++reinits_;
    if (!reinit_locked()) return -1;
    return read_metrics_amdsmi_locked(dv, s);
  }

 private:
  bool reinit_locked() {
    if (inited_) amdsmi_shut_down();
    inited_ = amdsmi_init(AMDSMI_INIT_AMD_GPUS) == AMDSMI_STATUS_SUCCESS;
    if (!inited_) return false;
    uint32_t nsock = 0;
    if (amdsmi_get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) return false;
    std::vector<amdsmi_socket_handle> socks(nsock);
    amdsmi_get_socket_handles(&nsock, socks.data());
    for (auto s : socks) {
      uint32_t np = 0;
      if (amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> hs(np);
      amdsmi_get_processor_handles(s, &np, hs.data());
      for (auto h : hs) {
        amdsmi_bdf_t bdf;
        if (amdsmi_get_gpu_device_bdf(h, &bdf) != AMDSMI_STATUS_SUCCESS) continue;
        const std::string b = fmt_bdf(bdf);
        for (auto& dv : devs_)
          if (dv->info.bdf == b) dv->h = h;
      }
    }
    return true;
  }

  static void open_files(Dev& d) {
    if (d.fd_metrics >= 0) close(d.fd_metrics);
    if (d.fd_vram_used >= 0) close(d.fd_vram_used);
    d.fd_metrics = d.fd_vram_used = -1;
    if (d.info.sysfs_dir.empty()) return;
    d.fd_metrics = open((d.info.sysfs_dir + "/gpu_metrics").c_str(), O_RDONLY | O_CLOEXEC);
    d.fd_vram_used = open((d.info.sysfs_dir + "/mem_info_vram_used").c_str(), O_RDONLY | O_CLOEXEC);
  }

  void add_device(amdsmi_processor_handle h, const std::string& sysfs_root) {
    auto d = std::make_unique<Dev>();
    d->h = h;
    DeviceInfo& in = d->info;
    in.index = static_cast<int>(devs_.size());
    amdsmi_bdf_t bdf;
    if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) in.bdf = fmt_bdf(bdf);
    char uuid[AMDSMI_GPU_UUID_SIZE + 1] = {};
    unsigned int ulen = AMDSMI_GPU_UUID_SIZE;
    if (amdsmi_get_gpu_device_uuid(h, &ulen, uuid) == AMDSMI_STATUS_SUCCESS) in.uuid = uuid;
    amdsmi_asic_info_t ai;
    std::memset(&ai, 0, sizeof ai);
    if (amdsmi_get_gpu_asic_info(h, &ai) == AMDSMI_STATUS_SUCCESS) {
      in.market_name = ai.market_name;
      in.serial = ai.asic_serial;
      in.num_cu = ai.num_of_compute_units == 0xFFFFFFFFu ? 0 : static_cast<int>(ai.num_of_compute_units);
      if (ai.target_graphics_version != ~0ull) {
        char g[32];
        std::snprintf(g, sizeof g, "gfx%llx", static_cast<unsigned long long>(ai.target_graphics_version));
        in.gfx_target = g;
      }
    }
    in.gpu_type = gpu_type_from_market_name(in.market_name);
    amdsmi_kfd_info_t kfd;
    if (amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS) {
      in.kfd_gpu_id = kfd.kfd_id;
      in.kfd_node = kfd.node_id == 0xFFFFFFFFu ? -1 : static_cast<int>(kfd.node_id);
      in.partition_id = kfd.current_partition_id == 0xFFFFFFFFu ? -1 : static_cast<int>(kfd.current_partition_id);
    }
    char part[64] = {};
    if (amdsmi_get_gpu_compute_partition(h, part, sizeof part - 1) == AMDSMI_STATUS_SUCCESS) in.compute_partition = part;
    std::memset(part, 0, sizeof part);
    if (amdsmi_get_gpu_memory_partition(h, part, sizeof part - 1) == AMDSMI_STATUS_SUCCESS) in.memory_partition = part;
    amdsmi_enumeration_info_t en;
    std::memset(&en, 0, sizeof en);
    if (amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
      in.drm_card = static_cast<int>(en.drm_card);
      in.hip_id = static_cast<int>(en.hip_id);
    }
    int32_t numa = -1;
    if (amdsmi_get_gpu_topo_numa_affinity(h, &numa) == AMDSMI_STATUS_SUCCESS) in.numa_node = numa;
    amdsmi_vram_info_t vi;
    std::memset(&vi, 0, sizeof vi);
    if (amdsmi_get_gpu_vram_info(h, &vi) == AMDSMI_STATUS_SUCCESS) in.vram_total_bytes = vi.vram_size * 1048576ull;

    in.sysfs_dir = find_sysfs_dir(sysfs_root, in.drm_card, in.bdf);
    if (!in.sysfs_dir.empty()) {
      open_files(*d);
      std::string tot;
      if (read_small_file(in.sysfs_dir + "/mem_info_vram_total", tot)) in.vram_total_bytes = std::strtoull(tot.c_str(), nullptr, 10);
    }
    // Probe the table once for the XCC count.  A compute partition (DPX/QPX/CPX)
    // is its own device over the physical GPU's table: it owns a contiguous
    // share of the XCCs by partition id (gpu_metrics.h restrict_to_xccs).
    GpuSample s;
    if (d->fd_metrics >= 0) {
      const ssize_t n = pread(d->fd_metrics, d->buf, sizeof d->buf, 0);
      if (n > 0 && parse_gpu_metrics_v1_8(d->buf, static_cast<size_t>(n), s) == 0) in.num_xcc = s.num_xcc;
    }
    const uint32_t parts = partitions_of_mode(in.compute_partition.c_str());
    if (parts > 1 && in.num_xcc >= parts && in.partition_id >= 0 && static_cast<uint32_t>(in.partition_id) < parts) {
      const uint32_t per = in.num_xcc / parts;
      in.xcc_first = per * static_cast<uint32_t>(in.partition_id);
      in.num_xcc = per;
      d->partitioned = true;
    }
    devs_.push_back(std::move(d));
  }

  static std::string find_sysfs_dir(const std::string& root, int card, const std::string& bdf) {
    auto matches = [&](const std::string& dir) {
      char rp[PATH_MAX];
      if (!realpath(dir.c_str(), rp)) return false;
      const std::string r(rp);
      return bdf.empty() || (r.size() >= bdf.size() && r.compare(r.size() - bdf.size(), bdf.size(), bdf) == 0);
    };
    if (card >= 0) {
      const std::string dir = root + "/class/drm/card" + std::to_string(card) + "/device";
      if (matches(dir)) return dir;
    }
    for (int c = 0; c < 256; ++c) {
      const std::string dir = root + "/class/drm/card" + std::to_string(c) + "/device";
      if (access(dir.c_str(), F_OK) == 0 && matches(dir)) return dir;
    }
    return std::string();
  }

  void read_vram(Dev& dv, GpuSample& s) {
    s.vram_total_bytes = dv.info.vram_total_bytes;
    if (dv.fd_vram_used >= 0) {
      char b[32];
      const ssize_t n = pread(dv.fd_vram_used, b, sizeof b - 1, 0);
      if (n > 0) {
        b[n] = 0;
        s.vram_used_bytes = std::strtoull(b, nullptr, 10);
        s.valid |= kFVram;
        return;
      }
    }
    amdsmi_vram_usage_t vu;
    std::lock_guard<std::mutex> g(smi_mu_);
    if (amdsmi_get_gpu_vram_usage(dv.h, &vu) == AMDSMI_STATUS_SUCCESS) {
      s.vram_used_bytes = static_cast<uint64_t>(vu.vram_used) * 1048576ull;
      s.vram_total_bytes = static_cast<uint64_t>(vu.vram_total) * 1048576ull;
      s.valid |= kFVram;
    }
  }

  // Generic path for any other table revision (e.g. a future driver).
  int read_metrics_amdsmi_locked(Dev& dv, GpuSample& s) {
    amdsmi_gpu_metrics_t m;
    std::memset(&m, 0, sizeof m);
    if (amdsmi_get_gpu_metrics_info(dv.h, &m) != AMDSMI_STATUS_SUCCESS) return -1;
    auto ok16 = [](uint16_t v) { return v != 0xFFFF; };
    if (ok16(m.temperature_hotspot)) { s.temp_hotspot_c = m.temperature_hotspot; s.valid |= kFTempHotspot; }
    if (ok16(m.temperature_mem)) { s.temp_mem_c = m.temperature_mem; s.valid |= kFTempMem; }
    if (ok16(m.temperature_vrsoc)) { s.temp_vrsoc_c = m.temperature_vrsoc; s.valid |= kFTempVrSoc; }
    if (ok16(m.current_socket_power)) { s.power_w = m.current_socket_power; s.valid |= kFPower; }
    else if (ok16(m.average_socket_power)) { s.power_w = m.average_socket_power; s.valid |= kFPower; }
    if (ok16(m.average_gfx_activity)) { s.gfx_busy_pct = m.average_gfx_activity; s.valid |= kFGfxBusy; }
    if (ok16(m.average_umc_activity)) { s.umc_busy_pct = m.average_umc_activity; s.valid |= kFUmcBusy; }
    if (m.energy_accumulator != ~0ull) { s.energy_acc = m.energy_accumulator; s.valid |= kFEnergy; }
    if (m.firmware_timestamp != ~0ull) { s.fw_ts = m.firmware_timestamp; s.valid |= kFFwTs; }
    if (m.gfx_activity_acc != 0xFFFFFFFFu && m.accumulation_counter != ~0ull) {
      s.gfx_activity_acc = m.gfx_activity_acc;
      s.mem_activity_acc = m.mem_activity_acc;
      s.accumulation_counter = m.accumulation_counter;
      s.valid |= kFAcc;
    }
    uint32_t nclk = 0;
    for (int x = 0; x < kMaxXcc && x < AMDSMI_MAX_NUM_GFX_CLKS; ++x)
      if (ok16(m.current_gfxclks[x])) s.gfxclk_mhz[nclk++] = m.current_gfxclks[x];
    if (nclk) s.valid |= kFGfxClk;
    if (ok16(m.current_uclk)) { s.uclk_mhz = m.current_uclk; s.valid |= kFUclk; }
    for (int l = 0; l < kMaxXgmi && l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
      s.xgmi_read_kb[l] = m.xgmi_read_data_acc[l] == ~0ull ? 0 : m.xgmi_read_data_acc[l];
      s.xgmi_write_kb[l] = m.xgmi_write_data_acc[l] == ~0ull ? 0 : m.xgmi_write_data_acc[l];
    }
    s.valid |= kFXgmi;
    return 0;
  }

  bool inited_ = false;
  std::string sysfs_root_;
  int64_t last_reinit_ns_ = 0;
  uint64_t reinits_ = 0;
  std::mutex smi_mu_;
  std::vector<std::unique_ptr<Dev>> devs_;
};

}  // namespace

std::unique_ptr<Backend> make_amdsmi_backend(std::string& err, const std::string& sysfs_root) {
  auto b = std::make_unique<AmdSmiBackend>();
  if (!b->init(err, sysfs_root)) return nullptr;
  return b;
}

}  // namespace kgs
