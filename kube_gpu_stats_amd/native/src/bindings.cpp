// pybind11 module `_kgs_native`: the Python control plane's handle on the
// native data plane.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <ctime>

#include "kgs/exporter.h"
#include "kgs/gpu_metrics.h"
#include "kgs/kfd_procs.h"

namespace py = pybind11;
using namespace kgs;

namespace {

int64_t mono_ns_now() {
  timespec ts{};
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

template <class T>
T get(const py::dict& d, const char* k, T dflt) {
  if (d.contains(k) && !d[k].is_none()) return d[k].cast<T>();
  return dflt;
}

ExporterConfig parse_config(const py::dict& d) {
  ExporterConfig c;
  c.backend = get<std::string>(d, "backend", c.backend);
  c.sysfs_root = get<std::string>(d, "sysfs_root", c.sysfs_root);
  if (d.contains("mock")) {
    py::dict m = d["mock"].cast<py::dict>();
    c.mock.n_gpus = get<int>(m, "n_gpus", c.mock.n_gpus);
    c.mock.fw_period_s = get<double>(m, "fw_period_s", c.mock.fw_period_s);
    c.mock.util_base = get<double>(m, "util_base", c.mock.util_base);
    c.mock.util_amp = get<double>(m, "util_amp", c.mock.util_amp);
    c.mock.util_period_s = get<double>(m, "util_period_s", c.mock.util_period_s);
    c.mock.fail_rate = get<double>(m, "fail_rate", c.mock.fail_rate);
    c.mock.stall_s = get<double>(m, "stall_s", c.mock.stall_s);
    c.mock.vanish_dev = get<int>(m, "vanish_dev", c.mock.vanish_dev);
    c.mock.vanish_after_s = get<double>(m, "vanish_after_s", c.mock.vanish_after_s);
    c.mock.vanish_for_s = get<double>(m, "vanish_for_s", c.mock.vanish_for_s);
    c.mock.energy_wrap_at = get<uint64_t>(m, "energy_wrap_at", c.mock.energy_wrap_at);
    c.mock.seed = get<uint64_t>(m, "seed", c.mock.seed);
    c.mock.ecc_correctable_per_s = get<uint64_t>(m, "ecc_correctable_per_s", c.mock.ecc_correctable_per_s);
    c.mock.square_duty = get<double>(m, "square_duty", c.mock.square_duty);
    c.mock.pmfw_busy_floor = get<double>(m, "pmfw_busy_floor", c.mock.pmfw_busy_floor);
    c.mock.ppt_frac = get<double>(m, "ppt_frac", c.mock.ppt_frac);
    c.mock.compute_partition = get<std::string>(m, "compute_partition", c.mock.compute_partition);
    c.mock.proc_latency_s = get<double>(m, "proc_latency_s", c.mock.proc_latency_s);
    c.mock.link_latency_s = get<double>(m, "link_latency_s", c.mock.link_latency_s);
    c.mock.health_latency_s = get<double>(m, "health_latency_s", c.mock.health_latency_s);
    c.mock.metrics_latency_s = get<double>(m, "metrics_latency_s", c.mock.metrics_latency_s);
    c.mock.proc_cu_share = get<std::vector<double>>(m, "proc_cu_share", c.mock.proc_cu_share);
    c.mock.proc_cu_fail = get<int>(m, "proc_cu_fail", c.mock.proc_cu_fail);
    c.mock.xgmi_bg = get<bool>(m, "xgmi_bg", c.mock.xgmi_bg);
    c.mock.xgmi_swap_dev = get<int>(m, "xgmi_swap_dev", c.mock.xgmi_swap_dev);
    c.mock.slow_fault_dev = get<int>(m, "slow_fault_dev", c.mock.slow_fault_dev);
    c.mock.slow_fault_tier = get<std::string>(m, "slow_fault_tier", c.mock.slow_fault_tier);
    c.mock.slow_fault_kind = get<std::string>(m, "slow_fault_kind", c.mock.slow_fault_kind);
    c.mock.slow_fault_after_s = get<double>(m, "slow_fault_after_s", c.mock.slow_fault_after_s);
    c.mock.slow_hang_s = get<double>(m, "slow_hang_s", c.mock.slow_hang_s);
  }
  if (d.contains("mock_pmc")) {
    py::dict m = d["mock_pmc"].cast<py::dict>();
    c.mock_pmc.clock_mhz = get<double>(m, "clock_mhz", c.mock_pmc.clock_mhz);
    c.mock_pmc.mfma_frac = get<double>(m, "mfma_frac", c.mock_pmc.mfma_frac);
    c.mock_pmc.vmem_frac = get<double>(m, "vmem_frac", c.mock_pmc.vmem_frac);
    c.mock_pmc.n_xcd = get<int>(m, "n_xcd", c.mock_pmc.n_xcd);
    c.mock_pmc.xcd_skew = get<double>(m, "xcd_skew", c.mock_pmc.xcd_skew);
    c.mock_pmc.freeze_after_s = get<double>(m, "freeze_after_s", c.mock_pmc.freeze_after_s);
    c.mock_pmc.slow_dev = get<int>(m, "slow_dev", c.mock_pmc.slow_dev);
    c.mock_pmc.slow_s = get<double>(m, "slow_s", c.mock_pmc.slow_s);
    c.mock_pmc.hang_dev = get<int>(m, "hang_dev", c.mock_pmc.hang_dev);
    c.mock_pmc.hang_after = get<uint64_t>(m, "hang_after", c.mock_pmc.hang_after);
    c.mock_pmc.hang_timeout_s = get<double>(m, "hang_timeout_s", c.mock_pmc.hang_timeout_s);
    c.mock_pmc.hang_heals_on_reset = get<bool>(m, "hang_heals_on_reset", c.mock_pmc.hang_heals_on_reset);
    c.mock_pmc.acquire_fail_dev = get<int>(m, "acquire_fail_dev", c.mock_pmc.acquire_fail_dev);
    c.mock_pmc.batch = get<int>(m, "batch", c.mock_pmc.batch);
    c.mock_pmc.cpc_read_us = get<double>(m, "cpc_read_us", c.mock_pmc.cpc_read_us);
    c.mock_pmc.wave_frac = get<double>(m, "wave_frac", c.mock_pmc.wave_frac);
    c.mock_pmc.lite_every = get<int>(m, "lite_every", c.mock_pmc.lite_every);
  }
  c.sampler.hz = get<double>(d, "hz", c.sampler.hz);
  c.sampler.pmfw_hz = get<double>(d, "pmfw_hz", c.sampler.pmfw_hz);
  c.sampler.proc_every = get<int>(d, "proc_every", c.sampler.proc_every);
  c.sampler.link_every = get<int>(d, "link_every", c.sampler.link_every);
  c.sampler.proc_period_s = get<double>(d, "proc_period_s", c.sampler.proc_period_s);
  c.sampler.link_period_s = get<double>(d, "link_period_s", c.sampler.link_period_s);
  c.sampler.pin_numa = get<bool>(d, "pin_numa", c.sampler.pin_numa);
  c.sampler.max_backoff_ms = get<int>(d, "max_backoff_ms", c.sampler.max_backoff_ms);
  c.sampler.pmc_reclaim_s = get<double>(d, "pmc_reclaim_s", c.sampler.pmc_reclaim_s);
  c.sampler.pmc_refresh_s = get<double>(d, "pmc_refresh_s", c.sampler.pmc_refresh_s);
  c.sampler.pmc_idle_hz = get<double>(d, "pmc_idle_hz", c.sampler.pmc_idle_hz);
  c.sampler.pmc_dispatch_hz = get<double>(d, "pmc_dispatch_hz", c.sampler.pmc_dispatch_hz);
  c.sampler.pmc_quiet_release_s = get<double>(d, "pmc_quiet_release_s", c.sampler.pmc_quiet_release_s);
  c.sampler.pmc_cp_only_min = get<double>(d, "pmc_cp_only_min", c.sampler.pmc_cp_only_min);
  c.sampler.pmc_dispatch_hold_s = get<double>(d, "pmc_dispatch_hold_s", c.sampler.pmc_dispatch_hold_s);
  c.sampler.devices = get<std::vector<int>>(d, "devices", c.sampler.devices);
  c.sampler.pmc_breaker_k = get<int>(d, "pmc_breaker_k", c.sampler.pmc_breaker_k);
  c.sampler.pmc_retry_s = get<double>(d, "pmc_retry_s", c.sampler.pmc_retry_s);
  c.sampler.pmc_retry_max_s = get<double>(d, "pmc_retry_max_s", c.sampler.pmc_retry_max_s);
  c.sampler.stop_timeout_s = get<double>(d, "stop_timeout_s", c.sampler.stop_timeout_s);
  c.sampler.tick_dither = get<double>(d, "tick_dither", c.sampler.tick_dither);
  c.bdfs = get<std::vector<std::string>>(d, "bdfs", c.bdfs);
  c.pmc_source = get<std::string>(d, "pmc_source", c.pmc_source);
  c.pmc_lib = get<std::string>(d, "pmc_lib", c.pmc_lib);
  c.pmc_pipeline = get<bool>(d, "pmc_pipeline", c.pmc_pipeline);
  c.pmc_set = get<std::string>(d, "pmc_set", c.pmc_set);
  c.pmc_lean = get<int>(d, "pmc_lean", c.pmc_lean);
  c.pmc_timeout_ms = get<int>(d, "pmc_timeout_ms", c.pmc_timeout_ms);
  c.pmc_batch = get<int>(d, "pmc_batch", c.pmc_batch);
  c.pmc_publish_us = get<int>(d, "pmc_publish_us", c.pmc_publish_us);
  c.pmc_lite = get<bool>(d, "pmc_lite", c.pmc_lite);
  c.hbm_bytes_per_s_at_full_umc = get<double>(d, "hbm_bytes_per_s_at_full_umc", c.hbm_bytes_per_s_at_full_umc);
  c.listen_addr = get<std::string>(d, "listen_addr", c.listen_addr);
  c.port = get<int>(d, "port", c.port);
  c.node_name = get<std::string>(d, "node_name", c.node_name);
  c.gpu_type_override = get<std::string>(d, "gpu_type_override", c.gpu_type_override);
  c.window_s = get<double>(d, "window_s", c.window_s);
  c.stale_s = get<double>(d, "stale_s", c.stale_s);
  c.per_process = get<bool>(d, "per_process", c.per_process);
  c.compat_series = get<bool>(d, "compat_series", c.compat_series);
  c.compat_unallocated = get<bool>(d, "compat_unallocated", c.compat_unallocated);
  c.sm_util_source = get<std::string>(d, "sm_util_source", c.sm_util_source);
  c.pcie_bytes_per_acc_unit = get<double>(d, "pcie_bytes_per_acc_unit", c.pcie_bytes_per_acc_unit);
  c.xgmi_bytes_per_acc_unit = get<double>(d, "xgmi_bytes_per_acc_unit", c.xgmi_bytes_per_acc_unit);
  c.control_http = get<bool>(d, "control_http", c.control_http);
  c.gzip_level = get<int>(d, "gzip_level", c.gzip_level);
  c.http_idle_s = get<double>(d, "http_idle_s", c.http_idle_s);
  c.http_max_conns = get<int>(d, "http_max_conns", c.http_max_conns);
  c.metric_allow = get<std::string>(d, "metric_allow", c.metric_allow);
  c.metric_deny = get<std::string>(d, "metric_deny", c.metric_deny);
  return c;
}

py::dict sample_dict(const GpuSample& s) {
  py::dict o;
  o["seq"] = s.seq;
  o["mono_ns"] = s.mono_ns;
  o["wall_ns"] = s.wall_ns;
  o["fw_ts"] = s.fw_ts;
  o["valid"] = s.valid;
  o["read_ns"] = s.read_ns;
  o["num_xcc"] = s.num_xcc;
  o["gfx_busy_pct"] = s.gfx_busy_pct;
  o["umc_busy_pct"] = s.umc_busy_pct;
  o["gfx_busy_xcc"] = std::vector<float>(s.gfx_busy_xcc, s.gfx_busy_xcc + s.num_xcc);
  o["gfx_busy_window_pct"] = s.gfx_busy_window_pct;
  o["gfx_busy_xcc_window"] = std::vector<float>(s.gfx_busy_xcc_window, s.gfx_busy_xcc_window + s.num_xcc);
  o["gfx_busy_acc_xcc"] = std::vector<uint64_t>(s.gfx_busy_acc_xcc, s.gfx_busy_acc_xcc + s.num_xcc);
  o["umc_busy_window_pct"] = s.umc_busy_window_pct;
  o["dt_s"] = s.dt_s;
  o["temp_hotspot_c"] = s.temp_hotspot_c;
  o["temp_mem_c"] = s.temp_mem_c;
  o["temp_vrsoc_c"] = s.temp_vrsoc_c;
  o["power_w"] = s.power_w;
  o["gfxclk_mhz"] = std::vector<uint32_t>(s.gfxclk_mhz, s.gfxclk_mhz + kMaxXcc);
  o["uclk_mhz"] = s.uclk_mhz;
  o["socclk_mhz"] = s.socclk_mhz;
  o["energy_acc"] = s.energy_acc;
  o["gfx_activity_acc"] = s.gfx_activity_acc;
  o["mem_activity_acc"] = s.mem_activity_acc;
  o["accumulation_counter"] = s.accumulation_counter;
  o["ppt_residency_acc"] = s.ppt_residency_acc;
  o["xgmi_read_kb"] = std::vector<uint64_t>(s.xgmi_read_kb, s.xgmi_read_kb + kMaxXgmi);
  o["xgmi_write_kb"] = std::vector<uint64_t>(s.xgmi_write_kb, s.xgmi_write_kb + kMaxXgmi);
  o["xgmi_link_up"] = std::vector<uint16_t>(s.xgmi_link_up, s.xgmi_link_up + kMaxXgmi);
  o["xgmi_link_speed_gbps"] = s.xgmi_link_speed_gbps;
  o["xgmi_link_width"] = s.xgmi_link_width;
  o["pcie_bw_acc_gb"] = s.pcie_bw_acc_gb;
  o["pcie_link_width"] = s.pcie_link_width;
  o["pcie_link_speed_01gts"] = s.pcie_link_speed_01gts;
  o["vram_used_bytes"] = s.vram_used_bytes;
  o["vram_total_bytes"] = s.vram_total_bytes;
  return o;
}

py::dict info_dict(const DeviceInfo& in) {
  py::dict o;
  o["index"] = in.index;
  o["bdf"] = in.bdf;
  o["uuid"] = in.uuid;
  o["serial"] = in.serial;
  o["market_name"] = in.market_name;
  o["gpu_type"] = in.gpu_type;
  o["gfx_target"] = in.gfx_target;
  o["numa_node"] = in.numa_node;
  o["num_cu"] = in.num_cu;
  o["num_xcc"] = in.num_xcc;
  o["vram_total_bytes"] = in.vram_total_bytes;
  o["kfd_gpu_id"] = in.kfd_gpu_id;
  o["kfd_node"] = in.kfd_node;
  o["drm_card"] = in.drm_card;
  o["hip_id"] = in.hip_id;
  o["compute_partition"] = in.compute_partition;
  o["memory_partition"] = in.memory_partition;
  o["partition_id"] = in.partition_id;
  o["xcc_first"] = in.xcc_first;
  o["sysfs_dir"] = in.sysfs_dir;
  return o;
}

class PyExporter {
 public:
  explicit PyExporter(const py::dict& cfg) : ex_(parse_config(cfg)) {
    if (!ex_.init()) throw std::runtime_error("exporter init failed: " + ex_.error());
  }
  void start() {
    py::gil_scoped_release r;
    ex_.start();
  }
  Sampler* sampler() const { return ex_.sampler(); }
  void stop() {
    py::gil_scoped_release r;
    ex_.stop();
  }
  std::string render() {
    std::string out;
    {
      py::gil_scoped_release r;
      ex_.render(out);
    }
    return out;
  }
  int port() const { return ex_.port(); }
  int device_count() const { return ex_.backend()->device_count(); }
  std::string backend_name() const { return ex_.backend()->name(); }
  std::string pmc_name() const { return ex_.counters() ? ex_.counters()->name() : std::string("none"); }
  std::string pmc_error() const { return ex_.pmc_error(); }
  std::string error() const { return ex_.error(); }
  py::list devices() const {
    py::list l;
    for (int d = 0; d < device_count(); ++d) l.append(info_dict(ex_.backend()->info(d)));
    return l;
  }
  py::object snapshot(int d) const {
    check(d);
    GpuSample s;
    if (!ex_.sampler()->state(d).latest.load(s)) return py::none();
    return sample_dict(s);
  }
  py::list samples(int d, int n) const {
    check(d);
    if (n < 1) n = 1;
    if (n > static_cast<int>(kRing) - 1) n = static_cast<int>(kRing) - 1;
    std::vector<GpuSample> buf(static_cast<size_t>(n));
    const size_t got = ex_.sampler()->state(d).ring.recent(buf.data(), static_cast<size_t>(n));
    py::list l;
    for (size_t i = got; i-- > 0;) l.append(sample_dict(buf[i]));
    return l;
  }
  py::dict integrals(int d) const {
    check(d);
    const Integrals I = ex_.sampler()->state(d).integrals();
    py::dict o;
    o["gfx_busy_seconds"] = I.gfx_busy_seconds;
    o["umc_busy_seconds"] = I.umc_busy_seconds;
    o["energy_joules"] = I.energy_joules;
    o["sampled_seconds"] = I.sampled_seconds;
    o["distinct_samples"] = I.distinct_samples;
    o["reads"] = I.reads;
    o["read_errors"] = I.read_errors;
    o["overruns"] = I.overruns;
    o["recoveries"] = I.recoveries;
    o["recover_attempts"] = I.recover_attempts;
    o["pmc_samples"] = I.pmc_samples;
    o["pmc_errors"] = I.pmc_errors;
    o["read_seconds"] = I.read_seconds;
    o["pmc_read_seconds"] = I.pmc_read_seconds;
    o["mfma_busy_seconds"] = I.mfma_busy_seconds;
    o["active_seconds"] = I.active_seconds;
    o["util_seconds"] = I.util_seconds;
    o["dispatch_seconds"] = I.dispatch_seconds;
    o["dispatch_drains"] = I.dispatch_drains;
    o["cpc_read_us"] = I.cpc_read_us;
    o["pmc_clk_idle_hz"] = I.pmc_clk_idle_hz;
    o["pmc_clk_busy_hz"] = I.pmc_clk_busy_hz;
    o["util_counter_seconds"] = I.util_counter_seconds;
    o["util_carry_seconds"] = I.util_carry_seconds;
    o["util_dropped_seconds"] = I.util_dropped_seconds;
    o["pmc_epoch"] = I.pmc_epoch;
    o["pmc_last_ns"] = I.pmc_last_ns;
    {
      py::dict t;
      for (int r = 0; r < kThrottleReasons; ++r) t[throttle_reason_name(r)] = I.throttle_seconds[r];
      o["throttle_seconds"] = t;
    }
    const DeviceState& st = ex_.sampler()->state(d);
    o["proc_reads"] = st.proc_reads.load();
    o["link_reads"] = st.link_reads.load();
    o["slow_read_seconds"] = st.slow_ns_total.load() * 1e-9;
    o["pmc_quiet"] = st.pmc_quiet.load();
    o["pmc_quiet_skips"] = st.pmc_quiet_skips.load();
    o["pmc_dispatch_skips"] = st.pmc_dbound_skips.load();
    o["pmc_parked"] = st.pmc_parked.load();
    o["pmc_parks"] = st.pmc_parks.load();
    {
      DeviceState::ParkTime pt;
      st.park_time.load(pt);
      const int64_t cur = pt.since_ns > 0 ? std::max<int64_t>(0, mono_ns_now() - pt.since_ns) : 0;
      o["pmc_parked_s"] = (pt.ended_ns + cur) * 1e-9;
    }
    {
      const int64_t lag = st.pmc_unpark_lag_ns.load();
      o["pmc_unpark_lag_s"] = lag >= 0 ? py::cast(lag * 1e-9) : py::none();
    }
    o["pmc_dispatch_bound"] = st.pmc_dbound.load();
    o["up"] = ex_.sampler()->state(d).up.load();
    o["cpu_pinned"] = ex_.sampler()->state(d).cpu_pinned.load();
    o["pmc_on"] = st.pmc_on.load();
    o["pmc_failed"] = st.pmc_failed.load();
    o["pmc_breaker_trips"] = st.pmc_breaker_trips.load();
    o["pmc_retries"] = st.pmc_retries.load();
    o["pmc_releases"] = st.pmc_releases.load();
    o["thread_hung"] = st.thread_hung.load();
    o["slow_hung"] = st.slow_hung.load();
    o["proc_errors"] = st.proc_errors.load();
    o["pmc_reordered"] = st.pmc_reordered.load();
    o["pmc_stalls_injected"] = st.pmc_stalls_injected.load();
    o["pmc_resets"] = ex_.counters() ? ex_.counters()->resets(d) : 0;
    return o;
  }
  py::object pmc(int d) const {
    check(d);
    PmcSample p;
    if (!ex_.sampler()->state(d).pmc_latest.load(p)) return py::none();
    py::dict o;
    o["seq"] = p.seq;
    o["mono_ns"] = p.mono_ns;
    o["read_ns"] = p.read_ns;
    py::dict v;
    for (int i = 0; i < kPmcCount; ++i)
      if (p.mask & (1u << i)) v[pmc_counter_name(i)] = p.value[i];
    o["values"] = v;
    if (p.n_xcd > 0) {
      o["xcd_active"] = std::vector<uint64_t>(p.xcd_active, p.xcd_active + p.n_xcd);
      o["xcd_mfma"] = std::vector<uint64_t>(p.xcd_mfma, p.xcd_mfma + p.n_xcd);
    }
    return o;
  }
  py::dict window(int d, double window_s) const {
    check(d);
    py::dict o;
    double g = 0, u = 0, util = 0;
    int n = 0;
    if (ex_.sampler()->window_busy(d, window_s, g, u, n, &util)) {
      o["gfx_busy_pct"] = g;
      o["umc_busy_pct"] = u;
      o["util_pct"] = util;
      o["n"] = n;
    }
    PmcRates r;
    if (ex_.sampler()->window_pmc(d, window_s, r)) {
      o["gpu_active_pct"] = r.gpu_active_pct;
      o["mfma_util_pct"] = r.mfma_util_pct;
      if (r.have_vmem) o["vmem_busy_pct"] = r.vmem_busy_pct;
      o["gpu_clock_mhz"] = r.gpu_clock_mhz;
      o["pmc_dt_s"] = r.dt_s;
      if (r.n_xcd > 0) {
        o["xcd_mfma_util_pct"] = std::vector<double>(r.xcd_mfma_util_pct, r.xcd_mfma_util_pct + r.n_xcd);
        o["xcd_active_pct"] = std::vector<double>(r.xcd_active_pct, r.xcd_active_pct + r.n_xcd);
        if (r.have_xcd_vmem)
          o["xcd_vmem_busy_pct"] = std::vector<double>(r.xcd_vmem_busy_pct, r.xcd_vmem_busy_pct + r.n_xcd);
      }
    }
    return o;
  }
  py::list procs(int d) const {
    check(d);
    py::list l;
    auto p = ex_.sampler()->state(d).get_procs();
    if (!p) return l;
    for (const ProcInfo& x : *p) {
      py::dict o;
      o["pid"] = x.pid;
      o["name"] = x.name;
      o["vram_bytes"] = x.vram_bytes;
      o["gtt_bytes"] = x.gtt_bytes;
      o["cpu_bytes"] = x.cpu_bytes;
      o["gfx_ns"] = x.gfx_ns;
      o["cu_occupancy"] = x.cu_occupancy;
      o["cu_valid"] = x.cu_valid;
      o["cu_seconds"] = x.cu_seconds;
      o["evicted_ms"] = x.evicted_ms;
      l.append(o);
    }
    return l;
  }
  py::list links(int d) const {
    check(d);
    py::list l;
    auto p = ex_.sampler()->state(d).get_links();
    if (!p) return l;
    for (const LinkInfo& x : *p) {
      py::dict o;
      o["link"] = x.link;
      o["peer_bdf"] = x.peer_bdf;
      o["link_type"] = x.link_type;
      o["bit_rate_gbps"] = x.bit_rate_gbps;
      o["max_bw_gbps"] = x.max_bw_gbps;
      o["read_kb"] = x.read_kb;
      o["write_kb"] = x.write_kb;
      l.append(o);
    }
    return l;
  }
  std::string topology_json() { return ex_.topology_json(); }
  std::string pmc_info(int d) const {
    check(d);
    return ex_.counters() ? ex_.counters()->info(d) : std::string("none");
  }
  void set_device_owners(int d, const py::list& owners) {
    check(d);
    std::vector<Owner> v;
    for (auto h : owners) {
      py::dict o = h.cast<py::dict>();
      v.push_back(Owner{get<std::string>(o, "pod", ""), get<std::string>(o, "namespace", ""),
                        get<std::string>(o, "container", "")});
    }
    ex_.set_device_owners(d, std::move(v));
  }
  // {(gpu, pid): {pod, namespace, container, pod_uid}}
  void set_pid_owners(const py::dict& m) {
    std::unordered_map<uint64_t, PidOwner> mm;
    for (auto kvp : m) {
      auto key = kvp.first.cast<std::pair<int, uint32_t>>();
      py::dict o = kvp.second.cast<py::dict>();
      mm[Exporter::pid_key(key.first, key.second)] =
          PidOwner{get<std::string>(o, "pod", ""), get<std::string>(o, "namespace", ""),
                   get<std::string>(o, "container", ""), get<std::string>(o, "pod_uid", "")};
    }
    ex_.set_pid_owners(std::move(mm));
  }
  void set_node_name(const std::string& n) { ex_.set_node_name(n); }
  void set_extra_metrics(const std::string& t) { ex_.set_extra_metrics(t); }
  py::dict stats() const {
    py::dict o;
    o["scrapes"] = ex_.scrapes.load();
    o["render_ns_total"] = ex_.render_ns_total.load();
    o["render_ns_last"] = ex_.render_ns_last.load();
    o["http_requests"] = ex_.http_requests.load();
    o["http_conns_open"] = ex_.http_conns_open.load();
    o["http_closed_idle"] = ex_.http_closed_idle.load();
    o["http_closed_limit"] = ex_.http_closed_limit.load();
    return o;
  }
  bool healthy() const { return ex_.healthy(); }
  void pause() {
    py::gil_scoped_release r;
    ex_.pause_sampling();
  }
  void resume() {
    py::gil_scoped_release r;
    ex_.resume_sampling();
  }
  void set_pmc_enabled(bool on, int gpu, bool drop_queue) {
    if (gpu >= 0) check(gpu);
    ex_.set_pmc_enabled(on, gpu, drop_queue);
  }
  void set_sample_rate(double hz) {
    bool ok;
    {
      py::gil_scoped_release r;
      ok = ex_.set_sample_rate(hz);
    }
    if (!ok) throw py::value_error("hz must be within (0, 100000]");
  }
  uint64_t abandoned_threads() const { return ex_.sampler()->abandoned_threads(); }
  int inject_xgmi(int src, int dst, uint64_t bytes) { return ex_.backend()->inject_xgmi(src, dst, bytes); }
  bool inject_pmc_stall(int d) {
    check(d);
    return ex_.sampler()->inject_pmc_stall(d);
  }
  double sample_rate() const { return ex_.sample_rate(); }
  uint64_t slow_passes() const { return ex_.sampler()->slow_passes(); }
  bool pmc_enabled() const { return ex_.pmc_enabled(); }
  bool sampling() const { return ex_.sampling(); }

 private:
  void check(int d) const {
    if (d < 0 || d >= device_count()) throw py::index_error("gpu index out of range");
  }
  Exporter ex_;
};

EstimatorParams sampler_estimator_params(int num_cu) { return estimator_params(SamplerConfig{}, num_cu); }

py::dict parse_metrics_blob(const py::bytes& b) {
  std::string s = b;
  GpuSample g;
  if (parse_gpu_metrics_v1_8(reinterpret_cast<const uint8_t*>(s.data()), s.size(), g) != 0)
    throw std::runtime_error("not a gpu_metrics v1.8 table");
  return sample_dict(g);
}

}  // namespace

PYBIND11_MODULE(_kgs_native, m) {
  m.doc() = "kube_gpu_stats_amd native data plane (C++17: sampler threads, seqlocks, renderer, HTTP)";
  py::class_<PyExporter>(m, "Exporter")
      .def(py::init<const py::dict&>())
      .def("start", &PyExporter::start)
      .def("stop", &PyExporter::stop)
      .def("render", &PyExporter::render)
      .def_property_readonly("port", &PyExporter::port)
      .def_property_readonly("device_count", &PyExporter::device_count)
      .def_property_readonly("backend_name", &PyExporter::backend_name)
      .def_property_readonly("pmc_name", &PyExporter::pmc_name)
      .def_property_readonly("pmc_error", &PyExporter::pmc_error)
      .def_property_readonly("error", &PyExporter::error)
      .def("devices", &PyExporter::devices)
      .def("snapshot", &PyExporter::snapshot)
      .def("samples", &PyExporter::samples, py::arg("gpu"), py::arg("n") = 100)
      .def("integrals", &PyExporter::integrals)
      .def("pmc", &PyExporter::pmc)
      .def("window", &PyExporter::window, py::arg("gpu"), py::arg("window_s") = 1.0)
      .def("procs", &PyExporter::procs)
      .def("links", &PyExporter::links)
      .def("topology_json", &PyExporter::topology_json)
      .def("pmc_info", &PyExporter::pmc_info)
      .def("set_device_owners", &PyExporter::set_device_owners)
      .def("set_pid_owners", &PyExporter::set_pid_owners)
      .def("set_node_name", &PyExporter::set_node_name)
      .def("set_extra_metrics", &PyExporter::set_extra_metrics)
      .def("stats", &PyExporter::stats)
      .def("healthy", &PyExporter::healthy)
      .def("pause", &PyExporter::pause)
      .def("resume", &PyExporter::resume)
      .def_property_readonly("sampling", &PyExporter::sampling)
      .def("set_pmc_enabled", &PyExporter::set_pmc_enabled, py::arg("on"), py::arg("gpu") = -1,
           py::arg("drop_queue") = false,
           "Hand the hardware counters to another profiler (False) or take them back (True); gpu=-1: every GPU; "
           "drop_queue (with False): also destroy the counter reader's READ queue")
      .def_property_readonly("abandoned_threads", &PyExporter::abandoned_threads,
                             "sampler threads stop() gave up on (stuck in a device call)")
      .def("inject_xgmi", &PyExporter::inject_xgmi, py::arg("src"), py::arg("dst"), py::arg("bytes"),
           "mock backend only: account a peer copy of `bytes` from GPU src to GPU dst on the link between them")
      .def("inject_pmc_stall", &PyExporter::inject_pmc_stall, py::arg("gpu"),
           "test hook: the GPU's counter thread wedges its reader's READ queue (a never-completing packet at its "
           "head) on its next tick; the circuit breaker must recover by recreating the queue")
      .def_property_readonly("pmc_enabled", &PyExporter::pmc_enabled)
      .def("set_sample_rate", &PyExporter::set_sample_rate, py::arg("hz"),
           "Change the sampler tick rate in place (threads restart; integrals continue)")
      .def_property_readonly("sample_rate", &PyExporter::sample_rate)
      .def_property(
          "pmc_idle_hz", [](const PyExporter& e) { return e.sampler() ? e.sampler()->pmc_idle_hz() : 0.0; },
          [](PyExporter& e, double hz) {
            if (e.sampler() && !e.sampler()->set_pmc_idle_hz(hz))
              throw py::value_error("pmc_idle_hz must be 0 or within [0.01, 100000]");
          },
          "Counter READ rate while the GPU has no wave (adaptive; 0 = every tick)")
      .def_property(
          "pmc_dispatch_hz", [](const PyExporter& e) { return e.sampler() ? e.sampler()->pmc_dispatch_hz() : 0.0; },
          [](PyExporter& e, double hz) {
            if (e.sampler() && !e.sampler()->set_pmc_dispatch_hz(hz))
              throw py::value_error("pmc_dispatch_hz must be within (0, 100000]");
          },
          "Counter READ rate while the CP dispatches with no wave in flight (--pmc-cp-only-min)")
      .def_property(
          "pmc_quiet_release_s",
          [](const PyExporter& e) { return e.sampler() ? e.sampler()->pmc_quiet_release_s() : 0.0; },
          [](PyExporter& e, double v) {
            if (e.sampler() && !e.sampler()->set_pmc_quiet_release_s(v))
              throw py::value_error("pmc_quiet_release_s must be within [0, 86400]");
          },
          "Seconds of quiet before the counter session is released (parked); 0 = never")
      .def_property_readonly("slow_passes", &PyExporter::slow_passes);
  // The utilisation estimators as pure units (util_estimator.h): the offline replay of
  // raw READ dumps runs the sampler's own code.
  py::class_<EstimatorParams>(m, "EstimatorParams")
      .def(py::init<>())
      .def_readwrite("quiet_active_frac", &EstimatorParams::quiet_active_frac)
      .def_readwrite("cpc_full_frac", &EstimatorParams::cpc_full_frac)
      .def_readwrite("clock_split_ns", &EstimatorParams::clock_split_ns)
      .def_readwrite("clock_ratio_lo", &EstimatorParams::clock_ratio_lo)
      .def_readwrite("clock_ratio_hi", &EstimatorParams::clock_ratio_hi)
      .def_readwrite("read_overlap_ns", &EstimatorParams::read_overlap_ns)
      .def_readwrite("time_split_ns", &EstimatorParams::time_split_ns)
      .def_readwrite("time_split_ratio_hi", &EstimatorParams::time_split_ratio_hi)
      .def_readwrite("time_split_weight", &EstimatorParams::time_split_weight)
      .def_readwrite("gap_clock_fresh_ns", &EstimatorParams::gap_clock_fresh_ns)
      .def_readwrite("read_only_bills_zero", &EstimatorParams::read_only_bills_zero)
      .def_readwrite("ewma", &EstimatorParams::ewma)
      .def_readwrite("quiet_hold_ns", &EstimatorParams::quiet_hold_ns)
      .def_readwrite("cp_only_min", &EstimatorParams::cp_only_min)
      .def_readwrite("dbound_hold_ns", &EstimatorParams::dbound_hold_ns)
      .def_readwrite("num_simds", &EstimatorParams::num_simds);
  m.def("sampler_estimator_params", &sampler_estimator_params, py::arg("num_cu") = 256,
        "The EstimatorParams the sampler runs with under the default SamplerConfig");
  py::class_<DrainStep>(m, "DrainStep")
      .def_readonly("interval", &DrainStep::interval)
      .def_readonly("span_s", &DrainStep::span_s)
      .def_readonly("active_s", &DrainStep::active_s)
      .def_readonly("mfma_s", &DrainStep::mfma_s)
      .def_readonly("have_dispatch", &DrainStep::have_dispatch)
      .def_readonly("dispatch_s", &DrainStep::dispatch_s)
      .def_readonly("cp_only_share", &DrainStep::cp_only_share)
      .def_readonly("learned", &DrainStep::learned)
      .def_readonly("quiet_interval", &DrainStep::quiet_interval)
      .def_readonly("dbound_interval", &DrainStep::dbound_interval)
      .def_readonly("quiet", &DrainStep::quiet)
      .def_readonly("dbound", &DrainStep::dbound);
  py::class_<DispatchEstimator>(m, "DispatchEstimator")
      .def(py::init<>())
      .def("restart", &DispatchEstimator::restart, py::arg("mono_ns"))
      .def("invalidate", &DispatchEstimator::invalidate, py::arg("mono_ns"))
      .def(
          "feed",
          [](DispatchEstimator& e, const EstimatorParams& p, int64_t mono_ns, uint64_t count, uint64_t spi,
             uint64_t cpc, py::object mfma, bool se_fresh, bool fresh_mode) {
            Drain d;
            d.mono_ns = mono_ns;
            d.count = count;
            d.spi = spi;
            d.cpc = cpc;
            d.mask = (1u << kPmcGrbmCount) | (1u << kPmcGrbmActive) | (1u << kPmcCpcBusy);
            if (!mfma.is_none()) {
              d.mfma = mfma.cast<uint64_t>();
              d.mask |= 1u << kPmcMfmaBusy;
            }
            d.se_fresh = se_fresh;
            d.fresh_mode = fresh_mode;
            return e.feed(d, p);
          },
          py::arg("params"), py::arg("mono_ns"), py::arg("count"), py::arg("spi"), py::arg("cpc"),
          py::arg("mfma") = py::none(), py::arg("se_fresh") = true, py::arg("fresh_mode") = false,
          "Fold one drain (cumulative counts since START); mfma=None: MFMA busy not in the set")
      .def(
          "replay",
          [](DispatchEstimator& e, const EstimatorParams& p, const std::vector<std::vector<double>>& rows) {
            // rows: [t_s, count, spi, cpc] (+ mfma, -1 = not read; + se_fresh): the integrals over the run.
            py::dict o;
            double disp = 0, act = 0, mfma = 0, span = 0;
            uint64_t learned = 0, quiet = 0, dbound = 0;
            for (const auto& r : rows) {
              if (r.size() < 4) throw py::value_error("each row needs t_s, count, spi, cpc");
              Drain d;
              d.mono_ns = static_cast<int64_t>(std::llround(r[0] * 1e9));
              d.count = static_cast<uint64_t>(r[1]);
              d.spi = static_cast<uint64_t>(r[2]);
              d.cpc = static_cast<uint64_t>(r[3]);
              d.mask = (1u << kPmcGrbmCount) | (1u << kPmcGrbmActive) | (1u << kPmcCpcBusy);
              if (r.size() > 4 && r[4] >= 0) {
                d.mfma = static_cast<uint64_t>(r[4]);
                d.mask |= 1u << kPmcMfmaBusy;
              }
              if (r.size() > 5) d.se_fresh = r[5] != 0;
              const DrainStep s = e.feed(d, p);
              disp += s.dispatch_s;
              act += s.active_s;
              mfma += s.mfma_s;
              span += s.span_s;
              learned += s.learned;
              quiet += s.quiet;
              dbound += s.dbound;
            }
            o["dispatch_s"] = disp;
            o["active_s"] = act;
            o["mfma_s"] = mfma;
            o["span_s"] = span;
            o["learned"] = learned;
            o["quiet_drains"] = quiet;
            o["dbound_drains"] = dbound;
            return o;
          },
          py::arg("params"), py::arg("rows"),
          "Fold a whole dump of drains (pipelined): rows [t_s, count, spi, cpc, mfma (-1: none), se_fresh]")
      .def_property_readonly("cpc_read_us", &DispatchEstimator::cpc_read_us)
      .def("read_cycles", &DispatchEstimator::read_cycles, py::arg("fresh_mode") = false, py::arg("full") = true)
      .def("read_spi_cycles", &DispatchEstimator::read_spi_cycles, py::arg("fresh_mode") = false,
           py::arg("full") = true)
      .def_property_readonly("clk_busy_hz", &DispatchEstimator::clk_busy_hz)
      .def_property_readonly("clk_idle_hz", &DispatchEstimator::clk_idle_hz)
      .def_property_readonly("last_plausible_ns", &DispatchEstimator::last_plausible_ns);
  py::class_<UtilBiller>(m, "UtilBiller")
      .def(py::init<>())
      .def(
          "bill",
          [](UtilBiller& b, double dt_s, double dgfx_s, bool ok, uint64_t epoch, double busy_s, double max_carry_s,
             bool dispatch, double share, double since_s, uint64_t drains) {
            CounterCover c;
            c.ok = ok;
            c.epoch = epoch;
            c.dispatch = dispatch;
            c.busy_s = busy_s;
            c.share = share;
            c.since_s = since_s;
            c.drains = drains;
            const UtilBiller::Bill r = b.bill(dt_s, dgfx_s, c, max_carry_s);
            return py::make_tuple(r.billed_s, r.from_counters);
          },
          py::arg("dt_s"), py::arg("dgfx_s"), py::arg("ok"), py::arg("epoch"), py::arg("busy_s"),
          py::arg("max_carry_s") = 1.0, py::arg("dispatch") = true, py::arg("share") = 0.0,
          py::arg("since_s") = 0.0, py::arg("drains") = 0,
          "Bill one PMFW interval: (seconds billed, billed from the counters?).  drains: the count of "
          "drains folded so far (a new drain restarts the run-on guess)")
      .def_property_readonly("carry_s", &UtilBiller::carry_s)
      .def_property_readonly("dropped_s", &UtilBiller::dropped_s)
      .def("drop_carry", &UtilBiller::drop_carry, "The GPU changed hands: drop the busy still carried");
  m.attr("MAX_UTIL_CARRY_S") = kMaxUtilCarryS;
  m.def("parse_gpu_metrics_v1_8", &parse_metrics_blob, "Parse a raw PMFW gpu_metrics v1.8 table");
  py::class_<DrmFdCache>(m, "DrmFdCache", "Per-process DRM fds between /proc/<pid>/fd walks (kgs/kfd_procs.h)")
      .def(py::init<>())
      .def_readonly("walks", &DrmFdCache::walks)
      .def_property_readonly("pids", [](const DrmFdCache& c) { return c.by_pid.size(); });
  m.attr("DRM_RESCAN_S") = kDrmRescanNs * 1e-9;
  m.def(
      "read_kfd_procs",
      [](const std::string& kfd_root, const std::string& proc_root, uint64_t gpu_id, const std::string& bdf,
         DrmFdCache* cache, double now_s) {
        std::vector<ProcInfo> v;
        if (read_kfd_procs(kfd_root, proc_root, gpu_id, bdf, v, cache, static_cast<int64_t>(now_s * 1e9)) != 0)
          return py::object(py::none());
        py::list l;
        for (const ProcInfo& x : v) {
          py::dict o;
          o["pid"] = x.pid;
          o["name"] = x.name;
          o["vram_bytes"] = x.vram_bytes;
          o["gtt_bytes"] = x.gtt_bytes;
          o["cpu_bytes"] = x.cpu_bytes;
          o["gfx_ns"] = x.gfx_ns;
          o["cu_occupancy"] = x.cu_occupancy;
          o["cu_valid"] = x.cu_valid;
          o["evicted_ms"] = x.evicted_ms;
          l.append(o);
        }
        return py::object(l);
      },
      py::arg("kfd_root"), py::arg("proc_root"), py::arg("gpu_id"), py::arg("bdf"), py::arg("cache") = nullptr,
      py::arg("now_s") = 0.0,
      "The processes with a KFD context on gpu_id, from the KFD sysfs + DRM fdinfo (None: no KFD root); with a "
      "DrmFdCache, a process's fd directory is walked at most every DRM_RESCAN_S of now_s");
  m.def("gpu_type_from_market_name", &gpu_type_from_market_name);
  m.def("pmc_counter_names", [] {
    std::vector<std::string> v;
    for (int i = 0; i < kPmcCount; ++i) v.push_back(pmc_counter_name(i));
    return v;
  });
}
