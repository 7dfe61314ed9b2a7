"""Metric catalogue: every family the exporter emits, with type, labels and meaning.

The reference consumes one GPU series and four kube-state-metrics series
(SURVEY.md §2.6).  The first entry below is that GPU series, kept label-compatible
so the reference's PromQL (gpu_util_stats.py:159) runs unchanged; the rest are the
MI355X-native families.  ``tests/test_schema.py`` checks the renderer against this
table, and ``docs/METRICS.md`` is generated from it (``python -m
kube_gpu_stats_amd.models.schema``).

It is also the only source of the HELP and TYPE lines: the native renderer looks them
up in ``native/include/kgs/metric_help.h``, generated from this table (``python -m
kube_gpu_stats_amd.models.schema --cpp-header``; the build regenerates it and
``tests/test_schema_cli.py`` checks the committed copy and every rendered HELP line).
A family whose meaning depends on ``--sm-util-source`` carries the non-default
modes' text in ``variants``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

DEVICE_LABELS = ("gpu", "uuid")  # everything else about a device: amdgpu_device_info
# the reference contract's labels (gpu_util_stats.py:45,71,159) and the pod's identity
CONTRACT = ("kubernetes_io_hostname", "nvidia_gpu_type", "pod_name", "namespace", "container_name", "gpu", "uuid")


@dataclass(frozen=True)
class Family:
    name: str
    type: str
    help: str
    labels: tuple[str, ...] = DEVICE_LABELS
    source: str = "pmfw"
    tier: str = "fast"
    extra: tuple[str, ...] = field(default=())
    # (mode, help) for the non-default --sm-util-source modes ("pmfw", "counters")
    variants: tuple[tuple[str, str], ...] = field(default=())

    def help_for(self, mode: str = "") -> str:
        return dict(self.variants).get(mode, self.help)


F = Family
CATALOG: tuple[Family, ...] = (
    # ---- reference contract ------------------------------------------------------------
    F("container_gpu_sm_util", "gauge",
      "Busy % of the GPU allocated to the pod (mean over the exporter window), not counting the exporter's own "
      "counter READs.  Default --sm-util-source auto: while the counter tier covers the PMFW interval, the "
      "dispatch-in-flight share from the hardware counters (CPC_CPC_STAT_BUSY less the CP time of the exporter's "
      "own READ packets, learned on intervals without waves; never below the GRBM_SPI_BUSY share), else the PMFW "
      "GFX busy (kgs_util_source_seconds_total says which).  Reference contract: consumed by "
      "`avg(container_gpu_sm_util) by (kubernetes_io_hostname, nvidia_gpu_type, pod_name)`.",
      CONTRACT, "pmfw+kubelet", "fast",
      variants=(("counters", "GPU-active % (GRBM_SPI_BUSY: a shader engine has waves) of the GPU allocated to the pod, "
                             "mean over the exporter window (--sm-util-source counters).  Reference contract: consumed by "
                             "`avg(container_gpu_sm_util) by (kubernetes_io_hostname, nvidia_gpu_type, pod_name)`."),
                ("pmfw", "GFX-engine busy % of the GPU allocated to the pod from the PMFW accumulators, mean over the "
                         "exporter window (--sm-util-source pmfw: a dispatch in flight, each counter READ packet of the "
                         "exporter included).  Reference contract: consumed by "
                         "`avg(container_gpu_sm_util) by (kubernetes_io_hostname, nvidia_gpu_type, pod_name)`."))),
    F("container_gpu_mfma_util", "gauge",
      "Matrix-core (MFMA) busy % of active cycles of the GPU allocated to the pod (window), same labels as "
      "container_gpu_sm_util.  GFX busy counts a GPU busy while any dispatch is in flight; this says how much of "
      "that was matrix work.  `kgs gpu-util-stats --util-metric container_gpu_mfma_util` reports it per pod.",
      CONTRACT,
      "counters+kubelet", "pmc"),
    F("container_gpu_busy_seconds_total", "counter",
      "Busy seconds of the GPU allocated to the pod, counted from the allocation: the integral behind "
      "container_gpu_sm_util.  Default --sm-util-source auto: the counter tier's dispatch-in-flight integral "
      "(CPC_CPC_STAT_BUSY less the learned CP time of the exporter's own READs, never below GRBM_SPI_BUSY) while "
      "that tier covers the PMFW interval, busy beyond one interval carried to the next so no rate loses time; the "
      "PMFW GFX busy otherwise.  "
      "`100 * avg(rate(container_gpu_busy_seconds_total[1h])) by (kubernetes_io_hostname, nvidia_gpu_type, pod_name)` "
      "is the exact hourly per-pod utilisation whatever the scrape interval — the default source of "
      "`kgs gpu-util-stats` (fixed mode).  Same labels as container_gpu_sm_util.",
      CONTRACT, "pmfw+kubelet", "fast",
      variants=(("counters", "GPU-active seconds (GRBM_SPI_BUSY) of the GPU allocated to the pod, counted from the "
                             "allocation (--sm-util-source counters); 100 * rate() = mean busy %.  Same labels as "
                             "container_gpu_sm_util."),
                ("pmfw", "GFX-engine busy seconds of the GPU allocated to the pod from the PMFW accumulators, counted "
                         "from the allocation (--sm-util-source pmfw); 100 * rate() = mean busy %.  Same labels as "
                         "container_gpu_sm_util."))),
    F("container_gpu_mfma_busy_seconds_total", "counter",
      "MFMA-busy seconds (all SIMDs busy with matrix work for 1 s = 1) of the GPU allocated to the pod, counted from "
      "the allocation (hardware counters).  Same labels as container_gpu_sm_util.",
      CONTRACT,
      "counters+kubelet", "pmc"),
    F("container_gpu_cu_seconds_total", "counter",
      "CU-occupancy seconds of the pod's own processes on the GPU (occupied CUs / all CUs, integrated by the "
      "per-process tier; processes that exited included), counted from the allocation.  100 * rate() is the pod's "
      "compute share: on a GPU shared by several pods each is billed its own share "
      "(`kgs gpu-util-stats --util-metric container_gpu_cu_seconds_total`), where container_gpu_busy_seconds_total "
      "bills each the whole GPU.  Same labels as container_gpu_sm_util.",
      CONTRACT,
      "amdsmi-procs+cgroups+kubelet", "procs"),
    F("container_gpu_energy_joules_total", "counter",
      "Socket energy of the GPU allocated to the pod, counted from the allocation (PMFW energy accumulator).  "
      "`sum(increase(container_gpu_energy_joules_total[1h])) by (kubernetes_io_hostname, namespace, pod_name)` is "
      "the pod's hourly energy; `kgs gpu-util-stats --energy` reports it in kWh.  A GPU shared by several pods "
      "counts in full for each; a compute partition (DPX/QPX/CPX) counts its XCCs' GFX-busy share of the socket's "
      "energy, so partitions add up to the socket.  Same labels as container_gpu_sm_util.",
      CONTRACT,
      "pmfw+kubelet", "fast"),
    F("kgs_gpu_owner", "gauge",
      "1 per (GPU, pod, container) allocation reported by the kubelet: the join target that puts pod labels on any "
      "amdgpu_* series (`... * on (gpu, uuid) group_left(pod_name, namespace) kgs_gpu_owner`).",
      CONTRACT,
      "kubelet", "attribution"),
    # ---- inventory / topology -------------------------------------------------------------
    F("amdgpu_device_info", "gauge", "Static device information (1).", extra=(
        "bdf", "gpu_type", "kubernetes_io_hostname", "serial", "market_name", "gfx_target", "numa_node", "num_cu", "num_xcc", "kfd_gpu_id", "hip_id",
        "compute_partition", "memory_partition", "partition_id"),
      source="amdsmi", tier="init"),
    F("amdgpu_topology_link", "gauge", "Pairwise link between visible GPUs (1).",
      extra=("peer_gpu", "peer_bdf", "link_type", "hops", "weight"), source="amdsmi", tier="init"),
    F("amdgpu_xgmi_link_info", "gauge", "Per-link peer PCI address and speed (1).",
      extra=("link", "peer_bdf", "link_type", "bit_rate_gbps", "max_bandwidth_gbps"), source="amdsmi", tier="slow"),
    # ---- utilisation ------------------------------------------------------------------------
    F("amdgpu_gfx_busy_percent", "gauge",
      "GPU busy %, time-weighted mean over the window — the source of container_gpu_sm_util (default auto: the "
      "counter tier's dispatch-in-flight share — CPC busy less the learned READ cost, never below SPI busy — while "
      "it covers the PMFW interval, PMFW GFX busy otherwise; never the exporter's own counter READs).",
      variants=(("counters", "GFX-engine busy %, time-weighted mean over the window (PMFW accumulators)."),
                ("pmfw", "GFX-engine busy %, time-weighted mean over the window (PMFW accumulators)."))),
    F("amdgpu_pmfw_gfx_busy_percent", "gauge",
      "Firmware (PMFW) GFX busy %, window mean from the PMFW accumulators: a dispatch in flight — and each counter "
      "READ packet of the exporter as ~80 us of work (99.7 % on an idle GPU READ at 8 kHz, profiles/r2/idle_busy/)."),
    F("amdgpu_gfx_busy_instant_percent", "gauge", "GFX busy % in the latest PMFW table."),
    F("amdgpu_gfx_busy_xcc_percent", "gauge",
      "Busy % per XCC over the last firmware interval, from the per-partition accumulators "
      "(instant value when those are absent).  Busy means a dispatch in flight on that XCC: a chip-wide kernel keeps "
      "all 8 at ~100 % even when waves run on a few; amdgpu_mfma_util_xcc_percent shows where they run.", extra=("xcc",)),
    F("amdgpu_umc_busy_percent", "gauge", "HBM memory-controller activity %, window mean."),
    F("amdgpu_gfx_busy_seconds_total", "counter",
      "∫ busy fraction dt of amdgpu_gfx_busy_percent's source (default auto: the READ-immune integral behind "
      "container_gpu_busy_seconds_total); rate() = exact mean utilisation.",
      variants=(("counters", "∫ PMFW GFX busy fraction dt; rate() = exact mean utilisation."),
                ("pmfw", "∫ PMFW GFX busy fraction dt; rate() = exact mean utilisation."))),
    F("amdgpu_pmfw_gfx_busy_seconds_total", "counter", "∫ PMFW GFX busy fraction dt (counts counter READs as work)."),
    F("kgs_util_source_seconds_total", "counter",
      "Firmware time the READ-immune busy integral (--sm-util-source auto) billed from each source: counters (the "
      "counter tier's dispatch integral — CPC_CPC_STAT_BUSY less the learned READ cost, never below GRBM_SPI_BUSY — "
      "covered the PMFW interval) or pmfw (counter tier off, handed over, failed or stale).",
      extra=("source",), source="self"),
    F("kgs_util_carry_seconds", "gauge",
      "Counter busy the READ-immune integral has received but not billed yet (negative: billed ahead of the last "
      "drain, run on at its share): a drain that lands after a PMFW interval's end is billed in the next one.",
      source="self"),
    F("kgs_util_dropped_seconds_total", "counter",
      "Counter busy beyond the carry cap (one freshness window), never billed: a firmware clock slower than the "
      "host's.  Should stay near 0.", source="self"),
    F("amdgpu_umc_busy_seconds_total", "counter", "∫ UMC busy fraction dt."),
    F("amdgpu_hbm_bandwidth_bytes_per_second", "gauge",
      "Estimated HBM (DRAM) read+write bandwidth, window mean, from UMC activity × the MI355X calibration "
      "(1 % = 84.1 GB/s): within ±2.5 % of the bytes streaming kernels move; random 64 B gathers read 2.0× their "
      "requested bytes (each costs a 128 B DRAM access, which is real HBM traffic); cache (L2 / MALL) hits are not "
      "counted (profiles/umc_calib.md)."),
    F("amdgpu_hbm_bytes_total", "counter",
      "HBM bytes moved (read+write), ∫ bandwidth dt from the UMC accumulators; rate() = bandwidth."),
    # ---- memory ------------------------------------------------------------------------------
    F("amdgpu_hbm_used_bytes", "gauge", "HBM3E bytes in use.", source="sysfs"),
    F("amdgpu_hbm_total_bytes", "gauge", "HBM3E capacity (288 GB on MI355X).", source="sysfs", tier="init"),
    # ---- thermals / power / clocks -----------------------------------------------------------
    F("amdgpu_temperature_celsius", "gauge", "Temperature by sensor (hotspot, hbm, vrsoc).", extra=("sensor",)),
    F("amdgpu_power_watts", "gauge", "Socket power."),
    F("amdgpu_energy_joules_total", "counter", "Energy since exporter start (wrap-safe); a compute partition counts "
      "its XCCs' GFX-busy share of the socket's energy."),
    F("amdgpu_clock_mhz", "gauge", "Current clock (gfx = mean over XCCs, mem, soc).", extra=("clock",)),
    F("amdgpu_throttle_seconds_total", "counter", "Seconds the GPU ran held back, per throttler (PMFW residency "
      "accumulators ÷ accumulation cycles × time); 100 * rate() = violation % (amdsmi PVIOL for reason=\"ppt\", TVIOL "
      "for reason=\"socket_thermal\").", extra=("reason",)),
    # ---- interconnect ------------------------------------------------------------------------
    F("amdgpu_xgmi_read_bytes_total", "counter", "Bytes received per xGMI link.", extra=("link",)),
    F("amdgpu_xgmi_write_bytes_total", "counter", "Bytes sent per xGMI link.", extra=("link",)),
    F("amdgpu_xgmi_link_up", "gauge", "xGMI link status per port.", extra=("link",)),
    F("amdgpu_pcie_bytes_total", "counter", "Bytes over the PCIe link, both directions: PMFW PCIe bandwidth "
      "accumulator × MI355X calibration (105.7 B/unit; H2D 102.65, D2H 108.74 measured, ±3 %; profiles/r2/pcie/)."),
    F("amdgpu_pcie_bandwidth_acc_total", "counter", "Raw PMFW PCIe bandwidth accumulator (amdsmi pcie_bandwidth_acc)."),
    # ---- RAS / link health -------------------------------------------------------------------
    F("amdgpu_ecc_block_errors_total", "counter",
      "Accumulated ECC errors per RAS block (umc = HBM, gfx, xgmi_wafl, ...) and type, for the blocks with ECC enabled.",
      extra=("block", "type"), source="amdsmi", tier="slow"),
    F("amdgpu_ecc_errors_total", "counter", "Accumulated ECC errors by type.", extra=("type",), source="amdsmi",
      tier="slow"),
    F("amdgpu_xgmi_error_status", "gauge", "xGMI error status (0 none, 1 error, 2 multiple).", source="amdsmi",
      tier="slow"),
    # ---- hardware counters (direct command-processor reader, native/counters/pmc_aqlprofile.cpp) --
    F("amdgpu_pmc_total", "counter", "Raw hardware counter since exporter start.", extra=("counter",),
      source="counters", tier="pmc"),
    F("amdgpu_mfma_util_percent", "gauge", "Matrix-core busy % of active cycles (window).", source="counters",
      tier="pmc"),
    F("amdgpu_gpu_active_seconds_total", "counter",
      "∫ GPU-active share of clocks dt (per drain: ΔGRBM_SPI_BUSY / ΔGRBM_COUNT · Δt); rate() = GPU-active fraction, "
      "blind to the exporter's own counter READs (the --sm-util-source counters integral).", source="counters",
      tier="pmc"),
    F("amdgpu_dispatch_busy_seconds_total", "counter",
      "∫ dispatch-in-flight share dt from the counter stream (per drain: CPC_CPC_STAT_BUSY share of the clocks less "
      "the exporter's own READ packet's CP time — counted once where it overlaps dispatch busy in intervals ≥ 400 us "
      "— never below the GRBM_SPI_BUSY share; an interval the CP was busy for ≥ 90 % counts whole, a READ-only one "
      "(no waves, no MFMA cycle) as nothing; intervals ≥ 400 us "
      "split busy from idle part in time — idle cycles at the learned idle clock, kgs_pmc_shader_clock_hz — blended "
      "0.6 with the cycle share unless READ-only intervals among the kernels just measured the gaps' clock); rate() = "
      "the READ-immune 'a kernel is running' fraction behind --sm-util-source auto.", source="counters", tier="pmc"),
    F("kgs_pmc_read_cp_seconds", "gauge", "Command-processor busy time of one full counter READ packet, learned on "
      "intervals without waves (what amdgpu_dispatch_busy_seconds_total subtracts per READ; lite READs are learned "
      "apart and cost less).", source="self",
      tier="pmc"),
    F("kgs_pmc_shader_clock_hz", "gauge",
      "Shader clock the dispatch estimator learned from GRBM_COUNT: kind=idle on intervals without waves, kind=busy "
      "on intervals the CP was busy for all of.  A long partial interval (low READ rate) prices its idle cycles at "
      "the idle clock (the time split behind amdgpu_dispatch_busy_seconds_total).", extra=("kind",), source="self",
      tier="pmc"),
    F("amdgpu_mfma_busy_seconds_total", "counter",
      "∫ MFMA-busy share of all SIMD cycles dt (per drain: ΔSQ_VALU_MFMA_BUSY_CYCLES / (SIMDs·ΔGRBM_COUNT) · Δt); "
      "rate() = matrix-core utilisation of wall time.", source="counters", tier="pmc"),
    F("amdgpu_gpu_active_percent", "gauge", "% of clocks a shader engine had waves to run (GRBM_SPI_BUSY, window); "
      "unlike the PMFW GFX busy it does not count the exporter's own counter READs.", source="counters", tier="pmc"),
    F("amdgpu_vmem_busy_percent", "gauge", "Vector-memory address unit (TA) busy % of active cycles (window).",
      source="counters", tier="pmc"),
    F("amdgpu_gpu_clock_effective_mhz", "gauge", "Effective shader clock from GRBM_COUNT (window).",
      source="counters", tier="pmc"),
    F("amdgpu_mfma_util_xcc_percent", "gauge",
      "Matrix-core busy % of one XCD's active SIMD cycles (window; aqlprofile reader, results placed on XCDs in "
      "the READ buffer's XCC-major order, verified against an XCC-gated load).  An XCD left idle while others "
      "saturate is a workgroup→XCD mapping problem, invisible in the device-wide gauges.",
      extra=("xcc",), source="counters", tier="pmc"),
    F("amdgpu_vmem_busy_xcc_percent", "gauge",
      "Vector-memory address unit (TA) busy % of one XCD's active cycles, mean over its CUs (window; --pmc-set full).",
      extra=("xcc",), source="counters", tier="pmc"),
    F("amdgpu_gpu_active_xcc_percent", "gauge",
      "GRBM SPI-busy % of clocks of one XCD (window): one of its shader engines has waves to run.  Unlike GUI-active "
      "(which reads ~100 % on every XCD while any chip-wide dispatch is in flight) it shows where waves run.",
      extra=("xcc",), source="counters", tier="pmc"),
    # ---- per process -------------------------------------------------------------------------
    F("amdgpu_process_hbm_bytes", "gauge", "HBM bytes held by a process.",
      extra=("pid", "process", "pod", "namespace", "container", "pod_uid"), source="amdsmi", tier="mid"),
    F("amdgpu_process_gtt_bytes", "gauge", "GTT bytes held by a process.",
      extra=("pid", "process", "pod", "namespace", "container", "pod_uid"), source="amdsmi", tier="mid"),
    F("amdgpu_process_cu_occupancy", "gauge", "CUs occupied by the process' waves.",
      extra=("pid", "process", "pod", "namespace", "container", "pod_uid"), source="amdsmi", tier="mid"),
    F("amdgpu_process_gfx_seconds_total", "counter", "GFX engine time of the process (driver-reported).",
      extra=("pid", "process", "pod", "namespace", "container", "pod_uid"), source="amdsmi", tier="mid"),
    F("amdgpu_process_cu_seconds_total", "counter", "∫ occupied-CU share dt; rate() = the process' compute share.",
      extra=("pid", "process", "pod", "namespace", "container", "pod_uid"), source="amdsmi", tier="mid"),
    # ---- exporter self-metrics ---------------------------------------------------------------
    F("kgs_up", "gauge", "1 if the device's last read succeeded.", source="self"),
    F("kgs_last_sample_age_seconds", "gauge", "Seconds since the last successful read.", source="self"),
    F("kgs_samples_total", "counter", "Distinct hardware samples (new PMFW firmware timestamp).", source="self"),
    F("kgs_reads_total", "counter", "Sampler reads attempted.", source="self"),
    F("kgs_read_errors_total", "counter", "Sampler reads that failed.", source="self"),
    F("kgs_sampler_overruns_total", "counter", "Ticks that overran the period.", source="self"),
    F("kgs_device_recoveries_total", "counter",
      "Backend re-opens / AMD SMI re-inits that restored reads after a failure streak (GPU reset).", source="self"),
    F("kgs_pmc_samples_total", "counter", "Hardware-counter drains completed.", source="self"),
    F("kgs_pmc_errors_total", "counter", "Hardware-counter drains that failed.", source="self"),
    F("kgs_pmc_read_seconds_total", "counter", "Time spent draining hardware counters.", source="self"),
    F("kgs_pmc_enabled", "gauge", "1 while the exporter holds the counters, 0 after handing them to another profiler "
      "(SIGUSR1; SIGUSR2 takes them back).", source="self"),
    F("kgs_pmc_releases_total", "counter", "Counter hand-overs to another profiler.", source="self"),
    F("kgs_pmc_stalled", "gauge", "1 while GRBM_COUNT shows no plausible clock: another profiler stopped or "
      "reprogrammed the counters (the counter-tier gauges are withheld meanwhile).", source="self"),
    F("kgs_pmc_reclaims_total", "counter", "Automatic counter re-STARTs after a stall of --pmc-reclaim-s.", source="self"),
    F("kgs_pmc_refreshes_total", "counter", "Periodic counter re-STARTs (--pmc-refresh-s): reprogram selects that "
      "another profiler may have changed without stalling GRBM_COUNT.", source="self"),
    F("kgs_pmc_quiet", "gauge", "1 while the last counter READ interval saw no wave and no MFMA cycle: READs drop to "
      "--pmc-idle-hz so the exporter's own packets do not read as GPU activity.", source="self"),
    F("kgs_pmc_quiet_skips_total", "counter", "Sampler ticks that skipped their counter READ on a quiet GPU.",
      source="self"),
    F("kgs_pmc_dispatch_bound", "gauge", "1 while the command processor dispatched with no wave in flight for at "
      "least --pmc-cp-only-min of the clocks for --pmc-dispatch-hold-ms (a stream of µs kernels, which each READ "
      "packet slows): READs drop to --pmc-dispatch-hz.", source="self"),
    F("kgs_process_cu_unavailable", "gauge", "Processes on the GPU whose CU occupancy could not be read in the last "
      "per-process pass (their KFD stats are gone: a process tearing down).  Their amdgpu_process_cu_occupancy line "
      "is withheld and nothing is integrated for them; a pod whose CU-seconds are all unknown gets no "
      "container_gpu_cu_seconds_total line rather than 0.", source="self"),
    F("kgs_pmc_parked", "gauge", "1 while the counter session is released because the GPU has been quiet for "
      "--pmc-quiet-release-s (no wave, no MFMA cycle): a programmed session and its READ queue keep an idle MI355X "
      "out of its low-power state (≈291 W against ≈258 W: +32 W per idle GPU, bench phase P).  Utilisation is "
      "billed from the PMFW GFX busy meanwhile (no READ inflates it), and the counter-tier gauges are withheld; the "
      "session is re-acquired as soon as one PMFW interval shows ≥ 10 % GFX busy or 100 ms of them ≥ 1 %.",
      source="self"),
    F("kgs_pmc_parks_total", "counter", "Quiet releases of the counter session (kgs_pmc_parked).", source="self"),
    F("kgs_pmc_parked_seconds_total", "counter", "Seconds the counter session has spent released by the quiet "
      "release (kgs_pmc_parked): × ≈32 W is the energy the release saved an idle MI355X.", source="self"),
    F("kgs_pmc_dispatch_skips_total", "counter", "Sampler ticks that skipped their counter READ in a dispatch-bound "
      "stream.", source="self"),
    F("kgs_pmc_failed", "gauge", "1 while the counter tier's circuit breaker is open: --pmc-breaker-k consecutive "
      "counter drains failed (a wedged command processor).  READs stop; after --pmc-retry-s (doubling to "
      "--pmc-retry-max-s) the reader's AQL queue is recreated and the counters re-STARTed.  The PMFW tier of the "
      "same GPU runs on its own thread and keeps reporting.", source="self"),
    F("kgs_pmc_breaker_trips_total", "counter", "Times the counter tier's circuit breaker opened.", source="self"),
    F("kgs_pmc_retries_total", "counter", "Reader resets + re-STARTs attempted while the breaker was open.",
      source="self"),
    F("kgs_pmc_publishes_total", "counter", "Counter READs that wrote the GPU's L2 back to publish their results "
      "to the host.  With --pmc-batch B at most one READ in B does (the writeback is about half of what a READ "
      "costs a training step); a READ never waits more than --pmc-publish-us for it, so at <= 1 kHz every READ "
      "publishes.", source="self"),
    F("kgs_pmc_unlanded_total", "counter", "Batched counter READs dropped because a result was still unwritten in "
      "host memory when their batch was folded (after a 200 us wait; the counters are cumulative, so the next sample "
      "covers the interval).  Should stay near 0 (a result dword that really reads 0xFFFFFFFF is dropped too, about "
      "one READ in 5e7); a steady rate means --pmc-batch 1.",
      source="self"),
    F("kgs_sampler_thread_hung", "gauge", "1 if a sampler thread of the device was stuck in a device call when "
      "sampling last stopped: it was abandoned (--stop-timeout) and that tier restarts once the call returns.",
      source="self"),
    F("kgs_sampled_seconds_total", "counter", "Firmware time covered by distinct samples.", source="self"),
    F("kgs_slow_reads_total", "counter",
      "Management-library reads by the device's slow thread kgs-slow<N> (tier=procs: process list; tier=links: xGMI "
      "link table + RAS).  They never run on the PMFW or counter threads.", extra=("tier",), source="self"),
    F("kgs_slow_read_seconds_total", "counter", "Time the device's slow thread spent in management-library calls.",
      source="self"),
    F("kgs_slow_errors_total", "counter", "Failed management-library reads of the device's slow thread, by tier "
      "(procs, links, health).", extra=("tier",), source="self"),
    F("kgs_slow_last_ok_age_seconds", "gauge",
      "Seconds since the tier's last good read on the device (-1 = never).  Past --stale-after (or three tier "
      "periods) its lines are dropped: per-process series (procs), amdgpu_xgmi_link_info (links), "
      "amdgpu_xgmi_error_status (health).  Other devices' tiers run on their own threads.",
      extra=("tier",), source="self"),
    F("kgs_slow_call_seconds", "gauge", "How long the device's slow thread has been inside its current "
      "management-library call (0 = none in flight): a call that never returns keeps growing here.", source="self"),
    F("kgs_slow_thread_hung", "gauge", "1 if the device's slow thread was stuck in a management-library call when "
      "sampling last stopped (abandoned after --stop-timeout; the slow tiers restart once the call returns).",
      source="self"),
    F("kgs_pmc_reordered_total", "counter", "Counter drains dropped because their command-processor time preceded "
      "the previous drain's (the cumulative counts of the next drain cover the interval).  Should stay 0.",
      source="self"),
    F("kgs_sample_read_seconds", "histogram", "Latency of one fast-tier backend read.", extra=("le",), source="self"),
    F("kgs_sampler_wake_lateness_seconds", "histogram", "How late the counter thread woke against each tick's "
      "absolute deadline (CPU contention, idle-state exit); a tick more than 4 periods late is skipped and counted "
      "in kgs_sampler_overruns_total.", extra=("le",), source="self"),
    F("kgs_scrapes_total", "counter", "Scrapes rendered.", ("kubernetes_io_hostname",), "self"),
    F("kgs_scrape_render_seconds_total", "counter", "Time spent rendering /metrics.", ("kubernetes_io_hostname",),
      "self"),
    F("kgs_scrape_render_last_seconds", "gauge", "Render time of the previous scrape.", ("kubernetes_io_hostname",),
      "self"),
    F("kgs_http_connections", "gauge", "HTTP connections held open by the exporter.", ("kubernetes_io_hostname",),
      "self"),
    F("kgs_http_connections_closed_total", "counter",
      "HTTP connections the exporter closed itself: idle past --http-idle-s (reason=idle) or evicted, least "
      "recently active first, to admit one past --http-max-conns (reason=limit).",
      ("kubernetes_io_hostname", "reason"), "self"),
    F("kgs_build_info", "gauge", "Build / configuration (1).",
      ("kubernetes_io_hostname", "version", "backend", "pmc_source", "sample_hz"), "self"),
    # ---- attribution loop (Python control plane, pushed via set_extra_metrics) ---------------
    F("kgs_attribution_updates_total", "counter", "Attribution passes completed.", (), "attribution", "attr"),
    F("kgs_attribution_errors_total", "counter", "Failed attribution passes / kubelet calls.", (), "attribution",
      "attr"),
    F("kgs_attribution_kubelet_reconnects_total", "counter", "Pod-resources client re-creations.", (),
      "attribution", "attr"),
    F("kgs_attribution_kubelet_connected", "gauge", "1 if a pod-resources client is open.", (), "attribution",
      "attr"),
    F("kgs_attribution_kubelet_age_seconds", "gauge", "Seconds since the last good kubelet List (-1: never).", (),
      "attribution", "attr"),
    F("kgs_attribution_allocated_gpus", "gauge", "GPUs with at least one owning container.", (), "attribution",
      "attr"),
)

BY_NAME = {f.name: f for f in CATALOG}
MODES = ("counters", "pmfw")  # --sm-util-source values with their own HELP variants (auto is the default text)


def _c(text: str) -> str:
    return '"' + text.replace("\\", "\\\\").replace('"', '\\"') + '"'


def cpp_header() -> str:
    """native/include/kgs/metric_help.h: the renderer's HELP / TYPE table."""
    rows = []
    for f in sorted(CATALOG, key=lambda f: f.name):
        rows.append(f"    {{{_c(f.name)}, {_c(f.type)}, {_c('')}, {_c(f.help)}}},")
        for mode, text in f.variants:
            rows.append(f"    {{{_c(f.name)}, {_c(f.type)}, {_c(mode)}, {_c(text)}}},")
    return ("// Generated by `python -m kube_gpu_stats_amd.models.schema --cpp-header` from\n"
            "// kube_gpu_stats_amd/models/schema.py (the metric catalogue).  Do not edit.\n"
            "#pragma once\n\n#include <cstddef>\n#include <cstring>\n\nnamespace kgs {\n\n"
            "struct MetricDoc {\n  const char* name;\n  const char* type;\n"
            "  const char* mode;  // \"\" = default (--sm-util-source auto); else that mode's text\n"
            "  const char* help;\n};\n\n"
            "inline constexpr MetricDoc kMetricDocs[] = {\n" + "\n".join(rows) + "\n};\n\n"
            "constexpr size_t kMetricDocCount = sizeof kMetricDocs / sizeof kMetricDocs[0];\n"
            "constexpr size_t kNoMetricDoc = ~size_t{0};\n\n"
            "constexpr bool metric_doc_streq(const char* a, const char* b) {\n"
            "  while (*a && *a == *b) {\n"
            "    ++a;\n"
            "    ++b;\n"
            "  }\n"
            "  return *a == *b;\n"
            "}\n\n"
            "// Index of the family's default entry (each default entry precedes its variants);\n"
            "// kNoMetricDoc if unknown.  Meant for constant evaluation: KGS_METRIC_DOC(\"name\").\n"
            "constexpr size_t metric_doc_index(const char* name) {\n"
            "  for (size_t i = 0; i < kMetricDocCount; ++i)\n"
            "    if (!*kMetricDocs[i].mode && metric_doc_streq(kMetricDocs[i].name, name)) return i;\n"
            "  return kNoMetricDoc;\n"
            "}\n\n"
            "// The entry at `i` in the text of `mode` (\"\" = default): the variants follow it.\n"
            "inline const MetricDoc& metric_doc_at(size_t i, const char* mode) {\n"
            "  if (*mode)\n"
            "    for (size_t j = i + 1; j < kMetricDocCount && std::strcmp(kMetricDocs[j].name, kMetricDocs[i].name) == 0; ++j)\n"
            "      if (std::strcmp(kMetricDocs[j].mode, mode) == 0) return kMetricDocs[j];\n"
            "  return kMetricDocs[i];\n"
            "}\n\n"
            "// A family's entry index, resolved at compile time; a name missing from the\n"
            "// catalogue does not compile.\n"
            "#define KGS_METRIC_DOC(name)                                                         \\\n"
            "  ([]() {                                                                           \\\n"
            "    constexpr size_t kgs_doc_i = ::kgs::metric_doc_index(name);                     \\\n"
            "    static_assert(kgs_doc_i != ::kgs::kNoMetricDoc, \"not in models/schema.py: \" name); \\\n"
            "    return kgs_doc_i;                                                               \\\n"
            "  }())\n\n"
            "// The family's HELP / TYPE for `mode` (falls back to the default text); nullptr if unknown.\n"
            "inline const MetricDoc* metric_doc(const char* name, const char* mode = \"\") {\n"
            "  for (size_t i = 0; i < kMetricDocCount; ++i)\n"
            "    if (!*kMetricDocs[i].mode && std::strcmp(kMetricDocs[i].name, name) == 0) return &metric_doc_at(i, mode);\n"
            "  return nullptr;\n"
            "}\n\n}  // namespace kgs\n")


def markdown() -> str:
    rows = ["| metric | type | labels | source / tier | meaning |", "|---|---|---|---|---|"]
    for f in CATALOG:
        labels = ", ".join(f.labels + f.extra)
        rows.append(f"| `{f.name}` | {f.type} | {labels} | {f.source} / {f.tier} | {f.help} |")
    return "\n".join(rows)


PREAMBLE = ("# Metric catalogue\n\nGenerated by `python -m kube_gpu_stats_amd.models.schema` from "
            "`kube_gpu_stats_amd/models/schema.py`; `tests/test_schema_cli.py` checks the renderer against it. Every "
            "series also carries `gpu` and `uuid`; device attributes (bdf, type, serial, NUMA node, …) are in "
            "`amdgpu_device_info`.\n\n")


if __name__ == "__main__":
    import sys

    if sys.argv[1:] == ["--cpp-header"]:
        sys.stdout.write(cpp_header())
    else:
        print(PREAMBLE + markdown())
