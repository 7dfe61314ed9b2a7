"""Grafana dashboard for the exporter, generated from code so its PromQL stays in
step with the metric catalogue (``schema.CATALOG``; ``tests/test_deploy.py``
checks every series name used here against it).

    python -m kube_gpu_stats_amd.models.dashboard > deploy/grafana-dashboard.json

Rows: fleet (allocation + the reference's per-pod utilisation), per-GPU
utilisation (PMFW window + per-XCC + matrix-core counters), memory / power /
thermals, xGMI, per-process, and exporter health.
"""
from __future__ import annotations

import json

_NODE = 'kubernetes_io_hostname=~"$node"'


def _panel(pid: int, title: str, exprs: list[tuple[str, str]], x: int, y: int, w: int = 12, h: int = 8,
           unit: str = "short", kind: str = "timeseries", maxv: float | None = None) -> dict:
    p = {
        "id": pid, "type": kind, "title": title, "datasource": {"type": "prometheus", "uid": "${datasource}"},
        "gridPos": {"x": x, "y": y, "w": w, "h": h},
        "targets": [{"refId": chr(ord("A") + i), "expr": e, "legendFormat": lg} for i, (e, lg) in enumerate(exprs)],
        "fieldConfig": {"defaults": {"unit": unit}, "overrides": []},
    }
    if maxv is not None:
        p["fieldConfig"]["defaults"]["max"] = maxv
        p["fieldConfig"]["defaults"]["min"] = 0
    return p


def _row(pid: int, title: str, y: int) -> dict:
    return {"id": pid, "type": "row", "title": title, "collapsed": False, "gridPos": {"x": 0, "y": y, "w": 24, "h": 1},
            "panels": []}


def _dev(metric: str) -> str:
    """A per-device family joined to its node through amdgpu_device_info (series carry gpu/uuid only)."""
    return (f"{metric} * on (instance, gpu) group_left (kubernetes_io_hostname) "
            f"max by (instance, gpu, kubernetes_io_hostname) (amdgpu_device_info{{{_NODE}}})")


def build() -> dict:
    panels: list[dict] = []
    pid = 0
    y = 0

    def add(p):
        nonlocal pid
        pid += 1
        p["id"] = pid
        panels.append(p)

    add(_row(0, "Fleet", y)); y += 1
    add(_panel(0, "Per-pod GPU utilisation (reference contract)",
               [(f"avg(container_gpu_sm_util{{{_NODE}}}) by (kubernetes_io_hostname, pod_name)",
                 "{{kubernetes_io_hostname}} / {{pod_name}}")], 0, y, unit="percent", maxv=100))
    add(_panel(0, "Allocated GPUs per node",
               [(f"count by (kubernetes_io_hostname) (container_gpu_sm_util{{{_NODE},pod_name!=\"\"}})",
                 "{{kubernetes_io_hostname}}")], 12, y))
    y += 8
    add(_panel(0, "Power drawn by each pod's GPUs",
               [(f"sum(rate(container_gpu_energy_joules_total{{{_NODE}}}[5m])) by (kubernetes_io_hostname, pod_name)",
                 "{{kubernetes_io_hostname}} / {{pod_name}}")], 0, y, unit="watt"))
    add(_panel(0, "Per-pod exact utilisation (busy-seconds counter)",
               [(f"100 * avg(rate(container_gpu_busy_seconds_total{{{_NODE}}}[5m])) by (kubernetes_io_hostname, pod_name)",
                 "{{kubernetes_io_hostname}} / {{pod_name}}")], 12, y, unit="percent", maxv=100))
    y += 8
    add(_row(0, "Utilisation", y)); y += 1
    add(_panel(0, "GFX busy (PMFW) vs GPU-active (waves, READ-immune)",
               [(_dev("100 * rate(amdgpu_gfx_busy_seconds_total[1m])"), "gfx busy {{kubernetes_io_hostname}} gpu{{gpu}}"),
                (_dev("100 * rate(amdgpu_gpu_active_seconds_total[1m])"),
                 "active {{kubernetes_io_hostname}} gpu{{gpu}}")],
               0, y, unit="percent", maxv=100))
    add(_panel(0, "Matrix-core (MFMA) busy",
               [(_dev("amdgpu_mfma_util_percent"), "{{kubernetes_io_hostname}} gpu{{gpu}}")], 12, y, unit="percent",
               maxv=100))
    y += 8
    add(_panel(0, "Per-XCD MFMA busy (workgroup→XCD imbalance)",
               [(_dev("amdgpu_mfma_util_xcc_percent"), "gpu{{gpu}} xcd{{xcc}}")], 0, y, unit="percent", maxv=100))
    add(_panel(0, "HBM bandwidth (UMC activity, MI355X calibration)",
               [(_dev("rate(amdgpu_hbm_bytes_total[1m])"), "gpu{{gpu}}")], 12, y, unit="Bps"))
    y += 8
    add(_panel(0, "HBM controller busy / vector-memory busy",
               [(_dev("amdgpu_umc_busy_percent"), "umc gpu{{gpu}}"),
                (_dev("amdgpu_vmem_busy_percent"), "vmem gpu{{gpu}}")], 0, y, unit="percent", maxv=100))
    y += 8
    add(_row(0, "Memory, power, thermals", y)); y += 1
    add(_panel(0, "HBM3E used", [(_dev("amdgpu_hbm_used_bytes"), "gpu{{gpu}}")], 0, y, w=8, unit="bytes"))
    add(_panel(0, "Power", [(_dev("amdgpu_power_watts"), "gpu{{gpu}}")], 8, y, w=8, unit="watt"))
    add(_panel(0, "Hotspot / HBM temperature",
               [(_dev('amdgpu_temperature_celsius{sensor=~"hotspot|hbm"}'), "gpu{{gpu}} {{sensor}}")], 16, y, w=8,
               unit="celsius"))
    y += 8
    add(_panel(0, "Energy per hour", [(_dev("3600 * rate(amdgpu_energy_joules_total[5m])"), "gpu{{gpu}}")], 0, y,
               w=12, unit="joule"))
    add(_panel(0, "Effective shader clock", [(_dev("amdgpu_gpu_clock_effective_mhz"), "gpu{{gpu}}")], 12, y, w=12,
               unit="MHz"))
    y += 8
    add(_panel(0, "Throttling by reason (PVIOL = ppt, TVIOL = socket_thermal)",
               [(_dev("100 * rate(amdgpu_throttle_seconds_total[1m])"), "gpu{{gpu}} {{reason}}")], 0, y, w=12,
               unit="percent", maxv=100))
    add(_panel(0, "PCIe traffic (host link)", [(_dev("rate(amdgpu_pcie_bytes_total[1m])"), "gpu{{gpu}}")], 12, y,
               w=12, unit="Bps"))
    y += 8
    add(_row(0, "xGMI and RAS", y)); y += 1
    add(_panel(0, "xGMI traffic per GPU (read + write, all links)",
               [(_dev("sum by (instance, gpu) (rate(amdgpu_xgmi_read_bytes_total[1m]) + "
                      "rate(amdgpu_xgmi_write_bytes_total[1m]))"), "gpu{{gpu}}")], 0, y, unit="Bps"))
    add(_panel(0, "xGMI errors", [(_dev("amdgpu_xgmi_error_status"), "gpu{{gpu}}")], 12, y, w=6))
    add(_panel(0, "ECC errors per RAS block (1 h)",
               [(_dev("sum by (instance, gpu, block, type) (increase(amdgpu_ecc_block_errors_total[1h]))"),
                 "gpu{{gpu}} {{block}} {{type}}")], 18, y, w=6))
    y += 8
    add(_row(0, "Processes", y)); y += 1
    add(_panel(0, "HBM per process", [("amdgpu_process_hbm_bytes", "{{pod}} pid {{pid}} gpu{{gpu}}")], 0, y,
               unit="bytes"))
    add(_panel(0, "Compute share per process (occupied-CU fraction)",
               [("rate(amdgpu_process_cu_seconds_total[1m])", "{{pod}} pid {{pid}} gpu{{gpu}}")], 12, y,
               unit="percentunit", maxv=1))
    y += 8
    add(_panel(0, "Shared GPUs: compute share per pod",
               [("sum by (kubernetes_io_hostname, gpu, namespace, pod) "
                 "(rate(amdgpu_process_cu_seconds_total{pod!=\"\"}[5m]))", "{{namespace}}/{{pod}} gpu{{gpu}}")],
               0, y, unit="percentunit", maxv=1))
    add(_panel(0, "Shared GPUs: HBM per pod",
               [("sum by (kubernetes_io_hostname, gpu, namespace, pod) (amdgpu_process_hbm_bytes{pod!=\"\"})",
                 "{{namespace}}/{{pod}} gpu{{gpu}}")], 12, y, unit="bytes"))
    y += 8
    add(_row(0, "Exporter health", y)); y += 1
    add(_panel(0, "Samples / s per GPU (PMFW distinct, counters)",
               [(_dev("rate(kgs_samples_total[1m])"), "pmfw gpu{{gpu}}"),
                (_dev("rate(kgs_pmc_samples_total[1m])"), "pmc gpu{{gpu}}"),
                (_dev("kgs_pmc_quiet"), "quiet (idle READ rate) gpu{{gpu}}"),
                (_dev("kgs_pmc_dispatch_bound"), "dispatch-bound (dispatch READ rate) gpu{{gpu}}"),
                (_dev("kgs_pmc_parked"), "parked (session released while quiet) gpu{{gpu}}"),
                (_dev("rate(kgs_pmc_parked_seconds_total[1h])"), "parked share, last hour gpu{{gpu}}")], 0, y, w=8))
    add(_panel(0, "Scrape render time / HTTP connections",
               [("kgs_scrape_render_last_seconds", "render s {{instance}}"),
                ("kgs_http_connections", "connections {{instance}}"),
                ("increase(kgs_http_connections_closed_total[1h])", "closed/h {{reason}} {{instance}}")],
               8, y, w=8))
    add(_panel(0, "Sampler up / recoveries / attribution age",
               [(_dev("kgs_up"), "up gpu{{gpu}}"), (_dev("increase(kgs_device_recoveries_total[1h])"),
                                                   "recoveries gpu{{gpu}}"),
                ("kgs_attribution_kubelet_age_seconds", "kubelet age {{instance}}")], 16, y, w=8))
    y += 8
    # batched READ publication: ~1000 writebacks/s per GPU at 8 kHz (--pmc-batch 8), every
    # READ at <= 1 kHz; dropped READs (results not in host memory) should stay at 0
    add(_panel(0, "Counter READ publication (L2 writebacks / s, dropped READs / s)",
               [(_dev("rate(kgs_pmc_publishes_total[1m])"), "writebacks gpu{{gpu}}"),
                (_dev("rate(kgs_pmc_unlanded_total[5m])"), "dropped gpu{{gpu}}")], 0, y, w=8))
    # host CPU contention: how late the counter threads wake (overruns skip ticks past 4 periods)
    add(_panel(0, "Sampler wake-up lateness p99 / overruns per s",
               [(_dev("histogram_quantile(0.99, rate(kgs_sampler_wake_lateness_seconds_bucket[5m]))"),
                 "p99 late s gpu{{gpu}}"),
                (_dev("rate(kgs_sampler_overruns_total[5m])"), "overruns/s gpu{{gpu}}")], 8, y, w=8))
    # the READ-immune utilisation's health: the share of firmware time billed from the
    # counter tier (< 1: hand-over, breaker or stale drains billed from PMFW), the counter
    # busy not yet billed, and the clocks the dispatch estimator prices idle cycles at
    add(_panel(0, "Utilisation from counters (share), billing carry, learned shader clocks",
               [(_dev('rate(kgs_util_source_seconds_total{source="counters"}[5m])'), "counters share gpu{{gpu}}"),
                (_dev("kgs_util_carry_seconds"), "carry s gpu{{gpu}}"),
                (_dev("kgs_pmc_shader_clock_hz / 1000000000"), "{{kind}} clock GHz gpu{{gpu}}")], 16, y, w=8))

    return {
        "title": "MI355X GPU stats (kube_gpu_stats_amd)",
        "uid": "kgs-mi355x",
        "schemaVersion": 39,
        "version": 1,
        "time": {"from": "now-6h", "to": "now"},
        "refresh": "30s",
        "tags": ["amd", "mi355x", "gpu"],
        "templating": {"list": [
            {"name": "datasource", "type": "datasource", "query": "prometheus"},
            {"name": "node", "type": "query", "datasource": {"type": "prometheus", "uid": "${datasource}"},
             "query": "label_values(amdgpu_device_info, kubernetes_io_hostname)", "includeAll": True,
             "multi": True, "current": {"text": "All", "value": "$__all"}},
        ]},
        "panels": panels,
    }


def exprs(d: dict | None = None) -> list[str]:
    d = d or build()
    return [t["expr"] for p in d["panels"] for t in p.get("targets", [])]


def render() -> str:
    return json.dumps(build(), indent=1, sort_keys=True) + "\n"


if __name__ == "__main__":
    print(render(), end="")
