"""``kgs dmon`` — live per-GPU view of one node exporter (an ``rocm-smi`` /
``nvidia-smi dmon`` analogue that needs no driver access on the caller's side).

The reference only looks at GPUs through Prometheus, after the fact
(gpu_util_stats.py:159) or as an allocation census (who_use_gpu.py:7-25).  This
reads one exporter directly: every ``--interval`` it scrapes ``/metrics`` and
prints one row per GPU.  Rates (xGMI and PCIe bytes/s, average power from the
energy counter) come from counter deltas between two polls.  With ``--counters`` it
also drains the full-rate counter stream (``/counters?since=``) and reports
the min / max of per-drain MFMA utilisation, the number of busy bursts and the
exact busy duty cycle inside each interval (``segments``).  At an 8 kHz tick
that exposes bursts the 1 s window gauges average away.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import urllib.parse
import urllib.request

from ..utils.scrape import Scraper, parse_text

COLS = [("gpu", "GPU", 3), ("pod", "POD", 18), ("gfx", "GFX%", 5), ("mfma", "MFMA%", 5), ("vmem", "VMEM%", 5),
        ("umc", "UMC%", 5), ("hbm_gb", "HBM_GB", 7), ("hbm_pct", "HBM%", 5), ("power_w", "PWR_W", 6),
        ("energy_w", "AVG_W", 6), ("temp_c", "TEMP", 4), ("clk_mhz", "MHZ", 5), ("xgmi_gbps", "XGMI_GB/s", 9),
        ("pcie_gbps", "PCIE_GB/s", 9), ("ppt_pct", "PVIOL%", 6), ("pmc", "PMC", 5), ("xcd_mfma", "MFMA%_PER_XCD", 31)]
BURST_COLS = [("mfma_min", "MFMA_MIN", 8), ("mfma_max", "MFMA_MAX", 8), ("bursts", "BURSTS", 6),
              ("duty", "DUTY%", 5), ("drains", "DRAINS", 6)]


def segments(samples: list[dict], key: str = "gpu_active_pct", hi: float = 60.0,
             lo: float = 20.0) -> tuple[list[tuple[int, int]], float, float]:
    """Busy segments of a full-rate counter stream (``/counters`` samples, oldest
    first, each covering ``dt_us`` up to its ``mono_ns``).

    Returns ``(segments, busy_s, span_s)``: the ``[start_ns, end_ns)`` runs where
    ``key`` rose to ≥ ``hi`` and had not yet fallen to ≤ ``lo`` (hysteresis, so a
    burst that straddles a drain boundary is one segment), the exact busy integral
    Σ key/100 · dt over the samples, and the time they span.  At an 8 kHz drain
    rate a 1 ms kernel is ~8 drains: the stream resolves each burst, where the
    ≈50 Hz PMFW table only sees their average."""
    segs: list[tuple[int, int]] = []
    busy = span = 0.0
    start = None
    for x in samples:
        if key not in x or "dt_us" not in x:
            continue
        v, dt_ns = float(x[key]), float(x["dt_us"]) * 1e3
        t1 = int(x["mono_ns"])
        t0 = int(t1 - dt_ns)
        busy += v * 0.01 * dt_ns * 1e-9
        span += dt_ns * 1e-9
        if start is None and v >= hi:
            start = t0
        elif start is not None and v <= lo:
            segs.append((start, t0))
            start = None
    if start is not None and samples:
        segs.append((start, int(samples[-1]["mono_ns"])))
    return segs, busy, span


def _by_gpu(m: dict, fam: str, **match) -> dict[str, float]:
    out: dict[str, float] = {}
    for lb, v in m.get(fam, []):
        if all(lb.get(k) == want for k, want in match.items()) and "gpu" in lb:
            out[lb["gpu"]] = v
    return out


def _sum_by_gpu(m: dict, *fams: str) -> dict[str, float]:
    out: dict[str, float] = {}
    for fam in fams:
        for lb, v in m.get(fam, []):
            if "gpu" in lb:
                out[lb["gpu"]] = out.get(lb["gpu"], 0.0) + v
    return out


def _pods(m: dict) -> dict[str, str]:
    """GPU → pod: the reference-compatible series first, else the pods of its processes."""
    pods: dict[str, set] = {}
    for lb, _ in m.get("container_gpu_sm_util", []):
        if lb.get("pod_name"):
            pods.setdefault(lb.get("gpu", ""), set()).add(f"{lb.get('namespace', '')}/{lb['pod_name']}".lstrip("/"))
    for lb, _ in m.get("amdgpu_process_hbm_bytes", []):
        if lb.get("pod") and lb.get("gpu") not in pods:
            pods.setdefault(lb["gpu"], set()).add(f"{lb.get('namespace', '')}/{lb['pod']}".lstrip("/"))
    return {g: ",".join(sorted(p)) for g, p in pods.items()}


def _xcd_split(m: dict, fam: str) -> dict[str, str]:
    """GPU → per-XCD values as "a/b/c/..." in XCD order (MI355X: 8)."""
    per: dict[str, dict[int, float]] = {}
    for lb, v in m.get(fam, []):
        if "gpu" in lb and lb.get("xcc", "").isdigit():
            per.setdefault(lb["gpu"], {})[int(lb["xcc"])] = v
    return {g: "/".join(f"{x[k]:.0f}" for k in sorted(x)) for g, x in per.items()}


def pmc_state(m: dict) -> dict[str, str]:
    """The counter tier per GPU, as one word: ``fail`` (breaker open), ``park`` (released
    by the quiet release), ``off`` (handed over / not configured), ``quiet`` (no wave:
    READ at the idle rate), ``dbnd`` (dispatch-bound: READ at the dispatch rate), ``on``."""
    out = {}
    for g, on in _by_gpu(m, "kgs_pmc_enabled").items():
        if _by_gpu(m, "kgs_pmc_failed").get(g):
            out[g] = "fail"
        elif _by_gpu(m, "kgs_pmc_parked").get(g):
            out[g] = "park"
        elif not on:
            out[g] = "off"
        elif _by_gpu(m, "kgs_pmc_quiet").get(g):
            out[g] = "quiet"
        elif _by_gpu(m, "kgs_pmc_dispatch_bound").get(g):
            out[g] = "dbnd"
        else:
            out[g] = "on"
    return out


def rows_from(prev: dict | None, cur: dict, dt: float) -> list[dict]:
    """One row per GPU from a scrape (and the previous one, for rates)."""
    gfx = _by_gpu(cur, "amdgpu_gfx_busy_percent")
    mfma = _by_gpu(cur, "amdgpu_mfma_util_percent")
    vmem = _by_gpu(cur, "amdgpu_vmem_busy_percent")
    umc = _by_gpu(cur, "amdgpu_umc_busy_percent")
    used = _by_gpu(cur, "amdgpu_hbm_used_bytes")
    total = _by_gpu(cur, "amdgpu_hbm_total_bytes")
    power = _by_gpu(cur, "amdgpu_power_watts")
    temp = _by_gpu(cur, "amdgpu_temperature_celsius", sensor="hotspot")
    clk = _by_gpu(cur, "amdgpu_gpu_clock_effective_mhz") or _by_gpu(cur, "amdgpu_clock_mhz", clock="gfx")
    energy = _by_gpu(cur, "amdgpu_energy_joules_total")
    xgmi = _sum_by_gpu(cur, "amdgpu_xgmi_read_bytes_total", "amdgpu_xgmi_write_bytes_total")
    pcie = _by_gpu(cur, "amdgpu_pcie_bytes_total")
    ppt = _by_gpu(cur, "amdgpu_throttle_seconds_total", reason="ppt")
    pppt = _by_gpu(prev, "amdgpu_throttle_seconds_total", reason="ppt") if prev else {}
    ppcie = _by_gpu(prev, "amdgpu_pcie_bytes_total") if prev else {}
    penergy = _by_gpu(prev, "amdgpu_energy_joules_total") if prev else {}
    pxgmi = _sum_by_gpu(prev, "amdgpu_xgmi_read_bytes_total", "amdgpu_xgmi_write_bytes_total") if prev else {}
    pods = _pods(cur)
    xcd = _xcd_split(cur, "amdgpu_mfma_util_xcc_percent")
    pmc = pmc_state(cur)
    gpus = sorted(set(gfx) | set(used) | set(power), key=lambda g: int(g) if g.isdigit() else 0)
    rows = []
    for g in gpus:
        r = {"gpu": g, "pod": pods.get(g, "-"), "gfx": gfx.get(g), "mfma": mfma.get(g), "vmem": vmem.get(g),
             "umc": umc.get(g), "hbm_gb": used[g] / 1e9 if g in used else None,
             "hbm_pct": 100.0 * used[g] / total[g] if total.get(g) and g in used else None,
             "power_w": power.get(g), "temp_c": temp.get(g), "clk_mhz": clk.get(g), "energy_w": None,
             "xgmi_gbps": None, "pcie_gbps": None, "ppt_pct": None, "pmc": pmc.get(g, "-"), "xcd_mfma": xcd.get(g)}
        if dt > 0 and g in penergy and g in energy and energy[g] >= penergy[g]:
            r["energy_w"] = (energy[g] - penergy[g]) / dt
        if dt > 0 and g in pxgmi and g in xgmi and xgmi[g] >= pxgmi[g]:
            r["xgmi_gbps"] = (xgmi[g] - pxgmi[g]) / dt / 1e9
        if dt > 0 and g in ppcie and g in pcie and pcie[g] >= ppcie[g]:
            r["pcie_gbps"] = (pcie[g] - ppcie[g]) / dt / 1e9
        if dt > 0 and g in pppt and g in ppt and ppt[g] >= pppt[g]:
            r["ppt_pct"] = 100.0 * (ppt[g] - pppt[g]) / dt  # package-power throttling (amdsmi PVIOL)
        rows.append(r)
    return rows


def _fmt(v, width: int) -> str:
    if v is None:
        s = "-"
    elif isinstance(v, str):
        s = v if len(v) <= width else v[: width - 1] + "~"
    elif abs(v) >= 100 or float(v).is_integer():
        s = f"{v:.0f}"
    else:
        s = f"{v:.1f}"
    return s.rjust(width)


def format_rows(rows: list[dict], cols) -> list[str]:
    return [" ".join(_fmt(r.get(k), w) for k, _, w in cols) for r in rows]


def header(cols) -> str:
    return " ".join(h.rjust(w) for _, h, w in cols)


class CounterStream:
    """Incremental reader of ``/counters?gpu=N&since=SEQ`` for every GPU."""

    def __init__(self, base: str):
        self.base = base.rstrip("/")
        self.since: dict[str, int] = {}

    def poll(self, gpus: list[str]) -> dict[str, dict]:
        out = {}
        for g in gpus:
            since = self.since.get(g, 0)
            url = f"{self.base}/counters?gpu={g}&" + (f"since={since}" if since else "n=1")
            body = json.loads(urllib.request.urlopen(url, timeout=5).read())
            s = body.get("samples", [])
            if s:
                self.since[g] = s[-1]["seq"]
            vals = [x["mfma_util_pct"] for x in s if "mfma_util_pct" in x]
            segs, busy, span = segments(s) if since else ([], 0.0, 0.0)
            out[g] = {"mfma_min": min(vals) if vals else None, "mfma_max": max(vals) if vals else None,
                      "bursts": len(segs) if since else None,
                      "duty": 100.0 * busy / span if span > 0 else None,
                      "drains": len(s) if since else None}
        return out


def build_parser(ap: argparse.ArgumentParser | None = None) -> argparse.ArgumentParser:
    ap = ap or argparse.ArgumentParser(prog="kgs dmon", description=__doc__.splitlines()[0])
    ap.add_argument("url", nargs="?", default="http://127.0.0.1:9400", help="exporter base URL")
    ap.add_argument("--interval", type=float, default=1.0, help="seconds between rows")
    ap.add_argument("--count", type=int, default=0, help="stop after N polls (0 = until interrupted)")
    ap.add_argument("--counters", action="store_true",
                    help="also drain the full-rate counter stream: min/max MFMA%% per interval")
    ap.add_argument("--json", action="store_true", help="one JSON object per GPU per poll")
    return ap


def run(a, out=sys.stdout) -> int:
    u = urllib.parse.urlsplit(a.url if "://" in a.url else "http://" + a.url)
    base = f"{u.scheme}://{u.netloc}"
    sc = Scraper(u.hostname or "127.0.0.1", u.port or 80)
    stream = CounterStream(base) if a.counters else None
    cols = COLS + (BURST_COLS if a.counters else [])
    prev, t_prev = None, 0.0
    n = 0
    try:
        while a.count <= 0 or n < a.count:
            t = time.monotonic()
            cur = parse_text(sc.scrape_once())
            rows = rows_from(prev, cur, t - t_prev if prev else 0.0)
            if stream is not None:
                burst = stream.poll([r["gpu"] for r in rows])
                for r in rows:
                    r.update(burst.get(r["gpu"], {}))
            if a.json:
                for r in rows:
                    out.write(json.dumps({"t": time.time(), **r}) + "\n")
            else:
                if n % 20 == 0:
                    out.write(header(cols) + "\n")
                out.write("\n".join(format_rows(rows, cols)) + "\n")
            out.flush()
            prev, t_prev = cur, t
            n += 1
            if a.count <= 0 or n < a.count:
                time.sleep(max(0.0, a.interval - (time.monotonic() - t)))
    except KeyboardInterrupt:
        pass
    return 0
