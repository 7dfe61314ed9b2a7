"""What phase B's scrapes show about the load: xGMI rates against the all-reduces' bytes, window
gauges, throttle residency and the counter thread's wake-up lateness."""
from __future__ import annotations



def xgmi_rates(before: dict, after: dict, win: float) -> dict:
    """xGMI bytes/s per GPU (all links, read + write) over the timed window, from the
    exporter's PMFW per-link accumulators."""
    def tot(m):
        out: dict = {}
        for fam in ("amdgpu_xgmi_read_bytes_total", "amdgpu_xgmi_write_bytes_total"):
            for lb, v in m.get(fam, []):
                out[lb["gpu"]] = out.get(lb["gpu"], 0.0) + v
        return out
    b, a_ = tot(before), tot(after)
    return {g: round((a_[g] - b.get(g, 0.0)) / win / 1e9, 3) for g in a_} if win > 0 else {}


def allreduce_GBps(load, a, n: int, win: float):
    """xGMI bytes/s per GPU that phase B's all-reduces imply (None without them)."""
    if getattr(load, "ar", None) is None or n < 2 or win <= 0:
        return None
    size = load.ar.numel() * load.ar.element_size()
    return round(2 * 2 * (n - 1) / n * size * a.steps * load.reps / win / 1e9, 3)


def allreduce_ratio(measured: dict, expected) -> dict | None:
    """Per GPU, the xGMI bytes its link counters saw during phase B ÷ the bytes its
    all-reduces must have moved (None without all-reduces)."""
    if not expected:
        return None
    return {g: round(v / expected, 4) for g, v in measured.items()}


def observed(m: dict) -> dict:
    """What the exporter saw of the load (window gauges of the last scrape), per GPU."""
    out: dict = {}
    for fam, key in (("amdgpu_gfx_busy_percent", "gfx_busy_pct"), ("amdgpu_umc_busy_percent", "umc_busy_pct"),
                     ("amdgpu_mfma_util_percent", "mfma_util_pct"), ("amdgpu_vmem_busy_percent", "vmem_busy_pct"),
                     ("amdgpu_power_watts", "power_w"), ("amdgpu_gpu_clock_effective_mhz", "clock_mhz")):
        for lb, v in m.get(fam, []):
            out.setdefault(lb["gpu"], {})[key] = round(v, 2)
    for lb, v in m.get("amdgpu_mfma_util_xcc_percent", []):  # XCD order 0..7
        out.setdefault(lb["gpu"], {}).setdefault("mfma_util_xcd_pct", []).append(round(v, 1))
    return out


def throttled(before: dict, after: dict, win: float) -> dict:
    """Per GPU and throttler, % of the timed window the GPU ran held back
    (amdgpu_throttle_seconds_total deltas; reason="ppt" is the package-power cap)."""
    out: dict = {}
    if win <= 0:
        return out
    b = {(lb["gpu"], lb["reason"]): v for lb, v in before.get("amdgpu_throttle_seconds_total", [])}
    for lb, v in after.get("amdgpu_throttle_seconds_total", []):
        d = v - b.get((lb["gpu"], lb["reason"]), v)
        if d > 0:
            out.setdefault(lb["gpu"], {})[lb["reason"]] = round(100.0 * d / win, 2)
    return out


def wake_lateness(before: dict, after: dict) -> dict:
    """Per GPU, how late the counter thread woke against its tick deadlines during
    phase B (kgs_sampler_wake_lateness_seconds deltas): the box's CPU contention,
    which is what makes phase B fall short of the nominal rate on some boxes."""
    out: dict = {}
    fam = "kgs_sampler_wake_lateness_seconds"
    b = {(lb["gpu"], lb["le"]): v for lb, v in before.get(fam + "_bucket", [])}
    buckets: dict = {}
    for lb, v in after.get(fam + "_bucket", []):
        le = float("inf") if lb["le"] == "+Inf" else float(lb["le"])
        buckets.setdefault(lb["gpu"], []).append((le, v - b.get((lb["gpu"], lb["le"]), 0.0)))
    sums = {lb["gpu"]: v for lb, v in after.get(fam + "_sum", [])}
    sums0 = {lb["gpu"]: v for lb, v in before.get(fam + "_sum", [])}
    for g, bl in buckets.items():
        bl.sort()
        n = bl[-1][1] if bl else 0
        if n <= 0:
            continue
        le = lambda t: max((c for x, c in bl if x <= t + 1e-12), default=0.0)  # noqa: E731  cumulative ≤ t
        out[g] = {"ticks": int(n), "share_within_10us": round(le(10e-6) / n, 4),
                  "share_within_100us": round(le(100e-6) / n, 4), "share_over_500us": round(1 - le(500e-6) / n, 5),
                  "share_over_2500us": round(1 - le(2500e-6) / n, 5),
                  "mean_us": round(1e6 * (sums.get(g, 0.0) - sums0.get(g, 0.0)) / n, 2)}
    return out
