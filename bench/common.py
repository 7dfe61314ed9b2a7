"""Shared pieces of the benchmark: repo paths, the metric name, statistics (95 % t-intervals), the
barrier-bracketed timed regions and the scrape helper every phase uses."""
from __future__ import annotations

import math
import os
import socket
import sys
import time

from kube_gpu_stats_amd.parallel import dist as D
from kube_gpu_stats_amd.utils.scrape import parse_text


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


METRIC = "counter samples/sec/GPU + p50 scrape latency at 8×MI355X; GPU-time overhead %"


PMC_READER = "aqlprofile"  # direct CP reads (native/counters/pmc_aqlprofile.cpp)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


T975 = {1: 12.706, 2: 4.303, 3: 3.182, 4: 2.776, 5: 2.571, 6: 2.447, 7: 2.365, 8: 2.306, 9: 2.262, 10: 2.228,
        11: 2.201, 12: 2.179, 13: 2.160, 14: 2.145, 15: 2.131, 16: 2.120, 17: 2.110, 18: 2.101, 19: 2.093,
        20: 2.086, 24: 2.064, 29: 2.045, 39: 2.023, 59: 2.001}


def t975(df: int) -> float:
    """Two-sided 95 % Student-t quantile (table; 1.96 beyond 60 degrees of freedom)."""
    if df <= 0:
        return float("nan")
    for k in sorted(T975):
        if df <= k:
            return T975[k]
    return 1.96


def mean_ci95(xs: list[float]) -> tuple[float, float, float]:
    """(mean, 95 % half-width, sample SD) of paired differences."""
    n = len(xs)
    if n == 0:
        return float("nan"), float("nan"), float("nan")
    m = sum(xs) / n
    if n == 1:
        return m, float("nan"), float("nan")
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (n - 1))
    return m, t975(n - 1) * sd / math.sqrt(n), sd


def pct(xs: list[float], q: float) -> float | None:
    if not xs:
        return None
    s = sorted(xs)
    return s[min(len(s) - 1, int(q * len(s)))]


PHASES: dict[str, list[float]] = {}


def timed(ctx, load, k: int, name: str = "") -> float:
    """Barrier + sync on both sides; returns the MAX over ranks of the wall time.

    The wall-clock (epoch) bounds of each named phase are kept in PHASES so a
    rocprofv3 kernel trace of the run can be split into exporter-off / -on
    phases (tools/rocprof_overhead.py)."""
    D.barrier(ctx)
    load.sync()
    w0 = time.time()
    t0 = time.perf_counter()
    for _ in range(k):
        load.step()
    load.sync()
    D.barrier(ctx)
    dt = time.perf_counter() - t0
    if name:
        PHASES[name] = [w0, time.time()]
    return D.all_reduce(ctx, [dt], "max")[0]


def calibrate_reps(ctx, load, step_ms: float) -> tuple[int, float]:
    """Units per step so one step lasts ≥ step_ms on the slowest rank."""
    load.unit()
    load.sync()
    D.barrier(ctx)
    t0 = time.perf_counter()
    load.unit()
    load.sync()
    unit_s = D.all_reduce(ctx, [time.perf_counter() - t0], "max")[0]
    return max(1, math.ceil(step_ms * 1e-3 / max(unit_s, 1e-6))), unit_s


def timed_block(ctx, load, k: int) -> tuple[float, float]:
    """One interleaved block: (this rank's own time to finish its k steps, the time
    until every rank has — the MAX-over-ranks wall time the headline uses)."""
    D.barrier(ctx)
    load.sync()
    t0 = time.perf_counter()
    for _ in range(k):
        load.step()
    load.sync()
    own = time.perf_counter() - t0
    D.barrier(ctx)
    return own, time.perf_counter() - t0


def scrape_at(sc) -> tuple[dict, float]:
    """One /metrics scrape and the time it was rendered (the request is sent at ``t``;
    the exporter renders within ~0.1 ms).  Count deltas between two scrapes cover
    exactly the interval between their ``t``s — timing after the parse instead would
    move the window by the parse time of the page (≈10 ms per GPU's worth of series)."""
    t = time.perf_counter()
    body = sc.get()
    return parse_text(body), t


RELEASED = -1.0  # interleaved condition: counter session STOPped, READ queue destroyed, sampler paused


def cond_label(c: float) -> str:
    return "released" if c < 0 else f"{c:g}"


def _r(x, nd=3):
    return None if x is None else round(float(x), nd)


def _pm(d: dict | None, k="overhead_pct", c="overhead_ci95_pct") -> list | None:
    return [_r(d.get(k)), _r(d.get(c))] if isinstance(d, dict) and d.get(k) is not None else None


def tiers(a) -> list[float]:
    """Every tick rate measured: the primary --hz plus --hz-list, ascending."""
    extra = [float(x) for x in str(a.hz_list).split(",") if x.strip()]
    return sorted({float(a.hz), *extra})


_T0 = time.monotonic()


def progress(ctx, msg: str) -> None:
    """One line to stderr on rank 0 per phase (and per round of the long ones): a run that
    prints nothing for minutes is taken for hung by the GPU harness; stdout stays the
    driver's one result line."""
    if ctx is None or getattr(ctx, "rank", 0) == 0:
        print(f"[bench +{time.monotonic() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)
