"""Phase Q — what the exporter does to an idle GPU (READ rate, PMFW busy, SPI share)."""
from __future__ import annotations

import time

from kube_gpu_stats_amd.parallel import dist as D

from .common import scrape_at


def quiet_gpu(ctx, load, exp, a) -> dict:
    """Phase Q — what the exporter does to an idle GPU (untimed).  Every counter READ
    is a command-processor packet that the PMFW GFX busy — the source of
    container_gpu_sm_util — counts as ≈80 µs of work, so a GPU READ every tick at
    8 kHz reads ~99 % busy while idle.  With the GPU idle on every rank, rank 0
    reads from the exporter's own counters, per GPU: the READ rate, the PMFW GFX
    busy (exact, from amdgpu_gfx_busy_seconds_total) and the SPI-busy share of
    clocks, first in the default adaptive mode (a quiet GPU is READ at
    --pmc-idle-hz) and then in profiling mode (every tick) for contrast."""
    if a.quiet_s <= 0:
        return {}
    D.barrier(ctx)
    load.sync()  # the barrier's own kernel is done: every GPU is idle from here
    out: dict = {}
    if exp is not None:
        default_idle = exp.set_idle_hz(-1)  # hz < 0 only reads the setting
        for mode, hz in (("adaptive", default_idle), ("profiling", 0.0)):
            exp.set_idle_hz(hz)
            time.sleep(0.2)
            m0, t0 = scrape_at(exp.sc)
            time.sleep(a.quiet_s)
            m1, t1 = scrape_at(exp.sc)
            dt = t1 - t0
            fam = lambda m, n, **kw: {lb["gpu"]: v for lb, v in m.get(n, [])  # noqa: E731
                                      if all(lb.get(k) == w for k, w in kw.items())}
            r0, r1 = fam(m0, "kgs_pmc_samples_total"), fam(m1, "kgs_pmc_samples_total")
            g0, g1 = fam(m0, "amdgpu_gfx_busy_seconds_total"), fam(m1, "amdgpu_gfx_busy_seconds_total")
            c0, c1 = fam(m0, "amdgpu_pmc_total", counter="GRBM_COUNT"), fam(m1, "amdgpu_pmc_total", counter="GRBM_COUNT")
            s0, s1 = (fam(m0, "amdgpu_pmc_total", counter="GRBM_SPI_BUSY"),
                      fam(m1, "amdgpu_pmc_total", counter="GRBM_SPI_BUSY"))
            out[mode] = {"pmc_idle_hz": hz, "per_gpu": {
                g: {"reads_per_s": round((r1[g] - r0.get(g, 0)) / dt, 1),
                    "pmfw_gfx_busy_pct": round(100 * (g1.get(g, 0) - g0.get(g, 0)) / dt, 3),
                    "gpu_active_pct": (round(100 * (s1[g] - s0.get(g, 0)) / (c1[g] - c0.get(g, 0)), 3)
                                       if g in s1 and g in c1 and c1[g] > c0.get(g, 0) else None)}
                for g in sorted(r1, key=int)}}
        exp.set_idle_hz(default_idle)
    D.cpu_barrier(ctx)  # the other ranks wait here without a spinning RCCL kernel on their GPUs
    return out
