"""Phase S — how far the counter tier goes past the primary rate."""
from __future__ import annotations

import time

from .common import scrape_at, timed
from .exporter import Rates


def capacity(ctx, load, exp, a) -> dict:
    """Phase S — how far the counter tier goes past the primary rate (untimed).  Under the
    same load, one ``--block-steps`` block at each ``--capacity-hz`` rate: delivered
    counter drains per GPU, the worst GPU's share of nominal, overruns per second and
    host µs per drain.  ``max_rate_hz_98pct`` is the highest rate tried (the primary one
    included) at which every GPU delivered ≥ 98 %: the headroom behind the headline
    number, which is the configured tick rate delivered."""
    rates = [float(x) for x in str(a.capacity_hz).split(",") if x.strip()]
    if not rates:
        return {}
    out: dict = {"block_steps": a.block_steps, "mode": "profiling (--pmc-idle-hz 0: every tick READs)",
                 "rates": {}}
    best = None
    # Profiling mode: a GPU idle at a block edge would otherwise be READ at the idle
    # rate until its first busy READ, which is the adaptive rate at work, not capacity.
    idle_hz = exp.set_idle_hz(-1) if exp is not None else 0.0
    if exp is not None:
        exp.set_idle_hz(0)
    for hz in [a.hz] + [r for r in rates if r != a.hz]:
        w0 = 0.0
        before: dict = {}
        if exp is not None:
            exp.set_rate(hz)
            time.sleep(0.05)
            before, w0 = scrape_at(exp.sc)
        dt = timed(ctx, load, a.block_steps)
        if exp is None:
            continue
        after, w1 = scrape_at(exp.sc)
        win = w1 - w0
        r = Rates()
        r.add(before, after, win)
        pg, src = r.per_gpu(exp.ready.get("pmc", "none") != "none")

        def delta(fam):
            b = {lb["gpu"]: v for lb, v in before.get(fam, [])}
            return {lb["gpu"]: v - b.get(lb["gpu"], 0.0) for lb, v in after.get(fam, [])}

        ov, rs = delta("kgs_sampler_overruns_total"), delta("kgs_pmc_read_seconds_total")
        worst = min(pg.values()) / hz if pg else 0.0
        out["rates"][f"{hz:g}"] = {
            "samples_per_sec_per_gpu": {g: round(v, 1) for g, v in pg.items()}, "sample_source": src,
            "worst_gpu_pct_of_nominal": round(100 * worst, 2),
            "overruns_per_s_per_gpu": round(sum(ov.values()) / max(1, len(ov)) / win, 1) if win > 0 else None,
            "host_us_per_drain": round(1e6 * sum(rs.values()) / max(1.0, sum(r.pmc.values())), 2),
            "block_s": round(dt, 4)}
        if worst >= 0.98:
            best = hz if best is None else max(best, hz)
    if exp is not None:
        exp.set_rate(a.hz)
        exp.set_idle_hz(idle_hz)
    out["max_rate_hz_98pct"] = best
    return out
