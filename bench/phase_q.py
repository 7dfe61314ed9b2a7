"""Phase Q — what the exporter does to an idle GPU (READ rate, PMFW busy, SPI share), and
phase P — what its counter session costs that GPU in socket power."""
from __future__ import annotations

import statistics
import time

from kube_gpu_stats_amd.parallel import dist as D

from .common import mean_ci95, progress, scrape_at
from .exporter import PmfwProbe


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


class MockPowerProbe:
    """PmfwProbe's interface for --mock runs: a 250 W idle socket on the host clock."""

    N = True

    def read(self) -> dict:
        t = time.monotonic()
        return {"fw_ts": int(t * 1e8), "energy_acc": int(250.0 * t * 65536.0), "accumulation_counter": int(t * 1e3),
                "ppt_residency_acc": 0}


def idle_power(ctx, load, exp, a) -> dict:
    """Phase P (untimed) — what the counter session costs an idle GPU in power, and what
    the quiet release saves.  With every rank's GPU idle, three
    conditions in blocks of --idle-power-s / --idle-power-rounds each, the block order
    cycling through every permutation:

    * ``session``  — the counter session programmed and the quiet GPU READ at
      --pmc-idle-hz (the exporter as rounds 1-5 shipped it: quiet release off);
    * ``released`` — the session STOPped and the READ queue destroyed while the PMFW and
      slow tiers keep sampling (the neutral base);
    * ``parked``   — the exporter's quiet release (--pmc-quiet-release-s, here 1 s)
      having released the session by itself;
    * ``absent``   — (--idle-power-absent 1) released and every sampling tier paused:
      nothing of the exporter touches the GPU.  Four conditions run in a Williams
      square (each order of neighbours once per four rounds).

    Each rank reads its own GPU's socket power from the PMFW energy accumulator at the
    block edges and halfway (PmfwProbe, not the exporter); per round, each condition is
    paired with that round's ``released`` block: mean ± 95 % CI
    (``summary.quiet_gpu.power_w``), and the same over the blocks' second halves
    (``late``).  An idle MI355X sits at one of two levels, ≈291 W or ≈257 W (r6h), and
    drops to the low one only ≈5 s after its last GPU work: measuring 1 s after the
    switch (r6b-r6g) billed that lag to whichever condition followed the session, so
    each block now starts --idle-power-settle-s after the switch.  A released GPU also
    leaves the low level by itself now and then (r6i: 2 of 12 blocks, each with a
    0.005 % PMFW busy blip that is not the exporter's), so the level difference is the
    median of the paired second halves (``*_minus_released_median_w``), and the floor —
    each condition's lowest settled block — against released's (``*_floor_w``)."""
    secs = float(getattr(a, "idle_power_s", 0.0) or 0.0)
    rounds = int(getattr(a, "idle_power_rounds", 6) or 0)
    if secs <= 0 or rounds <= 0:
        return {}
    import itertools

    block = secs / rounds
    # --mock: no power level to wait for
    settle = min(1.0, 0.2 * block) if a.mock else float(getattr(a, "idle_power_settle_s", 6.0))
    # --mock: the orchestration on CPU (every rank, every barrier), against a constant
    # synthetic socket power — no power number of a mock run means anything
    probe = MockPowerProbe() if a.mock else PmfwProbe(load.pci_bdf(ctx.local_rank))
    # every rank skips or none does: a rank leaving early would strand the others in a barrier
    if not all(D.all_gather_object(ctx, probe.N is not None)):
        return {"skipped": "no PMFW table probe on some rank"}
    if int(getattr(a, "idle_power_absent", 0) or 0):
        conds: tuple = ("session", "released", "parked", "absent")
        perms = [("session", "released", "absent", "parked"), ("released", "parked", "session", "absent"),
                 ("parked", "absent", "released", "session"), ("absent", "session", "parked", "released")]
    else:
        conds = ("session", "released", "parked")
        perms = list(itertools.permutations(conds))
    paused = False
    D.cpu_barrier(ctx)
    load.sync()
    default_qr = exp.set_quiet_release(-1) if ctx.local_rank == 0 and exp is not None else 0.0
    local: list[dict] = []
    blocks: list[dict] = []  # rank 0: the exporter's side of each block
    parked_ok = True
    for r in range(rounds):
        row: dict = {}
        progress(ctx, f"phase P round {r + 1}/{rounds}")
        for cond in perms[r % len(perms)]:
            if ctx.local_rank == 0 and exp is not None:
                if paused:
                    exp.resume()
                    paused = False
                if cond in ("released", "absent"):
                    exp.set_quiet_release(0)
                    exp.release(drop_queue=True)
                    if cond == "absent":
                        exp.pause()
                        paused = True
                elif cond == "session":
                    exp.set_quiet_release(0)
                    exp.acquire()
                else:
                    exp.set_quiet_release(1.0)
                    exp.acquire()
                    parked_ok &= exp.wait_parked(1.0 if a.mock else 10.0)
            D.cpu_barrier(ctx)
            time.sleep(settle)  # the power-state change after the switch
            m0 = scrape_at(exp.sc)[0] if ctx.local_rank == 0 and exp is not None else None
            p0 = probe.read()
            time.sleep(0.5 * block)
            pm = probe.read()
            time.sleep(0.5 * block)
            p1 = probe.read()
            row[cond] = PmfwProbe.delta(p0, p1)
            # the block's halves: a power state still settling after the switch shows here
            halves = [(PmfwProbe.delta(p0, pm) or {}).get("power_w"), (PmfwProbe.delta(pm, p1) or {}).get("power_w")]
            if row[cond] is not None:
                row[cond]["late_w"] = halves[1]
            if m0 is not None:  # what the exporter did in the block: parks, READs, PMFW busy
                m1 = scrape_at(exp.sc)[0]
                tot = lambda m, f: sum(v for _, v in m.get(f, []))  # noqa: E731
                blocks.append({"round": r, "cond": cond, "parks": tot(m1, "kgs_pmc_parks_total") - tot(m0, "kgs_pmc_parks_total"),
                               "reads_per_s": round((tot(m1, "kgs_pmc_samples_total") - tot(m0, "kgs_pmc_samples_total")) / block, 1),
                               "pmfw_busy_pct": round(100 * (tot(m1, "amdgpu_pmfw_gfx_busy_seconds_total")
                                                              - tot(m0, "amdgpu_pmfw_gfx_busy_seconds_total")) / block, 3),
                               "parked_at_end": tot(m1, "kgs_pmc_parked"),
                               "power_w": [None if w is None else round(w, 2) for w in halves],
                               "probe_gfx_busy_pct": (None if row[cond] is None or "gfx_busy_pct" not in row[cond]
                                                      else round(row[cond]["gfx_busy_pct"], 4))})
            D.cpu_barrier(ctx)
        local.append(row)
    if ctx.local_rank == 0 and exp is not None:
        if paused:
            exp.resume()
        exp.set_quiet_release(default_qr)
        exp.acquire()
    ranks = D.all_gather_object(ctx, local)
    per_rank = []
    for rk in ranks:
        one: dict = {}
        for cond in conds:
            ws = [rd[cond]["power_w"] for rd in rk if rd.get(cond)]
            if ws:
                one[f"{cond}_w"] = round(sum(ws) / len(ws), 2)
        for cond in (c for c in conds if c != "released"):
            for key, tag in (("power_w", ""), ("late_w", "late_")):
                d = [rd[cond][key] - rd["released"][key] for rd in rk
                     if rd.get(cond) and rd.get("released") and rd[cond].get(key) is not None
                     and rd["released"].get(key) is not None]
                if d:
                    m, ci, sd = mean_ci95(d)
                    one[f"{cond}_minus_released_{tag}w"] = [round(m, 3), round(ci, 3)]
                    if tag:  # the level: robust to a block caught in a stray excursion (r6i)
                        one[f"{cond}_minus_released_median_w"] = round(statistics.median(d), 3)
        # ... and the floor: each condition's lowest settled block.  The platform's own
        # excursions (≈ once per 30 s, r6l / r6t) only ever raise a block, and caught half
        # the parked blocks in r6x, where even the median moved; the floor is the level a
        # condition holds when nothing else wakes the GPU.
        floor = {c: min((rd[c]["late_w"] for rd in rk if rd.get(c) and rd[c].get("late_w") is not None),
                        default=None) for c in conds}
        for cond in (c for c in conds if c != "released"):
            if floor.get(cond) is not None and floor.get("released") is not None:
                one[f"{cond}_minus_released_floor_w"] = round(floor[cond] - floor["released"], 3)
        per_rank.append(one)
    out = {"secs_per_condition": secs, "rounds": rounds, "block_s": round(block, 2), "settle_s": settle,
           "parked_reached": parked_ok,
           "conditions": {"session": "counter session programmed, quiet GPU READ at --pmc-idle-hz, no quiet release",
                          "released": "session STOPped and READ queue destroyed; PMFW / slow tiers sampling",
                          "parked": "the exporter's quiet release (1 s here) released the session by itself",
                          "absent": "released, and every sampling tier paused"},
           "per_rank": per_rank, "blocks": blocks}
    for cond in conds:
        bl = [b for b in blocks if b["cond"] == cond]
        if bl:
            out.setdefault("exporter_by_condition", {})[cond] = {
                "parks_per_block": round(sum(b["parks"] for b in bl) / len(bl), 2),
                "reads_per_s": round(sum(b["reads_per_s"] for b in bl) / len(bl), 1),
                "pmfw_busy_pct": round(sum(b["pmfw_busy_pct"] for b in bl) / len(bl), 3)}
    for cond in (c for c in conds if c != "released"):
        for k in (f"{cond}_minus_released_w", f"{cond}_minus_released_late_w"):
            vals = [p[k] for p in per_rank if k in p]
            if vals:
                out[k] = [round(sum(v[0] for v in vals) / len(vals), 3), round(max(v[1] for v in vals), 3)]
        for k in (f"{cond}_minus_released_median_w", f"{cond}_minus_released_floor_w"):
            vals = [p[k] for p in per_rank if k in p]
            if vals:
                out[k] = round(statistics.median(vals), 3)
    return out
