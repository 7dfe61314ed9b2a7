#!/usr/bin/env python3
"""Replay raw counter READs through busy-estimator variants (offline, CPU).

Input: ``tools/cp_busy_probe.py --dump`` output — every READ of [GRBM_COUNT,
GRBM_SPI_BUSY, CPC busy, CPF busy] (max over XCCs) during known loads, with the
loads' event-timed GPU busy.  Each variant turns the READ intervals into a busy
integral the way the sampler's dispatch integral does (``sampler.cpp``, the
``dispatch_seconds`` block) and is scored against the kernels' own duty:

* ``shipped``  — the sampler from r4g: the whole interval if CPC busy ≥ 90 % of the
  clocks, else max(SPI − the READ's SPI blip, CPC − the READ's CP cost), share × Δt;
  both READ costs learned on every READ-only interval (SPI < 2 % of the clocks); from
  r4q a partial interval ≥ 400 µs long is split by the learned busy / idle clocks
  (share s → s·r / (1 − s + s·r), r = f_idle / f_busy);
* ``r4b``      — the same with a 97 % full threshold, no SPI-blip removal, and the READ
  cost learned only where SPI < 0.5 % of the clocks (rounds r4b–r4f: at 8 kHz that kept
  2 % of the READ-only intervals, the cheap ones);
* ``overlap``  — ``shipped``, but the READ's CP time counted once where it overlaps
  dispatch busy: busy = (CPC − r) / (1 − r/clk);
* ``timesplit``— ``shipped``, but busy time = Δt − idle cycles / idle clock, with the
  idle clock learned on READ-only intervals (cycle shares are clock-weighted: a burst
  under the power cap runs at a lower clock than the idle stretch around it).

``python tools/util_estimator_sim.py profiles/r4/r4e/cp_dump.json``
"""
from __future__ import annotations

import json
import sys

FULL = 0.90


def intervals(samples):
    for a, b in zip(samples, samples[1:]):
        dt = b[0] - a[0]
        clk = b[1] - a[1]
        if dt <= 0 or clk <= 0:
            continue
        yield dt, clk, max(0, b[2] - a[2]), max(0, b[3] - a[3])


QUIET_SPI = 0.02  # the sampler's kQuietActiveFrac: a READ alone shows ≈0.9 µs of SPI busy


def learn_read(ivs, quiet_spi: float = QUIET_SPI) -> tuple[float, float, float]:
    """READ cost in CPC cycles and in SPI cycles (means over intervals without waves
    and with the CP mostly idle) and the idle clock (cycles / s over the same)."""
    cyc, spi_c, clk_s, n = 0.0, 0.0, 0.0, 0
    for dt, clk, spi, cpc in ivs:
        if spi < quiet_spi * clk and cpc < 0.5 * clk:
            cyc += cpc
            spi_c += spi
            clk_s += clk / dt
            n += 1
    return (cyc / n, spi_c / n, clk_s / n) if n else (0.0, 0.0, 0.0)


def estimate(ivs, learned, variant: str) -> float:
    read_cyc, read_spi, idle_hz = learned
    full = 0.97 if variant == "r4b" else FULL
    if variant == "r4b":
        read_spi = 0.0
    tot, span = 0.0, 0.0
    f_busy, f_idle = 0.0, 0.0
    for dt, clk, spi, cpc in ivs:
        span += dt
        wav = max(0.0, spi - read_spi)  # the READ's own SPI blip is not a wave of the workload
        if spi < QUIET_SPI * clk and cpc < 0.5 * clk:
            f_idle = 0.95 * f_idle + 0.05 * clk / dt if f_idle else clk / dt
        if cpc >= full * clk:
            f_busy = 0.95 * f_busy + 0.05 * clk / dt if f_busy else clk / dt
            tot += dt
            continue
        if variant == "overlap":
            r = min(read_cyc, 0.5 * clk)
            busy = max(wav, max(0.0, (cpc - r) / (1.0 - r / clk)))
        else:
            busy = max(wav, max(0.0, cpc - read_cyc))
        if variant == "timesplit" and idle_hz > 0:
            tot += min(dt, max(0.0, dt - (clk - busy) / idle_hz))
        else:
            s = min(1.0, busy / clk)
            if variant == "shipped" and dt >= 400e-6 and s > 0 and f_busy and f_idle:
                r = min(1.1, max(0.9, f_idle / f_busy))
                s = s * r / (1.0 - s + s * r)
            tot += s * dt
    return 100.0 * tot / span if span else 0.0


def main(argv=None) -> int:
    path = (argv or sys.argv[1:])[0]
    d = json.load(open(path))
    out = {}
    for rate, loads in d["rates"].items():
        quiet = list(intervals(loads.get("idle", {}).get("samples", [])))
        learned = {"r4b": learn_read(quiet, 0.005), "shipped": learn_read(quiet)}
        rows = {f"read_us_{k}": round(1e6 * v[0] / v[2], 2) if v[2] else None for k, v in learned.items()}
        rows["read_spi_us"] = round(1e6 * learned["shipped"][1] / learned["shipped"][2], 3) if learned["shipped"][2] else None
        rows["idle_clock_mhz"] = round(learned["shipped"][2] / 1e6, 1)
        for name, L in loads.items():
            ivs = list(intervals(L["samples"]))
            if not ivs:
                continue
            wall = L["t1"] - L["t0"]
            row = {"duty_gpu_pct": round(100 * L["duty_gpu_s"] / wall, 2),
                   "busy_clock_mhz": round(sum(c for _, c, _, _ in ivs) / sum(t for t, _, _, _ in ivs) / 1e6, 1)}
            for v in ("shipped", "r4b", "overlap", "timesplit"):
                row[v] = round(estimate(ivs, learned["r4b" if v == "r4b" else "shipped"], v), 2)
            rows[name] = row
        out[rate] = rows
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
