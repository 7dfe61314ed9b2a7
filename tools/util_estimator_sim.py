#!/usr/bin/env python3
"""Replay raw counter READs through busy-estimator variants (offline, CPU).

Input: ``tools/cp_busy_probe.py --dump`` output — every READ of [GRBM_COUNT,
GRBM_SPI_BUSY, CPC busy, CPF busy] (max over XCCs) during known loads, with the
loads' event-timed GPU busy.  Each variant turns the READ intervals into a busy
integral the way the sampler's dispatch integral does (``sampler.cpp``, the
``dispatch_seconds`` block) and is scored against the kernels' own duty:

* ``subtract`` — per interval: the whole interval if CPC busy ≥ 97 % of the clocks,
  else max(SPI, CPC − learned READ cost), share × Δt (shipped);
* ``overlap``  — the same, but the READ's CP time is taken to land uniformly in the
  interval, counted once where the CP was busy anyway: busy = (CPC − r) / (1 − r/clk)
  (shipped in r4e only: phase U read 8 kHz burst trains up to 4.6 points high);
* ``carry``    — ``subtract``, but the part of an interval's READ-cost subtraction that
  the floor at SPI cut off is carried into the next intervals (zero-mean noise in
  the READ's own CP time then cancels instead of adding up);
* ``timesplit``— per interval, busy time = Δt − idle cycles / idle clock, with the
  idle clock learned on quiet intervals (cycle shares are clock-weighted: a burst
  under the power cap runs at a lower clock than the idle stretch around it).

``python tools/util_estimator_sim.py profiles/r4/r4e/cp_dump.json``
"""
from __future__ import annotations

import json
import sys

FULL = 0.97


def intervals(samples):
    for a, b in zip(samples, samples[1:]):
        dt = b[0] - a[0]
        clk = b[1] - a[1]
        if dt <= 0 or clk <= 0:
            continue
        yield dt, clk, max(0, b[2] - a[2]), max(0, b[3] - a[3])


def learn_read(ivs) -> tuple[float, float]:
    """READ cost in cycles (mean over intervals without waves and with the CP mostly
    idle) and the idle clock (cycles / s over the same intervals)."""
    cyc, clk_s, n = 0.0, 0.0, 0
    for dt, clk, spi, cpc in ivs:
        if spi < 0.005 * clk and cpc < 0.5 * clk:
            cyc += cpc
            clk_s += clk / dt
            n += 1
    return (cyc / n, clk_s / n) if n else (0.0, 0.0)


def estimate(ivs, read_cyc: float, idle_hz: float, variant: str) -> float:
    tot, span, carry = 0.0, 0.0, 0.0
    for dt, clk, spi, cpc in ivs:
        span += dt
        if variant == "timesplit" and idle_hz > 0:
            if cpc >= FULL * clk:
                tot += dt
                continue
            busy_cyc = max(spi, cpc - read_cyc)
            idle_s = max(0.0, (clk - busy_cyc) / idle_hz)
            tot += min(dt, max(0.0, dt - idle_s))
            continue
        if cpc >= FULL * clk:
            busy = clk
            carry = 0.0
        elif variant == "overlap":
            r = min(read_cyc, 0.5 * clk)
            busy = max(spi, max(0.0, (cpc - r) / (1.0 - r / clk)))
        elif variant == "carry":
            raw = cpc - read_cyc + carry
            busy = max(spi, raw)
            carry = min(0.0, raw - spi)
            carry = max(carry, -2 * read_cyc)  # never owe more than two READs
        else:
            busy = max(spi, max(0.0, cpc - read_cyc))
        tot += min(1.0, busy / clk) * dt
    return 100.0 * tot / span if span else 0.0


def main(argv=None) -> int:
    path = (argv or sys.argv[1:])[0]
    d = json.load(open(path))
    out = {}
    for rate, loads in d["rates"].items():
        quiet = list(intervals(loads.get("idle", {}).get("samples", [])))
        read_cyc, idle_hz = learn_read(quiet)
        rows = {"read_us": round(1e6 * read_cyc / idle_hz, 2) if idle_hz else None,
                "idle_clock_mhz": round(idle_hz / 1e6, 1)}
        for name, L in loads.items():
            ivs = list(intervals(L["samples"]))
            if not ivs:
                continue
            wall = L["t1"] - L["t0"]
            row = {"duty_gpu_pct": round(100 * L["duty_gpu_s"] / wall, 2),
                   "busy_clock_mhz": round(sum(c for _, c, _, _ in ivs) / sum(t for t, _, _, _ in ivs) / 1e6, 1)}
            for v in ("subtract", "overlap", "carry", "timesplit"):
                row[v] = round(estimate(ivs, read_cyc, idle_hz, v), 2)
            rows[name] = row
        out[rate] = rows
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
