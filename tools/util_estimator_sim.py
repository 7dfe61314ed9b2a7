#!/usr/bin/env python3
"""Replay raw counter READs through the sampler's own dispatch estimator (offline, CPU).

Input: ``tools/cp_busy_probe.py --dump`` output — every READ of [GRBM_COUNT,
GRBM_SPI_BUSY, CPC busy, ...] (max over XCCs) during known loads, with the loads'
event-timed GPU busy (``duty_gpu_s``).  Each load is folded READ by READ through
``_kgs_native.DispatchEstimator`` — the C++ class ``Sampler::run_pmc`` itself runs
(``native/include/kgs/util_estimator.h``), with the parameters of the default
``SamplerConfig`` (``_kgs_native.sampler_estimator_params``) — after the same rate's
idle READs have taught it the READ packet's cost, as the running sampler learns it on
the READ-only intervals between kernels.  There is no second model of the estimator
here: a change to the C++ class changes these numbers (tests/test_estimator_replay.py).

``python tools/util_estimator_sim.py profiles/r4/r4f/cp_dump.json [--set cpc_full_frac=0.97]``
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# Dump timestamps are seconds relative to each load's start (the first READs come a
# few ms before it): shift them onto a positive clock.
T_OFFSET_S = 10.0


def rows_of(load: dict, mfma_col: int | None = None, fresh_col: int | None = None,
            inside: bool = False) -> list[list[float]]:
    """[t_s, count, spi, cpc, mfma (-1: not in the set), se_fresh] per READ; ``inside``:
    only the READs taken while the load ran (its intervals lie wholly inside it)."""
    out = []
    wall = load.get("t1", 0.0) - load.get("t0", 0.0)
    for s in load["samples"]:
        if inside and not 0.0 <= s[0] <= wall:
            continue
        out.append([s[0] + T_OFFSET_S, s[1], s[2], s[3], s[mfma_col] if mfma_col is not None else -1,
                    s[fresh_col] if fresh_col is not None and fresh_col < len(s) else 1])
    return out


def replay_rate(N, loads: dict, params, mfma_col: int | None = None, fresh_col: int | None = None) -> dict:
    """Per load of one READ rate: the estimator's busy % of the load's wall time next to
    the event-timed duty, warmed on that rate's idle READs."""
    idle = rows_of(loads.get("idle", {"samples": []}), mfma_col, fresh_col)
    out = {}
    warm = N.DispatchEstimator()
    if idle:
        warm.replay(params, idle)
    out["read_us"] = round(warm.cpc_read_us, 2)
    out["idle_clock_mhz"] = round(warm.clk_idle_hz / 1e6, 1)
    for name, L in loads.items():
        rows = rows_of(L, mfma_col, fresh_col, inside=True)
        if len(rows) < 3:
            continue
        est = N.DispatchEstimator()
        if name != "idle" and idle:
            est.replay(params, idle)         # learn the READ cost first ...
            est.invalidate(int(rows[0][0] * 1e9))  # ... then baseline on the load's first READ
        r = est.replay(params, rows)
        wall = L["t1"] - L["t0"]
        # Busy as a share of the READ intervals inside the load (at 10 Hz the first and
        # last READ sit up to a period inside it), against the kernels' duty over the load.
        duty = 100 * L["duty_gpu_s"] / wall
        busy = 100 * r["dispatch_s"] / r["span_s"] if r["span_s"] > 0 else 0.0
        out[name] = {"duty_gpu_pct": round(duty, 2), "busy_pct": round(busy, 2), "err_pts": round(busy - duty, 2),
                     "active_pct": round(100 * r["active_s"] / r["span_s"], 2) if r["span_s"] > 0 else 0.0,
                     "reads": len(rows)}
    return out


def interval_classes(N, loads: dict, params, mfma_col: int | None = None, fresh_col: int | None = None) -> dict:
    """Per load: where the estimate comes from — READ intervals the CP was busy for ≥
    cpc_full_frac (counted whole), partial ones, and READ-only ones — as µs per second of
    load, with the kernels' duty for comparison (how r5aa / r5ab found the READ-only
    intervals' rectified scatter)."""
    idle = rows_of(loads.get("idle", {"samples": []}), mfma_col, fresh_col)
    out = {}
    for name, L in loads.items():
        rows = rows_of(L, mfma_col, fresh_col, inside=True)
        if name == "idle" or len(rows) < 3:
            continue
        est = N.DispatchEstimator()
        if idle:
            est.replay(params, idle)
        est.invalidate(int(rows[0][0] * 1e9))
        cls = {"full": [0, 0.0], "partial": [0, 0.0], "read_only": [0, 0.0]}
        prev, span = None, 0.0
        for r in rows:
            s = est.feed(params, int(r[0] * 1e9), int(r[1]), int(r[2]), int(r[3]), None if r[4] < 0 else int(r[4]),
                         bool(r[5]), False)
            if prev is not None and s.have_dispatch and r[1] > prev[1]:
                cpc = (r[3] - prev[3]) / (r[1] - prev[1])
                k = "full" if cpc >= params.cpc_full_frac else ("read_only" if s.learned else "partial")
                cls[k][0] += 1
                cls[k][1] += s.dispatch_s
                span += s.span_s
            prev = r
        if span <= 0:
            continue
        out[name] = {"duty_us_per_s": round(1e6 * L["duty_gpu_s"] / (L["t1"] - L["t0"]), 1),
                     **{k: {"intervals": n, "busy_us_per_s": round(1e6 * v / span, 1)} for k, (n, v) in cls.items()}}
    return out


def replay(path: str, overrides: dict | None = None, classes: bool = False) -> dict:
    from kube_gpu_stats_amd import load_native

    N = load_native()
    if path.endswith(".gz"):  # held-out dumps are committed compressed (profiles/r6/r6c)
        import gzip

        with gzip.open(path, "rt") as f:
            d = json.load(f)
    else:
        d = json.load(open(path))
    p = N.sampler_estimator_params()
    for k, v in (overrides or {}).items():
        t = type(getattr(p, k))
        setattr(p, k, str(v).lower() in ("1", "true", "yes") if t is bool else t(v))
    names = d.get("counters", [])
    mfma_col = 1 + names.index("SQ_VALU_MFMA_BUSY_CYCLES") if "SQ_VALU_MFMA_BUSY_CYCLES" in names else None
    cols = d.get("columns") or []
    fresh_col = cols.index("se_fresh") if "se_fresh" in cols else None
    if classes:
        return {rate: interval_classes(N, loads, p, mfma_col, fresh_col) for rate, loads in d["rates"].items()}
    return {rate: replay_rate(N, loads, p, mfma_col, fresh_col) for rate, loads in d["rates"].items()}


def replay_exporter_raw(path: str, overrides: dict | None = None) -> dict:
    """The irregular GPU test's raw 10 Hz capture (``irregular_raw_10hz.json``: the
    exporter's own drains from ``/counters`` and the kernels' event-timed intervals on the
    host monotonic clock) folded through the estimator drain by drain, warmed on the
    drains before the load: per load the dispatch integral against the kernels' union over
    the same drain intervals, and the intervals that err most."""
    from kube_gpu_stats_amd import load_native

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from kube_gpu_stats_amd.ops.irregular import union_seconds

    N = load_native()
    p = N.sampler_estimator_params()
    for k, v in (overrides or {}).items():
        t = type(getattr(p, k))
        setattr(p, k, str(v).lower() in ("1", "true", "yes") if t is bool else t(v))
    d = json.load(open(path))
    out = {}
    for name, rec in d.items():
        names = rec["counters"]["counters"]
        ix = {n: i for i, n in enumerate(names)}
        t_ref = rec["t_ref_mono_ns"] * 1e-9
        kern = [(t_ref + a, t_ref + b) for a, b in rec["kernels_s"]]
        k0, k1 = min(a for a, _ in kern), max(b for _, b in kern)
        est = N.DispatchEstimator()
        prev_t = None
        busy = truth = span = 0.0
        worst = []
        for smp in rec["counters"]["samples"]:
            v = smp["v"]
            t = smp["mono_ns"] * 1e-9
            mf = v[ix["SQ_VALU_MFMA_BUSY_CYCLES"]] if v[ix["SQ_VALU_MFMA_BUSY_CYCLES"]] is not None else None
            s = est.feed(p, smp["mono_ns"], int(v[ix["GRBM_COUNT"]]), int(v[ix["GRBM_SPI_BUSY"]]),
                         int(v[ix["CPC_CPC_STAT_BUSY"]]), None if mf is None else int(mf), bool(smp["se_fresh"]), False)
            if prev_t is not None and prev_t >= k0 - 0.2 and t <= k1 + 0.4:
                tr = union_seconds([(max(a, prev_t), min(b, t)) for a, b in kern if b > prev_t and a < t])
                busy += s.dispatch_s
                truth += tr
                span += t - prev_t
                worst.append((round(s.dispatch_s - tr, 5), round(prev_t - k0, 3), round(t - prev_t, 4),
                              round(tr / (t - prev_t), 3)))
            prev_t = t
        worst.sort(key=lambda x: abs(x[0]), reverse=True)
        out[name] = {"span_s": round(span, 3), "busy_pct": round(100 * busy / span, 2) if span else None,
                     "truth_pct": round(100 * truth / span, 2) if span else None,
                     "err_pts": round(100 * (busy - truth) / span, 2) if span else None,
                     "intervals": len(worst), "worst": worst[:8],
                     "idle_clock_mhz": round(est.clk_idle_hz / 1e6, 1), "busy_clock_mhz": round(est.clk_busy_hz / 1e6, 1)}
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("dump")
    ap.add_argument("--exporter-raw", action="store_true",
                    help="the dump is an irregular_raw_10hz.json capture of the exporter's own drains")
    ap.add_argument("--set", action="append", default=[], metavar="PARAM=VALUE",
                    help="override one EstimatorParams field (e.g. cpc_full_frac=0.97)")
    ap.add_argument("--classes", action="store_true",
                    help="instead: each load's estimate split by READ-interval class (full / partial / READ-only)")
    a = ap.parse_args(argv)
    ov = dict(kv.split("=", 1) for kv in a.set)
    if a.exporter_raw:
        print(json.dumps(replay_exporter_raw(a.dump, ov), indent=1))
        return 0
    print(json.dumps(replay(a.dump, ov, classes=a.classes), indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
