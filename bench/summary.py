"""The stdout result line: contract keys, config, and a ≤ 1.8 KB summary last."""
from __future__ import annotations

import json

from .common import _pm, _r


SUMMARY_MAX = 1800  # bytes of the summary object: the driver keeps the last ≈2.3 KB of stdout (BENCH_r04)


CONTRACT_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data")


def summarize(res: dict) -> dict:
    """The headline numbers in ≤ 1.5 KB: what a reader of the last few
    KB of stdout needs — value, scrape latency, overhead ± CI per tier (paired and
    position-adjusted), per load component and per rank, released vs paused, what the
    exporter delivered per component, phase U's utilisation accuracy and phase X's
    xGMI verdict."""
    inter = res.get("interleaved") or {}
    tiers = inter.get("tiers") or {}
    prim = f"{res.get('config', {}).get('hz', 0):g}"
    pa = inter.get("position_adjusted") or {}
    out: dict = {"value": _r(res.get("value"), 1), "samples_per_sec_per_gpu": _r(res.get("samples_per_sec_per_gpu"), 1),
                 "p50_scrape_ms": _r(res.get("p50_scrape_ms")), "p99_scrape_ms": _r(res.get("p99_scrape_ms")),
                 "scrapes": res.get("scrapes"), "overhead_pct": _pm(res)}
    out["overhead_by_tier"] = {h: _pm(t) for h, t in tiers.items()}
    out["overhead_median_by_tier"] = {h: _r(t.get("overhead_median_pct")) for h, t in tiers.items()}
    out["overhead_position_adjusted"] = {h: _pm(v) for h, v in pa.items() if isinstance(v, dict) and "overhead_pct" in v}
    # per tier and component: [vs paused, ± 95 %, vs released, ± 95 %] (the last two when
    # the run had the released condition)
    def comp(t: dict) -> dict:
        rel = t.get("overhead_by_component_vs_released") or {}
        return {c: (_pm(v) or [None, None]) + (_pm(rel.get(c)) or []) for c, v in
                (t.get("overhead_by_component") or {}).items()}

    out["overhead_by_component"] = {h: comp(t) for h, t in tiers.items()}
    out["overhead_by_rank"] = [_r(x.get("overhead_pct")) for x in (tiers.get(prim, {}).get("overhead_by_rank") or [])]
    rel = inter.get("released")
    if rel:
        pw = ((inter.get("power") or {}).get("by_condition") or {}).get("released", {})
        out["released"] = {"paused_vs_released": _pm(rel, "paused_vs_released_pct", "paused_vs_released_ci95_pct"),
                           **{k[:-len("_vs_released_pct")] + "_vs_released":
                              _pm(rel, k, k.replace("_pct", "_ci95_pct"))
                              for k in rel if k.endswith("_vs_released_pct") and not k.startswith("paused")},
                           "power_w_vs_paused": pw.get("power_w_vs_paused")}
    dbc = res.get("delivered_by_component") or {}
    out["delivered_by_component"] = {c: _r(min((v.get("samples_per_sec_per_gpu") or {"x": 0}).values()), 1)
                                     for c, v in dbc.items()}
    ua = res.get("util_accuracy") or {}
    if ua.get("per_rate"):
        def mean(xs):
            xs = [x for x in xs if x is not None]
            return _r(sum(xs) / len(xs), 1) if xs else None

        short = {"burst_1ms_every_5ms": "1ms/5ms", "burst_0.2ms_every_1ms": "0.2ms/1ms",
                 "triad_1ms_every_5ms": "triad1ms/5ms", "mfma_saturating": "sat", "random_kernels": "rand",
                 "two_stream_random": "rand2s", "train_step": "train"}
        out["util_accuracy"] = {
            "cols": "exported busy %, kernel duty %",
            **{hz: {short.get(ld, ld): [mean([r.get("busy_counter_pct") for r in pg.values()]),
                                        mean([r.get("duty_gpu_pct") for r in pg.values()])]
                    for ld, pg in per.items()} for hz, per in ua["per_rate"].items()},
            "worst_error_pts": {short.get(k, k): v for k, v in (ua.get("worst_error_pts") or {}).items()}}
        # what the auto source removes: the PMFW busy of the fastest rate's 0.2 ms train
        fast = max(ua["per_rate"], key=float)
        pg = ua["per_rate"][fast].get("burst_0.2ms_every_1ms") or {}
        out["util_accuracy"]["pmfw_busy_0.2ms_" + fast] = mean([r.get("pmfw_gfx_busy_pct") for r in pg.values()])
    q = res.get("quiet_gpu") or {}
    if q:
        out["quiet_gpu"] = {m: [_r(max(x.get("reads_per_s", 0) for x in v.get("per_gpu", {}).values()), 1),
                                _r(max(x.get("pmfw_gfx_busy_pct", 0) for x in v.get("per_gpu", {}).values()), 2)]
                            for m, v in q.items() if v.get("per_gpu")}
        ip = q.get("idle_power") or {}
        if "session_minus_released_w" in ip:  # phase P: W above released (± 95 %), and the released W
            out["quiet_gpu"]["power_w"] = {"session": ip["session_minus_released_w"],
                                           "parked": ip.get("parked_minus_released_w"),
                                           "released": (ip["per_rank"][0] or {}).get("released_w"),
                                           "median": [ip.get("session_minus_released_median_w"),
                                                      ip.get("parked_minus_released_median_w")],
                                           "floor": [ip.get("session_minus_released_floor_w"),
                                                     ip.get("parked_minus_released_floor_w")]}
    br = (res.get("burst_resolution") or {}).get("per_gpu") or {}
    if br:
        out["bursts_resolved"] = [sum(v.get("segments", 0) for v in br.values()), sum(v.get("launched", 0) for v in br.values())]
    out["capacity_max_hz_98pct"] = (res.get("capacity") or {}).get("max_rate_hz_98pct")
    out["exporter_cpu_cores"] = res.get("exporter_cpu_cores")
    out["xgmi_link_map_ok"] = res.get("xgmi_link_map_ok")
    out["xgmi_links_ok"] = res.get("xgmi_links_ok")
    out["xgmi_unit_ratio"] = res.get("xgmi_unit_ratio")
    out["xgmi_unit_ratio_min_max"] = res.get("xgmi_unit_ratio_min_max")
    if (res.get("xgmi_link_check") or {}).get("bad_links"):
        out["xgmi_bad_links"] = res["xgmi_link_check"]["bad_links"][:4]
    # keep the summary inside the driver's window: shed the side estimates first
    if len(json.dumps(out)) > SUMMARY_MAX:
        out.pop("overhead_position_adjusted", None)
    if len(json.dumps(out)) > SUMMARY_MAX and "util_accuracy" in out:
        out["util_accuracy"] = {"worst_error_pts": out["util_accuracy"].get("worst_error_pts")}
    return out


def compact(res: dict, full_path: str) -> dict:
    """The stdout line: the driver's contract keys, the config, where the full result
    is, and ``summary`` last."""
    line = {k: res.get(k) for k in CONTRACT_KEYS if k in res}
    if "error" in res:
        line["error"] = res["error"]
    cfg = res.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("model", "global_batch", "seq_len", "parallelism", "hz", "hz_tiers",
                                         "sample_source", "pmc_batch", "load") if k in cfg}
    line["full_result"] = full_path
    if res.get("value") is not None:
        line["summary"] = summarize(res)
    return line
