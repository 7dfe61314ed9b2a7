#!/usr/bin/env python3
"""Every measured bound of tests/test_gpu.py against what every kept hardware run
measured (a saturated MFMA stream's SPI share crossed a 0.9 threshold
on the driver's box, and that one thin margin cost the driver the evidence of 16 other
tests).

Sources, one *run* per profiles directory — the runs of the code the thresholds guard:
round 6's, and round 5's final tree (the tree the driver's round-5 record ran; runs of
earlier trees measured code that has since changed — the pre-carry biller read a
saturated 10 Hz window 12 points low in r5b — and are not box-to-box spread):
  * ``margins.jsonl`` — written by tests/test_gpu.py ``bound()`` on every GPU run since
    round 6: (test, quantity, value, lo, hi) per assertion;
  * the JSON files the tests ``_keep``-ed in rounds 2-5 (sm_util_read_immune.json,
    shipped_config_billing.json, dispatch_bound.json, ...), mapped onto the same
    quantity names by the extractors below (a run with a margins.jsonl is read from
    that file only).

Per quantity: the bound in force (the newest margins.jsonl's), every run's value, the
spread across runs (max − min), the margin (nearest observed value to the bound) and
margin ÷ spread.  ``ok`` needs margin ≥ 2 × spread over ≥ 2 runs (VERDICT r5 #2's rule);
``thin`` is below it; ``1 run`` cannot be judged yet.

    python tools/gpu_margins.py [--write profiles/gpu_test_margins.md]
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(REPO, "profiles")


def _sm_util_read_immune(d: dict):
    for k, r in d.items():
        if "/" not in k or not isinstance(r, dict):
            continue
        hz, name = k.split("/", 1)
        if name == "idle":
            yield f"read_immune_idle_busy_pct[{hz}]", r["busy_counter_pct"]
        elif name == "mfma_saturating":
            yield f"read_immune_saturated_busy_pct[{hz}]", r["busy_counter_pct"]
        else:
            yield f"read_immune_abs_err_pts[{hz}/{name}]", abs(r["busy_counter_pct"] - r["duty_gpu_pct"])
            if "gfx_busy_pct" in r:
                yield f"read_immune_gauge_vs_counter_pts[{hz}/{name}]", abs(r["gfx_busy_pct"] - r["busy_counter_pct"])


def _shipped(d: dict):
    for k, r in (d.get("rows") or {}).items():
        tag, name = k.split("/", 1)
        if name == "idle":
            yield f"shipped_idle_busy_pct[{tag}]", r["busy_counter_pct"]
            if r.get("report_pct") is not None:
                yield f"shipped_idle_report_pct[{tag}]", r["report_pct"]
        elif name == "mfma_saturating":
            if "load_only_busy_pct" in r:
                yield f"shipped_saturated_load_only_busy_pct[{tag}]", r["load_only_busy_pct"]
            yield f"shipped_saturated_abs_err_pts[{tag}]", abs(r["busy_counter_pct"] - r["duty_gpu_pct"])
            if r.get("report_pct") is not None:
                yield f"shipped_saturated_report_abs_err_pts[{tag}]", abs(r["report_pct"] - r["duty_gpu_pct"])
        else:
            yield f"shipped_abs_err_pts[{tag}/{name}]", abs(r["busy_counter_pct"] - r["duty_gpu_pct"])
            if r.get("report_pct") is not None:
                yield f"shipped_report_abs_err_pts[{tag}/{name}]", abs(r["report_pct"] - r["duty_gpu_pct"])


def _dispatch_bound(d: dict):
    g, k, st = d.get("tiny_graph") or {}, d.get("mfma") or {}, d.get("mfma_then_graph") or {}
    if "dispatch_bound_share" in g:
        yield "graph_dispatch_bound_share", g["dispatch_bound_share"]
        yield "graph_reads_per_s", g["reads_per_s"]
        yield "graph_dispatch_pct", g["dispatch_pct"]
    if "dispatch_bound_share" in k:
        yield "mfma_stream_reads_per_s", k["reads_per_s"]
        yield "mfma_stream_dispatch_bound_share", k["dispatch_bound_share"]
    if "reads_per_s" in st:
        yield "mfma_then_graph_reads_per_s", st["reads_per_s"]


def _idle_gpu(d: dict):
    a, p, ld = d.get("adaptive") or {}, d.get("profiling") or {}, d.get("mfma_load") or {}
    for q, row, key in (("idle_adaptive_reads_per_s", a, "reads_per_s"), ("idle_adaptive_pmfw_busy_pct", a, "pmfw_gfx_busy_pct"),
                        ("idle_adaptive_active_pct", a, "gpu_active_pct"), ("idle_profiling_reads_per_s", p, "reads_per_s"),
                        ("idle_profiling_pmfw_busy_pct", p, "pmfw_gfx_busy_pct"),
                        ("idle_profiling_active_pct", p, "gpu_active_pct"), ("loaded_reads_per_s", ld, "reads_per_s"),
                        ("loaded_active_pct", ld, "gpu_active_pct"), ("loaded_mfma_util_pct", ld, "mfma_util_pct")):
        if row.get(key) is not None:
            yield q, row[key]
    if ld.get("publishes_per_s") and ld.get("reads_per_s"):
        yield "loaded_publishes_per_read", ld["publishes_per_s"] / ld["reads_per_s"]
    if a.get("publishes_per_s") and a.get("reads_per_s"):
        yield "idle_publishes_per_read", a["publishes_per_s"] / a["reads_per_s"]


def _two_tenants(d: dict):
    pc, pb = d.get("pod_cu_share") or {}, d.get("pod_busy_share") or {}
    if "tenant-a" in pc:
        yield "pod_a_cu_share", pc["tenant-a"]
        yield "pod_b_cu_share", pc["tenant-b"]
    if "tenant-b" in pb:
        yield "pod_b_busy_share", pb["tenant-b"]
    ps = d.get("kgs_ps") or {}
    for t, k in (("tenant-a", "a"), ("tenant-b", "b")):
        row = ps.get(t) or {}
        if "hbm_gib" in row:
            yield f"ps_tenant_{k}_hbm_gib", row["hbm_gib"]
        if "cu_share_pct" in row:
            yield f"ps_tenant_{k}_cu_share_pct", row["cu_share_pct"]


def _lite(d: dict):
    f, lt = d.get("full") or {}, d.get("lite") or {}
    if "mfma_busy_pct" not in f or "mfma_busy_pct" not in lt:
        return
    yield "lite_full_mfma_busy_pct", f["mfma_busy_pct"]
    yield "lite_vs_full_mfma_busy_pts", abs(lt["mfma_busy_pct"] - f["mfma_busy_pct"])
    if "mfma_util_pct" in f and "mfma_util_pct" in lt:
        yield "lite_vs_full_mfma_util_pts", abs(lt["mfma_util_pct"] - f["mfma_util_pct"])
    for k, r in (("full", f), ("lite", lt)):
        if "dispatch_pct" in r:
            yield f"lite_dispatch_abs_err_pts[{k}]", abs(r["dispatch_pct"] - r["duty_gpu_pct"])
    yield "lite_reads_per_s", lt["reads_per_s"]


def _flops(d: dict):
    if "ratio" in d:
        yield "mfma_counter_flops_ratio", d["ratio"]
    if "measured_tflops" in d:
        yield "mfma_measured_flops", d["measured_tflops"] * 1e12


def _irregular(d: dict):
    for k, r in (d.get("rows") or {}).items():
        yield f"irregular_abs_err_pts[{k}]", abs(r["error_pts"])


# Round-5 runs of its final tree (profiles/r5/README.md; VERDICT r5 cites r5ac, r5ah, r5al).
FINAL_TREE_RUNS = {"r5/r5ac", "r5/r5ah", "r5/r5al", "r5/r5ai", "r5/r5an"}


def current(run: str) -> bool:
    return run.startswith("r6/") or run in FINAL_TREE_RUNS


EXTRACTORS = {"sm_util_read_immune.json": _sm_util_read_immune, "shipped_config_billing.json": _shipped,
              "dispatch_bound.json": _dispatch_bound, "idle_gpu_not_busy.json": _idle_gpu,
              "two_tenants.json": _two_tenants, "lite_reads.json": _lite, "mfma_flops_crosscheck.json": _flops,
              "irregular_billing.json": _irregular}


def run_dir(path: str) -> str:
    """The run a kept file belongs to: its profiles/rN/<run> directory."""
    rel = os.path.relpath(path, PROFILES).split(os.sep)
    return "/".join(rel[:2]) if len(rel) > 2 else rel[0]


def run_order(path: str) -> tuple:
    """Runs in the order they were taken: rN, then the tag as a spreadsheet column
    (r6z before r6aa), so the last margins.jsonl read holds the newest bounds."""
    parts = run_dir(path).split("/")
    rnd = parts[0][1:] if parts[0][:1] == "r" else ""
    tag = parts[1] if len(parts) > 1 else ""
    suffix = tag[len(parts[0]):] if tag.startswith(parts[0]) else tag
    return (int(rnd) if rnd.isdigit() else 0, len(suffix), suffix, path)


def collect(root: str = PROFILES) -> tuple[dict, dict]:
    """({(test, q): {run: value}}, {(test, q): (lo, hi)} — the newest bound)."""
    obs: dict = {}
    bounds: dict = {}
    test_of: dict = {}
    with_margins = set()
    for path in sorted(glob.glob(os.path.join(root, "**", "margins.jsonl"), recursive=True), key=run_order):
        run = run_dir(path)
        if not current(run):
            continue
        with_margins.add(run)
        for line in open(path):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            key = (r["test"], r["q"])
            if r.get("value") is None:
                continue
            obs.setdefault(key, {})[run] = r["value"]
            bounds[key] = (r.get("lo"), r.get("hi"))
            test_of[r["q"]] = r["test"]
    for name, fn in EXTRACTORS.items():
        for path in sorted(glob.glob(os.path.join(root, "**", name), recursive=True)):
            run = run_dir(path)
            if run in with_margins or not current(run):
                continue
            try:
                d = json.load(open(path))
                pairs = list(fn(d))
            except (ValueError, KeyError, TypeError, AttributeError):
                continue
            for q, v in pairs:
                t = test_of.get(q)
                if t is None or v is None:
                    continue  # no bound on record for it (any more)
                obs.setdefault((t, q), {})[run] = float(v)
    return obs, bounds


def table(obs: dict, bounds: dict) -> list[dict]:
    rows = []
    for key in sorted(bounds):
        lo, hi = bounds[key]
        vals = obs.get(key, {})
        xs = list(vals.values())
        mn, mx = (min(xs), max(xs)) if xs else (None, None)
        spread = (mx - mn) if xs else None
        margins = []
        if xs and lo is not None:
            margins.append(mn - lo)
        if xs and hi is not None:
            margins.append(hi - mx)
        margin = min(margins) if margins else None
        if not xs:
            status = "no runs"
        elif margin is not None and margin < 0:
            status = "FAILING"
        elif len(xs) < 2:
            status = "1 run"
        elif spread == 0 or margin >= 2 * spread:
            status = "ok"
        elif lo is not None and hi is None and mn > 0 and 0 <= lo <= 0.25 * mn:
            status = "ok (≤ ¼ of min)"  # a "clearly non-zero" bound on a noisy positive quantity
        else:
            status = "thin"
        rows.append({"test": key[0], "q": key[1], "lo": lo, "hi": hi, "runs": len(xs), "min": mn, "max": mx,
                     "spread": spread, "margin": margin,
                     "ratio": (math.inf if spread == 0 else margin / spread) if xs and margin is not None and spread is not None else None,
                     "status": status, "values": vals})
    return rows


def fmt(x) -> str:
    if x is None:
        return ""
    if isinstance(x, float) and math.isinf(x):
        return "∞"
    ax = abs(x)
    if ax >= 1e9:
        return f"{x:.3g}"
    if ax >= 100:
        return f"{x:.0f}"
    if ax >= 1:
        return f"{x:.2f}"
    return f"{x:.3g}"


def markdown(rows: list[dict]) -> str:
    n_runs = len({r for row in rows for r in row["values"]})
    counts: dict = {}
    for r in rows:
        counts[r["status"]] = counts.get(r["status"], 0) + 1
    out = ["# GPU test margins (VERDICT r5 #2)", "",
           "Generated by `python tools/gpu_margins.py --write profiles/gpu_test_margins.md` from every kept "
           "hardware run under `profiles/` (round 6's `margins.jsonl` from `tests/test_gpu.py` `bound()`, and the "
           "JSON files earlier rounds kept).  *spread* = max − min over runs (boxes); *margin* = distance from the "
           "nearest observed value to the bound; **ok** = margin ≥ 2 × spread over ≥ 2 runs, or a lower bound at "
           "most ¼ of the smallest value seen (a clearly-non-zero check on a noisy share).  Runs: round 6's and "
           "round 5's final tree (`FINAL_TREE_RUNS`); earlier trees measured code that has since changed.", "",
           f"{len(rows)} bounds, {n_runs} runs: " + ", ".join(f"{k} {v}" for k, v in sorted(counts.items())), "",
           "| test | quantity | bound | runs | min | max | spread | margin | margin/spread | status |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        b = " ".join(x for x in ((f"≥ {fmt(r['lo'])}" if r["lo"] is not None else ""),
                                 (f"≤ {fmt(r['hi'])}" if r["hi"] is not None else "")) if x)
        out.append(f"| {r['test'].replace('test_', '', 1)} | `{r['q']}` | {b} | {r['runs']} | {fmt(r['min'])} | "
                   f"{fmt(r['max'])} | {fmt(r['spread'])} | {fmt(r['margin'])} | {fmt(r['ratio'])} | {r['status']} |")
    return "\n".join(out) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--write", default="", help="write the markdown table here")
    ap.add_argument("--json", action="store_true", help="print the rows as JSON")
    a = ap.parse_args(argv)
    rows = table(*collect())
    if a.json:
        print(json.dumps(rows, indent=1, default=str))
    md = markdown(rows)
    if a.write:
        with open(a.write, "w") as f:
            f.write(md)
    elif not a.json:
        sys.stdout.write(md)
    return 0


if __name__ == "__main__":
    sys.exit(main())
