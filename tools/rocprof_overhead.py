"""Split a rocprofv3 kernel trace of ``bench.py`` by exporter condition and compare
per-kernel GPU time: no exporter process (phases A, C), sampling at 8 kHz (B), and
the interleaved blocks (paused / 100 Hz / 8 kHz).

bench.py launches, per rank, in this order (``load`` units: one
``mfma_bf16_kernel``, ``--triads`` ``triad_f32_kernel``, one replay of the
``--tiny-kernels`` copy graph):

* ``calibrate()``: 1 mfma, 1 triad, 1 graph replay (after 1 eager warm-up copy);
* ``calibrate_reps()``: 2 units;
* warm-up W steps, A K steps, B K steps, the phase-R burst train (MFMA kernels
  only, ``burst_resolution.per_gpu.*.launched``), the interleaved blocks in
  ``interleaved.block_seconds`` order (``block_steps`` steps each), the phase-S
  capacity blocks, phase K (each component alone,
  ``delivered_by_component.*.launches``), C K steps — every step
  ``config.units_per_step`` units.

Kernels are assigned to segments by launch order, so no clock translation between
rocprofv3 and Python is needed.  The interleaved blocks come in rounds of one block
per condition (bench.py's order design), so each tier's per-kernel difference to the
paused block of the same round gives one paired value per round; the tables report
their mean with a 95 % CI (t-quantile 1.96 · sd / sqrt(rounds)).

    python tools/rocprof_overhead.py <trace dir> <bench.json> [--out md]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def find_trace(d: str) -> str:
    c = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True), key=os.path.getsize)
    if not c:
        raise SystemExit(f"no *kernel_trace.csv under {d}")
    return c[-1]


def segments(res: dict, triads: int, tiny: int) -> list[tuple[str, int, dict]]:
    """(label, units, extra launches per kernel kind) in launch order after the
    calibration launches."""
    reps = res["config"]["units_per_step"]
    k, w = res["steps"], res["warmup"]
    inter = res.get("interleaved") or {}
    bs = inter.get("block_steps", 0)
    bursts = max((g.get("launched", 0) for g in ((res.get("burst_resolution") or {}).get("per_gpu") or {}).values()),
                 default=0)
    seg = [("calib_reps", 2, {}), ("warmup", w * reps, {}), ("A_off", k * reps, {}), ("B_on_8k", k * reps, {}),
           ("R_bursts", 0, {"mfma": bursts})]
    seg += [(f"I_{'paused' if c == '0' else c + 'Hz'}", bs * reps, {}) for c, _ in inter.get("block_seconds", [])]
    cap = res.get("capacity") or {}
    seg += [(f"S_{hz}Hz", cap.get("block_steps", 0) * reps, {}) for hz in cap.get("rates", {})]
    # phase K: each component alone (``delivered_by_component.<name>.launches``)
    kk = res.get("delivered_by_component") or {}
    launches = lambda n: int((kk.get(n) or {}).get("launches", 0))  # noqa: E731
    seg += [("K_mfma", 0, {"mfma": launches("mfma")}), ("K_triad", 0, {"triad": launches("triad")}),
            ("K_tiny_graph", 0, {"copy": launches("tiny_graph") * tiny})]
    seg += [("C_off", k * reps, {})]
    return seg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("bench_json")
    ap.add_argument("--triads", type=int, default=2)
    ap.add_argument("--tiny", type=int, default=2000)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    with open(a.bench_json) as f:
        res = json.loads(f.read().strip().splitlines()[-1])
    path = find_trace(a.dir)
    by = {"mfma": [], "triad": [], "copy": []}
    with open(path) as f:
        rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                       for r in csv.DictReader(f)), key=lambda x: x[0])
    for t0, t1, name in rows:
        dur = (t1 - t0) * 1e-3  # µs
        if "mfma_bf16_kernel" in name:
            by["mfma"].append(dur)
        elif "triad_f32_kernel" in name:
            by["triad"].append(dur)
        elif "copy_f32_kernel" in name:
            by["copy"].append(dur)
    per_unit = {"mfma": 1, "triad": a.triads, "copy": a.tiny}
    calib = {"mfma": 1, "triad": 1, "copy": 1 + a.tiny}
    seg = segments(res, a.triads, a.tiny)
    out = {"trace": os.path.relpath(path), "kernels_total": len(rows), "kernels": {}}
    for kind, xs in by.items():
        if per_unit[kind] == 0:
            continue
        i = calib[kind]
        groups: dict[str, list[float]] = {}
        blocks: list[tuple[str, float]] = []  # interleaved blocks in order: (label, mean µs)
        for label, units, extra in seg:
            n = units * per_unit[kind] + extra.get(kind, 0)
            groups.setdefault(label, []).extend(xs[i:i + n])
            if label.startswith("I_") and n:
                blocks.append((label, statistics.fmean(xs[i:i + n])))
            i += n
        if i != len(xs):
            out["kernels"][kind] = {"error": f"expected {i} launches, found {len(xs)}"}
            continue
        mean = {g: statistics.fmean(v) for g, v in groups.items() if v}
        base_abc = 0.5 * (mean["A_off"] + mean["C_off"])
        r = {"mean_us": {g: round(m, 3) for g, m in mean.items()},
             "launches": {g: len(v) for g, v in groups.items()},
             "B_vs_AC_pct": 100.0 * (mean["B_on_8k"] / base_abc - 1.0)}
        if "I_paused" in mean:
            for g in mean:
                if g.startswith("I_") and g != "I_paused":
                    r[f"{g}_vs_paused_pct"] = 100.0 * (mean[g] / mean["I_paused"] - 1.0)
            ncond = len({lb for lb, _ in blocks})
            rounds = [dict(blocks[j:j + ncond]) for j in range(0, len(blocks) - ncond + 1, ncond)]
            for g in mean:
                if not g.startswith("I_") or g == "I_paused":
                    continue
                d = [100.0 * (rd[g] / rd["I_paused"] - 1.0) for rd in rounds if g in rd and "I_paused" in rd]
                if len(d) >= 2:
                    r[f"{g}_vs_paused_paired_pct"] = statistics.fmean(d)
                    r[f"{g}_vs_paused_ci95_pct"] = 1.96 * statistics.stdev(d) / len(d) ** 0.5
                    r["rounds"] = len(d)
        out["kernels"][kind] = r
    print(json.dumps(out, indent=1))
    if a.out:
        conds = ["A_off", "B_on_8k", "C_off", "I_paused", "I_100Hz", "I_8000Hz"]
        lines = ["# Per-kernel GPU time by exporter condition (rocprofv3 kernel trace of bench.py)", "",
                 f"Trace: `{out['trace']}` ({out['kernels_total']} kernels), assigned to bench segments by "
                 "launch order (`tools/rocprof_overhead.py`).  A / C: no exporter process; B: sampling at 8 kHz; "
                 "I_*: interleaved blocks, exporter paused or sampling at 100 Hz / 8 kHz.", "",
                 "| kernel | " + " | ".join(f"{c} mean µs" for c in conds) + " | B vs A/C % | 100 Hz vs paused % | "
                 "8 kHz vs paused % | 100 Hz paired (95 % CI) | 8 kHz paired (95 % CI) |", "|---" * (len(conds) + 6) + "|"]
        for kind, r in out["kernels"].items():
            if "error" in r:
                lines.append(f"| {kind} | {r['error']} |")
                continue
            m = r["mean_us"]
            cells = " | ".join(f"{m[c]:.3f}" if c in m else "" for c in conds)
            pair = lambda g: (f"{r[g + '_vs_paused_paired_pct']:+.3f} ± {r[g + '_vs_paused_ci95_pct']:.3f}"  # noqa: E731
                              if g + "_vs_paused_ci95_pct" in r else "")
            lines.append(f"| {kind} | {cells} | {r['B_vs_AC_pct']:+.3f} | {r.get('I_100Hz_vs_paused_pct', 0):+.3f} | "
                         f"{r.get('I_8000Hz_vs_paused_pct', 0):+.3f} | {pair('I_100Hz')} | {pair('I_8000Hz')} |")
        if any("rounds" in r for r in out["kernels"].values()):
            lines += ["", f"Paired: {max(r.get('rounds', 0) for r in out['kernels'].values())} rounds, each tier's "
                      "block against the paused block of the same round."]
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
