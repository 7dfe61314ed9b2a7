"""Split a rocprofv3 kernel trace of ``bench.py`` into its phases and compare
per-kernel GPU time with the exporter off (A, C) and on (B).

bench.py launches, per rank: W warm-up steps, one calibration step, then K steps
in each of phases A, B, C; a step is one ``mfma_bf16_kernel`` followed by
``--triads`` ``triad_f32_kernel`` launches.  Kernels are assigned to phases by
launch order, so no clock translation between rocprofv3 and Python is needed.

    python tools/rocprof_overhead.py <trace dir> --warmup W --steps K [--triads 2] [--out md]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--triads", type=int, default=2)
    ap.add_argument("--tiny", type=int, default=2000, help="tiny copy kernels per step (bench --tiny-kernels)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    path = find_trace(a.dir)
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = {"mfma": [], "triad": [], "copy": []}
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3  # µs
        if "mfma_bf16_kernel" in name:
            by["mfma"].append(dur)
        elif "triad_f32_kernel" in name:
            by["triad"].append(dur)
        elif "copy_f32_kernel" in name:
            by["copy"].append(dur)
    res = {"trace": os.path.relpath(path), "kernels_total": len(rows)}
    kinds = [("mfma", 1), ("triad", a.triads)] + ([("copy", a.tiny)] if a.tiny else [])
    for kind, per_step in kinds:
        xs = by[kind]
        # the calibration step launches one mfma + one triad (+ one graph replay);
        # the tiny-kernel graph is preceded by one eager warm-up copy
        skip = a.warmup * per_step + (1 if kind != "copy" else 1 + per_step)
        n = a.steps * per_step
        ph = {"A_off": xs[skip:skip + n], "B_on": xs[skip + n:skip + 2 * n], "C_off": xs[skip + 2 * n:skip + 3 * n]}
        if any(len(v) != n for v in ph.values()):
            res[kind] = {"error": f"expected {3 * n + skip} launches, found {len(xs)}"}
            continue
        med = {k: statistics.median(v) for k, v in ph.items()}
        mean = {k: statistics.fmean(v) for k, v in ph.items()}
        off = 0.5 * (mean["A_off"] + mean["C_off"])
        res[kind] = {"median_us": med, "mean_us": mean, "launches_per_phase": n,
                     "gpu_time_overhead_pct": 100.0 * (mean["B_on"] / off - 1.0)}
    print(json.dumps(res, indent=1))
    if a.out:
        lines = ["# GPU-time overhead from a rocprofv3 kernel trace of bench.py", "",
                 f"Trace: `{res['trace']}` ({res['kernels_total']} kernels). Phases by launch order: "
                 f"warm-up {a.warmup} + 1 calibration step, then {a.steps} steps each of A (exporter off), "
                 "B (exporter on), C (exporter off).", "",
                 "| kernel | launches/phase | A off mean µs | B on mean µs | C off mean µs | overhead % (B vs mean(A,C)) |",
                 "|---|---|---|---|---|---|"]
        for kind, _ in kinds:
            r = res[kind]
            if "error" in r:
                lines.append(f"| {kind} | {r['error']} | | | | |")
                continue
            m = r["mean_us"]
            lines.append(f"| {kind} | {r['launches_per_phase']} | {m['A_off']:.1f} | {m['B_on']:.1f} | "
                         f"{m['C_off']:.1f} | {r['gpu_time_overhead_pct']:+.3f} |")
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
