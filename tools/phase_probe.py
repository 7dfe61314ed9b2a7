#!/usr/bin/env python3
"""GPU probe: does the READ phase lock onto a periodic workload?

A train of ``--burst-ms`` MFMA kernels every ``--period-ms`` with absolute deadlines keeps one
phase against a fixed counter tick for seconds (1 ms against 125 µs at 8 kHz), so the
estimator's per-interval rules (the ≥ 90 % full-interval rule, the READ cost subtracted
from partial intervals) err the same way on every kernel of a window — and a different
way in the next window, whose phase is another.  For each ``--dither`` value the exporter
runs in this process (amdsmi, aqlprofile, ``--hz``, batch 8, lite READs) and the probe runs
``--windows`` windows of ``--window-s``, each started at a random offset within a period:
per window, the dispatch integral's increment against the kernels' event-timed time.
The spread of the per-window error across windows is the phase-lock effect.

``python tools/phase_probe.py --out gpurun_out/phase.json``
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--hz", type=float, default=8000.0)
    ap.add_argument("--burst-ms", type=float, default=0.2)
    ap.add_argument("--period-ms", type=float, default=1.0)
    ap.add_argument("--windows", type=int, default=12)
    ap.add_argument("--window-s", type=float, default=1.0)
    ap.add_argument("--dither", default="0,0.25")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "phase.json"))
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if not a.child:
        # one process per dither value: the counter reader opens the GPU agent once per process
        import subprocess

        out: dict = {"hz": a.hz, "burst_ms": a.burst_ms, "period_ms": a.period_ms, "window_s": a.window_s,
                     "by_dither": {}}
        for dither in a.dither.split(","):
            r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", "--dither", dither,
                                "--hz", str(a.hz), "--burst-ms", str(a.burst_ms), "--period-ms", str(a.period_ms),
                                "--windows", str(a.windows), "--window-s", str(a.window_s), "--seed", str(a.seed)],
                               capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not line:
                out["by_dither"][dither] = {"error": r.stderr[-500:]}
                break
            res = json.loads(line[-1])
            out["by_dither"][f"{float(dither):g}"] = res
            print(json.dumps(res), flush=True)
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
        return 0

    import torch

    from kube_gpu_stats_amd import load_native
    from kube_gpu_stats_amd.native import pmc_lib_path
    from kube_gpu_stats_amd.ops import load
    from kube_gpu_stats_amd.ops.load import LoadStep

    N = load_native()
    ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=1 << 26)
    ls.run_mfma()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    load.mfma_bf16(ls.A, ls.B, ls.C, 2048, 4000)
    e1.record()
    torch.cuda.synchronize()
    iters = max(10, int(a.burst_ms / (e0.elapsed_time(e1) / 4000)))
    rnd = random.Random(a.seed)
    for dither in [float(a.dither)]:
        ex = N.Exporter({"backend": "amdsmi", "hz": a.hz, "port": -1, "pmc_source": "aqlprofile",
                         "pmc_lib": pmc_lib_path("aqlprofile"), "proc_period_s": 0, "link_period_s": 0,
                         "pmc_batch": 8, "tick_dither": dither})
        assert not ex.pmc_error, ex.pmc_error
        ex.start()
        errs = []
        try:
            time.sleep(1.0)  # READ cost and clocks learned on the idle GPU
            for _ in range(a.windows):
                time.sleep(0.3 + rnd.uniform(0, a.period_ms * 1e-3))
                i0, t0 = ex.integrals(0), time.monotonic()
                gpu, nxt = 0.0, time.monotonic()
                end = nxt + a.window_s
                ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                while time.monotonic() < end:
                    ea.record()
                    load.mfma_bf16(ls.A, ls.B, ls.C, 2048, iters)
                    eb.record()
                    eb.synchronize()
                    gpu += ea.elapsed_time(eb) * 1e-3
                    nxt += a.period_ms * 1e-3
                    d = nxt - time.monotonic()
                    if d > 0:
                        time.sleep(d)
                time.sleep(0.02)  # the last drains publish (≤ 1 ms) inside the window
                i1, t1 = ex.integrals(0), time.monotonic()
                win = t1 - t0
                errs.append(round(100 * ((i1["dispatch_seconds"] - i0["dispatch_seconds"]) - gpu) / win, 3))
            reads = ex.integrals(0)["pmc_samples"]
        finally:
            ex.stop()
        print(json.dumps({"dither": dither, "error_pts": errs, "mean": round(statistics.mean(errs), 3),
                          "sd": round(statistics.stdev(errs), 3) if len(errs) > 1 else 0.0,
                          "worst": round(max(errs, key=abs), 3), "reads": reads}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
