#!/usr/bin/env python3
"""GPU probe: the billed busy integral at a low counter rate, against the kernels' own time.

At ``--hz`` (default 10, the DaemonSet's) the exporter runs in this process (amdsmi
backend, aqlprofile counters, default flags) while a train of ``--burst-ms`` MFMA
kernels every ``--period-ms`` runs for ``--load-s`` between idle stretches.  Every
50 ms the probe records the exporter's integrals (``util_seconds`` — what
container_gpu_busy_seconds_total bills —, ``dispatch_seconds``, ``sampled_seconds``,
the biller's carry, the last drain's time) next to the cumulative event-timed GPU time
of the kernels, and it keeps every counter drain of the window (``/counters``-style
rows: t, GRBM_COUNT, GRBM_SPI_BUSY, CPC busy, MFMA busy, se_fresh) so the estimator can
be replayed offline (``tools/util_estimator_sim.py``).  Output: JSON.

``python tools/lowrate_probe.py --hz 10 --out gpurun_out/lowrate.json``
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
# the DispatchEstimator.replay row order: t_s, count, spi, cpc, mfma, se_fresh
DRAIN_COLS = ("GRBM_COUNT", "GRBM_SPI_BUSY", "CPC_CPC_STAT_BUSY", "SQ_VALU_MFMA_BUSY_CYCLES")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--hz", type=float, default=10.0)
    ap.add_argument("--burst-ms", type=float, default=1.0)
    ap.add_argument("--period-ms", type=float, default=5.0)
    ap.add_argument("--idle-s", type=float, default=2.0)
    ap.add_argument("--load-s", type=float, default=8.0)
    ap.add_argument("--batch", type=int, default=8, help="the exporter's --pmc-batch")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "lowrate.json"))
    a = ap.parse_args(argv)

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
    ms_per_iter = e0.elapsed_time(e1) / 4000
    iters = max(10, int(a.burst_ms / ms_per_iter))

    ex = N.Exporter({"backend": "amdsmi", "hz": a.hz, "port": -1, "pmc_source": "aqlprofile",
                     "pmc_lib": pmc_lib_path("aqlprofile"), "proc_period_s": 0, "link_period_s": 0,
                     "pmc_batch": a.batch})
    assert not ex.pmc_error, ex.pmc_error
    ex.start()
    gpu_busy = [0.0]
    trace: list[dict] = []
    stop = threading.Event()
    t_base = time.monotonic()

    drains: list[list] = []
    t_base_ns = time.monotonic_ns()

    def sampler():
        seq = -1
        while not stop.is_set():
            i = ex.integrals(0)
            trace.append({"t": round(time.monotonic() - t_base, 4), "gpu_s": round(gpu_busy[0], 6),
                          "util_s": i["util_seconds"], "dispatch_s": i["dispatch_seconds"],
                          "pmfw_s": i["gfx_busy_seconds"], "sampled_s": i["sampled_seconds"],
                          "carry_s": i["util_carry_seconds"], "from_counters_s": i["util_counter_seconds"],
                          "drains": i["pmc_samples"]})
            p = ex.pmc(0)
            if p is not None and p["seq"] != seq:  # at <= 20 Hz every drain is seen
                seq = p["seq"]
                v = p["values"]
                # at <= 1 kHz every READ publishes and reads the per-SE counters: se_fresh 1
                drains.append([(p["mono_ns"] - t_base_ns) * 1e-9] + [v.get(k, -1) for k in DRAIN_COLS] + [1])
            time.sleep(0.02)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    marks = {}
    try:
        time.sleep(a.idle_s)
        marks["load_start"] = time.monotonic() - t_base
        a_ev, b_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        nxt = time.monotonic()
        end = nxt + a.load_s
        while time.monotonic() < end:
            a_ev.record()
            load.mfma_bf16(ls.A, ls.B, ls.C, 2048, iters)
            b_ev.record()
            b_ev.synchronize()
            gpu_busy[0] += a_ev.elapsed_time(b_ev) * 1e-3
            nxt += a.period_ms * 1e-3
            d = nxt - time.monotonic()
            if d > 0:
                time.sleep(d)
        marks["load_end"] = time.monotonic() - t_base
        time.sleep(a.idle_s)
    finally:
        stop.set()
        th.join(timeout=5)
        ex.stop()
    # lag: after the load ends, when does the billed integral reach its final value?
    fin = trace[-1]["util_s"]
    after = [r for r in trace if r["t"] >= marks["load_end"]]
    settle = next((r["t"] - marks["load_end"] for r in after if fin - r["util_s"] < 1e-3), None)
    s0 = next(r for r in trace if r["t"] >= marks["load_start"] - 0.5)
    s1 = trace[-1]
    out = {"hz": a.hz, "burst_ms": a.burst_ms, "period_ms": a.period_ms, "marks": marks,
           "gpu_busy_s": gpu_busy[0], "billed_s": s1["util_s"] - s0["util_s"],
           "dispatch_s": s1["dispatch_s"] - s0["dispatch_s"], "settle_after_load_s": settle,
           "pmfw_s": s1["pmfw_s"] - s0["pmfw_s"], "drain_cols": ["t"] + list(DRAIN_COLS) + ["se_fresh"],
           "trace": trace, "drains": drains}
    out["billed_minus_gpu_s"] = round(out["billed_s"] - out["gpu_busy_s"], 4)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f)
    print(json.dumps({k: v for k, v in out.items() if k not in ("trace", "drains")}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
