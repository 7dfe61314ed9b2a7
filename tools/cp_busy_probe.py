#!/usr/bin/env python3
"""Is there a READ-immune "a dispatch is in flight" signal?  (follow-up)

tools/sm_util_probe.py showed that GRBM_SPI_BUSY ("a shader engine has waves") is blind
to the exporter's READs but reads a HIP graph of µs kernels at ≈42 % while kernels are
in flight back to back (the PMFW GFX busy, like NVML's utilisation, reads ≈100 %).  The
command processor's own busy counters (CPC_CPC_STAT_BUSY, CPF_CPF_STAT_BUSY) read
≈100 % whenever any kernel is in flight (profiles/r3/README.md r3b) and count each READ
packet for a short, fixed time — unlike the PMFW busy, whose per-READ cost grows with
the READ rate until it saturates.  If that per-READ cost is small and additive, the
CP busy minus (READs × cost) is a dispatch-in-flight signal that the exporter's own
READs cannot fake.

A child process reads [GRBM_COUNT, GRBM_SPI_BUSY, CPC_CPC_STAT_BUSY, CPF_CPF_STAT_BUSY]
(GRBM and CP busy max-reduced over the XCCs) through libkgs_pmc_aql.so at a fixed READ
rate and prints every sample; the parent runs known loads — idle, back-to-back MFMA
kernels, HBM triads, bf16 GEMMs, a graph of µs copies, MFMA burst trains — and reports,
per READ rate and load, each counter's share of wall time (Σ per-interval share × Δt)
next to the kernels' own GPU time (HIP events).  ``python tools/cp_busy_probe.py --out
gpurun_out/cp_busy_probe.json`` on a GPU box.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

NAMES = ["GRBM_COUNT", "GRBM_SPI_BUSY", "CPC:25", "CPF:23"]
# --exporter-set 1: the exporter's base set, in this column order (4th column MFMA busy, not CPF)
EXPORTER_NAMES = ["GRBM_COUNT", "GRBM_SPI_BUSY", "CPC:25", "SQ_VALU_MFMA_BUSY_CYCLES"]
KEYS = ["count", "spi", "cpc", "cpf"]


def kfd_gpu_id() -> int:
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")):
        try:
            v = int(open(p).read().strip() or 0)
        except OSError:
            continue
        if v:
            return v
    raise RuntimeError("no KFD GPU node")


def child(hz: float, secs: float, pipelined: bool, batch: int = 1, lite: int = 0, exporter_set: int = 0) -> int:
    from kube_gpu_stats_amd.native import pmc_lib_path

    L = ctypes.CDLL(pmc_lib_path("aqlprofile"))
    err = ctypes.create_string_buffer(512)
    L.kgs_pmc_configure(b"batch", batch)  # as the exporter configures the reader (--pmc-batch, --pmc-lite)
    L.kgs_pmc_configure(b"lite", lite)
    if L.kgs_pmc_init(err, 512) != 0:
        print(json.dumps({"error": "init: " + err.value.decode()}), flush=True)
        return 1
    # the exporter's base set in the dump's column order (the 4th column is then MFMA busy, not CPF)
    names = EXPORTER_NAMES if exporter_set else NAMES
    n = len(names)
    arr = (ctypes.c_char_p * n)(*[s.encode() for s in names])
    red = (ctypes.c_int * n)(*([1, 1, 1, 0] if exporter_set else [1] * n))  # max over XCCs; MFMA summed
    L.kgs_pmc_open.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p,
                               ctypes.c_int]
    h = L.kgs_pmc_open(kfd_gpu_id(), arr, red, n, err, 512)
    if h < 0:
        print(json.dumps({"error": "open: " + err.value.decode()}), flush=True)
        return 1
    if pipelined:  # the exporter's 8 kHz mode: each call returns the previous READ, stamped at its CP time
        if L.kgs_pmc_set_pipelined(h, 1, err, 512) != 0:
            print(json.dumps({"error": "pipelined: " + err.value.decode()}), flush=True)
            return 1
    print(json.dumps({"ready": True}), flush=True)
    out = (ctypes.c_uint64 * n)()
    rns = ctypes.c_uint32()
    sns = ctypes.c_int64()
    period = 1.0 / hz
    t_end = time.perf_counter() + secs
    nxt = time.perf_counter()
    buf = []
    while True:
        now = time.perf_counter()
        if now >= t_end:
            break
        if now < nxt:
            if nxt - now > 3e-4:
                time.sleep(nxt - now - 2e-4)
            continue
        rc = L.kgs_pmc_sample_ts(h, out, n, ctypes.byref(rns), ctypes.byref(sns))
        if rc == 0:
            # the time the CP read the values (pipelined: the previous call's READ), on the wall clock;
            # then whether that READ read the per-SE counters (lite READs: 0)
            buf.append((time.time() - (time.monotonic_ns() - sns.value) * 1e-9, list(out) + [L.kgs_pmc_se_fresh(h)]))
        nxt += period
        if nxt < now - 10 * period:
            nxt = now
        if len(buf) >= 2000:
            print(json.dumps(buf), flush=True)
            buf = []
    if buf:
        print(json.dumps(buf), flush=True)
    L.kgs_pmc_close(h)
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--rates", default="100,1000,8000")
    ap.add_argument("--secs", type=float, default=2.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--batch", type=int, default=1, help="reader batch (the exporter's --pmc-batch)")
    ap.add_argument("--lite", type=int, default=0, choices=[0, 1], help="lite READs (the exporter's --pmc-lite)")
    ap.add_argument("--exporter-set", type=int, default=0, choices=[0, 1],
                    help="read the exporter's base set (4th column MFMA busy instead of CPF busy)")
    ap.add_argument("--pipelined", type=int, default=0, choices=[0, 1],
                    help="READ pipelined, as the exporter does above its idle rate")
    ap.add_argument("--dump", default="", help="write every raw sample of the --dump-rates runs here (JSON)")
    ap.add_argument("--dump-rates", default="8000")
    ap.add_argument("--irregular", type=int, default=0, choices=[0, 1],
                    help="also the out-of-sample loads of ops/irregular.py (VERDICT r5 #3): seeded random MFMA "
                    "kernels and gaps on one and two streams, and a bf16 training step (profiler-timed)")
    ap.add_argument("--only-irregular", type=int, default=0, choices=[0, 1],
                    help="with --irregular: idle + the irregular loads only (the held-out dumps)")
    ap.add_argument("--child", type=float, default=0.0, help=argparse.SUPPRESS)
    ap.add_argument("--child-secs", type=float, default=0.0, help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.child:
        return child(a.child, a.child_secs, bool(a.pipelined), a.batch, a.lite, a.exporter_set)

    import torch

    sys.path.insert(0, os.path.join(REPO, "tools"))
    from sm_util_probe import Loads

    loads = Loads(torch)
    names = ["idle", "mfma", "triad", "gemm", "tiny_graph", "burst_1_5", "burst_02_1"]
    irr = train = None
    if a.irregular:
        from kube_gpu_stats_amd.ops.irregular import IrregularLoad, mfma_launcher, profiled_busy

        irr = IrregularLoad(torch, mfma_launcher(torch, loads.ls, loads.ms_per_iter))
        import bench

        ta = bench.parse_args(["--train-dim", "2048", "--train-layers", "4", "--train-batch", "4", "--train-seq", "1024"])
        train = bench.TrainLoad(ta, 0, None)
        for _ in range(2):
            train.unit()
        torch.cuda.synchronize()
        names = (["idle"] if a.only_irregular else names) + ["random_kernels", "two_stream_random", "train_step"]
    seeds = {"random_kernels": (71, 1), "two_stream_random": (72, 2)}

    def gpu_busy(name: str, secs: float) -> float:
        """Event-timed kernel seconds (bursts: event-timed too, not host-timed)."""
        if name.startswith("burst"):
            ms, per = (1.0, 5.0) if name == "burst_1_5" else (0.2, 1.0)
            iters = max(20, int(ms / loads.ms_per_iter))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            busy, nxt = 0.0, time.monotonic()
            end = nxt + secs
            while time.monotonic() < end:
                e0.record()
                loads.L.mfma_bf16(loads.ls.A, loads.ls.B, loads.ls.C, 2048, iters)
                e1.record()
                e1.synchronize()
                busy += e0.elapsed_time(e1) * 1e-3
                nxt += per * 1e-3
                d = nxt - time.monotonic()
                if d > 0:
                    time.sleep(d)
            return busy
        if name in seeds:
            return irr.run(secs, seeds[name][0], seeds[name][1])["busy_s"]
        if name == "train_step":
            return profiled_busy(torch, train.unit, secs)[0]
        return getattr(loads, "run_" + name)(secs)

    out: dict = {"counters": NAMES, "rates": {}, "pipelined": a.pipelined}
    dumps: dict = {}
    # the profiler-timed training step returns seconds after its last kernel (trace
    # post-processing): the reader must outlive every load's window, or the replay
    # compares busy over a short READ span with the duty over the whole window
    total = len(names) * (a.secs + 0.6) + 2.0 + (30.0 if a.irregular else 0.0)
    for hz in [float(x) for x in a.rates.split(",")]:
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", str(hz), "--child-secs",
                              str(total), "--pipelined", str(a.pipelined), "--batch", str(a.batch), "--lite", str(a.lite),
                              "--exporter-set", str(a.exporter_set)], stdout=subprocess.PIPE, text=True,
                             cwd=REPO)
        first = json.loads(p.stdout.readline())
        if "error" in first:
            out["rates"][f"{hz:g}"] = first
            p.wait()
            continue
        # Drain the child's stdout while the loads run: a full pipe would block its
        # print, and with it the sampling, until the loads end.
        lines: list[str] = []
        reader = threading.Thread(target=lambda: lines.extend(p.stdout), daemon=True)
        reader.start()
        time.sleep(0.5)
        marks = {}
        for name in names:
            time.sleep(0.3)
            t0 = time.time()
            busy = gpu_busy(name, a.secs)
            t1 = time.time()
            marks[name] = (t0, t1, busy)
        p.wait()
        reader.join(timeout=30)
        samples = []
        for line in lines:
            samples.extend(json.loads(line))
        res = {}
        for name, (t0, t1, busy) in marks.items():
            win = [s for s in samples if t0 <= s[0] <= t1]
            if len(win) < 3:
                continue
            acc = {k: 0.0 for k in KEYS[1:]}
            for (ta, va), (tb, vb) in zip(win, win[1:]):
                dc = vb[0] - va[0]
                if dc <= 0:
                    continue
                for i, k in enumerate(KEYS[1:], start=1):
                    acc[k] += min(1.0, max(0.0, (vb[i] - va[i]) / dc)) * (tb - ta)
            span = win[-1][0] - win[0][0]
            res[name] = {"duty_gpu_pct": round(100 * busy / (t1 - t0), 2),
                         **{f"{k}_pct": round(100 * v / span, 2) for k, v in acc.items()},
                         "reads_per_s": round(len(win) / span, 1)}
        # CP busy per READ on the idle GPU
        if "idle" in res:
            r = res["idle"]
            res["cpc_us_per_read_idle"] = round(1e4 * r["cpc_pct"] / r["reads_per_s"], 2) if r["reads_per_s"] else None
            res["cpf_us_per_read_idle"] = round(1e4 * r["cpf_pct"] / r["reads_per_s"], 2) if r["reads_per_s"] else None
        out["rates"][f"{hz:g}"] = res
        if a.dump and f"{hz:g}" in a.dump_rates.split(","):
            raw = {name: {"t0": t0, "t1": t1, "duty_gpu_s": busy,
                          "samples": [[round(ts - t0, 7)] + v for ts, v in samples if t0 - 0.01 <= ts <= t1 + 0.01]}
                   for name, (t0, t1, busy) in marks.items()}
            dumps[f"{hz:g}"] = raw
        print(json.dumps({f"{hz:g}": res}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    if a.dump:
        os.makedirs(os.path.dirname(os.path.abspath(a.dump)), exist_ok=True)
        with open(a.dump, "w") as f:
            names = EXPORTER_NAMES if a.exporter_set else NAMES
            json.dump({"counters": names, "columns": ["t_s", *names, "se_fresh"], "pipelined": a.pipelined,
                       "batch": a.batch, "lite": a.lite, "rates": dumps}, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
