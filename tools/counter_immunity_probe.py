#!/usr/bin/env python3
"""Which device-mode counters see real work but not the sampler's own READs?

Every counter READ is a PM4 packet on the command processor, and GRBM_GUI_ACTIVE
(and the PMFW GFX busy) count it as ≈190 µs (≈80 µs) of work on an idle MI355X
(tools/idle_busy_probe.py).  An activity signal that a high-rate sampler can trust
must stay at 0 while only READs run, and rise with kernels.  SQ_BUSY_CYCLES /
SQ_WAVES would be ideal but read 0 in device mode (only waves dispatched with the
perf-count enable count, profiles/pmc_probe.md), so this tries the SPI and GRBM
wave-presence counters.

Opens libkgs_pmc_aql.so directly (ctypes, no HIP in this process), samples at
--hz with pipelined READs through three phases: idle (READs only), a child process
running an MFMA load, idle again.  Prints per-phase rates of each counter as a
fraction of GRBM_COUNT.

    python tools/counter_immunity_probe.py --out gpurun_out/immunity.json
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "kube_gpu_stats_amd", "lib", "libkgs_pmc_aql.so")

# one session per set (GRBM has two counter slots per XCC)
SETS = {
    "spi": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SPI:225", "SPI:1", "SPI:7", "SPI:13", "SPI:19"],
    "grbm_spi": ["GRBM_COUNT", "GRBM:11", "SQ_VALU_MFMA_BUSY_CYCLES", "TA_TA_BUSY"],
    "grbm_cp": ["GRBM_COUNT", "GRBM:3", "SQ:3", "SQ:4"],
    # the exporter's base set, and variants of it
    "product": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SPI_CSC_WAVE_CNT_BUSY"],
    "product_num": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SPI:225"],
    "spi_first": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SPI:225", "SQ_VALU_MFMA_BUSY_CYCLES"],
    "no_sq": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SPI_CSC_WAVE_CNT_BUSY"],
    "grbm_spi": ["GRBM_COUNT", "GRBM:11", "SQ_VALU_MFMA_BUSY_CYCLES"],
    "grbm_spi_mfma": ["GRBM_COUNT", "GRBM:11", "SQ_VALU_MFMA_BUSY_CYCLES", "SPI_CSC_WAVE_CNT_BUSY"],
}
LOAD = r"""
import sys, time, torch
sys.path.insert(0, %r)
from kube_gpu_stats_amd.ops.load import LoadStep
ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=1 << 30)
ls.run_mfma(); torch.cuda.synchronize()
if "--wait" in sys.argv:  # the queue exists (and has run a kernel) before the counting session starts
    print("ready", flush=True)
    sys.stdin.readline()
print("start", time.monotonic_ns(), flush=True)
t0 = time.time()
while time.time() - t0 < 1.5:
    ls.run_mfma(); torch.cuda.synchronize()
print("end", time.monotonic_ns(), flush=True)
"""


def kfd_gpu_id() -> int:
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")):
        try:
            with open(p) as f:
                v = int(f.read().strip() or 0)
        except OSError:  # nodes of GPUs outside this lease
            continue
        if v:
            return v
    raise SystemExit("no KFD GPU node")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hz", type=float, default=8000)
    ap.add_argument("--sets", default=",".join(SETS))
    ap.add_argument("--pre-queue", action="store_true",
                    help="the load process creates its queue and runs a kernel BEFORE the session starts")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    L = ctypes.CDLL(LIB)
    err = ctypes.create_string_buffer(512)
    if L.kgs_pmc_init(err, 512) != 0:
        raise SystemExit("init: " + err.value.decode())
    gid = kfd_gpu_id()
    out = {"hz": a.hz, "kfd_gpu_id": gid, "pre_queue": a.pre_queue, "sets": {}}
    for name in a.sets.split(","):
        child = None
        if a.pre_queue:
            child = subprocess.Popen([sys.executable, "-c", LOAD % REPO, "--wait"], stdin=subprocess.PIPE,
                                     stdout=subprocess.PIPE, text=True)
            assert child.stdout.readline().strip() == "ready"
        names = SETS[name]
        n = len(names)
        arr = (ctypes.c_char_p * n)(*[x.encode() for x in names])
        red = (ctypes.c_int * n)(*[1 if x.startswith("GRBM") else 2 for x in names])
        h = L.kgs_pmc_open(ctypes.c_uint64(gid), arr, red, n, err, 512)
        if h < 0:
            out["sets"][name] = {"error": err.value.decode()}
            print(name, "open failed:", err.value.decode(), flush=True)
            continue
        L.kgs_pmc_set_pipelined(h, 1, err, 512)
        info = ctypes.create_string_buffer(4096)
        L.kgs_pmc_info(h, info, 4096)
        vals = (ctypes.c_uint64 * n)()
        rns = ctypes.c_uint32()
        sns = ctypes.c_int64()
        samples = []  # (t_ns, values)
        if child is None:
            child = subprocess.Popen([sys.executable, "-c", LOAD % REPO], stdout=subprocess.PIPE, text=True)
        else:
            child.stdin.write("go\n")
            child.stdin.flush()
        marks = {}
        period = 1.0 / a.hz
        t_end = time.monotonic() + 60
        nxt = time.monotonic()
        done_at = None
        os.set_blocking(child.stdout.fileno(), False)
        buf = ""
        while time.monotonic() < t_end:
            if L.kgs_pmc_sample_ts(h, vals, n, ctypes.byref(rns), ctypes.byref(sns)) == 0 and sns.value > 0:
                samples.append((sns.value, list(vals)))
            try:
                chunk = child.stdout.read()
            except (BlockingIOError, TypeError):
                chunk = None
            if chunk:
                buf += chunk
                for ln in buf.splitlines():
                    k, _, v = ln.partition(" ")
                    if k in ("start", "end") and v.strip().isdigit():
                        marks[k] = int(v)
            if "end" in marks and done_at is None:
                done_at = time.monotonic()
            if done_at is not None and time.monotonic() - done_at > 1.0:
                break
            nxt += period
            d = nxt - time.monotonic()
            if d > 0:
                time.sleep(d)
            else:
                nxt = time.monotonic()
        child.wait(timeout=30)
        L.kgs_pmc_close(h)
        s0, e0 = marks.get("start", 0), marks.get("end", 0)

        def rates(lo, hi):
            pts = [s for s in samples if lo <= s[0] <= hi]
            if len(pts) < 2:
                return None
            dv = [b - a_ for a_, b in zip(pts[0][1], pts[-1][1])]
            cnt = dv[0] or 1
            return {"drains": len(pts), "secs": (pts[-1][0] - pts[0][0]) * 1e-9,
                    **{names[k]: dv[k] / cnt for k in range(1, n)}}
        first = samples[0][0] if samples else 0
        res = {"names": names, "info": info.value.decode(), "phases": {
            "idle_reads_only": rates(first + 200_000_000, s0 - 100_000_000) if s0 else None,
            "mfma_load": rates(s0 + 100_000_000, e0 - 100_000_000) if s0 and e0 else None,
            "idle_after": rates(e0 + 200_000_000, samples[-1][0]) if e0 and samples else None}}
        out["sets"][name] = res
        print(json.dumps({name: res}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
