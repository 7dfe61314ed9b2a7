"""GPU probe: which hardware counters count device-wide through the direct
aqlprofile reader (libkgs_pmc_aql.so), under known synthetic loads.

Parent (this script): runs idle / MFMA / triad / copy phases with the gfx950
load kernels and records phase boundaries.  Child (``--child``): opens the
counter set on the GPU through the same C ABI the exporter uses and prints one
JSON line of cumulative values every 20 ms.  Per-phase rates are written to
gpurun_out/aql_probe.json.  Expected bytes per phase are known from the kernels
(triad: 2 reads + 1 write of N floats; copy: 1 + 1), so TCC request counts can
be checked against them (64 B / 128 B requests).
"""
from __future__ import annotations

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)

import ctypes
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SETS = {
    "tcc_size": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "TCC:42", "TCC:43", "TCC:30", "TCC:31"],
    "tcc_dram": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "TCC:108", "TCC:109", "TCC:62", "TCC:44"],
    "tcc_req": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "TCC:6", "TCC:21", "TCC:23", "TCC:45"],
    "sq": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ:4", "SQ:26", "SQ:3", "SQ_VALU_MFMA_BUSY_CYCLES"],
    "tcp": ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "TCP:68", "TCP:69", "TA_TA_BUSY"],
    # Round 3: is there a device-wide "command processor is the bottleneck" signal?
    # CPC_ADC_DISPATCH_ALLOC_DONE (4) / CPC_TG_SEND (62) count dispatches and
    # workgroups, which the exporter's own PM4 READs are not; the busy counters
    # (CPC_CPC_STAT_BUSY 25, ME1 packet decode 13, CPF_CPF_STAT_BUSY 23, GRBM_CP*_BUSY)
    # would also count the READs.  counter_defs.yaml, architectures: gfx950.
    "cpc_dispatch": ["GRBM_COUNT", "GRBM_SPI_BUSY", "CPC:4", "CPC:62"],
    "cpc_busy": ["GRBM_COUNT", "GRBM_SPI_BUSY", "CPC:25", "CPC:13", "CPF:23", "CPF:25"],
    "cpc_gd": ["GRBM_COUNT", "GRBM_SPI_BUSY", "CPC:61", "CPC:33"],
    "grbm_cp": ["GRBM:3", "GRBM:30"],
    "spi_csn": ["GRBM_COUNT", "GRBM_SPI_BUSY", "SPI:49", "SPI:52"],
    # Round 5: a counter-tier HBM bandwidth (BASELINE config 4)?  TCC's DRAM request
    # counters need per-dispatch perf enables other processes' kernels lack; the memory
    # controllers' own blocks, if aqlprofile programs them on gfx950, would not.  No
    # event list ships for them (counter_defs.yaml has none for gfx950): try the low ids.
    "umc_a": ["GRBM_COUNT", "GRBM_SPI_BUSY", "UMC:0", "UMC:1", "UMC:2", "UMC:3"],
    "umc_b": ["GRBM_COUNT", "GRBM_SPI_BUSY", "UMC:4", "UMC:5", "UMC:6", "UMC:7"],
    "mmea": ["GRBM_COUNT", "GRBM_SPI_BUSY", "MMEA:0", "MMEA:1", "MMEA:2", "MMEA:3"],
    "gcea": ["GRBM_COUNT", "GRBM_SPI_BUSY", "GCEA:0", "GCEA:1", "GCEA:2", "GCEA:3"],
    # r5d: UMC and MMEA validate no event on gfx950; GCEA takes two counters per session
    **{f"gcea{i}": ["GRBM_COUNT", "GRBM_SPI_BUSY", f"GCEA:{2 * i}", f"GCEA:{2 * i + 1}"] for i in range(8)},
}


def kfd_gpu_ids() -> list[int]:
    ids = []
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")):
        try:
            v = int(open(p).read().strip() or 0)
        except OSError:
            continue
        if v:
            ids.append(v)
    return ids


def child(names: list[str], secs: float) -> int:
    from kube_gpu_stats_amd.native import pmc_lib_path

    L = ctypes.CDLL(pmc_lib_path("aqlprofile"))
    err = ctypes.create_string_buffer(512)
    if L.kgs_pmc_init(err, 512) != 0:
        print(json.dumps({"error": "init: " + err.value.decode()}), flush=True)
        return 1
    n = len(names)
    arr = (ctypes.c_char_p * n)(*[s.encode() for s in names])
    # GRBM is max-reduced, everything else summed (TA busy is a mean over CUs).
    red = (ctypes.c_int * n)(*[1 if s.startswith("GRBM_") else (2 if s == "TA_TA_BUSY" else 0) for s in names])
    gid = kfd_gpu_ids()[0]
    L.kgs_pmc_open.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p,
                               ctypes.c_int]
    h = L.kgs_pmc_open(gid, arr, red, n, err, 512)
    if h < 0:
        print(json.dumps({"error": "open: " + err.value.decode()}), flush=True)
        return 1
    info = ctypes.create_string_buffer(2048)
    L.kgs_pmc_info(h, info, 2048)
    print(json.dumps({"ready": True, "info": info.value.decode()}), flush=True)
    out = (ctypes.c_uint64 * n)()
    rns = ctypes.c_uint32()
    t_end = time.time() + secs
    while time.time() < t_end:
        rc = L.kgs_pmc_sample(h, out, n, ctypes.byref(rns))
        print(json.dumps({"t": time.time(), "rc": rc, "v": list(out), "read_us": rns.value / 1e3}), flush=True)
        time.sleep(0.02)
    L.kgs_pmc_close(h)
    return 0


def parent(sets: list[str]) -> int:
    import torch

    from kube_gpu_stats_amd.ops import load
    from kube_gpu_stats_amd.ops.load import LoadStep

    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=6 << 30)
    ls()
    torch.cuda.synchronize()
    nflt = ls.a.numel()
    # Dispatch-bound phases: a HIP graph of 500 tiny copies (≈575 k kernels/s, the
    # bench's worst case) and the same copies launched eagerly (host-bound).
    tsrc = torch.rand(16384, device="cuda")
    tdst = torch.empty_like(tsrc)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        load.copy_f32(tsrc, tdst, nblocks=64, stream=s)
        s.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(500):
                load.copy_f32(tsrc, tdst, nblocks=64, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    def eager():
        for _ in range(200):
            load.copy_f32(tsrc, tdst, nblocks=64)

    phases_def = {
        "idle": (lambda: time.sleep(0.05), 0.0, 0.0, 0),
        "mfma": (ls.run_mfma, 0.0, 0.0, 1),
        "triad": (lambda: load.triad_f32(ls.a, ls.b, ls.c, 1.5), 8.0 * nflt, 4.0 * nflt, 1),
        "copy": (lambda: load.copy_f32(ls.b, ls.a), 4.0 * nflt, 4.0 * nflt, 1),
        "tiny_graph": (g.replay, 0.0, 0.0, 500),
        "tiny_eager": (eager, 0.0, 0.0, 200),
    }
    result = {}
    for sname in sets:
        names = SETS[sname]
        p = subprocess.Popen([sys.executable, __file__, "--child", json.dumps(names), "18"], stdout=subprocess.PIPE,
                             text=True, cwd=REPO)
        first = json.loads(p.stdout.readline())
        if "error" in first:
            result[sname] = {"error": first["error"]}
            p.wait()
            print(sname, first, flush=True)
            continue
        time.sleep(0.5)
        marks = {}
        for ph, (fn, rd, wr, kern) in phases_def.items():
            t0 = time.time()
            k = 0
            while time.time() - t0 < 2.0:
                fn()
                torch.cuda.synchronize()
                k += 1
            el = time.time() - t0
            marks[ph] = (t0 + 0.2, time.time() - 0.2, k, rd * k / el, wr * k / el, kern * k / el)
        rows = [json.loads(line) for line in p.stdout]
        p.wait()
        rows = [r for r in rows if r.get("rc") == 0]
        res = {"info": first["info"], "read_us_mean": sum(r["read_us"] for r in rows) / max(1, len(rows))}
        for ph, (a, b, k, rd_bps, wr_bps, kps) in marks.items():
            win = [r for r in rows if a <= r["t"] <= b]
            if len(win) < 2:
                continue
            dt = win[-1]["t"] - win[0]["t"]
            rates = {names[i]: (win[-1]["v"][i] - win[0]["v"][i]) / dt for i in range(len(names))}
            rates["expected_read_Bps"] = rd_bps
            rates["expected_write_Bps"] = wr_bps
            rates["kernels_per_s"] = kps
            res[ph] = rates
        result[sname] = res
        print(sname, json.dumps(res), flush=True)
    out = os.environ.get("KGS_AQL_PROBE_OUT", os.path.join(REPO, "gpurun_out", "aql_probe.json"))
    json.dump(result, open(out, "w"), indent=1)
    return 0


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        sys.exit(child(json.loads(sys.argv[2]), float(sys.argv[3])))
    # optional: comma-separated set names (default: every set)
    sys.exit(parent(sys.argv[1].split(",") if len(sys.argv) > 1 else list(SETS)))
