"""GPU probe: is there a kernel perf PMU for the MI355X data fabric / xGMI links that a
DaemonSet exporter could read at a high rate (VERDICT r2 missing #5)?

Lists every PMU under /sys/bus/event_source/devices (type, cpumask, event and format
names), reads /proc/sys/kernel/perf_event_paranoid, and for every amdgpu-looking PMU
tries perf_event_open(2) (system-wide: pid = -1 on the PMU's first CPU) on each of
its events. Any event that opens is read across 1 s idle and 1 s of an HBM triad
load (ops/hip/load_kernels.hip), so a byte counter that moves is visible.

Output: one JSON document on stdout (and ``--out``).
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import struct
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SYS_PERF_EVENT_OPEN = 298  # x86_64
PERF_ATTR_SIZE_VER5 = 112


def read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.strerror}>"


def parse_event(spec: str, fmt: dict[str, str]) -> dict[str, int]:
    """'event=0x12,umask=0x3' → {'config': ..., 'config1': ..., 'config2': ...} using format/."""
    cfg = {"config": 0, "config1": 0, "config2": 0}
    for term in spec.split(","):
        term = term.strip()
        if not term:
            continue
        k, _, v = term.partition("=")
        val = int(v, 0) if v else 1
        f = fmt.get(k)
        if not f:
            continue
        field, _, bits = f.partition(":")
        lo, _, hi = bits.partition("-")
        lo = int(lo)
        cfg[field] |= val << lo
    return cfg


def perf_open(pmu_type: int, cfg: dict[str, int], cpu: int) -> tuple[int, int]:
    libc = ctypes.CDLL(None, use_errno=True)
    attr = bytearray(PERF_ATTR_SIZE_VER5)
    struct.pack_into("IIQQ", attr, 0, pmu_type, PERF_ATTR_SIZE_VER5, cfg["config"], 0)
    struct.pack_into("Q", attr, 56, cfg["config1"])  # config1 (bp_addr union)
    struct.pack_into("Q", attr, 64, cfg["config2"])  # config2 (bp_len union)
    buf = (ctypes.c_char * len(attr)).from_buffer(attr)
    fd = libc.syscall(SYS_PERF_EVENT_OPEN, buf, -1, cpu, -1, 0)
    return fd, ctypes.get_errno()


def read_count(fd: int) -> int | None:
    try:
        return struct.unpack("Q", os.read(fd, 8))[0]
    except OSError:
        return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--load", type=int, default=1, help="run the HBM triad phase (needs the HIP load library)")
    a = ap.parse_args()
    out: dict = {"perf_event_paranoid": read("/proc/sys/kernel/perf_event_paranoid"),
                 "uid": os.getuid(), "pmus": {}}
    for d in sorted(glob.glob("/sys/bus/event_source/devices/*")):
        name = os.path.basename(d)
        ev = sorted(os.listdir(os.path.join(d, "events"))) if os.path.isdir(os.path.join(d, "events")) else []
        fm = sorted(os.listdir(os.path.join(d, "format"))) if os.path.isdir(os.path.join(d, "format")) else []
        out["pmus"][name] = {"type": read(os.path.join(d, "type")), "cpumask": read(os.path.join(d, "cpumask")),
                             "n_events": len(ev), "events": ev[:64], "format": fm}
    amd = {k: v for k, v in out["pmus"].items()
           if k.startswith("amdgpu") or "xgmi" in k or k.startswith("amd_df") or "df" in k.split("_")}
    out["amdgpu_like"] = sorted(amd)
    opened: list[tuple[str, str, int]] = []
    tries = []
    for name in sorted(amd):
        d = f"/sys/bus/event_source/devices/{name}"
        fmt = {f: read(os.path.join(d, "format", f)) for f in out["pmus"][name]["format"]}
        cpus = out["pmus"][name]["cpumask"]
        cpu = int(cpus.split(",")[0].split("-")[0]) if cpus and cpus[0].isdigit() else 0
        for e in out["pmus"][name]["events"]:
            spec = read(os.path.join(d, "events", e))
            try:
                cfg = parse_event(spec, fmt)
                fd, err = perf_open(int(out["pmus"][name]["type"]), cfg, cpu)
            except (ValueError, KeyError) as x:
                tries.append({"pmu": name, "event": e, "spec": spec, "error": str(x)})
                continue
            tries.append({"pmu": name, "event": e, "spec": spec, "fd": fd,
                          "errno": err, "strerror": os.strerror(err) if fd < 0 else ""})
            if fd >= 0:
                opened.append((name, e, fd))
    out["open_attempts"] = tries
    if opened:
        c0 = {f"{p}/{e}": read_count(fd) for p, e, fd in opened}
        time.sleep(1.0)
        c1 = {f"{p}/{e}": read_count(fd) for p, e, fd in opened}
        phases = {"idle_1s": {k: (c1[k] - c0[k]) if c0[k] is not None and c1[k] is not None else None for k in c0}}
        if a.load:
            try:
                import torch

                from kube_gpu_stats_amd.ops.load import LoadStep

                ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=2000, stream_bytes=4 << 30)
                ls.run_stream()
                torch.cuda.synchronize()
                c0 = {f"{p}/{e}": read_count(fd) for p, e, fd in opened}
                t0 = time.time()
                k = 0
                while time.time() - t0 < 1.0:
                    ls.run_stream()
                    torch.cuda.synchronize()
                    k += 1
                c1 = {f"{p}/{e}": read_count(fd) for p, e, fd in opened}
                phases["triad_1s"] = {kk: (c1[kk] - c0[kk]) if c0[kk] is not None and c1[kk] is not None else None
                                      for kk in c0}
                phases["triad_bytes"] = k * ls.bytes
            except Exception as x:  # noqa: BLE001 - record, do not fail the probe
                phases["triad_error"] = repr(x)
        out["counts"] = phases
        for _, _, fd in opened:
            os.close(fd)
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
