"""Which exporter tier, if any, wakes an idle MI355X out of its low-power level.

An idle MI355X sits at one of two socket-power levels, ≈291 W or ≈258-261 W, and drops to
the lower one ≈5 s after its last GPU work (bench phase P, profiles/r6/r6h-r6k).  In r6k a
released exporter (no counter session; PMFW and slow tiers sampling) let the GPU leave the
low level in 4 of 16 blocks, each time with 0.003-0.0045 % of PMFW GFX busy, and the
exporter-absent blocks never showed GFX busy.  This probe runs the exporter with the
counter tier off (``--pmc none``) in one tier configuration at a time, on a GPU held by an
idle process (this one: a torch context, as an idle pod would hold it), and reads the
socket power and the GFX busy from the PMFW table itself in short slices:

* ``none``      — no exporter;
* ``pmfw``      — the PMFW table tier only (``--proc-every 0 --link-every 0``);
* ``proc``      — + the per-process tier at the DaemonSet's 1 Hz (KFD sysfs, DRM fdinfo);
* ``link``      — + the xGMI link / RAS tier, here every second (the DaemonSet: 10 s);
* ``daemonset`` — the DaemonSet's tiers (``--proc-period 1 --link-period 10``).

Per configuration: mean power, the share of slices above the low level (+10 W), and the
GFX busy µs per second.  Two rounds, the second in reverse order.

usage: python tools/idle_tier_probe.py [--secs 30] [--slice 2] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CONFIGS = {
    "none": None,
    "pmfw": ["--proc-every", "0", "--link-every", "0"],
    "proc": ["--proc-period", "1", "--link-every", "0"],
    "link": ["--proc-every", "0", "--link-period", "1"],
    "daemonset": ["--proc-period", "1", "--link-period", "10"],
}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--secs", type=float, default=30.0, help="measured seconds per configuration and round")
    ap.add_argument("--slice", type=float, default=2.0, help="seconds per power / busy slice")
    ap.add_argument("--settle", type=float, default=8.0, help="seconds after each switch before measuring")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--out", default="gpurun_out/idle_tier_probe.json")
    a = ap.parse_args(argv)

    import torch

    from bench.exporter import PmfwProbe

    torch.ones(1, device="cuda").sum().item()  # an idle process holding a GPU context and its queues
    torch.cuda.synchronize()
    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    probe = PmfwProbe(bdf)
    if probe.N is None:
        print(json.dumps({"skipped": "no PMFW table probe"}))
        return 0
    names = [c for c in a.configs.split(",") if c in CONFIGS]
    slices: list[dict] = []
    t_start = time.monotonic()
    for r in range(a.rounds):
        for name in (names if r % 2 == 0 else names[::-1]):
            proc = None
            if CONFIGS[name] is not None:
                cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
                       "--hz", "10", "--pmc", "none", "--bdfs", bdf, "--node-name", "probe", *CONFIGS[name]]
                proc = subprocess.Popen(cmd, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                end = time.monotonic() + 60
                ready = False
                while time.monotonic() < end and not ready:
                    line = proc.stdout.readline()
                    if not line:
                        break
                    ready = '"event": "ready"' in line
                if not ready:
                    proc.kill()
                    print(json.dumps({"error": f"exporter not ready ({name})"}))
                    return 1
            print(f"[{time.monotonic() - t_start:6.1f}s] round {r + 1} {name}", flush=True)
            time.sleep(a.settle)
            prev = probe.read()
            t_end = time.monotonic() + a.secs
            while time.monotonic() < t_end:
                time.sleep(a.slice)
                cur = probe.read()
                d = PmfwProbe.delta(prev, cur)
                prev = cur
                if d:
                    slices.append({"round": r, "config": name, "power_w": round(d["power_w"], 2),
                                   "gfx_busy_pct": round(d.get("gfx_busy_pct", 0.0), 5)})
            if proc is not None:
                proc.terminate()
                try:
                    proc.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    proc.kill()
                    proc.wait()
    low = min(s["power_w"] for s in slices)
    out = {"low_level_w": low, "slice_s": a.slice, "secs": a.secs, "settle_s": a.settle, "configs": {}}
    for name in names:
        ss = [s for s in slices if s["config"] == name]
        if not ss:
            continue
        out["configs"][name] = {
            "slices": len(ss),
            "power_w_mean": round(sum(s["power_w"] for s in ss) / len(ss), 2),
            "high_share": round(sum(s["power_w"] > low + 10 for s in ss) / len(ss), 3),
            "gfx_busy_us_per_s": round(1e4 * sum(s["gfx_busy_pct"] for s in ss) / len(ss), 2),
            "slices_with_busy": sum(s["gfx_busy_pct"] > 0 for s in ss)}
    out["slices"] = slices
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "slices"}, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
