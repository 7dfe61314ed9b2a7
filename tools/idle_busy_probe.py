#!/usr/bin/env python3
"""Does the exporter's own sampling make an idle GPU look busy?

The counter tier puts one PM4 READ packet per tick on a private AQL queue of the
command processor.  GRBM_GUI_ACTIVE and the PMFW GFX-activity accumulator
(``amdgpu_gfx_busy_percent``, which backs ``container_gpu_sm_util``) both count
the graphics pipe busy while *any* packet is in flight, so a READ that keeps the CP
occupied is indistinguishable from work.  (The exporter's ``amdgpu_gpu_active_percent``
is GRBM_SPI_BUSY since round 2, which needs waves.)

With the GPU idle (this process initialises HIP to find the PCI address, then
launches nothing), start the exporter once per configuration and read what it
reports.  One JSON line per configuration; summary to --out.

    python tools/idle_busy_probe.py --out gpurun_out/idle_busy.json
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
import urllib.request

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text  # noqa: E402

# (label, hz, pmc reader, extra exporter flags[, extra env]) — the rate sweep
SWEEP = [
    ("pmfw_only_100", 100, "none", []),
    ("aql_100", 100, "aqlprofile", ["--pmc-idle-hz", "0"]),
    ("aql_1k", 1000, "aqlprofile", ["--pmc-idle-hz", "0"]),
    ("aql_4k", 4000, "aqlprofile", ["--pmc-idle-hz", "0"]),
    ("aql_8k", 8000, "aqlprofile", ["--pmc-idle-hz", "0"]),
    ("aql_8k_lean0", 8000, "aqlprofile", ["--pmc-idle-hz", "0", "--pmc-lean", "0"]),
    ("aql_8k_sync", 8000, "aqlprofile", ["--pmc-idle-hz", "0", "--no-pmc-pipeline"]),
    # the default: a quiet GPU (no wave, no MFMA cycle) is READ at --pmc-idle-hz only
    ("aql_8k_adaptive_100", 8000, "aqlprofile", []),
    ("aql_8k_adaptive_10", 8000, "aqlprofile", ["--pmc-idle-hz", "10"]),
]
# what in a READ costs the busy time: all at 1 kHz, PMFW GFX busy is the judge
# (modes 4/5 return stale counters, so GUI-active cannot be trusted there)
COST = [
    ("pmfw_only_1k", 1000, "none", []),
    ("lean2_default", 1000, "aqlprofile", ["--pmc-idle-hz", "0"]),
    ("lean0_as_built", 1000, "aqlprofile", ["--pmc-idle-hz", "0"], {"KGS_AQL_LEAN": "0"}),
    ("lean1_no_flush", 1000, "aqlprofile", ["--pmc-idle-hz", "0"], {"KGS_AQL_LEAN": "1"}),
    ("lean3_no_acquire", 1000, "aqlprofile", ["--pmc-idle-hz", "0"], {"KGS_AQL_LEAN": "3"}),
    ("lean4_no_copies", 1000, "aqlprofile", ["--pmc-idle-hz", "0"], {"KGS_AQL_LEAN": "4"}),
    ("lean5_all_nop", 1000, "aqlprofile", ["--pmc-idle-hz", "0"], {"KGS_AQL_LEAN": "5"}),
    ("fence_none_agent", 1000, "aqlprofile", ["--pmc-idle-hz", "0"], {"KGS_AQL_FENCE": "none,agent"}),
    ("fence_none_none", 1000, "aqlprofile", ["--pmc-idle-hz", "0"], {"KGS_AQL_FENCE": "none,none"}),
    ("full_set", 1000, "aqlprofile", ["--pmc-idle-hz", "0", "--pmc-set", "full"]),
    ("sync_reads", 1000, "aqlprofile", ["--pmc-idle-hz", "0", "--no-pmc-pipeline"]),
]
SETS = {"sweep": SWEEP, "cost": COST}


def bdf0() -> str:
    import torch

    p = torch.cuda.get_device_properties(0)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


def one(label: str, hz: float, pmc: str, extra: list[str], bdf: str, secs: float, env: dict | None = None) -> dict:
    cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0", "--hz", str(hz),
           "--pmc", pmc, "--control-stdin", "--bdfs", bdf, "--window", str(secs * 0.8), "--proc-every", "0",
           "--link-every", "0", *extra]
    p = subprocess.Popen(cmd, cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, env=dict(os.environ, KGS_NO_BUILD="1", **(env or {})))
    try:
        ready = json.loads(p.stdout.readline())
        if ready.get("event") != "ready":
            return {"config": label, "error": ready}
        time.sleep(secs)
        m = parse_text(Scraper("127.0.0.1", ready["port"]).get())
        g = lambda f: m[f][0][1] if m.get(f) else None  # noqa: E731
        out = {"config": label, "hz": hz, "pmc": ready.get("pmc"), "extra": extra, "env": env or {},
               "pmfw_gfx_busy_pct": g("amdgpu_pmfw_gfx_busy_percent"), "gpu_active_pct": g("amdgpu_gpu_active_percent"),
               "mfma_util_pct": g("amdgpu_mfma_util_percent"), "power_w": g("amdgpu_power_watts"),
               "clock_mhz": g("amdgpu_gpu_clock_effective_mhz"), "quiet": g("kgs_pmc_quiet"),
               "reads_total": g("kgs_pmc_samples_total")}
        if ready.get("pmc") not in (None, "none"):
            s = json.load(urllib.request.urlopen(f"http://127.0.0.1:{ready['port']}/counters?gpu=0&n=2000",
                                                 timeout=10))["samples"]
            act = [x["gpu_active_pct"] for x in s if "gpu_active_pct" in x]
            out["stream_active_mean"] = sum(act) / len(act) if act else None
            out["stream_active_p10_p50_p90"] = ([sorted(act)[int(q * (len(act) - 1))] for q in (0.1, 0.5, 0.9)]
                                                if act else None)
        return out
    finally:
        try:
            p.stdin.write("quit\n")
            p.stdin.flush()
            p.communicate(timeout=30)
        except Exception:  # noqa: BLE001
            p.kill()
            p.communicate()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=2.5)
    ap.add_argument("--set", default="sweep", choices=sorted(SETS))
    ap.add_argument("--only", default="", help="comma-separated config labels")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    bdf = bdf0()
    rows = []
    for label, hz, pmc, extra, *env in SETS[a.set]:
        if a.only and label not in a.only.split(","):
            continue
        r = one(label, hz, pmc, extra, bdf, a.secs, env[0] if env else None)
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"bdf": bdf, "set": a.set, "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
