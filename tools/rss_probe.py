"""GPU probe: where the exporter's resident memory goes.

Starts the exporter on GPU 0 in a few configurations (AMD SMI only; + the aqlprofile
counter reader; + the reader at 8 kHz), lets it sample for a few seconds and sums
``/proc/<pid>/smaps`` Rss by mapping (file path, or [heap] / [anon] / device node).

    python tools/rss_probe.py --out gpurun_out/rss_probe.json
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


def smaps_by_mapping(pid: int) -> dict:
    out: dict = {}
    name = "[anon]"
    with open(f"/proc/{pid}/smaps") as f:
        for ln in f:
            parts = ln.split()
            if not parts:
                continue
            if "-" in parts[0] and len(parts) >= 5 and not parts[0].endswith(":"):
                name = parts[5] if len(parts) >= 6 else "[anon]"
            elif parts[0] == "Rss:":
                out[name] = out.get(name, 0) + int(parts[1])
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/rss_probe.json")
    ap.add_argument("--seconds", type=float, default=4.0)
    a = ap.parse_args()
    import torch  # only to name GPU 0's PCI address; the exporter runs in its own process

    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    configs = {"amdsmi_only_10hz": ["--hz", "10", "--pmc", "none"],
               "aqlprofile_10hz": ["--hz", "10", "--pmc", "aqlprofile"],
               "aqlprofile_8khz": ["--hz", "8000", "--pmc", "aqlprofile"]}
    res: dict = {}
    for name, extra in configs.items():
        proc = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
                                 "--control-stdin", "--bdfs", bdf, *extra], cwd=REPO, stdin=subprocess.PIPE,
                                stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        try:
            ready = json.loads(proc.stdout.readline())
            time.sleep(a.seconds)
            m = smaps_by_mapping(proc.pid)
            total = sum(m.values())
            top = sorted(m.items(), key=lambda kv: -kv[1])[:15]
            res[name] = {"pmc": ready.get("pmc"), "rss_mib": round(total / 1024, 1),
                         "top_mib": [[k, round(v / 1024, 1)] for k, v in top]}
            print(name, json.dumps(res[name]), flush=True)
        finally:
            try:
                proc.stdin.write("quit\n")
                proc.stdin.flush()
                proc.communicate(timeout=30)
            except Exception:  # noqa: BLE001
                proc.kill()
                proc.communicate()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
