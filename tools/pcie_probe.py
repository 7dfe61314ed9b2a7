#!/usr/bin/env python3
"""What does the PMFW ``pcie_bandwidth_acc`` count?  amdsmi.h:1945 says "PCIE
accumulated bandwidth (GB/sec)": either GB moved, or a sum of per-cycle GB/s
readings like the activity accumulators (then Δacc / Δaccumulation_counter is the
mean GB/s).  Move a known number of bytes host→device and device→host (pinned
memory) and compare both readings with the truth.

    python tools/pcie_probe.py --out gpurun_out/pcie_probe.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0, help="size of one copy")
    ap.add_argument("--secs", type=float, default=3.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from kube_gpu_stats_amd import load_native

    N = load_native()
    ex = N.Exporter({"backend": "amdsmi", "port": -1, "hz": 100, "proc_every": 0, "link_every": 0})
    ex.start()
    n = int(a.gib * (1 << 30)) // 4
    host = torch.empty(n, dtype=torch.float32).pin_memory()
    dev = torch.empty(n, dtype=torch.float32, device="cuda")
    dev.copy_(host)
    torch.cuda.synchronize()
    small_n = n // 8
    s_h2d, s_d2h = torch.cuda.Stream(), torch.cuda.Stream()
    host2 = torch.empty(n, dtype=torch.float32).pin_memory()
    dev2 = torch.empty(n, dtype=torch.float32, device="cuda")
    cases = [("idle", 0), ("h2d", n), ("d2h", n), ("h2d", small_n), ("d2h", small_n), ("both", n)]
    rows = []
    for direction, m in cases:
        time.sleep(0.3)
        s0, t0 = ex.snapshot(0), time.time()
        moved = 0
        while time.time() - t0 < a.secs:
            if direction == "h2d":
                dev[:m].copy_(host[:m], non_blocking=True)
            elif direction == "d2h":
                host[:m].copy_(dev[:m], non_blocking=True)
            elif direction == "both":  # full duplex: one copy each way on its own stream
                with torch.cuda.stream(s_h2d):
                    dev.copy_(host, non_blocking=True)
                with torch.cuda.stream(s_d2h):
                    host2.copy_(dev2, non_blocking=True)
                m = 2 * n
            else:
                time.sleep(0.05)
                continue
            torch.cuda.synchronize()
            moved += m * 4
        wall = time.time() - t0
        time.sleep(0.1)
        s1 = ex.snapshot(0)
        dacc = s1["pcie_bw_acc_gb"] - s0["pcie_bw_acc_gb"]
        dcnt = s1["accumulation_counter"] - s0["accumulation_counter"]
        dfw = (s1["fw_ts"] - s0["fw_ts"]) * 1e-8
        r = {"direction": direction, "copy_bytes": m * 4, "bytes_moved": moved, "wall_s": round(wall, 3),
             "true_GBps": moved / wall / 1e9, "d_pcie_bw_acc": dacc, "d_accumulation_counter": dcnt,
             "d_fw_s": round(dfw, 3), "acc_per_cycle": dacc / dcnt if dcnt else None,
             "bytes_per_acc_unit": moved / dacc if dacc and moved else None,
             "link": [s1["pcie_link_width"], s1["pcie_link_speed_01gts"]]}
        print(json.dumps(r), flush=True)
        rows.append(r)
    ex.stop()
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
