#!/usr/bin/env python3
"""What does 8 kHz cost a dispatch-bound kernel stream, per reader variant?  

Every counter READ is one more AQL packet for the command processor that also
dispatches the workload's kernels.  Long kernels hide it; a HIP graph of µs kernels
does not (bench.py's tiny_graph component: +0.3 … +1.1 % at 8 kHz in round 3).  This
probe measures only that component, for several exporter variants on the same box:

* ``default``   — the shipped exporter: batched READs, and the dispatch-bound READ
  rate (--pmc-cp-only-min 0.3: a GPU whose CP dispatches with no wave in flight for
  ≥ 30 % of the clocks is READ at --pmc-dispatch-hz, 1 kHz);
* ``full_rate`` — --pmc-cp-only-min 0: every tick READs, whatever the workload (the
  round-4 r4c reader: +3.8 % at 8 kHz; the KGS_AQL_NOBARRIER and low-priority READ
  queue variants measured the same there and were deleted);
* ``batch1``    — --pmc-cp-only-min 0 --pmc-batch 1 (every READ writes the L2 back);
* ``hz1000`` / ``hz100`` — the full-rate reader at 1 kHz / 100 Hz;
* ``util_set``  — full rate, --pmc-set util (24 register reads per READ instead of 56);
* ``lite``      — full rate, --pmc-lite (7 of 8 READs without the 32 per-SE MFMA reads;
  the default from r4k, so ``full_rate`` is the same since);
* ``nolite``    — full rate, --no-pmc-lite (every READ full).

Per variant one exporter process (--hz 8000, --control-http) and ``--rounds`` paired
rounds of two blocks — exporter paused / sampling, order alternating (ABBA) — each
block ``--replays`` replays of a graph of ``--kernels`` 64 KiB copies, timed with HIP
events.  Overhead per round = t_on / t_paused − 1; reported as mean ± 95 % CI, with
the counter samples/s the exporter delivered while sampling.  ``python
tools/graph_cost_probe.py --out gpurun_out/graph_cost.json`` on a GPU box.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

VARIANTS = {
    "default": ({}, []),
    "full_rate": ({}, ["--pmc-cp-only-min", "0"]),
    "batch1": ({}, ["--pmc-cp-only-min", "0", "--pmc-batch", "1"]),
    "hz1000": ({}, ["--pmc-cp-only-min", "0", "--hz", "1000"]),
    "hz100": ({}, ["--pmc-cp-only-min", "0", "--hz", "100"]),
    "util_set": ({}, ["--pmc-cp-only-min", "0", "--pmc-set", "util"]),
    "lite": ({}, ["--pmc-cp-only-min", "0", "--pmc-lite"]),
    "nolite": ({}, ["--pmc-cp-only-min", "0", "--no-pmc-lite"]),
}
T975 = {5: 2.571, 7: 2.365, 11: 2.201, 15: 2.131, 23: 2.069, 31: 2.040, 47: 2.012}


def ci95(xs: list[float]) -> tuple[float, float]:
    n = len(xs)
    m = sum(xs) / n
    if n < 2:
        return m, float("nan")
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (n - 1))
    t = next((v for k, v in sorted(T975.items()) if n - 1 <= k), 1.96)
    return m, t * sd / math.sqrt(n)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--variants", default="default,full_rate,batch1,hz1000,hz100")
    ap.add_argument("--rounds", type=int, default=24)
    ap.add_argument("--replays", type=int, default=120, help="graph replays per block (≈3.5 ms each)")
    ap.add_argument("--kernels", type=int, default=2000)
    ap.add_argument("--hz", type=float, default=8000)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    import torch

    from kube_gpu_stats_amd.ops import load as L
    from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

    dev = torch.device("cuda", 0)
    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    src = torch.rand(16384, device=dev)
    dst = torch.empty_like(src)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        L.copy_f32(src, dst, nblocks=64, stream=s)
        s.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(a.kernels):
                L.copy_f32(src, dst, nblocks=64, stream=s)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def block() -> float:
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.replays):
            graph.replay()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3

    for _ in range(3):
        block()
    out: dict = {"kernels_per_graph": a.kernels, "replays_per_block": a.replays, "hz": a.hz, "variants": {}}
    for name in a.variants.split(","):
        env_extra, flags = VARIANTS[name]
        env = dict(os.environ, **env_extra)
        cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0", "--hz",
               f"{a.hz:g}", "--pmc", "aqlprofile", "--bdfs", bdf, "--proc-every", "0", "--link-every", "0",
               "--control-stdin", "--control-http", *flags]
        proc = subprocess.Popen(cmd, cwd=REPO, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        try:
            ready = json.loads(proc.stdout.readline())
            assert ready.get("event") == "ready" and ready.get("pmc") == "aqlprofile", ready
            sc = Scraper("127.0.0.1", ready["port"])
            diffs, on_s, samples, t_on, dbound = [], [], 0.0, 0.0, []
            for r in range(a.rounds):
                t = {}
                for cond in (("off", "on") if r % 2 == 0 else ("on", "off")):
                    sc.get("/control/pause" if cond == "off" else "/control/resume")
                    time.sleep(0.02)
                    if cond == "on":
                        m0, w0 = parse_text(sc.get()), time.monotonic()
                    t[cond] = block()
                    if cond == "on":
                        m1, w1 = parse_text(sc.get()), time.monotonic()
                        samples += m1["kgs_pmc_samples_total"][0][1] - m0["kgs_pmc_samples_total"][0][1]
                        dbound.append(m1.get("kgs_pmc_dispatch_bound", [({}, 0)])[0][1])
                        t_on += w1 - w0
                diffs.append(100.0 * (t["on"] / t["off"] - 1.0))
                on_s.append(t["on"])
            m, ci = ci95(diffs)
            info = ready.get("pmc_info", [""])[0]
            out["variants"][name] = {"overhead_pct": round(m, 4), "overhead_ci95_pct": round(ci, 4),
                                     "samples_per_s_while_on": round(samples / t_on, 1) if t_on else None,
                                     "dispatch_bound_share_of_scrapes": round(sum(dbound) / len(dbound), 3),
                                     "block_s_mean": round(sum(on_s) / len(on_s), 5),
                                     "kernels_per_s": round(a.kernels * a.replays / (sum(on_s) / len(on_s)), 0),
                                     "reader": ";".join(x for x in info.split(";")
                                                        if x.split("=")[0] in ("batch", "lean")),
                                     "per_round_pct": [round(d, 4) for d in diffs]}
            print(json.dumps({name: {k: v for k, v in out["variants"][name].items() if k != "per_round_pct"}}),
                  flush=True)
        finally:
            try:
                proc.stdin.write("quit\n")
                proc.stdin.flush()
                proc.communicate(timeout=30)
            except Exception:  # noqa: BLE001
                proc.kill()
                proc.communicate()
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
