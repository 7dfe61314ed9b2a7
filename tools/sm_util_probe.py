#!/usr/bin/env python3
"""What does each busy signal say a GPU is doing?  ("check that first")

The reference-contract series ``container_gpu_sm_util`` must mean "a kernel is
running" (reference gpu_util_stats/gpu_util_stats.py:159 averages it per pod).  Two
sources can back it on MI355X:

* the PMFW GFX-activity accumulator (``amdgpu_gfx_busy_seconds_total``): counts a
  dispatch in flight, but also every counter READ packet (≈80 µs each,
  profiles/r2/idle_busy/);
* the counter tier's GRBM_SPI_BUSY (``amdgpu_gpu_active_seconds_total``): a shader
  engine has waves; blind to READs.

This probe runs one exporter per configuration (``--configs hz:idle_hz,...``) next
to a set of loads whose true busy share the host knows — GPU-bound streams of long
MFMA kernels, HBM triads, hipBLASLt bf16 GEMMs and a graph of µs kernels (event-timed
kernel time / wall time), MFMA burst trains (host-timed duty) and an idle GPU — and
reports every signal's busy % next to the truth.  ``python tools/sm_util_probe.py
--out gpurun_out/sm_util_probe.json`` on a GPU box.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def bdf0(torch) -> str:
    p = torch.cuda.get_device_properties(0)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


class Loads:
    """GPU loads with a host-known busy share.  Each ``run_<name>(secs)`` returns the
    GPU-busy seconds the host measured (HIP events around every kernel, or the
    host-timed bursts)."""

    def __init__(self, torch):
        from kube_gpu_stats_amd.ops import load as L
        from kube_gpu_stats_amd.ops.load import LoadStep

        self.torch, self.L = torch, L
        dev = torch.device("cuda", 0)
        self.ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=3 << 30)
        g = torch.Generator().manual_seed(3)
        self.ga = torch.randn(8192, 8192, generator=g).to(torch.bfloat16).to(dev)
        self.gb = torch.randn(8192, 8192, generator=g).to(torch.bfloat16).to(dev)
        self.gc = torch.empty(8192, 8192, dtype=torch.bfloat16, device=dev)
        # the first mm initialises hipBLASLt (≈0.2 s of host time no HIP event sees):
        # warm it here, not inside the first configuration's GEMM row
        torch.mm(self.ga, self.gb, out=self.gc)
        self.tsrc = torch.rand(16384, device=dev)
        self.tdst = torch.empty_like(self.tsrc)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            L.copy_f32(self.tsrc, self.tdst, nblocks=64, stream=s)
            s.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=s):
                for _ in range(2000):
                    L.copy_f32(self.tsrc, self.tdst, nblocks=64, stream=s)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        # ms per MFMA iteration, for the burst lengths
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.ls.run_mfma()
        e0.record()
        L.mfma_bf16(self.ls.A, self.ls.B, self.ls.C, 2048, 4000)
        e1.record()
        torch.cuda.synchronize()
        self.ms_per_iter = e0.elapsed_time(e1) / 4000

    def _stream(self, secs: float, launch) -> float:
        """Launch `launch` back to back (≤ 8 in flight) for `secs`: Σ event-timed kernel time."""
        torch = self.torch
        ev = []
        t0 = time.monotonic()
        while time.monotonic() - t0 < secs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch()
            b.record()
            ev.append((a, b))
            if len(ev) >= 8:
                ev[-8][1].synchronize()
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) * 1e-3

    def run_mfma(self, secs):
        return self._stream(secs, self.ls.run_mfma)

    def run_triad(self, secs):
        return self._stream(secs, self.ls.run_stream)

    def run_gemm(self, secs):
        return self._stream(secs, lambda: self.torch.mm(self.ga, self.gb, out=self.gc))

    def run_tiny_graph(self, secs):
        return self._stream(secs, self.graph.replay)

    def bursts(self, secs: float, burst_ms: float, period_ms: float) -> float:
        """Host-timed MFMA bursts (launch → synchronize) of ≈burst_ms every period_ms."""
        iters = max(20, int(burst_ms / self.ms_per_iter))
        busy = 0
        nxt = time.monotonic()
        t_end = nxt + secs
        while time.monotonic() < t_end:
            a = time.monotonic_ns()
            self.L.mfma_bf16(self.ls.A, self.ls.B, self.ls.C, 2048, iters)
            self.torch.cuda.synchronize()
            busy += time.monotonic_ns() - a
            nxt += period_ms * 1e-3
            d = nxt - time.monotonic()
            if d > 0:
                time.sleep(d)
        return busy * 1e-9

    def run_burst_1_5(self, secs):
        return self.bursts(secs, 1.0, 5.0)

    def run_burst_02_1(self, secs):
        return self.bursts(secs, 0.2, 1.0)

    def run_idle(self, secs):
        time.sleep(secs)
        return 0.0


def one(m: dict, fam: str, **kw) -> float | None:
    for lb, v in m.get(fam, []):
        if all(lb.get(k) == w for k, w in kw.items()):
            return v
    return None


def measure(loads: Loads, sc, names: list[str], secs: float) -> dict:
    from kube_gpu_stats_amd.utils.scrape import parse_text

    rows = {}
    for name in names:
        time.sleep(0.3)
        m0, s0 = parse_text(sc.get()), time.monotonic()
        busy_s = getattr(loads, "run_" + name)(secs)
        m1, s1 = parse_text(sc.get()), time.monotonic()
        wall = s1 - s0
        d = lambda f, **kw: (one(m1, f, **kw) or 0.0) - (one(m0, f, **kw) or 0.0)  # noqa: E731
        clk = d("amdgpu_pmc_total", counter="GRBM_COUNT")
        row = {"host_busy_pct": round(100 * busy_s / wall, 2),
               "pmfw_gfx_busy_pct": round(100 * d("amdgpu_pmfw_gfx_busy_seconds_total") / wall, 2),
               "spi_active_pct": round(100 * d("amdgpu_gpu_active_seconds_total") / wall, 2),
               "dispatch_pct": round(100 * d("amdgpu_dispatch_busy_seconds_total") / wall, 2),
               "read_cp_us": round(1e6 * (one(m1, "kgs_pmc_read_cp_seconds") or 0.0), 2),
               "spi_share_of_clocks_pct": round(100 * d("amdgpu_pmc_total", counter="GRBM_SPI_BUSY") / clk, 2)
               if clk > 0 else None,
               "mfma_busy_pct": round(100 * d("amdgpu_mfma_busy_seconds_total") / wall, 2),
               "sm_util_gauge": one(m1, "container_gpu_sm_util"),
               "busy_counter_pct": round(100 * d("container_gpu_busy_seconds_total") / wall, 2),
               "reads_per_s": round(d("kgs_pmc_samples_total") / wall, 1), "wall_s": round(wall, 3)}
        rows[name] = row
        print(json.dumps({name: row}), flush=True)
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--configs", default="100:0,8000:100,1000:100",
                    help="exporter configurations hz:pmc_idle_hz[:sm_util_source], comma-separated")
    ap.add_argument("--loads", default="idle,mfma,triad,gemm,tiny_graph,burst_1_5,burst_02_1")
    ap.add_argument("--secs", type=float, default=2.5)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    import torch

    from kube_gpu_stats_amd.utils.scrape import Scraper

    loads = Loads(torch)
    bdf = bdf0(torch)
    tmp = tempfile.mkdtemp()
    owners = os.path.join(tmp, "owners.json")
    with open(owners, "w") as f:
        json.dump({bdf: {"pod": "probe-0", "namespace": "ml", "container": "main"}}, f)
    out = {"ms_per_mfma_iter": loads.ms_per_iter, "configs": {}}
    for spec in a.configs.split(","):
        parts = spec.split(":")
        hz, idle = parts[0], parts[1]
        src = parts[2] if len(parts) > 2 else ""
        cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0", "--hz", hz,
               "--pmc", "aqlprofile", "--pmc-idle-hz", idle, "--bdfs", bdf, "--proc-every", "0", "--link-every", "0",
               "--window", str(a.secs), "--static-owners", owners, "--pod-resources-socket", "", "--node-name", "n",
               "--control-stdin"] + (["--sm-util-source", src] if src else [])
        proc = subprocess.Popen(cmd, cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        try:
            ready = json.loads(proc.stdout.readline())
            assert ready.get("event") == "ready", ready
            time.sleep(0.5)
            sc = Scraper("127.0.0.1", ready["port"])
            out["configs"][spec] = measure(loads, sc, a.loads.split(","), a.secs)
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
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
