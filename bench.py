#!/usr/bin/env python3
"""Headline benchmark: counter samples/s per GPU, p50 /metrics scrape latency and
GPU-time overhead %, under synthetic gfx950 load (BASELINE.json "metric").

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One rank per GPU.  A *step* is one fixed block of synthetic load on every GPU
(an MFMA-bound bf16 kernel + HBM triads, ops/hip/load_kernels.hip, + a HIP
graph of 2000 tiny copies: the dispatch-bound part, where the counter reader's
command-processor packets would cost the workload time).  Phases:

  A  K steps, no exporter running                       (baseline, untimed for the result line)
  B  K steps with the node exporter sampling every used GPU at --hz (PMFW table,
     HBM, per-process list, xGMI, and hardware counters through rocprofiler-sdk)
     while rank 0 scrapes /metrics at --scrape-hz      (THE timed region)
  C  K steps, exporter stopped again                    (second baseline)

``value`` = counter samples/s summed over the N GPUs (weak scaling: per-GPU work
and sampling rate are fixed).  A counter sample is one hardware-counter drain
(GRBM/SQ/TCC values advance on every drain) when rocprofiler-sdk counting is
available, else one distinct PMFW table (new firmware timestamp).  Overhead % =
100 · (t_B / mean(t_A, t_C) − 1), same device, same process.  Scrape latency is
request → last body byte on a keep-alive connection, as a Prometheus server sees
it (utils/scrape.py; body decoding happens after the clock stops).

The exporter runs as its own process (as in production: DaemonSet vs workload),
launched by local rank 0 over the PCI addresses of every local rank's GPU.
``--mock`` runs the same flow on CPU with the mock provider (tests only).
"""
from __future__ import annotations

import argparse
import json
import os
import select
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from kube_gpu_stats_amd.parallel import dist as D  # noqa: E402
from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text  # noqa: E402

METRIC = "counter samples/sec/GPU + p50 scrape latency at 8×MI355X; GPU-time overhead %"
AUTO_PMC = "aqlprofile"  # direct CP reads: same counters, ≈10× less exporter CPU than rocprofiler-sdk


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--hz", type=float, default=8000.0,
                    help="sampler tick rate per GPU: one hardware-counter drain per tick (PMFW table ≤100 Hz); "
                    "8 kHz costs ≈0.08 exporter cores/GPU with pipelined reads (profiles/r1/pipelined)")
    ap.add_argument("--pmc", default="auto", choices=["auto", "aqlprofile", "rocprofiler", "none"],
                    help="counter reader (auto = %s)" % AUTO_PMC)
    ap.add_argument("--pmc-pipeline", type=int, default=1, choices=[0, 1],
                    help="aqlprofile reader: pipelined READs (1) or submit-and-wait per sample (0)")
    ap.add_argument("--pmc-set", default="base", choices=["base", "full"],
                    help="counter set: base (GRBM + MFMA busy) or full (+ TA busy, 10x the CP register reads)")
    ap.add_argument("--pmc-lean", type=int, default=2, choices=[0, 1, 2, 3],
                    help="aqlprofile READ packet mode (exporter --pmc-lean; 0 = as aqlprofile builds it)")
    ap.add_argument("--scrape-hz", type=float, default=10.0)
    ap.add_argument("--mfma-iters", type=int, default=150000, help="≈40 ms of MFMA work per step on MI355X")
    ap.add_argument("--mfma-blocks", type=int, default=2048)
    ap.add_argument("--stream-gib", type=float, default=6.0)
    ap.add_argument("--triads", type=int, default=2)
    ap.add_argument("--tiny-kernels", type=int, default=2000,
                    help="dispatch-bound part of each step: a HIP graph of this many 64 KiB copies (≈1.7 µs each); "
                    "it is where counter READs on the command processor would show up (0 = off)")
    ap.add_argument("--load", default="synthetic", choices=["synthetic", "train"],
                    help="GPU work per step: the synthetic gfx950 kernels (default) or a PyTorch bf16 "
                    "decoder training step (forward + backward + AdamW, DDP when N > 1)")
    ap.add_argument("--train-dim", type=int, default=4096)
    ap.add_argument("--train-layers", type=int, default=4)
    ap.add_argument("--train-batch", type=int, default=4)
    ap.add_argument("--train-seq", type=int, default=2048)
    ap.add_argument("--train-vocab", type=int, default=32768)
    ap.add_argument("--xgmi-mib", type=int, default=256, help="RCCL all-reduce size per step when N > 1 (0 = off)")
    ap.add_argument("--interleave", type=int, default=4,
                    help="after phase B: this many off/on block pairs (ABBA order; exporter paused vs sampling "
                    "and scraped, --steps/4 steps per block) -> overhead_interleaved_pct, which cancels the "
                    "slow thermal/power drift that an A-B-C comparison sees (0 = off)")
    ap.add_argument("--settle", type=float, default=1.0, help="seconds between exporter start and phase B")
    ap.add_argument("--mock", action="store_true", help="CPU plumbing run with the mock provider")
    ap.add_argument("--mock-step-ms", type=float, default=20.0)
    ap.add_argument("--out", default="", help="also write the result JSON here")
    ap.add_argument("--attach", default="", help="host:port of an exporter started with --control-http; it is "
                    "paused for phases A/C instead of being spawned (lets rocprofv3 trace the bench alone)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- load
class GpuLoad:
    def __init__(self, a, device: int, ctx=None):
        import torch

        from kube_gpu_stats_amd.ops.load import LoadStep

        self.torch = torch
        self.ls = LoadStep(device=device, mfma_blocks=a.mfma_blocks, mfma_iters=a.mfma_iters,
                           stream_bytes=int(a.stream_gib * (1 << 30)))
        self.triads = a.triads
        # Dispatch-bound component: back-to-back tiny kernels replayed from a HIP
        # graph.  Long kernels hide command-processor contention; these expose it.
        self.graph = None
        self.tiny = int(a.tiny_kernels)
        if self.tiny > 0:
            from kube_gpu_stats_amd.ops import load as L

            self.tsrc = torch.rand(16384, device=torch.device("cuda", device))
            self.tdst = torch.empty_like(self.tsrc)
            s = torch.cuda.Stream(device=device)
            s.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(s):
                L.copy_f32(self.tsrc, self.tdst, nblocks=64, stream=s)
                s.synchronize()
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph, stream=s):
                    for _ in range(self.tiny):
                        L.copy_f32(self.tsrc, self.tdst, nblocks=64, stream=s)
            torch.cuda.current_stream(device).wait_stream(s)
        # xGMI traffic for N > 1: one RCCL all-reduce per step over the
        # point-to-point xGMI mesh, so the exporter's per-link counters move.
        self.ar = None
        if ctx is not None and ctx.is_dist and a.xgmi_mib > 0:
            self.ar = torch.ones(int(a.xgmi_mib) << 18, dtype=torch.float32, device=torch.device("cuda", device))

    def step(self):
        self.ls.run_mfma()
        for _ in range(self.triads):
            self.ls.run_stream()
        if self.graph is not None:
            self.graph.replay()
        if self.ar is not None:
            import torch.distributed as dist

            dist.all_reduce(self.ar)
            self.ar.mul_(0.5)  # keep values bounded across steps

    def sync(self):
        self.torch.cuda.synchronize()

    def calibrate(self) -> dict:
        """Per-kernel throughput (events), outside every timed region."""
        torch = self.torch
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record()
        self.ls.run_mfma()
        e[1].record()
        self.ls.run_stream()
        e[2].record()
        if self.graph is not None:
            self.graph.replay()
        e[3].record()
        torch.cuda.synchronize()
        mfma_s = e[0].elapsed_time(e[1]) * 1e-3
        tri_s = e[1].elapsed_time(e[2]) * 1e-3
        out = {"mfma_ms": mfma_s * 1e3, "mfma_tflops": self.ls.flops / mfma_s / 1e12,
               "triad_ms": tri_s * 1e3, "triad_tbps": self.ls.bytes / tri_s / 1e12}
        if self.graph is not None:
            g_s = e[2].elapsed_time(e[3]) * 1e-3
            out.update({"tiny_graph_ms": g_s * 1e3, "tiny_kernels_per_s": self.tiny / g_s})
        return out

    def pci_bdf(self, device: int) -> str:
        p = self.torch.cuda.get_device_properties(device)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


class TrainLoad(GpuLoad):
    """``--load train``: one PyTorch bf16 training step per bench step instead of the
    synthetic kernels: a decoder stack (RMSNorm, causal SDPA, SwiGLU MLP) forward +
    backward + AdamW, DDP over RCCL when N > 1.  Hundreds of library kernels
    (hipBLASLt GEMMs, flash attention, elementwise) per step, which is the kind of
    workload a DaemonSet exporter shares the GPU with.  Random-init weights and
    synthetic tokens; the exporter is measured exactly as with the synthetic load."""

    def __init__(self, a, device: int, ctx=None):
        import torch
        import torch.nn as nn
        import torch.nn.functional as F

        self.torch = torch
        dev = torch.device("cuda", device) if device >= 0 else torch.device("cpu")  # cpu: tests only
        d, h, L, ff = a.train_dim, a.train_dim // 128, a.train_layers, int(a.train_dim * 8 / 3 / 256 + 0.5) * 256
        self.batch, self.seq, self.vocab = a.train_batch, a.train_seq, a.train_vocab

        class Block(nn.Module):
            def __init__(self):
                super().__init__()
                self.n1 = nn.RMSNorm(d)
                self.qkv = nn.Linear(d, 3 * d, bias=False)
                self.o = nn.Linear(d, d, bias=False)
                self.n2 = nn.RMSNorm(d)
                self.up = nn.Linear(d, 2 * ff, bias=False)
                self.down = nn.Linear(ff, d, bias=False)

            def forward(self, x):
                B, S, _ = x.shape
                q, k, v = self.qkv(self.n1(x)).view(B, S, 3, h, d // h).permute(2, 0, 3, 1, 4)
                y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
                x = x + self.o(y.transpose(1, 2).reshape(B, S, d))
                g, u = self.up(self.n2(x)).chunk(2, dim=-1)
                return x + self.down(F.silu(g) * u)

        class Model(nn.Module):
            def __init__(self, vocab):
                super().__init__()
                self.emb = nn.Embedding(vocab, d)
                self.blocks = nn.ModuleList(Block() for _ in range(L))
                self.norm = nn.RMSNorm(d)
                self.head = nn.Linear(d, vocab, bias=False)

            def forward(self, t):
                x = self.emb(t)
                for b in self.blocks:
                    x = b(x)
                return self.head(self.norm(x))

        torch.manual_seed(1234)
        model = Model(self.vocab).to(device=dev, dtype=torch.bfloat16)
        self.params = sum(p.numel() for p in model.parameters())
        if ctx is not None and ctx.is_dist:
            from torch.nn.parallel import DistributedDataParallel

            model = DistributedDataParallel(model, device_ids=[device], bucket_cap_mb=256)
        self.model = model
        self.opt = torch.optim.AdamW(model.parameters(), lr=1e-4, fused=dev.type == "cuda")
        g = torch.Generator(device=dev).manual_seed(1234 + (ctx.rank if ctx is not None else 0))
        self.tok = torch.randint(0, self.vocab, (self.batch, self.seq + 1), device=dev, generator=g)
        self.F = F

    def step(self):
        logits = self.model(self.tok[:, :-1])
        loss = self.F.cross_entropy(logits.float().view(-1, self.vocab), self.tok[:, 1:].reshape(-1))
        loss.backward()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)

    def calibrate(self) -> dict:
        torch = self.torch
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        self.step()
        e1.record()
        torch.cuda.synchronize()
        s = e0.elapsed_time(e1) * 1e-3
        toks = self.batch * self.seq
        # 6·N·T for the dense weights + causal attention (fwd 2·S·d per token per layer, x3 with bwd)
        return {"train_step_ms": s * 1e3, "train_tokens_per_s": toks / s, "train_params": self.params,
                "train_tflops": 6.0 * self.params * toks / s / 1e12}


class MockLoad:
    def __init__(self, a, device: int):
        self.dt = a.mock_step_ms * 1e-3

    def step(self):
        time.sleep(self.dt)  # releases the GIL like a GPU sync would

    def sync(self):
        pass

    def calibrate(self) -> dict:
        return {"mock_step_ms": self.dt * 1e3}

    def pci_bdf(self, device: int) -> str:
        return f"0000:{0x11 + 0x10 * device:02x}:00.0"  # mock provider's BDF scheme


PHASES: dict[str, list[float]] = {}


def timed(ctx, load, k: int, name: str = "") -> float:
    """Barrier + sync on both sides; returns the MAX over ranks of the wall time.

    The wall-clock (epoch) bounds of each phase are kept in PHASES so a
    rocprofv3 kernel trace of the run can be split into exporter-off / -on
    phases (tools/rocprof_overhead.py)."""
    D.barrier(ctx)
    load.sync()
    w0 = time.time()
    t0 = time.perf_counter()
    for _ in range(k):
        load.step()
    load.sync()
    D.barrier(ctx)
    dt = time.perf_counter() - t0
    if name:
        PHASES[name] = [w0, time.time()]
    return D.all_reduce(ctx, [dt], "max")[0]


def interleaved(ctx, load, exp, a) -> dict:
    """Off/on blocks in ABBA order (off,on, on,off, ...) with the exporter process up:
    *off* = sampling paused (no PMFW / counter reads, no scrapes), *on* = sampling at
    --hz and scraped at --scrape-hz.  Pairs of adjacent blocks see the same thermal
    and power state, so slow drift cancels; the A-B-C phases cannot do that."""
    if a.interleave <= 0:
        return {}
    blk = max(3, a.steps // 4)
    t_on = t_off = 0.0
    blocks = []
    for r in range(a.interleave):
        for on in ((False, True) if r % 2 == 0 else (True, False)):
            sc = None
            if exp is not None:
                if on:
                    exp.resume()
                    sc = Scraper("127.0.0.1", exp.port).start(a.scrape_hz)
                else:
                    exp.pause()
            D.barrier(ctx)
            dt = timed(ctx, load, blk)
            if sc is not None:
                sc.stop()
            blocks.append([int(on), round(dt, 6)])
            if on:
                t_on += dt
            else:
                t_off += dt
    if exp is not None:
        exp.resume()
    return {"overhead_interleaved_pct": 100.0 * (t_on / t_off - 1.0), "interleave_blocks": blocks,
            "interleave_steps_per_block": blk}


# ----------------------------------------------------------------------------- exporter
class AttachedExporter:
    """An already-running exporter (``--control-http``) driven over HTTP."""

    def __init__(self, hostport: str):
        host, _, port = hostport.rpartition(":")
        self.port = int(port)
        self.sc = Scraper(host or "127.0.0.1", self.port)
        m = parse_text(self.sc.get())
        info = m.get("kgs_build_info", [({}, 0)])[0][0]
        self.ready = {"pmc": info.get("pmc_source", "none"), "pmc_error": "",
                      "hz": float(info.get("sample_hz", "0") or 0)}

    def pause(self):
        self.sc.get("/control/pause")

    def resume(self):
        self.sc.get("/control/resume")

    def stop(self) -> dict:
        self.pause()
        m = parse_text(self.sc.get())
        fam = lambda n: {lb["gpu"]: v for lb, v in m.get(n, [])}  # noqa: E731
        reads, rs, pmc, prs = (fam("kgs_reads_total"), fam("kgs_read_seconds_total"),
                               fam("kgs_pmc_samples_total"), fam("kgs_pmc_read_seconds_total"))
        hist = fam("kgs_sample_read_seconds_sum")
        return {"integrals": [{"gpu": g, "reads": reads[g], "read_seconds": hist.get(g, rs.get(g, 0.0)),
                               "pmc_samples": pmc.get(g, 0), "pmc_read_seconds": prs.get(g, 0.0),
                               "overruns": fam("kgs_sampler_overruns_total").get(g, 0)} for g in sorted(reads)]}


class ExporterProc:
    def __init__(self, a, bdfs: list[str], log_path: str):
        cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
               "--hz", str(a.hz), "--proc-every", str(max(1, int(a.hz // 10))),
               "--link-every", str(max(1, int(a.hz))), "--control-stdin", "--control-http", "--node-name", "bench-node",
               "--bdfs", ",".join(bdfs)]
        if a.mock:
            cmd += ["--backend", "mock", "--mock-gpus", str(max(8, len(bdfs))), "--pmc", "mock"]
        else:
            pmc = AUTO_PMC if a.pmc == "auto" else a.pmc
            cmd += ["--pmc", pmc, "--pmc-pipeline" if a.pmc_pipeline else "--no-pmc-pipeline", "--pmc-set", a.pmc_set,
                    "--pmc-lean", str(a.pmc_lean)]
        env = dict(os.environ)
        env.setdefault("KGS_NO_BUILD", "1")
        env.setdefault("PYTHONFAULTHANDLER", "1")  # a native fault leaves a trace in the exporter log
        if not a.mock and "--pmc" in cmd and cmd[cmd.index("--pmc") + 1] == "rocprofiler" \
                and env.get("ROCP_TOOL_LIBRARIES"):
            # Running under rocprofv3: rocprofiler configuration closes before the
            # exporter could force-register, so join as a listed tool library.
            from kube_gpu_stats_amd.native import pmc_lib_path

            env["ROCP_TOOL_LIBRARIES"] = env["ROCP_TOOL_LIBRARIES"] + ":" + pmc_lib_path()
            env["KGS_PMC_AS_TOOL"] = "1"
        self.log = open(log_path, "w")
        self.p = subprocess.Popen(cmd, cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=self.log,
                                  text=True, env=env)
        self.ready = self._wait_ready(120.0)
        self.port = int(self.ready["port"])
        self.sc = Scraper("127.0.0.1", self.port)

    def pause(self):
        self.sc.get("/control/pause")

    def resume(self):
        self.sc.get("/control/resume")

    def _wait_ready(self, timeout: float) -> dict:
        end = time.time() + timeout
        while time.time() < end:
            r, _, _ = select.select([self.p.stdout], [], [], 1.0)
            if r:
                line = self.p.stdout.readline()
                if not line:
                    break
                try:
                    msg = json.loads(line)
                except ValueError:
                    continue
                if msg.get("event") == "ready":
                    return msg
                if msg.get("event") == "error":
                    raise RuntimeError("exporter failed: " + msg.get("error", ""))
            if self.p.poll() is not None:
                break
        raise RuntimeError(f"exporter did not become ready (rc={self.p.poll()}); see {self.log.name}")

    def stop(self) -> dict:
        try:
            self.p.stdin.write("quit\n")
            self.p.stdin.flush()
        except OSError:
            pass
        try:
            out, _ = self.p.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            self.p.kill()
            out, _ = self.p.communicate()
        self.log.close()
        for line in out.splitlines():
            try:
                msg = json.loads(line)
                if msg.get("event") == "stopped":
                    return msg
            except ValueError:
                pass
        return {}


def proc_cpu_seconds(pid: int) -> float:
    """utime + stime of a process (all threads), seconds; 0 if unreadable."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return 0.0


def thread_cpu_seconds(pid: int) -> dict:
    """Per-thread utime + stime, keyed ``<comm>/<tid>`` (finds spinning helper threads)."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"/proc/{pid}/task/{tid}/stat") as f:
                raw = f.read()
            comm = raw[raw.index("(") + 1:raw.rindex(")")]
            fields = raw.rsplit(")", 1)[1].split()
            out[f"{comm}/{tid}"] = (int(fields[11]) + int(fields[12])) / tck
        except (OSError, ValueError, IndexError):
            continue
    return out


def sample_counts(m: dict) -> tuple[dict, dict]:
    pmfw = {lb["gpu"]: v for lb, v in m.get("kgs_samples_total", [])}
    pmc = {lb["gpu"]: v for lb, v in m.get("kgs_pmc_samples_total", [])}
    return pmfw, pmc


def xgmi_rates(before: dict, after: dict, win: float) -> dict:
    """xGMI bytes/s per GPU (all links, read + write) over the timed window, from the
    exporter's PMFW per-link accumulators."""
    def tot(m):
        out: dict = {}
        for fam in ("amdgpu_xgmi_read_bytes_total", "amdgpu_xgmi_write_bytes_total"):
            for lb, v in m.get(fam, []):
                out[lb["gpu"]] = out.get(lb["gpu"], 0.0) + v
        return out
    b, a_ = tot(before), tot(after)
    return {g: round((a_[g] - b.get(g, 0.0)) / win / 1e9, 3) for g in a_} if win > 0 else {}


def observed(m: dict) -> dict:
    """What the exporter saw of the load (window gauges of the last scrape), per GPU."""
    out: dict = {}
    for fam, key in (("amdgpu_gfx_busy_percent", "gfx_busy_pct"), ("amdgpu_umc_busy_percent", "umc_busy_pct"),
                     ("amdgpu_mfma_util_percent", "mfma_util_pct"), ("amdgpu_vmem_busy_percent", "vmem_busy_pct"),
                     ("amdgpu_power_watts", "power_w"), ("amdgpu_gpu_clock_effective_mhz", "clock_mhz")):
        for lb, v in m.get(fam, []):
            out.setdefault(lb["gpu"], {})[key] = round(v, 2)
    for lb, v in m.get("amdgpu_mfma_util_xcc_percent", []):  # XCD order 0..7
        out.setdefault(lb["gpu"], {}).setdefault("mfma_util_xcd_pct", []).append(round(v, 1))
    return out


# ----------------------------------------------------------------------------- main
def main(argv=None) -> int:
    a = parse_args(argv)
    use_cuda = not a.mock
    ctx = D.init_from_env(use_cuda)
    if ctx.world != a.gpus:
        if ctx.rank == 0:
            print(f"warning: --gpus {a.gpus} but WORLD_SIZE {ctx.world}; using WORLD_SIZE", file=sys.stderr)
    n = ctx.world
    if ctx.local_rank == 0 and not a.attach:
        # The exporter child runs with KGS_NO_BUILD=1: make sure its artefacts exist
        # (incremental no-op when the in-tree .so files are current).
        from kube_gpu_stats_amd.native import build as B

        B.build_native()
        if not a.mock:
            B.build_pmc()
            B.build_pmc_aql()
    if a.mock:
        load = MockLoad(a, ctx.local_rank)
    elif a.load == "train":
        load = TrainLoad(a, ctx.local_rank, ctx)
    else:
        load = GpuLoad(a, ctx.local_rank, ctx)

    for _ in range(a.warmup):
        load.step()
    load.sync()
    calib = load.calibrate()

    # phase A: no exporter (an attached exporter is paused: process up, no reads)
    attached = None
    if a.attach and ctx.local_rank == 0:
        attached = AttachedExporter(a.attach)
        attached.pause()
    t_a = timed(ctx, load, a.steps, "A_off")

    # start the node exporter over every local rank's GPU
    bdfs = D.all_gather_object(ctx, (ctx.local_rank, load.pci_bdf(ctx.local_rank)))
    bdfs = [b for _, b in sorted(set(bdfs))]
    exp = None
    err = ""
    if ctx.local_rank == 0:
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        try:
            if attached is not None:
                attached.resume()
                exp = attached
            else:
                exp = ExporterProc(a, bdfs, os.path.join(REPO, "gpurun_out", f"bench_exporter_r{ctx.rank}.log"))
        except Exception as e:  # noqa: BLE001
            err = str(e)
    err = D.broadcast_object(ctx, err)
    if err:
        if ctx.rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "error": err}))
        D.destroy(ctx)
        return 1
    time.sleep(a.settle)

    scraper = None
    before = after = {}
    t_w0 = t_w1 = 0.0
    exp_pid = int(exp.ready.get("pid", 0) or 0) if exp is not None else 0
    cpu0 = cpu1 = 0.0
    thr0: dict = {}
    thr1: dict = {}
    if exp is not None:
        scraper = Scraper("127.0.0.1", exp.port)
        before = parse_text(scraper.get())
        cpu0 = proc_cpu_seconds(exp_pid)
        thr0 = thread_cpu_seconds(exp_pid)
        t_w0 = time.perf_counter()
        scraper.start(a.scrape_hz)
    # phase B: exporter on (timed)
    t_b = timed(ctx, load, a.steps, "B_on")
    if exp is not None:
        scraper.stop()
        after = parse_text(scraper.get())
        t_w1 = time.perf_counter()
        cpu1 = proc_cpu_seconds(exp_pid)
        thr1 = thread_cpu_seconds(exp_pid)
    inter = interleaved(ctx, load, exp, a)
    stopped = exp.stop() if exp is not None else {}

    # phase C: exporter off again
    t_c = timed(ctx, load, a.steps, "C_off")

    result = None
    if exp is not None:
        b_pmfw, b_pmc = sample_counts(before)
        a_pmfw, a_pmc = sample_counts(after)
        win = t_w1 - t_w0
        gpus = sorted(a_pmfw, key=int)
        pmfw_rate = {g: (a_pmfw[g] - b_pmfw.get(g, 0)) / win for g in gpus}
        pmc_rate = {g: (a_pmc.get(g, 0) - b_pmc.get(g, 0)) / win for g in gpus}
        pmc_on = exp.ready.get("pmc", "none") != "none" and sum(pmc_rate.values()) > 0
        # Per GPU: its counter stream if it delivered one, else its PMFW table rate, so one
        # device whose counter tier failed to open lowers the total by its own share only.
        per_gpu = {g: (pmc_rate[g] if pmc_on and pmc_rate[g] > 0 else pmfw_rate[g]) for g in gpus}
        n_pmc = sum(1 for g in gpus if pmc_on and pmc_rate[g] > 0)
        source = "pmc" if n_pmc == len(gpus) else ("pmfw" if n_pmc == 0 else f"pmc on {n_pmc}/{len(gpus)} GPUs")
        total = sum(per_gpu.values())
        t_off = 0.5 * (t_a + t_c)
        result = {
            "metric": METRIC,
            "value": total,
            "unit": "samples/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": t_b * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": ("synthetic mock provider (CPU plumbing)" if a.mock
                     else f"synthetic tokens, random-init {a.train_layers}-layer d={a.train_dim} bf16 decoder "
                     "training step (fwd + bwd + AdamW) as the GPU load" if a.load == "train"
                     else "synthetic (gfx950 MFMA bf16 + HBM triad + HIP-graph tiny-kernel load; random-init operands)"),
            "config": {"model": "node exporter: PMFW table + HBM + per-PID + xGMI + rocprofiler PMC, "
                                f"{a.hz:g} Hz/GPU, /metrics scraped at {a.scrape_hz:g} Hz",
                       "global_batch": n, "seq_len": a.steps, "parallelism": f"dp{n}",
                       "hz": exp.ready.get("hz") or a.hz, "sample_source": source,
                       "exporter": "attached" if a.attach else "spawned",
                       "load": "mock" if a.mock else a.load},
            "samples_per_sec_per_gpu": total / max(1, len(per_gpu)),
            "pmc_samples_per_sec_per_gpu": {g: round(v, 2) for g, v in pmc_rate.items()},
            "pmfw_distinct_samples_per_sec_per_gpu": {g: round(v, 2) for g, v in pmfw_rate.items()},
            "p50_scrape_ms": scraper.percentile(0.5) * 1e3,
            "p99_scrape_ms": scraper.percentile(0.99) * 1e3,
            "scrapes": len(scraper.latencies_s),
            "scrape_errors": scraper.errors,
            "scrape_bytes_avg": scraper.bytes / max(1, len(scraper.latencies_s)),
            "overhead_pct": 100.0 * (t_b / t_off - 1.0),
            "t_off_a_s": t_a,
            "t_on_s": t_b,
            "t_off_c_s": t_c,
            **inter,
            "exporter_cpu_cores": round((cpu1 - cpu0) / win, 4) if win > 0 and exp_pid else None,
            "exporter_cpu_cores_by_thread": {k: round((v - thr0.get(k, 0.0)) / win, 4) for k, v in thr1.items()
                                             if win > 0 and v - thr0.get(k, 0.0) > 0.005 * win},
            "pmc_source": exp.ready.get("pmc"),
            "pmc_error": exp.ready.get("pmc_error"),
            "load": calib,
            "observed_during_load": observed(after),
            "xgmi_GBps_per_gpu": xgmi_rates(before, after, win),
            "phases_wall": PHASES,
            "pmc_read_us_mean": 1e6 * sum(i.get("pmc_read_seconds", 0) for i in stopped.get("integrals") or [])
            / max(1, sum(i.get("pmc_samples", 0) for i in stopped.get("integrals") or [])),
            "pmfw_read_us_mean": 1e6 * sum(i.get("read_seconds", 0) for i in stopped.get("integrals") or [])
            / max(1, sum(i.get("reads", 0) for i in stopped.get("integrals") or [])),
            "exporter_integrals": stopped.get("integrals"),
        }
    # make the result visible to rank 0 if the exporter lived elsewhere (single node: it is rank 0)
    result = D.broadcast_object(ctx, result)
    if ctx.rank == 0 and result is not None:
        line = json.dumps(result)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    D.destroy(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
