"""GPU work the exporter is measured under: the synthetic gfx950 unit (MFMA + HBM triads + a HIP
graph of µs copies, ops/hip/load_kernels.hip), a bf16 decoder training step, and the CPU mock."""
from __future__ import annotations

import time



class Load:
    """A step = ``reps`` back-to-back units (set by calibrate_reps)."""

    reps = 1
    timing = False  # per-component event timing (interleaved blocks)

    def step(self):
        for _ in range(self.reps):
            self.unit()

    def components_start(self) -> None:
        self.timing = True

    def components_end(self) -> dict:
        """Seconds of GPU time per load component since components_start (synced)."""
        self.timing = False
        return {}


class EventTimer:
    """HIP events bracketing each load component inside a timed block: a component's
    GPU time per block, so the paired overheads can be split by what the exporter
    could slow down — a long MFMA kernel, HBM streams, or the dispatch-bound graph of
    tiny kernels.  Events are recorded in every condition alike."""

    def __init__(self, torch):
        self.torch = torch
        self.pool: list = []
        self.used: list[tuple[str, int]] = []

    def mark(self, name: str) -> None:
        """Record the event that opens (or closes) ``name``; components alternate open/close."""
        i = len(self.used)
        if i >= len(self.pool):
            self.pool.append(self.torch.cuda.Event(enable_timing=True))
        self.pool[i].record()
        self.used.append((name, i))

    def collect(self) -> dict:
        self.torch.cuda.synchronize()
        out: dict[str, float] = {}
        for (name, a), (_, b) in zip(self.used[0::2], self.used[1::2]):
            out[name] = out.get(name, 0.0) + self.pool[a].elapsed_time(self.pool[b]) * 1e-3
        self.used.clear()
        return out


class GpuLoad(Load):
    def __init__(self, a, device: int, ctx=None):
        import torch

        from kube_gpu_stats_amd.ops.load import LoadStep

        self.torch = torch
        self.a, self.device = a, device
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
        self.ev = EventTimer(torch)

    def unit(self):
        t = self.timing
        if t:
            self.ev.mark("mfma")
        self.ls.run_mfma()
        if t:
            self.ev.mark("mfma")
            self.ev.mark("triad")
        for _ in range(self.triads):
            self.ls.run_stream()
        if t:
            self.ev.mark("triad")
        if self.graph is not None:
            if t:
                self.ev.mark("tiny_graph")
            self.graph.replay()
            if t:
                self.ev.mark("tiny_graph")
        if self.ar is not None:
            import torch.distributed as dist

            if t:
                self.ev.mark("allreduce")
            dist.all_reduce(self.ar)
            self.ar.mul_(0.5)  # keep values bounded across steps
            if t:
                self.ev.mark("allreduce")

    def components_end(self) -> dict:
        self.timing = False
        return self.ev.collect()

    def component_names(self) -> list[str]:
        return ["mfma", "triad"] + (["tiny_graph"] if self.graph is not None else [])

    def run_component(self, name: str) -> None:
        """One launch of a single load component (phase K)."""
        if name == "mfma":
            self.ls.run_mfma()
        elif name == "triad":
            self.ls.run_stream()
        elif name == "tiny_graph":
            self.graph.replay()

    def sync(self):
        self.torch.cuda.synchronize()

    def burst(self, ms: float) -> None:
        """One MFMA kernel of ≈``ms`` milliseconds, waited for (phase R)."""
        from kube_gpu_stats_amd.ops import load as L

        iters = max(50, int(self.ls.mfma_iters * ms / max(self.mfma_ms, 1e-3)))
        L.mfma_bf16(self.ls.A, self.ls.B, self.ls.C, self.ls.mfma_blocks, iters)
        self.torch.cuda.synchronize()

    def burst_timed(self, ms: float) -> float:
        """burst(), returning the kernel's own GPU time (HIP events), seconds (phase U)."""
        from kube_gpu_stats_amd.ops import load as L

        torch = self.torch
        if not hasattr(self, "_bev"):
            self._bev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        e0, e1 = self._bev
        iters = max(10, int(self.ls.mfma_iters * ms / max(self.mfma_ms, 1e-3)))
        e0.record()
        L.mfma_bf16(self.ls.A, self.ls.B, self.ls.C, self.ls.mfma_blocks, iters)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3

    def triad_burst_timed(self, ms: float) -> float:
        """One HBM triad of ≈``ms`` milliseconds (a slice of the stream buffers), waited for:
        its own GPU time (HIP events), seconds (phase U: a memory-bound kernel, which runs
        at the full shader clock where an MFMA burst is power-capped)."""
        from kube_gpu_stats_amd.ops import load as L

        torch = self.torch
        if not hasattr(self, "_bev"):
            self._bev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        e0, e1 = self._bev
        a, b, c = self.ls.a, self.ls.b, self.ls.c
        if not hasattr(self, "_triad_per_ms"):  # elements per ms, from a warm 1/8-buffer triad
            n = a.numel() // 32 * 4
            for _ in range(2):  # the first pass pays first-touch and TLB misses
                e0.record()
                L.triad_f32(a[:n], b[:n], c[:n], 1.5)
                e1.record()
                e1.synchronize()
            self._triad_per_ms = n / max(e0.elapsed_time(e1), 1e-3)
        n = min(a.numel(), max(1 << 20, int(self._triad_per_ms * ms))) // 4 * 4  # float4 accesses
        e0.record()
        L.triad_f32(a[:n], b[:n], c[:n], 1.5)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3

    def saturate(self, secs: float) -> float:
        """MFMA kernels back to back (two in flight) for ``secs``: Σ their GPU time (phase U)."""
        torch = self.torch
        ev = []
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < secs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.ls.run_mfma()
            e1.record()
            ev.append((e0, e1))
            if len(ev) >= 2:
                ev[-2][1].synchronize()
        torch.cuda.synchronize()
        return sum(x.elapsed_time(y) for x, y in ev) * 1e-3

    def irregular(self, secs: float, seed: int, streams: int = 1) -> float:
        """Seeded random MFMA kernels (5 µs - 20 ms) and gaps on ``streams`` streams for
        ``secs``: the union of the kernels' event-timed intervals, seconds (phase U)."""
        from kube_gpu_stats_amd.ops.irregular import IrregularLoad, mfma_launcher

        if not hasattr(self, "_irr"):
            per_iter = self.mfma_ms / max(1, self.ls.mfma_iters)
            self._irr = IrregularLoad(self.torch, mfma_launcher(self.torch, self.ls, per_iter), self.device)
        r = self._irr.run(secs, seed, streams)
        self.last_irregular = r
        return r["busy_s"]

    def prepare_train(self) -> None:
        if not hasattr(self, "_train"):
            self._train = TrainLoad(self.a, self.device, None)
            self._train.unit()  # allocator growth, kernel selection
            self._train.unit()
            self.torch.cuda.synchronize()

    def train_timed(self, secs: float) -> float:
        """bf16 decoder training steps (TrainLoad, no DDP) for ``secs``: the union of the
        step kernels' execution intervals from the PyTorch profiler, seconds (phase U)."""
        from kube_gpu_stats_amd.ops.irregular import profiled_busy

        self.prepare_train()
        busy, steps, kernels = profiled_busy(self.torch, self._train.unit, secs)
        self.last_train = {"steps": steps, "kernels": kernels}
        return busy

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
        self.mfma_ms = mfma_s * 1e3
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

    burst_timed = None  # no MFMA burst kernel of known length: phase U is skipped

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

        self.ev = EventTimer(torch) if dev.type == "cuda" else None

    burst = None  # phase R runs on the synthetic load only

    def component_names(self) -> list[str]:
        return []  # one component (the whole step): phase K has nothing to split

    def unit(self):
        t = self.timing and self.ev is not None
        if t:
            self.ev.mark("train_step")
        logits = self.model(self.tok[:, :-1])
        loss = self.F.cross_entropy(logits.float().view(-1, self.vocab), self.tok[:, 1:].reshape(-1))
        loss.backward()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        if t:
            self.ev.mark("train_step")

    def components_end(self) -> dict:
        self.timing = False
        return self.ev.collect() if self.ev is not None else {}

    def calibrate(self) -> dict:
        torch = self.torch
        self.unit()  # first step: allocator growth, kernel selection; not representative
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.unit()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        s = sorted(ts)[1]
        toks = self.batch * self.seq
        # 6·N·T for the dense weights + causal attention (fwd 2·S·d per token per layer, x3 with bwd)
        return {"train_step_ms": s * 1e3, "train_tokens_per_s": toks / s, "train_params": self.params,
                "train_tflops": 6.0 * self.params * toks / s / 1e12}


class MockLoad(Load):
    def __init__(self, a, device: int):
        self.dt = a.mock_step_ms * 1e-3

    def unit(self):
        t0 = time.perf_counter()
        time.sleep(self.dt)  # releases the GIL like a GPU sync would
        if self.timing:
            self.comp["mock"] = self.comp.get("mock", 0.0) + time.perf_counter() - t0

    def components_start(self) -> None:
        self.timing = True
        self.comp: dict[str, float] = {}

    def components_end(self) -> dict:
        self.timing = False
        return dict(self.comp)

    def burst(self, ms: float) -> None:
        time.sleep(ms * 1e-3)  # plumbing only: the mock counters do not follow the host

    def burst_timed(self, ms: float) -> float:
        self.burst(ms)
        return ms * 1e-3

    triad_burst_timed = burst_timed

    def saturate(self, secs: float) -> float:
        time.sleep(secs)
        return secs

    def irregular(self, secs: float, seed: int, streams: int = 1) -> float:
        time.sleep(secs)  # plumbing only: the mock counters do not follow the host
        return 0.5 * secs

    def train_timed(self, secs: float) -> float:
        time.sleep(secs)
        return 0.9 * secs

    def sync(self):
        pass

    def calibrate(self) -> dict:
        return {"mock_unit_ms": self.dt * 1e3}

    def pci_bdf(self, device: int) -> str:
        return f"0000:{0x11 + 0x10 * device:02x}:00.0"  # mock provider's BDF scheme
