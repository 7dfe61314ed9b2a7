"""Irregular GPU loads with an event-timed duty.

Phase U and the GPU tests used to check the exported utilisation on strictly periodic,
single-stream trains only — the loads the estimator's constants were fitted on.  Real
tenants run kernels of every length, with gaps of every length, on several streams.
This module drives such loads from a seed, so a run can be repeated, and measures the
truth the exporter is compared with: the union over time of every kernel's own
execution interval (HIP events around each launch; on two streams the intervals
overlap, and "a kernel is in flight" is their union — what container_gpu_sm_util's
dispatch-in-flight source measures, and what the reference bills each pod the mean of,
gpu_util_stats/gpu_util_stats.py:78).

* ``random``     — one stream; each kernel ≈ log-uniform [5 µs, 20 ms] of MFMA work, each
                   idle gap log-uniform [5 µs, 20 ms] (gaps under 0.1 ms: the next kernel
                   is queued behind the previous one, so the GPU sees only launch gaps);
* ``two_stream`` — the same on two streams at once, independently seeded;
* ``train``      — a bf16 training step (bench's decoder), its kernels timed by the
                   PyTorch profiler (bench/phase_u.py; per-kernel events cannot bracket
                   library kernels from the outside).

Everything but ``union_seconds`` needs torch and a GPU; the pieces are pure functions
of their inputs so the CPU tests pin the schedule and the union.
"""
from __future__ import annotations

import math
import random
import time

# Log-uniform ranges (ms) of one kernel and one idle gap (5 µs – 20 ms).
KERNEL_MS = (0.005, 20.0)
GAP_MS = (0.005, 20.0)
# A gap shorter than this is not slept: the next kernel is queued at once (host sleeps
# cannot time tens of µs; the GPU then idles only for the launch gap).
QUEUE_BELOW_MS = 0.1
MAX_QUEUED = 4  # kernels in flight per stream when queued back to back


def loguniform(rnd: random.Random, lo: float, hi: float) -> float:
    return math.exp(rnd.uniform(math.log(lo), math.log(hi)))


def schedule(seed: int, n: int, kernel_ms=KERNEL_MS, gap_ms=GAP_MS) -> list[tuple[float, float]]:
    """The first n (kernel ms, following gap ms) pairs of seed's schedule."""
    rnd = random.Random(seed)
    return [(loguniform(rnd, *kernel_ms), loguniform(rnd, *gap_ms)) for _ in range(n)]


def union_seconds(intervals: list[tuple[float, float]]) -> float:
    """Length of the union of [start, end] intervals (any order, any overlap)."""
    total, cur_s, cur_e = 0.0, None, None
    for s, e in sorted(intervals):
        if e <= s:
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                total += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        total += cur_e - cur_s
    return total


class IrregularLoad:
    """Seeded random MFMA kernels on one or more streams, each bracketed by HIP events.

    ``launch(ms, stream, k)`` launches one kernel of ≈ms milliseconds on ``stream``
    (k: the stream's index, for a per-stream output buffer).  ``run`` returns the
    union of the kernels' execution intervals over the run (``busy_s``), their plain
    sum (``sum_s``: larger than the union where two streams overlap), the kernel count
    and the host wall time from the first launch to the end of the last kernel."""

    def __init__(self, torch, launch, device: int = 0):
        self.torch = torch
        self.launch = launch
        self.device = device
        self.streams = [torch.cuda.Stream(device=device) for _ in range(2)]

    def run(self, secs: float, seed: int, streams: int = 1, kernel_ms=KERNEL_MS, gap_ms=GAP_MS) -> dict:
        torch = self.torch
        ss = self.streams[:streams]
        for s in ss:
            s.wait_stream(torch.cuda.current_stream(self.device))
        rnds = [random.Random(seed * 1000 + k) for k in range(streams)]
        ref = torch.cuda.Event(enable_timing=True)
        ref.record(ss[0])
        ref.synchronize()
        t_ref_ns = time.monotonic_ns()  # host CLOCK_MONOTONIC at the reference stamp (± µs)
        for s in ss[1:]:
            s.wait_event(ref)  # no kernel of stream k starts before the reference stamp
        events: list[tuple] = []
        # per stream: events of kernels queued and not yet known complete; time the next launch is due
        inflight: list[list] = [[] for _ in ss]
        due = [time.perf_counter()] * streams
        gap_after: list[float] = [0.0] * streams
        t0 = time.perf_counter()
        end = t0 + secs
        while True:
            now = time.perf_counter()
            if now >= end:
                break
            for k, s in enumerate(ss):
                # a stream waiting out a gap: the gap starts when its last kernel ends
                if inflight[k] and gap_after[k] >= QUEUE_BELOW_MS:
                    if not inflight[k][-1].query():
                        continue
                    inflight[k].clear()
                    due[k] = time.perf_counter() + gap_after[k] * 1e-3
                    gap_after[k] = 0.0
                    continue
                inflight[k] = [e for e in inflight[k] if not e.query()] if len(inflight[k]) >= MAX_QUEUED else inflight[k]
                if now < due[k] or len(inflight[k]) >= MAX_QUEUED:
                    continue
                kms, gms = loguniform(rnds[k], *kernel_ms), loguniform(rnds[k], *gap_ms)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                self.launch(kms, s, k)
                e1.record(s)
                events.append((e0, e1))
                inflight[k].append(e1)
                gap_after[k] = gms
                if gms < QUEUE_BELOW_MS:
                    due[k] = now
            wait = min(due) - time.perf_counter()
            time.sleep(min(max(wait, 0.0), 2e-4) if wait > 5e-5 else 2e-5)
        for s in ss:
            s.synchronize()
        wall = time.perf_counter() - t0
        iv = [(ref.elapsed_time(a) * 1e-3, ref.elapsed_time(b) * 1e-3) for a, b in events]
        return {"busy_s": union_seconds(iv), "sum_s": sum(b - a for a, b in iv), "kernels": len(iv),
                "wall_s": wall, "streams": streams, "seed": seed, "t_ref_mono_ns": t_ref_ns, "intervals": iv}


def mfma_launcher(torch, ls, ms_per_iter: float, blocks: int = 2048):
    """launch(ms, stream, k) for IrregularLoad: the in-tree MFMA kernel
    (ops/hip/load_kernels.hip) with its iteration count scaled to ≈ms, writing a
    per-stream output buffer."""
    from kube_gpu_stats_amd.ops import load as L

    outs = [ls.C, torch.empty_like(ls.C)]

    def launch(ms: float, stream, k: int) -> None:
        L.mfma_bf16(ls.A, ls.B, outs[k], blocks, max(1, int(ms / max(ms_per_iter, 1e-9))), stream=stream)

    return launch


def kernel_intervals_from_profile(prof) -> list[tuple[float, float]]:
    """GPU kernel [start, end] intervals (seconds) of a torch.profiler run: the truth a
    training step's duty is taken from (bench/phase_u.py)."""
    out = []
    for ev in prof.events():
        dt = getattr(ev, "device_type", None)
        if dt is None or "CUDA" not in str(dt) and "HIP" not in str(dt):
            continue
        tr = getattr(ev, "time_range", None)
        if tr is None:
            continue
        out.append((tr.start * 1e-6, tr.end * 1e-6))  # µs → s
    return out


def profiled_busy(torch, step, secs: float, queue: int = 2) -> tuple[float, int, int]:
    """Run ``step()`` repeatedly for ``secs`` under the PyTorch profiler (at most ``queue``
    steps in flight): (union of the GPU kernels' execution intervals in seconds, steps,
    kernels).  The duty of a workload whose kernels come from libraries (a training
    step's GEMMs, attention, optimizer) that no event pair can bracket one by one."""
    from torch.profiler import ProfilerActivity, profile

    steps = 0
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < secs:
            step()
            steps += 1
            if steps % queue == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
    iv = kernel_intervals_from_profile(prof)
    if not iv:
        raise RuntimeError("the profiler recorded no GPU kernel")
    return union_seconds(iv), steps, len(iv)
