"""Phase R — what the primary rate resolves of a train of ≈1 ms MFMA bursts."""
from __future__ import annotations

import json
import time

from kube_gpu_stats_amd.parallel import dist as D


RING = 8190  # drains /counters returns at most (native kPmcRing 8192, less the write slot)


def burst_train(ctx, load, exp, a) -> dict:
    """Phase R — what the primary rate resolves ("the headline value is a
    dial").  Every rank fires a train of ≈``--burst-ms`` MFMA kernels, one every
    ``--burst-period-ms``, for ``--burst-s``; the node exporter keeps sampling at the
    primary rate.  Rank 0 then reads each GPU's full-rate ``/counters`` stream and
    counts busy segments (reports/dmon.py ``segments``): at 8 kHz every launched
    burst is its own segment and the busy integral matches the host's duty cycle,
    where the ≈50 Hz PMFW table only sees the average.  Untimed; not in any overhead."""
    if a.burst_s <= 0 or getattr(load, "burst", None) is None:
        return {}
    idle_hz = exp.set_idle_hz(-1) if exp is not None else 0.0  # hz < 0 only reads the setting
    if exp is not None:
        exp.set_idle_hz(0)  # profiling mode: READ every tick
    D.barrier(ctx)
    period = a.burst_period_ms * 1e-3
    # /counters keeps the last RING drains: the train must fit in them (8190 drains are
    # 1.0 s at 8 kHz, 0.51 s at 16 kHz — r5i resolved 102 of 120 bursts of a 0.6 s train)
    train_s = min(a.burst_s, 0.8 * RING / a.hz) if a.hz > 0 else a.burst_s
    bursts: list[tuple[int, int]] = []
    nxt = time.monotonic()
    t_end = nxt + train_s
    while time.monotonic() < t_end:
        t0 = time.monotonic_ns()
        load.burst(a.burst_ms)
        bursts.append((t0, time.monotonic_ns()))
        nxt += period
        d = nxt - time.monotonic()
        if d > 0:
            time.sleep(d)
    everyone = D.all_gather_object(ctx, (load.pci_bdf(ctx.local_rank), bursts))
    if exp is None:
        return {}
    exp.set_idle_hz(idle_hz)
    import urllib.request

    from kube_gpu_stats_amd.reports.dmon import segments

    base = f"http://127.0.0.1:{exp.port}"
    gpu_of = {d["bdf"]: str(d["gpu"]) for d in json.load(urllib.request.urlopen(base + "/devices", timeout=10))}
    per: dict[str, dict] = {}
    for bdf, bs in everyone:
        g = gpu_of.get(bdf)
        if g is None or not bs:
            continue
        body = json.load(urllib.request.urlopen(f"{base}/counters?gpu={g}&n={RING}", timeout=10))
        lo, hi = bs[0][0] - 2_000_000, bs[-1][1] + 2_000_000
        win = [x for x in body.get("samples", []) if lo <= x["mono_ns"] <= hi]
        segs, busy, span = segments(win)
        med = lambda xs: sorted(xs)[len(xs) // 2] * 1e-6 if xs else None  # noqa: E731
        per[g] = {"launched": len(bs), "segments": len(segs), "drains": len(win),
                  "drains_per_s": round(len(win) / span, 1) if span else None,
                  "covered_s": round(span, 4),
                  "median_burst_ms_host": med([e - s for s, e in bs]),
                  "median_segment_ms": med([e - s for s, e in segs]),
                  "duty_host": round(sum(e - s for s, e in bs) * 1e-9 / span, 4) if span else None,
                  "duty_counters": round(busy / span, 4) if span else None}
    return {"burst_ms": a.burst_ms, "period_ms": a.burst_period_ms, "train_s": round(train_s, 3),
            "mode": "profiling (--pmc-idle-hz 0: every tick READs)", "mock": bool(a.mock), "per_gpu": per}
