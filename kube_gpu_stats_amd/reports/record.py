"""``kgs record`` — capture one exporter's full-rate counter stream as a timeline.

The exporter keeps every counter drain of the last ≈1 s per GPU (``/counters``,
8192 drains at 8 kHz).  This polls ``/counters?gpu=N&since=SEQ`` for every GPU
and writes what it drained as a Chrome trace-event JSON file: open it in
Perfetto (ui.perfetto.dev) or chrome://tracing.  Each GPU is a process with
counter tracks — GPU-active % (GRBM_SPI_BUSY: waves to run), MFMA util % of the
active cycles, shader clock — and a ``busy`` track of the segments where work
ran (``dmon.segments``), so a 1 ms kernel burst shows up as a 1 ms block.
Nothing here touches a GPU; it is an HTTP client of a running exporter.

``--profiling`` switches the exporter to READ every tick for the capture
(``/control/pmc/idle?hz=0``, loopback only) and restores its idle rate after:
full time resolution on quiet stretches, at the cost of the PMFW GFX busy
counting the READs as work meanwhile (profiles/r2/idle_busy/README.md).

A gap in the sequence numbers between two polls means the ring wrapped before
it was drained (poll faster); it is counted per GPU as ``lost``.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import urllib.parse
import urllib.request

from .dmon import segments


def _get(base: str, path: str):
    return json.loads(urllib.request.urlopen(base + path, timeout=10).read())


def capture(base: str, seconds: float, poll_s: float, gpus: list[str] | None = None) -> dict:
    """{gpu: {"samples": [...], "lost": n, "counters": [...]}} drained over ``seconds``."""
    if gpus is None:
        gpus = [str(d["gpu"]) for d in _get(base, "/devices")]
    out = {g: {"samples": [], "lost": 0, "counters": []} for g in gpus}
    since: dict[str, int] = {}
    t_end = time.monotonic() + seconds
    while True:
        for g in gpus:
            q = f"/counters?gpu={g}&" + (f"since={since[g]}" if g in since else "n=1")
            body = _get(base, q)
            s = body.get("samples", [])
            out[g]["counters"] = body.get("counters", out[g]["counters"])
            if s:
                if g in since and s[0]["seq"] > since[g] + 1:
                    out[g]["lost"] += s[0]["seq"] - since[g] - 1
                if g in since:  # the first poll only anchors the sequence
                    out[g]["samples"].extend(s)
                since[g] = s[-1]["seq"]
        if time.monotonic() >= t_end:
            break
        time.sleep(poll_s)
    return out


def chrome_trace(cap: dict, devices: dict | None = None) -> dict:
    """Chrome trace-event JSON (counter tracks + busy segments) from ``capture``."""
    t0 = min((d["samples"][0]["mono_ns"] for d in cap.values() if d["samples"]), default=0)
    us = lambda ns: (ns - t0) / 1e3  # noqa: E731
    ev: list[dict] = []
    for g, d in cap.items():
        pid = int(g)
        name = f"GPU {g}" + (f" ({devices[g]})" if devices and g in devices else "")
        ev.append({"name": "process_name", "ph": "M", "pid": pid, "args": {"name": name}})
        ev.append({"name": "thread_name", "ph": "M", "pid": pid, "tid": 1, "args": {"name": "busy segments"}})
        for x in d["samples"]:
            if "gpu_active_pct" not in x:
                continue
            ts = us(x["mono_ns"])
            ev.append({"name": "GPU active %", "ph": "C", "ts": ts, "pid": pid,
                       "args": {"active": round(x["gpu_active_pct"], 2)}})
            if "mfma_util_pct" in x:  # fresh drains only (lite READs: the publishing ones)
                ev.append({"name": "MFMA util %", "ph": "C", "ts": ts, "pid": pid,
                           "args": {"mfma": round(x["mfma_util_pct"], 2)}})
            ev.append({"name": "shader clock MHz", "ph": "C", "ts": ts, "pid": pid,
                       "args": {"mhz": round(x.get("gpu_clock_mhz", 0.0), 1)}})
        segs, _, _ = segments(d["samples"])
        for s0, s1 in segs:
            ev.append({"name": "busy", "ph": "X", "ts": us(s0), "dur": (s1 - s0) / 1e3, "pid": pid, "tid": 1})
    return {"traceEvents": ev, "displayTimeUnit": "ms"}


def summary(cap: dict) -> dict:
    out = {}
    for g, d in cap.items():
        s = d["samples"]
        segs, busy, span = segments(s)
        gaps = [(b["mono_ns"] - a["mono_ns"]) * 1e-6 for a, b in zip(s, s[1:])]
        out[g] = {"drains": len(s), "lost": d["lost"], "span_s": round(span, 4),
                  "drains_per_s": round(len(s) / span, 1) if span else None,
                  "max_gap_ms": round(max(gaps), 3) if gaps else None,
                  "busy_segments": len(segs), "duty_pct": round(100 * busy / span, 2) if span else None}
    return out


def build_parser(ap: argparse.ArgumentParser | None = None) -> argparse.ArgumentParser:
    ap = ap or argparse.ArgumentParser(prog="kgs record", description=__doc__.splitlines()[0])
    ap.add_argument("url", nargs="?", default="http://127.0.0.1:9400", help="exporter base URL")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--poll-ms", type=float, default=200.0,
                    help="poll period per GPU; keep it under the ring's span (≈1 s at 8 kHz)")
    ap.add_argument("--gpu", action="append", default=None, help="GPU index to record (repeatable; default all)")
    ap.add_argument("--profiling", action="store_true",
                    help="READ every tick during the capture (exporter control endpoint; loopback only)")
    ap.add_argument("--out", default="kgs_trace.json", help="Chrome trace-event JSON output")
    return ap


def run(a, out=sys.stdout) -> int:
    u = urllib.parse.urlsplit(a.url if "://" in a.url else "http://" + a.url)
    base = f"{u.scheme}://{u.netloc}"
    devices = {str(d["gpu"]): d.get("bdf", "") for d in _get(base, "/devices")}
    restore = None
    if a.profiling:
        restore = _get(base, "/control/pmc/idle?hz=-1").get("pmc_idle_hz")
        _get(base, "/control/pmc/idle?hz=0")
    try:
        cap = capture(base, a.seconds, a.poll_ms / 1e3, a.gpu)
    finally:
        if restore is not None:
            _get(base, f"/control/pmc/idle?hz={restore:g}")
    with open(a.out, "w") as f:
        json.dump(chrome_trace(cap, devices), f)
    out.write(json.dumps({"out": a.out, "gpus": summary(cap)}) + "\n")
    return 0
