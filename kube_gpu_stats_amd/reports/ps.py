"""``kgs ps`` — which processes (and pods) are using a node's GPUs right now.

The reference answers "who holds GPUs" from the allocation side only: pod specs
(who_use_gpu.py:27-49) and kube-state-metrics requests (gpu_util_stats.py:137).
A card that a pod was granted but that another process actually runs on, or a
pod that holds HBM without computing, is invisible there.  This reads one node
exporter's per-process families — AMD SMI process list on the node-wide slow
tier, each line already attributed to its pod (attribution/attributor.py) — and
prints one row per (GPU, process): HBM held, CU occupancy now, and the compute
share over the interval (``rate(amdgpu_process_cu_seconds_total)`` from two
scrapes ``--interval`` apart).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import urllib.parse

from ..utils.scrape import Scraper, parse_text
from .table import render, render_csv

HEADER = ["GPU", "PID", "Process", "Namespace", "Pod", "Container", "HBM GiB", "CU share %", "CUs now"]


def _key(lb: dict) -> tuple[str, str]:
    return lb.get("gpu", ""), lb.get("pid", "")


def rows_from(prev: dict | None, cur: dict, dt: float) -> list[dict]:
    """One row per (GPU, PID) of the current scrape; ``cu_share_pct`` needs ``prev``."""
    hbm = {_key(lb): (lb, v) for lb, v in cur.get("amdgpu_process_hbm_bytes", [])}
    occ = {_key(lb): v for lb, v in cur.get("amdgpu_process_cu_occupancy", [])}
    cus = {_key(lb): v for lb, v in cur.get("amdgpu_process_cu_seconds_total", [])}
    pcus = {_key(lb): v for lb, v in prev.get("amdgpu_process_cu_seconds_total", [])} if prev else {}
    rows = []
    for k, (lb, v) in hbm.items():
        share = None
        if dt > 0 and k in pcus and k in cus and cus[k] >= pcus[k]:
            share = 100.0 * (cus[k] - pcus[k]) / dt
        rows.append({"gpu": lb.get("gpu", ""), "pid": int(lb["pid"]) if lb.get("pid", "").isdigit() else lb.get("pid"),
                     "process": lb.get("process", ""), "namespace": lb.get("namespace", ""),
                     "pod": lb.get("pod", ""), "container": lb.get("container", ""),
                     "hbm_gib": v / float(1 << 30), "cu_share_pct": share, "cu_occupancy": occ.get(k)})
    rows.sort(key=lambda r: (int(r["gpu"]) if str(r["gpu"]).isdigit() else 0, -r["hbm_gib"]))
    return rows


def _cells(r: dict) -> list:
    f = lambda x, fmt: "-" if x is None else fmt.format(x)  # noqa: E731
    return [r["gpu"], r["pid"], r["process"] or "-", r["namespace"] or "-", r["pod"] or "-", r["container"] or "-",
            f(r["hbm_gib"], "{:.2f}"), f(r["cu_share_pct"], "{:.1f}"),
            "-" if r["cu_occupancy"] is None else int(r["cu_occupancy"])]


def build_parser(ap: argparse.ArgumentParser | None = None) -> argparse.ArgumentParser:
    ap = ap or argparse.ArgumentParser(prog="kgs ps", description=__doc__.splitlines()[0])
    ap.add_argument("url", nargs="?", default="http://127.0.0.1:9400", help="exporter base URL")
    ap.add_argument("--interval", type=float, default=1.0,
                    help="seconds between the two scrapes the compute share is measured over (0 = one scrape, "
                         "no share)")
    ap.add_argument("--gpu", default="", help="only this GPU index")
    ap.add_argument("--pod", default="", help="only processes of this pod")
    ap.add_argument("--format", default="table", choices=["table", "json", "csv"])
    return ap


def run(a, out=sys.stdout) -> int:
    u = urllib.parse.urlsplit(a.url if "://" in a.url else "http://" + a.url)
    sc = Scraper(u.hostname or "127.0.0.1", u.port or 80)
    prev, dt = None, 0.0
    if a.interval > 0:
        t0 = time.monotonic()  # the exporter renders right after the request
        prev = parse_text(sc.scrape_once())
        time.sleep(max(0.0, a.interval - (time.monotonic() - t0)))
    t1 = time.monotonic()
    cur = parse_text(sc.scrape_once())
    if prev is not None:
        dt = t1 - t0
    rows = rows_from(prev, cur, dt)
    rows = [r for r in rows if (not a.gpu or r["gpu"] == a.gpu) and (not a.pod or r["pod"] == a.pod)]
    if a.format == "json":
        out.write(json.dumps(rows) + "\n")
    elif a.format == "csv":
        out.write(render_csv(HEADER, [_cells(r) for r in rows]) + "\n")
    else:
        out.write(render(HEADER, [_cells(r) for r in rows]) + "\n")
    return 0
