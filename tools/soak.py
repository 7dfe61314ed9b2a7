"""GPU soak: the exporter at its defaults (8 kHz, batched READs, 100 Hz PMFW thread)
for several minutes on a real MI355X, under a load that keeps changing.

Every cycle of the load is (1) 2 s of back-to-back MFMA + HBM triad steps, (2) 2 s of
short bursts with 20 ms idle gaps (the counter tier goes quiet and back: synchronous
READs at the idle rate, then a fresh batched rotation), (3) 1 s idle.  The exporter's
own periodic re-START (--pmc-refresh-s 20 here) and a counter hand-over
(``/control/pmc/release`` + ``acquire``) every 30 s run on top.  Scraped at 10 Hz.

Per 10 s window: counter samples/s, PMFW distinct tables/s, READ writebacks/s, dropped
READs, counter errors, breaker trips, sampler overruns, exporter RSS and CPU, render time.
The run fails (exit 1) on any counter error, dropped READ, breaker trip or hung thread,
or an RSS that grows by more than 8 MiB after the first minute.

With ``--idle-s 4 --quiet-release-s 2`` every cycle's idle stretch parks the counter tier
(the quiet release) and the next busy phase takes it back, under the same re-STARTs and
hand-overs; the run then also fails unless it parked and woke every cycle or so.

    python tools/soak.py --seconds 240 --out gpurun_out/soak.json
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
import urllib.request

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def rss_mib(pid: int) -> float:
    with open(f"/proc/{pid}/status") as f:
        for ln in f:
            if ln.startswith("VmRSS:"):
                return int(ln.split()[1]) / 1024.0
    return 0.0


def cpu_s(pid: int) -> float:
    with open(f"/proc/{pid}/stat") as f:
        parts = f.read().rsplit(")", 1)[1].split()
    return (int(parts[11]) + int(parts[12])) / os.sysconf("SC_CLK_TCK")


def thread_cpu(pid: int) -> dict:
    """Per-thread utime + stime in seconds, keyed ``<comm>/<tid>``."""
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
            fields = raw.rsplit(")", 1)[1].split()
            out[f"{raw[raw.index('(') + 1:raw.rindex(')')]}/{tid}"] = (int(fields[11]) + int(fields[12])) / tck
        except (OSError, ValueError, IndexError):
            continue
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--hz", type=float, default=8000)
    ap.add_argument("--window", type=float, default=10.0)
    ap.add_argument("--out", default="gpurun_out/soak.json")
    ap.add_argument("--mock", action="store_true", help="mock GPU and counters, no load (CPU rehearsal of the script)")
    ap.add_argument("--idle-s", type=float, default=1.0, help="idle stretch of each load cycle")
    ap.add_argument("--quiet-release-s", type=float, default=None,
                    help="the exporter's --pmc-quiet-release-s (default: the exporter's own)")
    a = ap.parse_args()

    from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

    if a.mock:
        src = ["--backend", "mock", "--mock-gpus", "1", "--pmc", "mock", "--no-pin-numa"]
        ls = burst = lambda: time.sleep(0.005)  # noqa: E731
        sync = lambda: None  # noqa: E731
    else:
        import torch

        from kube_gpu_stats_amd.ops.load import LoadStep

        p = torch.cuda.get_device_properties(0)
        src = ["--pmc", "aqlprofile", "--bdfs", f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"]
        ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=4000, stream_bytes=1 << 30)
        burst = LoadStep(device=0, mfma_blocks=2048, mfma_iters=200, stream_bytes=1 << 24)
        sync = torch.cuda.synchronize
        ls()
        burst()
        sync()

    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    err = open(os.path.splitext(a.out)[0] + "_exporter.err", "w")  # a pipe nobody drains could block the exporter
    proc = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
                             "--hz", f"{a.hz:g}", *src, "--control-stdin", "--control-http",
                             "--pmc-refresh-s", "20", "--window", "1",
                             *([] if a.quiet_release_s is None else ["--pmc-quiet-release-s", f"{a.quiet_release_s:g}"])],
                            cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=err, text=True)
    windows: list[dict] = []
    fail: list[str] = []
    try:
        ready = json.loads(proc.stdout.readline())
        assert ready["event"] == "ready" and ready["pmc"] == ("mock" if a.mock else "aqlprofile"), ready
        base = f"http://127.0.0.1:{ready['port']}"
        sc = Scraper("127.0.0.1", ready["port"])
        one = lambda m, f: m[f][0][1] if m.get(f) else 0.0  # noqa: E731
        fams = ("kgs_pmc_samples_total", "kgs_samples_total", "kgs_pmc_publishes_total", "kgs_pmc_unlanded_total",
                "kgs_pmc_errors_total", "kgs_pmc_breaker_trips_total", "kgs_sampler_overruns_total",
                "kgs_pmc_refreshes_total", "kgs_pmc_releases_total", "kgs_scrape_render_seconds_total",
                "kgs_scrapes_total", "kgs_sampler_thread_hung", "amdgpu_gpu_active_seconds_total",
                "kgs_pmc_parks_total", "kgs_pmc_parked_seconds_total")
        snap = lambda: {f: one(parse_text(sc.get()), f) for f in fams}  # noqa: E731
        t_start = time.time()
        w_t0, w_m0, w_cpu0, w_thr0 = t_start, snap(), cpu_s(proc.pid), thread_cpu(proc.pid)
        w_loaded = 0.0
        last_handover = t_start
        next_scrape = t_start
        phase_t0, phase = t_start, 0
        while time.time() - t_start < a.seconds:
            now = time.time()
            # load cycle: 2 s continuous, 2 s bursts with 20 ms gaps, --idle-s idle
            if phase == 0:
                ls()
                sync()
                w_loaded += time.time() - now
                if time.time() - phase_t0 >= 2.0:
                    phase, phase_t0 = 1, time.time()
            elif phase == 1:
                burst()
                sync()
                time.sleep(0.02)
                if time.time() - phase_t0 >= 2.0:
                    phase, phase_t0 = 2, time.time()
            else:
                time.sleep(0.05)
                if time.time() - phase_t0 >= a.idle_s:
                    phase, phase_t0 = 0, time.time()
            if now >= next_scrape:
                sc.get()
                next_scrape = now + 0.1
            if now - last_handover >= 30.0:
                urllib.request.urlopen(base + "/control/pmc/release", timeout=10).read()
                time.sleep(0.2)
                urllib.request.urlopen(base + "/control/pmc/acquire", timeout=10).read()
                last_handover = time.time()
            if now - w_t0 >= a.window:
                m1, t1, c1, thr1 = snap(), time.time(), cpu_s(proc.pid), thread_cpu(proc.pid)
                dt = t1 - w_t0
                d = {f: m1[f] - w_m0[f] for f in fams}
                w = {"t": round(t1 - t_start, 1), "pmc_samples_per_s": round(d["kgs_pmc_samples_total"] / dt, 1),
                     "pmfw_tables_per_s": round(d["kgs_samples_total"] / dt, 1),
                     "writebacks_per_s": round(d["kgs_pmc_publishes_total"] / dt, 1),
                     "gpu_active_share": round(d["amdgpu_gpu_active_seconds_total"] / dt, 3),
                     "loaded_share": round(w_loaded / dt, 3),
                     "dropped": d["kgs_pmc_unlanded_total"], "pmc_errors": d["kgs_pmc_errors_total"],
                     "breaker_trips": d["kgs_pmc_breaker_trips_total"], "overruns": d["kgs_sampler_overruns_total"],
                     "refreshes": d["kgs_pmc_refreshes_total"], "handovers": d["kgs_pmc_releases_total"],
                     "parks": d["kgs_pmc_parks_total"], "parked_share": round(d["kgs_pmc_parked_seconds_total"] / dt, 3),
                     "render_ms": round(1e3 * d["kgs_scrape_render_seconds_total"] / max(d["kgs_scrapes_total"], 1), 3),
                     "rss_mib": round(rss_mib(proc.pid), 1), "cpu_cores": round((c1 - w_cpu0) / dt, 4),
                     "thread_hung": m1["kgs_sampler_thread_hung"],
                     # the threads that used ≥ 1 % of a core in the window
                     "cpu_by_thread": {k: round((v - w_thr0.get(k, 0.0)) / dt, 4) for k, v in thr1.items()
                                       if v - w_thr0.get(k, 0.0) >= 0.01 * dt}}
                windows.append(w)
                print(json.dumps(w), flush=True)
                w_t0, w_m0, w_cpu0, w_thr0, w_loaded = t1, m1, c1, thr1, 0.0
    finally:
        try:
            proc.stdin.write("quit\n")
            proc.stdin.flush()
            proc.communicate(timeout=30)
        except Exception:  # noqa: BLE001
            proc.kill()
            proc.communicate()
        err.close()
    if not windows:
        fail.append("no window completed")
    for w in windows:
        for k in ("dropped", "pmc_errors", "breaker_trips", "thread_hung"):
            if w[k]:
                fail.append(f"t={w['t']}: {k}={w[k]}")
    # a park per cycle expected (not on --mock: its GPU never goes quiet)
    if a.quiet_release_s and a.idle_s > a.quiet_release_s + 0.5 and not a.mock:
        cycles = a.seconds / (4.0 + a.idle_s)
        parks = sum(w["parks"] for w in windows)
        if parks < 0.5 * cycles:
            fail.append(f"{parks:g} parks in {cycles:.0f} cycles whose idle stretch outlasts the quiet release")
    after = [w["rss_mib"] for w in windows if w["t"] >= 60]
    if after and max(after) - after[0] > 8.0:
        fail.append(f"RSS grew {max(after) - after[0]:.1f} MiB after the first minute")
    # the counter tier is READ every tick while the load runs; quiet stretches READ at 100 Hz
    full = [w for w in windows if w["handovers"] == 0]
    res = {"seconds": a.seconds, "hz": a.hz, "windows": windows, "fail": fail,
           "rss_mib_first_last": [windows[0]["rss_mib"], windows[-1]["rss_mib"]] if windows else None,
           "pmc_samples_per_s_min_max": [min(w["pmc_samples_per_s"] for w in full),
                                         max(w["pmc_samples_per_s"] for w in full)] if full else None,
           "refreshes": sum(w["refreshes"] for w in windows), "handovers": sum(w["handovers"] for w in windows),
           "parks": sum(w["parks"] for w in windows),
           "cpu_cores_mean": round(sum(w["cpu_cores"] for w in windows) / len(windows), 4) if windows else None}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "windows"}))
    return 1 if fail else 0


if __name__ == "__main__":
    sys.exit(main())
