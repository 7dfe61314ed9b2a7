"""Mock-provider scaling of the native exporter on CPU (BASELINE.json config 1 and
the 2/4/8-GPU fan-out rehearsal of SURVEY.md §4.3).  NOT hardware numbers.

For N mock GPUs × tick rate: achieved samples/s/GPU (counter tier, worst GPU),
sampler overruns per GPU per second, p50/p99 /metrics latency over keep-alive
HTTP, body size, and exporter CPU cost (process CPU seconds per wall second).
Rows with the latency model use AMD SMI call latencies measured on MI355X
(exporter/main.py MOCK_LATENCY, profiles/r2/amdsmi_latency.md) under one
process-wide lock — the
per-process tier at 10 Hz and the link tier at 1 Hz run on the node-wide slow
thread, never on the per-GPU threads (profiles/r2/mock_scaling.md).
    python tools/mock_scaling.py [--latency] [--out profiles/r2/mock_scaling.md]
"""
import argparse
import json
import os
import resource
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kube_gpu_stats_amd import load_native  # noqa: E402
from kube_gpu_stats_amd.utils.scrape import Scraper  # noqa: E402


def cpu_s() -> float:
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


from kube_gpu_stats_amd.exporter.main import MOCK_LATENCY as LATENCY  # noqa: E402  (MI355X-measured)


def one(N, n_gpus: int, hz: float, latency: bool, secs: float = 2.0, scrapes: int = 200) -> dict:
    mock = {"n_gpus": n_gpus, **(LATENCY if latency else {})}
    ex = N.Exporter({"backend": "mock", "mock": mock, "hz": hz, "port": 0, "pmc_source": "mock",
                     "node_name": "mock-node", "pin_numa": False, "proc_period_s": 0.1, "link_period_s": 1.0})
    ex.start()
    time.sleep(0.3)
    c0, w0 = cpu_s(), time.time()
    i0 = [ex.integrals(g) for g in range(n_gpus)]
    time.sleep(secs)
    c1, w1 = cpu_s(), time.time()
    i1 = [ex.integrals(g) for g in range(n_gpus)]
    sc = Scraper("127.0.0.1", ex.port)
    for _ in range(scrapes):
        sc.scrape_once()
    ex.stop()
    dt = w1 - w0
    rates = [(b["pmc_samples"] - a["pmc_samples"]) / dt for a, b in zip(i0, i1)]
    over = [(b["overruns"] - a["overruns"]) / dt for a, b in zip(i0, i1)]
    procs = sum(b["proc_reads"] - a["proc_reads"] for a, b in zip(i0, i1)) / dt / n_gpus
    return {"n_gpus": n_gpus, "hz": hz, "latency_model": latency,
            "samples_per_s_per_gpu": round(sum(rates) / n_gpus, 1), "worst_gpu_pct_of_nominal": round(100 * min(rates) / hz, 2),
            "overruns_per_s_per_gpu": round(sum(over) / n_gpus, 1), "proc_reads_per_s_per_gpu": round(procs, 1),
            "p50_scrape_ms": round(sc.percentile(0.5) * 1e3, 3), "p99_scrape_ms": round(sc.percentile(0.99) * 1e3, 3),
            "body_kb": round(sc.bytes / scrapes / 1024, 1), "exporter_cpu_cores": round((c1 - c0) / dt, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--rates", default="100,1000,8000")
    ap.add_argument("--gpus", default="1,2,4,8")
    a = ap.parse_args()
    N = load_native()
    rows = [one(N, n, float(hz), lat) for lat in (False, True) for hz in a.rates.split(",")
            for n in (int(x) for x in a.gpus.split(","))]
    for r in rows:
        print(json.dumps(r), flush=True)
    if a.out:
        lines = ["# Mock-provider scaling on CPU (not hardware numbers)", "",
                 f"`tools/mock_scaling.py` in the build container ({os.cpu_count()} CPUs): native exporter, mock "
                 "N-GPU provider + mock counter source, one sampler thread per GPU plus the node-wide slow thread "
                 "(per-process tier 10 Hz, link + RAS tier 1 Hz), 200 keep-alive scrapes of /metrics per row.  "
                 "`latency` rows model AMD SMI with the call latencies measured on MI355X "
                 "(`profiles/r2/amdsmi_latency.md`: process list 0.5 ms, link table 1 ms, RAS 0.75 ms under ONE "
                 "process-wide lock, PMFW table read 0.125 ms unlocked).", "",
                 "| GPUs | tick Hz | AMD SMI latency model | samples/s/GPU | worst GPU % of nominal | overruns/s/GPU | "
                 "proc-list reads/s/GPU | p50 scrape ms | p99 scrape ms | /metrics KiB | exporter CPU cores |",
                 "|---|---|---|---|---|---|---|---|---|---|---|"]
        for r in rows:
            lines.append(f"| {r['n_gpus']} | {r['hz']:g} | {'on' if r['latency_model'] else 'off'} | "
                         f"{r['samples_per_s_per_gpu']} | {r['worst_gpu_pct_of_nominal']} | {r['overruns_per_s_per_gpu']} | "
                         f"{r['proc_reads_per_s_per_gpu']} | {r['p50_scrape_ms']} | {r['p99_scrape_ms']} | "
                         f"{r['body_kb']} | {r['exporter_cpu_cores']} |")
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
