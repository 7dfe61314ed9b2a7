"""Mock-provider scaling of the native exporter on CPU (BASELINE.json config 1 and
the 2/4/8-GPU fan-out rehearsal of SURVEY.md §4.3).  NOT hardware numbers.

For N mock GPUs × tick rate: achieved samples/s/GPU (counter tier), p50/p99
/metrics latency over keep-alive HTTP, body size, and exporter CPU cost
(process CPU seconds per wall second while sampling).
    python tools/mock_scaling.py [--out profiles/r1/mock_scaling.md]
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


def one(N, n_gpus: int, hz: float, secs: float = 2.0, scrapes: int = 200) -> dict:
    ex = N.Exporter({"backend": "mock", "mock": {"n_gpus": n_gpus}, "hz": hz, "port": 0, "pmc_source": "mock",
                     "node_name": "mock-node", "pin_numa": False, "proc_every": max(1, int(hz // 10)),
                     "link_every": max(1, int(hz))})
    ex.start()
    time.sleep(0.3)
    c0, w0 = cpu_s(), time.time()
    i0 = [ex.integrals(g)["pmc_samples"] for g in range(n_gpus)]
    time.sleep(secs)
    c1, w1 = cpu_s(), time.time()
    i1 = [ex.integrals(g)["pmc_samples"] for g in range(n_gpus)]
    sc = Scraper("127.0.0.1", ex.port)
    for _ in range(scrapes):
        sc.scrape_once()
    ex.stop()
    rate = sum(b - a for a, b in zip(i0, i1)) / (w1 - w0) / n_gpus
    return {"n_gpus": n_gpus, "hz": hz, "samples_per_s_per_gpu": round(rate, 1),
            "p50_scrape_ms": round(sc.percentile(0.5) * 1e3, 3), "p99_scrape_ms": round(sc.percentile(0.99) * 1e3, 3),
            "body_kb": round(sc.bytes / scrapes / 1024, 1), "exporter_cpu_cores": round((c1 - c0) / (w1 - w0), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    N = load_native()
    rows = [one(N, n, hz) for hz in (1, 100, 1000) for n in (1, 2, 4, 8)]
    for r in rows:
        print(json.dumps(r))
    if a.out:
        lines = ["# Mock-provider scaling on CPU (not hardware numbers)", "",
                 "`tools/mock_scaling.py` in the build container (8 CPUs): native exporter, mock N-GPU provider + mock "
                 "counter source, one sampler thread per GPU, 200 keep-alive scrapes of /metrics per row.", "",
                 "| GPUs | tick Hz | samples/s/GPU | p50 scrape ms | p99 scrape ms | /metrics KiB | exporter CPU cores |",
                 "|---|---|---|---|---|---|---|"]
        for r in rows:
            lines.append(f"| {r['n_gpus']} | {r['hz']:g} | {r['samples_per_s_per_gpu']} | {r['p50_scrape_ms']} | "
                         f"{r['p99_scrape_ms']} | {r['body_kb']} | {r['exporter_cpu_cores']} |")
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
