"""GPU probe: per-call latency of the management-library reads the exporter's
node-wide slow thread makes (process list, link metrics, ECC, xGMI status) and
of the PMFW table pread of the fast tier, so the mock's latency model
(exporter/main.py MOCK_LATENCY) is grounded in MI355X numbers.

    python tools/probe_amdsmi_latency.py > gpurun_out/r2/amdsmi_latency.json
"""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=200):
    xs = []
    for _ in range(n):
        t0 = time.perf_counter()
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - e.g. AMDSMI_STATUS_INVAL: not supported on this part
            return {"error": repr(e)[:200]}
        xs.append((time.perf_counter() - t0) * 1e6)
    xs.sort()
    return {"n": n, "p50_us": round(xs[n // 2], 1), "p99_us": round(xs[int(n * 0.99)], 1),
            "mean_us": round(statistics.mean(xs), 1)}


def main() -> None:
    import amdsmi as A

    from kube_gpu_stats_amd import load_native

    A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
    h = A.amdsmi_get_processor_handles()[0]
    out = {"python_binding": {
        "process_list": timeit(lambda: A.amdsmi_get_gpu_process_list(h)),
        "link_metrics": timeit(lambda: A.amdsmi_get_link_metrics(h)),
        "total_ecc_count": timeit(lambda: A.amdsmi_get_gpu_total_ecc_count(h)),
        "xgmi_error_status": timeit(lambda: A.amdsmi_gpu_xgmi_error_status(h)),
        "gpu_metrics_info": timeit(lambda: A.amdsmi_get_gpu_metrics_info(h)),
    }}
    A.amdsmi_shut_down()
    # Native path (what the exporter really pays): slow-thread seconds per read.
    N = load_native()
    ex = N.Exporter({"backend": "amdsmi", "port": -1, "hz": 100, "proc_period_s": 0.05, "link_period_s": 0.05})
    ex.start()
    time.sleep(3.0)
    ex.stop()
    i = ex.integrals(0)
    reads = i["proc_reads"] + i["link_reads"]
    out["native"] = {"proc_reads": i["proc_reads"], "link_reads": i["link_reads"],
                     "slow_read_seconds": i["slow_read_seconds"],
                     "mean_us_per_slow_read": round(1e6 * i["slow_read_seconds"] / max(1, reads), 1),
                     "pmfw_read_us_mean": round(1e6 * i["read_seconds"] / max(1, i["reads"]), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
