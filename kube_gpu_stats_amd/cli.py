"""``kgs`` command line: exporter | who-use-gpu | gpu-util-stats | ps | dmon | record | topo | pmc | scrape | bench.

The reference ships two scripts with no arguments (who_use_gpu.py:61-62,
gpu_util_stats.py:165-166).  They become subcommands here, every hard-coded
constant a flag (utils/config.py), with ``--compat`` reproducing the reference
output byte-for-byte where SURVEY.md §2.8 pins it.
"""
from __future__ import annotations

import argparse
import json
import sys


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="kgs", description=__doc__.splitlines()[0])
    sub = ap.add_subparsers(dest="cmd", required=True)

    from .exporter import main as exporter_main
    from .reports import dmon, gpu_util_stats, ps, record, who_use_gpu

    exporter_main.build_parser(sub.add_parser("exporter", help="run the node exporter"))
    who_use_gpu.build_parser(sub.add_parser("who-use-gpu", help="per-pod GPU allocation census (F1)"))
    gpu_util_stats.build_parser(sub.add_parser("gpu-util-stats", help="per-pod / per-node utilisation report (F2-F4)"))
    ps.build_parser(sub.add_parser("ps", help="processes using a node's GPUs now: pod, HBM, compute share (from one "
                                              "exporter)"))
    dmon.build_parser(sub.add_parser("dmon", help="live per-GPU rows from one exporter (util, MFMA, HBM, power, xGMI)"))
    record.build_parser(sub.add_parser("record", help="capture an exporter's full-rate counter stream as a Chrome / "
                                                      "Perfetto trace (GPU-active, MFMA, clock, busy segments)"))
    tp = sub.add_parser("topo", help="print device inventory + xGMI topology as JSON")
    tp.add_argument("--backend", default="amdsmi")
    tp.add_argument("--mock-gpus", type=int, default=8)
    tp.add_argument("--format", default="json", choices=["json", "prom"],
                    help="json inventory, or amdgpu_xgmi_neighbor{bdf,peer_bdf} lines (node topology export)")
    tp.add_argument("--node-name", default="")
    pm = sub.add_parser("pmc", help="hand the hardware counters of a running exporter to another profiler (release) "
                                    "or back (acquire); run inside the exporter pod: kubectl exec <pod> -- kgs pmc release")
    pm.add_argument("action", choices=["release", "acquire", "status"])
    pm.add_argument("--exporter", default="127.0.0.1:9400", help="host:port of the exporter (loopback only)")
    pm.add_argument("--pid-file", default="", help="signal the PID in this file instead of using HTTP")
    pm.add_argument("--gpu", type=int, default=-1, help="this GPU only (exporter index; default every GPU). Each "
                    "GPU's own sampler thread acts, so a hung GPU never delays the others")
    sub.add_parser("bench", help="run the headline benchmark (bench.py; flags pass through)", add_help=False)
    sp = sub.add_parser("scrape", help="scrape an exporter once and print selected families")
    sp.add_argument("url", nargs="?", default="http://127.0.0.1:9400/metrics")
    sp.add_argument("--match", default="")

    if argv and argv[0] == "bench":
        import os
        import runpy

        bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
        sys.argv = [bench] + argv[1:]
        runpy.run_path(bench, run_name="__main__")
        return 0
    a = ap.parse_args(argv)
    if a.cmd == "exporter":
        return exporter_main.run(a)
    if a.cmd == "who-use-gpu":
        return who_use_gpu.run(a)
    if a.cmd == "gpu-util-stats":
        return gpu_util_stats.run(a)
    if a.cmd == "ps":
        return ps.run(a)
    if a.cmd == "dmon":
        return dmon.run(a)
    if a.cmd == "record":
        return record.run(a)
    if a.cmd == "topo":
        from .parallel.topology import discover, prometheus_lines

        topo = discover(a.backend, a.mock_gpus)
        if a.format == "prom":
            print("# HELP amdgpu_xgmi_neighbor Direct xGMI link between two GPUs of this node (1)")
            print("# TYPE amdgpu_xgmi_neighbor gauge")
            print("\n".join(prometheus_lines(topo, a.node_name or topo.get("node", ""))))
        else:
            print(json.dumps(topo, indent=2))
        return 0
    if a.cmd == "pmc":
        return pmc_control(a)
    if a.cmd == "scrape":
        import urllib.request

        body = urllib.request.urlopen(a.url, timeout=10).read().decode()
        for line in body.splitlines():
            if not a.match or a.match in line:
                print(line)
        return 0
    return 1


def pmc_control(a) -> int:
    """Counter hand-over from inside the exporter's pod.  The DaemonSet runs with
    hostPID, so PID 1 there is the host's init — never signal it; use the exporter's
    loopback-only /control/pmc/* endpoints, or the PID it wrote to --pid-file."""
    if a.pid_file:
        import os
        import signal

        if a.gpu >= 0:
            raise SystemExit("--gpu needs the HTTP control endpoint (drop --pid-file)")
        with open(a.pid_file) as f:
            pid = int(f.read().strip())
        if a.action != "status":
            os.kill(pid, signal.SIGUSR1 if a.action == "release" else signal.SIGUSR2)
        print(json.dumps({"pid": pid, "action": a.action}))
        return 0
    import urllib.request

    path = {"release": "/control/pmc/release", "acquire": "/control/pmc/acquire"}.get(a.action)
    if path:
        q = f"?gpu={a.gpu}" if a.gpu >= 0 else ""
        print(urllib.request.urlopen(f"http://{a.exporter}{path}{q}", timeout=10).read().decode())
        return 0
    body = urllib.request.urlopen(f"http://{a.exporter}/metrics", timeout=10).read().decode()
    print("\n".join(ln for ln in body.splitlines()
                    if ln.startswith(("kgs_pmc_enabled", "kgs_pmc_stalled", "kgs_pmc_failed", "kgs_pmc_quiet ",
                                       "kgs_pmc_quiet{", "kgs_pmc_dispatch_bound", "kgs_pmc_parked", "kgs_sampler_thread_hung",
                                       "kgs_pmc_publishes_total", "kgs_pmc_unlanded_total"))
                    and (a.gpu < 0 or f'gpu="{a.gpu}"' in ln)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
