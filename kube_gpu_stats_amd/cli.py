"""``kgs`` command line: exporter | who-use-gpu | gpu-util-stats | dmon | topo | scrape | bench.

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
    from .reports import dmon, gpu_util_stats, who_use_gpu

    exporter_main.build_parser(sub.add_parser("exporter", help="run the node exporter"))
    who_use_gpu.build_parser(sub.add_parser("who-use-gpu", help="per-pod GPU allocation census (F1)"))
    gpu_util_stats.build_parser(sub.add_parser("gpu-util-stats", help="per-pod / per-node utilisation report (F2-F4)"))
    dmon.build_parser(sub.add_parser("dmon", help="live per-GPU rows from one exporter (util, MFMA, HBM, power, xGMI)"))
    tp = sub.add_parser("topo", help="print device inventory + xGMI topology as JSON")
    tp.add_argument("--backend", default="amdsmi")
    tp.add_argument("--mock-gpus", type=int, default=8)
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
    if a.cmd == "dmon":
        return dmon.run(a)
    if a.cmd == "topo":
        from .parallel.topology import discover

        print(json.dumps(discover(a.backend, a.mock_gpus), indent=2))
        return 0
    if a.cmd == "scrape":
        import urllib.request

        body = urllib.request.urlopen(a.url, timeout=10).read().decode()
        for line in body.splitlines():
            if not a.match or a.match in line:
                print(line)
        return 0
    return 1


if __name__ == "__main__":
    sys.exit(main())
