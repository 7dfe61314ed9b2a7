"""GPU probe: what the 1-GPU lease shows of the node's xGMI fabric.

Prints (JSON) the native exporter's link table (amdsmi_get_link_metrics), its
topology JSON, the PMFW xGMI fields of one table, and the amdsmi Python view of
the same device, so the hardware tests can assert on what really exists.

    python tools/probe_xgmi.py > gpurun_out/xgmi_probe.json
"""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kube_gpu_stats_amd import load_native  # noqa: E402


def main() -> None:
    N = load_native()
    ex = N.Exporter({"backend": "amdsmi", "port": -1, "hz": 20, "link_every": 1, "proc_every": 0})
    ex.start()
    time.sleep(1.0)
    out = {"devices": ex.devices(), "links": {}, "snap": {}}
    for d in range(ex.device_count):
        out["links"][d] = ex.links(d)
        s = ex.snapshot(d) or {}
        out["snap"][d] = {k: s.get(k) for k in ("xgmi_read_kb", "xgmi_write_kb", "xgmi_link_up",
                                                "xgmi_link_speed_gbps", "pcie_link_width", "valid")}
    out["topology"] = json.loads(ex.topology_json())
    ex.stop()
    try:
        import amdsmi as A

        A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
        hs = A.amdsmi_get_processor_handles()
        out["amdsmi_n"] = len(hs)
        m = A.amdsmi_get_gpu_metrics_info(hs[0])
        out["amdsmi_metrics_xgmi"] = {k: m.get(k) for k in m if "xgmi" in k}
        try:
            out["amdsmi_link_metrics"] = A.amdsmi_get_link_metrics(hs[0])
        except Exception as e:  # noqa: BLE001
            out["amdsmi_link_metrics_error"] = repr(e)
        try:
            out["amdsmi_topo_numa"] = A.amdsmi_topo_get_numa_node_number(hs[0])
        except Exception as e:  # noqa: BLE001
            out["amdsmi_topo_numa_error"] = repr(e)
        A.amdsmi_shut_down()
    except Exception as e:  # noqa: BLE001
        out["amdsmi_error"] = repr(e)
    print(json.dumps(out, indent=1, default=str))


if __name__ == "__main__":
    main()
