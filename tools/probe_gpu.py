"""Feasibility probe for the MI355X sampler design.

Runs on a gpurun box (non-root). Answers, with measurements, the questions the
100 Hz design depends on:

* device count / ASIC info / BDF / NUMA of every GPU amdsmi can see;
* latency of each amdsmi call the sampler uses;
* how often the PMFW ``firmware_timestamp`` advances (caps honest samples/s);
* whether the per-process list works as a non-root user (with a live HIP
  process on the card);
* raw sysfs ``gpu_metrics`` availability + pread latency;
* xGMI link metrics / topology.

Writes ``gpurun_out/probe.json``.
"""
from __future__ import annotations

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)

import glob
import json
import os
import subprocess
import sys
import time

OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
os.makedirs(OUT, exist_ok=True)
res: dict = {"uid": os.getuid()}


def timed(fn, *a, n=50):
    ts = []
    v = None
    err = None
    for _ in range(n):
        t0 = time.perf_counter()
        try:
            v = fn(*a)
        except Exception as e:  # noqa: BLE001 - probe records everything
            err = repr(e)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return {"p50_us": ts[len(ts) // 2] * 1e6, "min_us": ts[0] * 1e6, "err": err}, v


def jsonable(v):
    try:
        json.dumps(v)
        return v
    except Exception:  # noqa: BLE001
        return repr(v)[:4000]


def main():
    # sysfs survey first (no driver library)
    cards = sorted(glob.glob("/sys/class/drm/card*/device/gpu_metrics"))
    res["sysfs_gpu_metrics"] = cards
    sys_files = {}
    for c in cards[:1]:
        d = os.path.dirname(c)
        sys_files["listing"] = sorted(os.listdir(d))
        for f in ["gpu_busy_percent", "mem_busy_percent", "mem_info_vram_used",
                  "mem_info_vram_total", "unique_id", "current_link_width", "numa_node",
                  "product_name", "xgmi_device_id", "xgmi_hive_id"]:
            p = os.path.join(d, f)
            try:
                with open(p) as fh:
                    sys_files[f] = fh.read().strip()[:200]
            except Exception as e:  # noqa: BLE001
                sys_files[f] = "ERR " + repr(e)
        fd = os.open(c, os.O_RDONLY)
        buf = os.pread(fd, 4096, 0)
        sys_files["gpu_metrics_len"] = len(buf)
        sys_files["gpu_metrics_hdr"] = list(buf[:4])
        sys_files["gpu_metrics_hex"] = buf.hex()
        st, _ = timed(lambda: os.pread(fd, 4096, 0), n=200)
        sys_files["gpu_metrics_pread"] = st
        # how fast does the raw table change? (bytes 16..24 hold system_clock_counter on v1.x)
        seen = set()
        t_end = time.time() + 1.0
        n = 0
        while time.time() < t_end:
            b = os.pread(fd, 4096, 0)
            seen.add(b)
            n += 1
        sys_files["gpu_metrics_distinct_tables_per_s"] = len(seen)
        sys_files["gpu_metrics_reads_per_s"] = n
        os.close(fd)
    res["sysfs"] = sys_files

    import amdsmi as A

    t0 = time.perf_counter()
    A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
    res["init_ms"] = (time.perf_counter() - t0) * 1e3
    hs = A.amdsmi_get_processor_handles()
    res["n_gpus"] = len(hs)
    devs = []
    for i, h in enumerate(hs):
        d = {"index": i}
        for name in ["amdsmi_get_gpu_asic_info", "amdsmi_get_gpu_device_bdf",
                     "amdsmi_get_gpu_device_uuid", "amdsmi_get_gpu_kfd_info",
                     "amdsmi_get_gpu_enumeration_info", "amdsmi_get_gpu_vram_info",
                     "amdsmi_get_gpu_board_info", "amdsmi_get_power_info",
                     "amdsmi_get_gpu_activity", "amdsmi_get_gpu_vram_usage",
                     "amdsmi_get_gpu_process_list", "amdsmi_get_link_metrics",
                     "amdsmi_get_gpu_xgmi_link_status", "amdsmi_get_gpu_metrics_info",
                     "amdsmi_get_gpu_topo_numa_affinity"]:
            fn = getattr(A, name, None)
            if fn is None:
                d[name] = "missing"
                continue
            st, v = timed(fn, h, n=20 if i == 0 else 2)
            d[name] = {"lat": st, "value": jsonable(v)}
        try:
            st, v = timed(A.amdsmi_get_temp_metric, h, A.AmdSmiTemperatureType.HOTSPOT,
                          A.AmdSmiTemperatureMetric.CURRENT, n=20)
            d["temp_hotspot"] = {"lat": st, "value": v}
        except Exception as e:  # noqa: BLE001
            d["temp_hotspot"] = repr(e)
        devs.append(d)
        if i >= 1:
            break
    res["devices"] = devs

    h = hs[0]
    # firmware timestamp cadence
    fw = []
    t_end = time.time() + 2.0
    nloop = 0
    while time.time() < t_end:
        m = A.amdsmi_get_gpu_metrics_info(h)
        fw.append((time.perf_counter(), m.get("firmware_timestamp"), m.get("system_clock_counter")))
        nloop += 1
    distinct = sorted({x[1] for x in fw if isinstance(x[1], int)})
    res["fw_ts"] = {"loops_per_2s": nloop, "distinct_fw_ts": len(distinct),
                    "distinct_sys_clk": len({x[2] for x in fw}),
                    "fw_deltas_10ns": [b - a for a, b in zip(distinct, distinct[1:])][:50]}

    # process list under load: spawn a HIP process
    child = subprocess.Popen([sys.executable, "-c", (
        "import torch,time;x=torch.randn(8192,8192,device='cuda',dtype=torch.bfloat16);"
        "t=time.time()\n"
        "while time.time()-t<12: y=x@x\n"
        "torch.cuda.synchronize()")])
    time.sleep(7)
    try:
        pl = A.amdsmi_get_gpu_process_list(h)
        res["proc_list_under_load"] = jsonable(pl)
    except Exception as e:  # noqa: BLE001
        res["proc_list_under_load"] = "ERR " + repr(e)
    try:
        res["activity_under_load"] = jsonable(A.amdsmi_get_gpu_activity(h))
        m = A.amdsmi_get_gpu_metrics_info(h)
        res["metrics_under_load"] = jsonable(m)
    except Exception as e:  # noqa: BLE001
        res["activity_under_load"] = "ERR " + repr(e)
    child.wait(timeout=60)
    res["child_rc"] = child.returncode

    topo = []
    for a in range(min(len(hs), 8)):
        row = []
        for b in range(min(len(hs), 8)):
            if a == b:
                row.append("self")
                continue
            try:
                row.append(jsonable(A.amdsmi_topo_get_link_type(hs[a], hs[b])))
            except Exception as e:  # noqa: BLE001
                row.append("ERR " + repr(e))
        topo.append(row)
    res["topo"] = topo
    A.amdsmi_shut_down()


if __name__ == "__main__":
    try:
        main()
    finally:
        with open(os.path.join(OUT, "probe.json"), "w") as f:
            json.dump(res, f, indent=1, default=str)
        print(json.dumps({k: (v if k != "devices" else "...") for k, v in res.items()
                          if k not in ("sysfs",)}, default=str)[:3000])
