"""GPU probe: how much resident host memory the HSA runtime takes at hsa_init, and
which runtime switch changes it (the exporter's counter reader initialises HSA; with
it the exporter's RSS goes from 36 to 391 MiB, 360 MiB of it anonymous — r3s).

Each variant runs in a fresh child: load libhsa-runtime64, hsa_init(), then read
VmRSS / RssAnon; the reader variants step through the exporter's counter reader
(init, open + START on GPU 0, 400 pipelined samples) with the READ queue created
without / with ROCr's default scratch and LDS segment sizes.

    python tools/hsa_rss_probe.py --out gpurun_out/hsa_rss.json
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

VARIANTS = {
    "default": {},
    "no_fragment_allocator": {"HSA_DISABLE_FRAGMENT_ALLOCATOR": "1"},
    "no_sdma": {"HSA_ENABLE_SDMA": "0"},
    "no_interrupt": {"HSA_ENABLE_INTERRUPT": "0"},
    "no_scratch_reclaim": {"HSA_ENABLE_SCRATCH_ASYNC_RECLAIM": "0"},
}


def status() -> dict:
    out = {}
    with open("/proc/self/status") as f:
        for ln in f:
            k = ln.split(":")[0]
            if k in ("VmRSS", "RssAnon", "RssFile", "VmSize"):
                out[k] = round(int(ln.split()[1]) / 1024, 1)
    return out


def child() -> None:
    r = {"before": status()}
    hsa = ctypes.CDLL("/opt/rocm/lib/libhsa-runtime64.so.1", mode=ctypes.RTLD_GLOBAL)
    rc = hsa.hsa_init()
    r["hsa_init_rc"] = rc
    r["after_init"] = status()
    print(json.dumps(r))


def reader_child() -> None:
    """The exporter's counter reader step by step (libkgs_pmc_aql.so, in-tree)."""
    import glob
    import time

    r = {"before": status()}
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kube_gpu_stats_amd",
                                   "lib", "libkgs_pmc_aql.so"))
    err = ctypes.create_string_buffer(512)
    r["init_rc"] = lib.kgs_pmc_init(err, 512)
    r["after_init"] = status()
    gpu_id = 0
    for f in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")):
        try:
            v = int(open(f).read().strip() or 0)
        except OSError:
            continue
        if v:
            gpu_id = v
            break
    names = (ctypes.c_char_p * 3)(b"GRBM_COUNT", b"GRBM_SPI_BUSY", b"SQ_VALU_MFMA_BUSY_CYCLES")
    is_max = (ctypes.c_int * 3)(1, 1, 0)
    h = lib.kgs_pmc_open(ctypes.c_uint64(gpu_id), names, is_max, 3, err, 512)
    r["open_handle"], r["open_err"] = h, err.value.decode(errors="replace")
    r["after_open"] = status()
    if h >= 0:
        lib.kgs_pmc_set_pipelined(h, 1, err, 512)
        out = (ctypes.c_uint64 * 3)()
        rns = ctypes.c_uint32()
        for _ in range(400):
            lib.kgs_pmc_sample(h, out, 3, ctypes.byref(rns))
            time.sleep(0.000125)
        r["after_400_samples"] = status()
        lib.kgs_pmc_close(h)
    print(json.dumps(r))


def queue_child() -> None:
    """RSS after creating one, then a second, AQL queue on the GPU agent (is the
    per-queue context save/restore area the reader's cost, and per queue?)."""
    r = {"before": status()}
    hsa = ctypes.CDLL("/opt/rocm/lib/libhsa-runtime64.so.1", mode=ctypes.RTLD_GLOBAL)
    r["hsa_init_rc"] = hsa.hsa_init()
    r["after_init"] = status()
    agents = []
    CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)

    def on_agent(handle, _data):
        dev = ctypes.c_uint32()
        hsa.hsa_agent_get_info(ctypes.c_uint64(handle), 17, ctypes.byref(dev))  # HSA_AGENT_INFO_DEVICE
        if dev.value == 1:  # HSA_DEVICE_TYPE_GPU
            agents.append(handle)
        return 0

    cb = CB(on_agent)
    hsa.hsa_iterate_agents(cb, None)
    r["gpu_agents"] = len(agents)
    qs = []
    for i in range(2):
        q = ctypes.c_void_p()
        rc = hsa.hsa_queue_create(ctypes.c_uint64(agents[0]), ctypes.c_uint32(64), ctypes.c_uint32(1), None, None,
                                  ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.byref(q))
        r[f"queue{i + 1}_rc"] = rc
        r[f"after_queue{i + 1}"] = status()
        qs.append(q)
    for q in qs:
        if q.value:
            hsa.hsa_queue_destroy(q)
    r["after_destroy"] = status()
    print(json.dumps(r))


QUEUE_VARIANTS = {
    "default": {},
    "queue_dev_mem": {"HSA_ALLOCATE_QUEUE_DEV_MEM": "1"},
    "no_pc_sampling": {"HSA_DISABLE_PC_SAMPLING": "1"},
    "no_coredump": {"HSA_DISABLE_COREDUMP_ON_EXCEPTION": "1"},
}

READER_VARIANTS = {
    "reader_queue_segments_0": {},
    "reader_queue_segments_max": {"KGS_AQL_QUEUE_SEGMENTS": "max"},
}


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "--queue-child":
        queue_child()
        return 0
    if len(sys.argv) > 1 and sys.argv[1] == "--reader-child":
        reader_child()
        return 0
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/hsa_rss.json")
    a = ap.parse_args()
    res = {}
    runs = [(n, v, "--child") for n, v in VARIANTS.items()] + [(n, v, "--reader-child") for n, v in READER_VARIANTS.items()]
    runs += [(f"two_queues_{n}", v, "--queue-child") for n, v in QUEUE_VARIANTS.items()]
    for name, env, mode in runs:
        e = dict(os.environ)
        e.update(env)
        p = subprocess.run([sys.executable, os.path.abspath(__file__), mode], env=e, capture_output=True, text=True,
                           timeout=120)
        try:
            res[name] = {"env": env, **json.loads(p.stdout.strip().splitlines()[-1])}
        except (ValueError, IndexError):
            res[name] = {"env": env, "error": (p.stderr or p.stdout)[-400:]}
        print(name, json.dumps(res[name]), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
