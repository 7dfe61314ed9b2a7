"""GPU probe: how much resident host memory the HSA runtime takes at hsa_init, and
which runtime switch changes it (the exporter's counter reader initialises HSA; with
it the exporter's RSS goes from 36 to 391 MiB, 360 MiB of it anonymous — r3s).

Each variant runs in a fresh child: load libhsa-runtime64, hsa_init(), then read
VmRSS / RssAnon.

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


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        return 0
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/hsa_rss.json")
    a = ap.parse_args()
    res = {}
    for name, env in VARIANTS.items():
        e = dict(os.environ)
        e.update(env)
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=e, capture_output=True, text=True,
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
