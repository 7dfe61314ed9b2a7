"""GPU probe: how PMFW UMC (memory-controller) activity relates to measured HBM
bandwidth.  The exporter (amdsmi backend, in process, no counters) integrates
UMC activity exactly from the PMFW accumulators; this runs stream kernels at
several bandwidths (grid size varies the achieved TB/s) and compares the
exporter's UMC % over each phase with the bytes the kernels moved.
Writes gpurun_out/umc_calib.json."""
from __future__ import annotations

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)

import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    import torch

    from kube_gpu_stats_amd import load_native
    from kube_gpu_stats_amd.ops import load
    from kube_gpu_stats_amd.ops.load import LoadStep

    N = load_native()
    ex = N.Exporter({"backend": "amdsmi", "hz": 100, "port": -1, "proc_every": 0, "link_every": 0})
    ex.start()
    ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=6 << 30)
    ls()
    torch.cuda.synchronize()
    n = ls.a.numel()

    def phase(name, fn, bytes_per_call, secs=2.0):
        time.sleep(0.1)
        i0 = ex.integrals(0)
        t0 = time.time()
        k = 0
        while time.time() - t0 < secs:
            fn()
            torch.cuda.synchronize()
            k += 1
        wall = time.time() - t0
        time.sleep(0.05)
        i1 = ex.integrals(0)
        ds = i1["sampled_seconds"] - i0["sampled_seconds"]
        row = {"phase": name, "calls": k, "wall_s": wall, "bytes_per_s": bytes_per_call * k / wall,
               "umc_pct": 100 * (i1["umc_busy_seconds"] - i0["umc_busy_seconds"]) / ds if ds > 0 else None,
               "gfx_pct": 100 * (i1["gfx_busy_seconds"] - i0["gfx_busy_seconds"]) / ds if ds > 0 else None}
        print(json.dumps(row), flush=True)
        return row

    rows = [phase("idle", lambda: time.sleep(0.05), 0)]
    for blocks in (64, 256, 1024, 8192):
        rows.append(phase(f"triad_b{blocks}", lambda b=blocks: load.triad_f32(ls.a, ls.b, ls.c, 1.5, nblocks=b),
                          12.0 * n))
    for blocks in (256, 8192):
        rows.append(phase(f"copy_b{blocks}", lambda b=blocks: load.copy_f32(ls.b, ls.a, nblocks=b), 8.0 * n))
    rows.append(phase("read_only_sum", lambda: ls.b.sum(), 4.0 * n))
    rows.append(phase("mfma", ls.run_mfma, 0))
    ex.stop()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "umc_calib.json"), "w") as f:
        json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
