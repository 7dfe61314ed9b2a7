"""GPU diagnostic: raw rocprofiler counter deltas per synthetic-load phase, and
stream-kernel variants (nt vs default loads, grid sizes).  Writes
gpurun_out/pmc_debug.json."""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import json
import os
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from kube_gpu_stats_amd.ops import load  # noqa: E402
from kube_gpu_stats_amd.ops.load import LoadStep  # noqa: E402
from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text  # noqa: E402

out = {}
ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=6 << 30)
ls()
torch.cuda.synchronize()

# stream variants
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
var = {}
for nt in (True, False):
    for blocks in (1024, 2048, 4096, 8192, 16384):
        load.triad_f32(ls.a, ls.b, ls.c, 1.5, nblocks=blocks, nt=nt)
        ev[0].record()
        for _ in range(5):
            load.triad_f32(ls.a, ls.b, ls.c, 1.5, nblocks=blocks, nt=nt)
        ev[1].record()
        torch.cuda.synchronize()
        var[f"nt={int(nt)},blocks={blocks}"] = ls.bytes * 5 / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e12
out["triad_tbps"] = var
print(json.dumps(var), flush=True)

p = torch.cuda.get_device_properties(0)
bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
proc = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
                         "--hz", "100", "--pmc", "rocprofiler", "--control-stdin", "--bdfs", bdf],
                        cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
ready = json.loads(proc.stdout.readline())
out["ready"] = {k: ready.get(k) for k in ("pmc", "pmc_error", "pmc_info")}
print(json.dumps(out["ready"]), flush=True)
sc = Scraper("127.0.0.1", ready["port"])


def totals():
    m = parse_text(sc.get())
    return {lb["counter"]: v for lb, v in m.get("amdgpu_pmc_total", [])}, m


def phase(name, fn, secs=1.5):
    t0c, _ = totals()
    t0 = time.time()
    n = 0
    while time.time() - t0 < secs:
        fn()
        torch.cuda.synchronize()
        n += 1
    t1c, m = totals()
    dt = time.time() - t0
    d = {k: (t1c.get(k, 0) - t0c.get(k, 0)) / dt for k in t1c}
    g = {k: [v for _, v in m.get(k, [])] for k in ("amdgpu_mfma_util_percent", "amdgpu_gpu_active_percent",
                                                   "amdgpu_hbm_read_bytes_per_second",
                                                   "amdgpu_hbm_write_bytes_per_second", "amdgpu_cu_busy_percent")}
    out[name] = {"per_s": d, "gauges": g, "iters": n}
    print(name, json.dumps(out[name]), flush=True)


phase("idle", lambda: time.sleep(0.05))
phase("mfma", ls.run_mfma)
phase("triad_nt", lambda: load.triad_f32(ls.a, ls.b, ls.c, 1.5, nt=True))
phase("triad_plain", lambda: load.triad_f32(ls.a, ls.b, ls.c, 1.5, nt=False))
phase("copy", lambda: load.copy_f32(ls.a, ls.c))
proc.stdin.write("quit\n")
proc.stdin.flush()
proc.wait(timeout=30)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", "pmc_debug.json"), "w") as f:
    json.dump(out, f, indent=1)
