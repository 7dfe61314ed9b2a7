"""Which kernels does the exporter's GPU-active counter (GRBM_SPI_BUSY) see?  An exporter
in profiling mode (every tick READs) samples this process' MFMA, triad and matmul
kernels — on a queue created before the counting session started — then a child
process' load; prints the per-phase mean GPU-active and MFMA util from /counters.

    python tools/activity_diag.py
"""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import json, os, subprocess, sys, time, urllib.request
sys.path.insert(0, ".")
import torch
from kube_gpu_stats_amd.ops import load
from kube_gpu_stats_amd.ops.load import LoadStep
p = torch.cuda.get_device_properties(0)
bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
torch.ones(1, device="cuda").sum().item()  # this process' queue predates the counting session
exp = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0", "--hz", "4000",
                        "--pmc", "aqlprofile", "--pmc-idle-hz", "0", "--control-stdin", "--bdfs", bdf, "--proc-every", "0",
                        "--link-every", "0"], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
ready = json.loads(exp.stdout.readline())
base = f"http://127.0.0.1:{ready['port']}"
def phase(name, fn, secs=0.5):
    t0 = time.monotonic_ns()
    t = time.time()
    n = 0
    while time.time() - t < secs:
        fn(); n += 1
    t1 = time.monotonic_ns()
    time.sleep(0.02)
    s = json.load(urllib.request.urlopen(base + "/counters?gpu=0&n=4000", timeout=10))["samples"]
    w = [x for x in s if t0 <= x["mono_ns"] <= t1 and "gpu_active_pct" in x]
    res = {"phase": name, "calls": n, "drains": len(w),
           "active_mean": sum(x["gpu_active_pct"] for x in w) / max(1, len(w)),
           "mfma_mean": sum(x["mfma_util_pct"] for x in w) / max(1, len(w)),
           "active_raw_first_last": [w[0]["v"][1], w[-1]["v"][1]] if w else None}
    print(json.dumps(res), flush=True)
ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=1 << 28)
ls.run_mfma(); torch.cuda.synchronize()
phase("loadstep_mfma_sync", lambda: (ls.run_mfma(), torch.cuda.synchronize()))
g = torch.Generator().manual_seed(5)
A = torch.randn(16, 32, generator=g).to(torch.bfloat16).cuda()
B = torch.randn(32, 64, generator=g).to(torch.bfloat16).cuda()
C = torch.empty(2048 * 4 * 16 * 64, device="cuda")
phase("direct_mfma_3400", lambda: (load.mfma_bf16(A, B, C, 2048, 3400), torch.cuda.synchronize()))
phase("direct_mfma_20000", lambda: (load.mfma_bf16(A, B, C, 2048, 20000), torch.cuda.synchronize()))
phase("triad", lambda: (ls.run_stream(), torch.cuda.synchronize()))
x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
phase("torch_matmul", lambda: (x @ x, torch.cuda.synchronize()))
phase("idle", lambda: time.sleep(0.01))
child = r'''
import sys, time, torch
sys.path.insert(0, ".")
from kube_gpu_stats_amd.ops.load import LoadStep
ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=1 << 28)
ls.run_mfma(); torch.cuda.synchronize()
print(time.monotonic_ns(), flush=True)
t = time.time()
while time.time() - t < 0.6:
    ls.run_mfma(); torch.cuda.synchronize()
print(time.monotonic_ns(), flush=True)
'''
out = subprocess.run([sys.executable, "-c", child], capture_output=True, text=True).stdout.split()
t0, t1 = int(out[0]), int(out[1])
time.sleep(0.02)
s = json.load(urllib.request.urlopen(base + "/counters?gpu=0&n=4000", timeout=10))["samples"]
w = [x for x in s if t0 <= x["mono_ns"] <= t1 and "gpu_active_pct" in x]
print(json.dumps({"phase": "child_process_loadstep", "drains": len(w),
                  "active_mean": sum(x["gpu_active_pct"] for x in w) / max(1, len(w)),
                         "mfma_mean": sum(x["mfma_util_pct"] for x in w) / max(1, len(w))}), flush=True)
exp.stdin.write("quit\n"); exp.stdin.flush(); exp.communicate(timeout=30)
