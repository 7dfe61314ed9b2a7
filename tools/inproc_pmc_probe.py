"""Probe: the aqlprofile counter reader inside a process that already runs HIP
(torch) — what smoke() needs to exercise the counter tier in-process."""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kube_gpu_stats_amd import load_native  # noqa: E402
from kube_gpu_stats_amd.native import pmc_lib_path  # noqa: E402
from kube_gpu_stats_amd.ops import load  # noqa: E402

N = load_native()
dev = torch.device("cuda", 0)
A = torch.randn(16, 32).to(torch.bfloat16).to(dev)
B = torch.randn(32, 64).to(torch.bfloat16).to(dev)
C = torch.empty(2048 * 4 * 16 * 64, device=dev)
load.mfma_bf16(A, B, C, 2048, 2000)
torch.cuda.synchronize()
ex = N.Exporter({"backend": "amdsmi", "hz": 1000, "port": -1, "pmc_source": "aqlprofile",
                 "pmc_lib": pmc_lib_path("aqlprofile"), "proc_period_s": 0, "link_period_s": 0})
ex.start()
print(json.dumps({"pmc_error": ex.pmc_error}), flush=True)
t0 = time.time()
while time.time() - t0 < 1.5:
    load.mfma_bf16(A, B, C, 2048, 20000)
    torch.cuda.synchronize()
w = ex.window(0, 1.0)
i = ex.integrals(0)
ex.stop()
print(json.dumps({"window": w, "pmc_samples": i.get("pmc_samples"), "pmc_errors": i.get("pmc_errors")}), flush=True)
