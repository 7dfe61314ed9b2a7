"""Workload for a rocprofv3 --pmc profile of the hand-written gfx950 load kernels.

Runs each kernel a few times with known work: the MFMA loop (exact FLOPs), the HBM
triad (exact bytes: two 4-byte reads and one write per element) and the 64 KiB copy
of the dispatch-bound graph.  tools/gpu_run48.sh profiles it in separate counter
passes and tools/pmc_kernels_report.py compares the counters with the known work.
"""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import json
import sys
import time

sys.path.insert(0, ".")

import torch  # noqa: E402

from kube_gpu_stats_amd.ops import load  # noqa: E402
from kube_gpu_stats_amd.ops.load import LoadStep  # noqa: E402

ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=3 << 30)
src = torch.rand(16384, device="cuda")
dst = torch.empty_like(src)
torch.cuda.synchronize()
for _ in range(3):
    ls.run_mfma()
for _ in range(3):
    ls.run_stream()
for _ in range(3):
    load.copy_f32(src, dst, nblocks=64)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
e[0].record()
ls.run_mfma()
e[1].record()
ls.run_stream()
e[2].record()
torch.cuda.synchronize()
print(json.dumps({"mfma_flops": ls.flops, "mfma_ms": e[0].elapsed_time(e[1]), "triad_bytes": ls.bytes,
                  "triad_ms": e[1].elapsed_time(e[2]), "copy_bytes": 2 * src.numel() * 4,
                  "time": time.time()}))
