"""Command line and rank launch: ``python bench.py --gpus N --steps K --warmup W``."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

from kube_gpu_stats_amd.parallel import dist as D

from .common import PMC_READER, REPO, free_port
from .phase_x import xgmi_child
from .run import run
from .summary import compact


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--hz", type=float, default=8000.0,
                    help="primary sampler tick rate per GPU (phase B): one hardware-counter drain per tick "
                    "(PMFW table ≤ 100 Hz); 8 kHz costs ≈0.05 exporter cores/GPU; 16 kHz (with --pmc-batch 16) "
                    "≈0.07 and +0.1 %% GPU time vs paused, +0.01 %% vs released (profiles/r5/r5o)")
    ap.add_argument("--hz-list", default="100",
                    help="further tick rates measured in the interleaved rounds (BASELINE config 4 = 100 Hz); "
                    "'' = primary only")
    ap.add_argument("--pmc", default="auto", choices=["auto", "aqlprofile", "none"],
                    help="counter reader (auto = %s)" % PMC_READER)
    ap.add_argument("--pmc-pipeline", type=int, default=1, choices=[0, 1],
                    help="aqlprofile reader: pipelined READs (1) or submit-and-wait per sample (0)")
    ap.add_argument("--pmc-set", default="base", choices=["base", "full"],
                    help="counter set: base (GRBM clocks + SPI busy + MFMA busy) or full (+ TA busy, 10x the CP register "
                    "reads)")
    ap.add_argument("--pmc-dispatch-hz", type=float, default=1000.0,
                    help="exporter --pmc-dispatch-hz: READ rate while the CP dispatches with no wave in flight")
    ap.add_argument("--pmc-batch", type=int, default=8,
                    help="exporter --pmc-batch: counter READs per L2 writeback (8 at 8 kHz: one per ms)")
    ap.add_argument("--pmc-publish-us", type=int, default=1000, help="exporter --pmc-publish-us")
    ap.add_argument("--pmc-lean", type=int, default=2, choices=[0, 1, 2, 3],
                    help="aqlprofile READ packet mode (exporter --pmc-lean; 0 = as aqlprofile builds it)")
    ap.add_argument("--scrape-hz", type=float, default=20.0)
    ap.add_argument("--step-ms", type=float, default=500.0,
                    help="each step repeats the load unit until it lasts at least this long")
    ap.add_argument("--rounds", type=int, default=48,
                    help="interleaved rounds (0 = off); 48 x 3 blocks of ~1 s put the 95 %% CI of the "
                         "overhead under 0.1 %% on a power-capped MI355X (per-round sd 0.18-0.28 %%: r2ag, r2aj)")
    ap.add_argument("--block-steps", type=int, default=2, help="steps per interleaved block")
    ap.add_argument("--mfma-iters", type=int, default=150000, help="≈40 ms of MFMA work per unit on MI355X")
    ap.add_argument("--mfma-blocks", type=int, default=2048)
    ap.add_argument("--stream-gib", type=float, default=6.0)
    ap.add_argument("--triads", type=int, default=2)
    ap.add_argument("--tiny-kernels", type=int, default=2000,
                    help="dispatch-bound part of each unit: a HIP graph of this many 64 KiB copies (≈1.7 µs each); "
                    "it is where counter READs on the command processor would show up (0 = off)")
    ap.add_argument("--load", default="synthetic", choices=["synthetic", "train"],
                    help="GPU work per unit: the synthetic gfx950 kernels (default) or a PyTorch bf16 "
                    "decoder training step (forward + backward + AdamW, DDP when N > 1)")
    ap.add_argument("--train-dim", type=int, default=4096)
    ap.add_argument("--train-layers", type=int, default=4)
    ap.add_argument("--train-batch", type=int, default=4)
    ap.add_argument("--train-seq", type=int, default=2048)
    ap.add_argument("--train-vocab", type=int, default=32768)
    ap.add_argument("--xgmi-mib", type=int, default=256, help="RCCL all-reduce size per unit when N > 1 (0 = off)")
    ap.add_argument("--xgmi-check-mib", type=int, default=2048,
                    help="phase X (N > 1): bytes of each GPU 0 → GPU k peer copy that checks the link map and unit")
    ap.add_argument("--xgmi-check-settle", type=float, default=0.5,
                    help="phase X: seconds between a round of peer copies and the scrape that reads its link counters")
    ap.add_argument("--xgmi-check-budget-s", type=float, default=120.0,
                    help="phase X: start no further round of peer copies after this many seconds")
    ap.add_argument("--mock-xgmi-swap", type=int, default=-1,
                    help="mock: GPU whose link table reports two ports' peers swapped (phase X must flag it)")
    ap.add_argument("--xgmi-child", type=int, default=0, help=argparse.SUPPRESS)  # phase X child: exporter port
    ap.add_argument("--xgmi-bdfs", default="", help=argparse.SUPPRESS)
    ap.add_argument("--settle", type=float, default=1.0, help="seconds between exporter start and phase B")
    ap.add_argument("--burst-s", type=float, default=0.6,
                    help="phase R: length of the MFMA burst train read back from /counters (0 = off; cut to "
                    "what the full-rate ring holds: ≈1 s at 8 kHz, 0.5 s at 16 kHz)")
    ap.add_argument("--burst-ms", type=float, default=1.0, help="phase R: length of one burst")
    ap.add_argument("--burst-period-ms", type=float, default=5.0, help="phase R: burst period")
    ap.add_argument("--capacity-hz", default="16000,24000,32000",
                    help="phase S: tick rates above --hz to try under the load, one block each ('' = off)")
    ap.add_argument("--quiet-s", type=float, default=1.5,
                    help="phase Q: seconds of idle GPU per exporter mode (adaptive / profiling; 0 = off)")
    ap.add_argument("--idle-power-s", type=float, default=36.0,
                    help="phase P: seconds per condition (session programmed / released / parked by the quiet "
                    "release) of an idle GPU, in --idle-power-rounds rounds of every order (0 = off)")
    ap.add_argument("--idle-power-rounds", type=int, default=6)
    ap.add_argument("--idle-power-absent", type=int, default=0, choices=[0, 1],
                    help="phase P: a fourth condition, 'absent' — session released and every sampling tier "
                    "paused, so nothing of the exporter touches the GPU")
    ap.add_argument("--idle-power-settle-s", type=float, default=6.0,
                    help="phase P: wait after each switch before measuring — an idle MI355X drops to its "
                    "low-power state ≈5 s after its last GPU work (r6h)")
    ap.add_argument("--component-s", type=float, default=1.0,
                    help="phase K: seconds each load component runs alone while the exporter samples (0 = off)")
    ap.add_argument("--released", type=int, default=1, choices=[0, 1],
                    help="phase I: a fourth interleaved condition, 'released' — counter session STOPped and the "
                    "reader's READ queue destroyed for the block (1 = on)")
    ap.add_argument("--util-s", type=float, default=1.5,
                    help="phase U: seconds of each load (idle, two MFMA burst trains, saturating MFMA) while the "
                    "exported container_gpu_sm_util / busy counter is checked against the host-known duty (0 = off)")
    ap.add_argument("--util-irregular", type=int, default=1, choices=[0, 1],
                    help="phase U: also the out-of-sample loads — seeded random 5 µs-20 ms kernels and gaps on one and "
                    "on two streams, and a bf16 training step (VERDICT r5 #3)")
    ap.add_argument("--util-seed", type=int, default=6, help="phase U: seed of the random kernel schedules")
    ap.add_argument("--util-hz", default="1000,10",
                    help="phase U: tick rates besides the primary --hz ('' = primary only); 10 Hz is the "
                    "DaemonSet's (deploy/daemonset.yaml), each load there runs at least 30 drain periods")
    ap.add_argument("--mock", action="store_true", help="CPU plumbing run with the mock provider")
    ap.add_argument("--mock-step-ms", type=float, default=20.0, help="mock: duration of one load unit")
    ap.add_argument("--mock-latency", type=int, default=1, choices=[0, 1],
                    help="mock: model AMD SMI call latency under one global lock (profiles/r2/mock_scaling.md)")
    ap.add_argument("--out", default="", help="write the full result JSON here (default gpurun_out/bench_result_n<N>.json); the "
                    "exporter log goes next to it")
    ap.add_argument("--attach", default="", help="host:port of an exporter started with --control-http; it is "
                    "paused for phases A/C instead of being spawned (lets rocprofv3 trace the bench alone)")
    return ap.parse_args(argv)


def spawn_ranks(a, argv: list[str]) -> int:
    """``--gpus N`` without a torchrun environment: start N ranks (one per GPU) with
    torch.distributed.run as a child process and return its exit status.  This
    process never initialises a GPU (no HIP call happens before the children run),
    so nothing here is replaced by exec and no device is held twice."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"), *argv]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, cwd=REPO, env=env)


def main(argv=None) -> int:
    import faulthandler
    import signal

    # `kill -USR1 <rank pid>` dumps every thread's stack to stderr (a hung rank says where)
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse_args(argv)
    if a.xgmi_child:
        return xgmi_child(a)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(a, argv)
    ctx = D.init_from_env(not a.mock)
    if ctx.world != a.gpus and ctx.rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {ctx.world}; measuring {ctx.world} rank(s)", file=sys.stderr)
    result = run(a, ctx)
    # make the result visible to rank 0 if the exporter lived elsewhere (single node: it is rank 0)
    result = D.broadcast_object(ctx, result)
    rc = 0
    if ctx.rank == 0 and result is not None:
        # The full result (per-round blocks, per-GPU tables, ...) goes to a side file;
        # stdout gets one compact line whose last key is ``summary``, so the part a
        # driver keeps of stdout (its last few KB) holds every headline number.
        full = a.out or os.path.join(REPO, "gpurun_out", f"bench_result_n{ctx.world}.json")
        os.makedirs(os.path.dirname(os.path.abspath(full)), exist_ok=True)
        with open(full, "w") as f:
            f.write(json.dumps(result) + "\n")
        print(json.dumps(compact(result, os.path.relpath(full, REPO))), flush=True)
        rc = 1 if result.get("value") is None else 0
    D.destroy(ctx)
    return rc
