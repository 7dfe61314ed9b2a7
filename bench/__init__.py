"""Headline benchmark (``python bench.py``; this package holds its phases): counter samples/s per GPU, p50 /metrics scrape latency and
GPU-time overhead %, under synthetic gfx950 load (BASELINE.json "metric").

    python bench.py --gpus N --steps K --warmup W

With N > 1 and no torchrun environment, bench.py starts N rank processes itself
(``torch.distributed.run``, 127.0.0.1) before anything touches a GPU, and exits
with their status; under torchrun it is one of those ranks.  One rank per GPU;
rank 0 prints the result line.

A *step* is a fixed block of synthetic load on every GPU: a *unit* (an MFMA-bound
bf16 kernel + HBM triads, ops/hip/load_kernels.hip, + a HIP graph of 2000 tiny
copies — the dispatch-bound part, where the counter reader's command-processor
packets would cost the workload time) repeated until the step lasts ≥ --step-ms
(default 500 ms), so every timed region is long against timer and DVFS noise.

  A  K steps, no exporter process                       (baseline)
  B  K steps, node exporter sampling every GPU at --hz (PMFW table, HBM, per-process
     list, xGMI, hardware counters) and scraped at --scrape-hz      (THE timed region)
  R  untimed: a train of ~1 ms MFMA bursts every 5 ms on every GPU, read back from the
     exporter's full-rate /counters stream — how many bursts the primary rate resolves
     (``burst_resolution``)
  Q  untimed: every GPU idle; the exporter's READ rate, the PMFW GFX busy and the
     SPI-busy share it reports, in the default adaptive mode and in profiling mode
     (``quiet_gpu``) — the cost of sampling that GPU-time overhead cannot show
  I  --rounds rounds of one block per condition — exporter paused, then each rate of
     --hz-list — in alternating order (off,100,8k | 8k,100,off | ...), --block-steps
     steps per block, scraped while sampling.  Per round, overhead = t_on/t_off − 1;
     the result is the mean over rounds ± a 95 % t-interval.  Adjacent blocks share
     thermal and power state, so slow drift cancels (A/B/C cannot do that).  The bench
     reads the PMFW table itself at every block edge: power and package-power throttle
     residency per condition (``interleaved.power``; profiles/r2/r2aq).
  S  untimed: one block at each --capacity-hz rate in profiling mode — delivered drains,
     overruns, host µs per drain (``capacity``)
  C  K steps, exporter stopped                           (second baseline)

``value`` = counter samples/s summed over the N GPUs (the driver's contract: the
whole-job aggregate; weak scaling, per-GPU rate fixed).  ``samples_per_sec_per_gpu``
is the per-GPU figure the metric name refers to.  A counter sample is one hardware-
counter drain (values advance on every drain), or one distinct PMFW table where
the counter tier is unavailable.  Scrape latency is request → last body byte on a
keep-alive connection, as a Prometheus server sees it (utils/scrape.py).

The exporter runs as its own process (as in production: DaemonSet vs workload),
launched by local rank 0 over the PCI addresses of every local rank's GPU.
``--mock`` runs the same flow on CPU with the mock provider (tests only).
"""

from __future__ import annotations

from kube_gpu_stats_amd.parallel import dist as D  # noqa: F401  (tests monkeypatch the collectives)

from .cli import main, parse_args  # noqa: F401
from .common import METRIC, REPO, free_port, mean_ci95, tiers  # noqa: F401
from .exporter import AttachedExporter, ExporterProc, PmfwProbe, Rates  # noqa: F401
from .loads import GpuLoad, MockLoad, TrainLoad  # noqa: F401
from .observe import allreduce_GBps, allreduce_ratio  # noqa: F401
from .phase_x import _pair_rounds, _xgmi_rank0, xgmi_link_check  # noqa: F401
from .summary import compact, summarize  # noqa: F401

# Module map (one phase per module):
#   cli       flags, rank launch, main          run      A / B / C and the result dict
#   common    paths, statistics, timed regions  summary  the stdout line
#   loads     synthetic / train / mock load     exporter the exporter under test
#   observe   phase-B side readings             phase_i  interleaved overhead rounds
#   phase_r   burst resolution                  phase_q  idle GPU (+ idle power)
#   phase_u   utilisation accuracy              phase_k  per-component delivery
#   phase_s   capacity                          phase_x  xGMI link map
