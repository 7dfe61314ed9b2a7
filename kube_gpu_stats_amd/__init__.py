"""kube_gpu_stats_amd — MI355X-native Kubernetes GPU statistics.

Capabilities of kanglanglang/kube_gpu_stats (reference: ``who_use_gpu/who_use_gpu.py``
and ``gpu_util_stats/gpu_util_stats.py``), rebuilt for AMD Instinct MI355X:

* ``exporter``  – per-node DaemonSet exporter: one C++ sampler thread per GPU
  reading the PMFW metrics table, HBM occupancy, per-process usage, xGMI links and
  (optionally) hardware counters through rocprofiler-sdk; serves Prometheus
  ``/metrics`` including the reference's ``container_gpu_sm_util`` contract.
* ``attribution`` – GPU → pod mapping via the kubelet pod-resources API, PID →
  pod via cgroups.
* ``reports``   – the reference's two reports (``who-use-gpu`` census and the
  daily ``gpu-util-stats`` accounting) with a ``--compat`` golden mode.
* ``ops``       – gfx950 HIP synthetic-load kernels used by the overhead bench.

Subpackages: ``models`` (metric schema), ``ops`` (HIP kernels), ``parallel``
(device fan-out, topology, distributed bench helpers), ``utils``.
"""

__version__ = "0.1.0"


def load_native():
    """The compiled C++ data plane (built in-tree on first use)."""
    from .native import load

    return load()
