"""``kgs exporter`` — the per-node DaemonSet exporter process.

Native data plane (C++ sampler threads + epoll HTTP, see native/include/kgs/*.h)
plus the Python control plane (flags/env, attribution loop, lifecycle).  Prints
one ``{"event": "ready", ...}`` JSON line on stdout once ``/metrics`` is being
served, then runs until SIGTERM/SIGINT (or ``quit`` on stdin with
``--control-stdin``).

Run it in its own process: with ``--pmc aqlprofile`` it initialises HSA and
opens a private AQL queue per GPU for its counter READs, which must not share a
process with a workload's HIP runtime.

One counter reader ships: the direct aqlprofile CP reader.  The rocprofiler-sdk
device-counting reader (``native/counters/pmc_rocprofiler.cpp``) is a test-only
cross-check of its numbers: ``--pmc rocprofiler`` is refused unless
``KGS_PMC_CROSSCHECK=1`` (tests/test_gpu.py sets it) — no runtime choice of
backends in the product.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import threading

from ..native import load as load_native
from ..native import pmc_lib_path
from ..utils import log
from ..utils.config import add_flag

L = log.get("exporter")

# AMD SMI call latencies of the mock's latency model, from the per-call latencies
# measured on MI355X (profiles/r2/amdsmi_latency.md): link metrics p99 0.99 ms, ECC
# count p99 0.75 ms, PMFW table pread mean 0.125 ms; the process list (p50 74 µs with
# one process) is modelled at 0.5 ms for a node with many GPU processes.
MOCK_LATENCY = {"proc_latency_s": 5e-4, "link_latency_s": 1e-3, "health_latency_s": 7.5e-4,
                "metrics_latency_s": 1.25e-4}


def build_parser(ap: argparse.ArgumentParser | None = None) -> argparse.ArgumentParser:
    ap = ap or argparse.ArgumentParser(prog="kgs exporter", description=__doc__.splitlines()[0])
    add_flag(ap, "backend", "amdsmi", "device provider: amdsmi (MI355X) or mock")
    add_flag(ap, "mock-gpus", 8, "mock provider: number of GPUs")
    add_flag(ap, "mock-fail-rate", 0.0, "mock provider: injected read-failure probability")
    add_flag(ap, "mock-latency", False, "mock provider: model AMD SMI latency as measured on MI355X (process list "
                                        "0.5 ms, link table 1 ms, RAS 0.75 ms, under one global lock; PMFW table "
                                        "read 0.125 ms, unlocked)")
    add_flag(ap, "mock-xgmi-swap", -1, "mock provider: this GPU's link table reports its first two xGMI ports' "
                                       "peers swapped (a wrong link map for the bench's phase X self-check)")
    add_flag(ap, "mock-partition", "SPX", "mock provider: compute partition mode (SPX | DPX | QPX | CPX)")
    add_flag(ap, "hz", 10.0, "sampler tick rate per GPU (1/10/100 Hz tiers; hardware counters every tick)")
    add_flag(ap, "pmfw-hz", 100.0, "cap on PMFW metrics-table reads/s (firmware refreshes it every ~20 ms)")
    add_flag(ap, "proc-every", 10, "per-process tier every N fast ticks, at most 10 Hz (0 = off)")
    add_flag(ap, "link-every", 100, "xGMI link tier every N fast ticks, at most 1 Hz (0 = off)")
    add_flag(ap, "proc-period", 0.0, "per-process tier period in seconds (overrides --proc-every; survives rate "
                                     "changes)")
    add_flag(ap, "link-period", 0.0, "xGMI link + RAS tier period in seconds (overrides --link-every)")
    add_flag(ap, "pmc", "none", "hardware counters: none | aqlprofile (direct CP reads on a private AQL queue) "
                                "| mock (tests)")
    add_flag(ap, "pmc-lib", "", "counter reader library (default: the in-tree one for --pmc)")
    add_flag(ap, "pmc-lean", 2, "aqlprofile READ packet: 0 as built (per-XCC CS_PARTIAL_FLUSH + full cache "
                                "invalidate), 1 no flushes, 2 no flushes + L2 writeback only (default), 3 no cache op")
    add_flag(ap, "pmc-set", "base", "counter set: base (GRBM clocks/active + MFMA busy + CPC busy, 56 register "
                                    "reads) | full (+ TA vector-memory busy, 568 reads: costs dispatch-bound workloads more) | util (GRBM "
                                    "count + SPI + CPC busy, 24 reads: the utilisation only, no MFMA / per-XCD gauges, "
                                    "each READ cheaper for a µs-kernel stream)")
    add_flag(ap, "pmc-pipeline", True, "aqlprofile reader: overlap each counter READ's CP round trip with the "
                                       "tick sleep (the sample is stamped with the CP read time)")
    add_flag(ap, "pmc-reclaim-s", 10.0, "re-START the counters after they stalled this long (a foreign profiler "
                                        "stopped or reprogrammed them; 0 = never, SIGUSR1 hand-over disables it)")
    add_flag(ap, "pmc-refresh-s", 60.0, "re-START (reprogram) the counters this often, in case another profiler "
                                        "changed their selects (0 = never; SIGUSR1 hand-over disables it)")
    add_flag(ap, "pmc-idle-hz", 100.0, "counter READ rate while the GPU has no wave in flight: every READ is a "
                                       "command-processor packet that GFX busy / GUI-active count as work (≈80 / "
                                       "190 µs each), so a quiet GPU is read at this rate and a busy one every tick "
                                       "(0 = every tick: profiling mode)")
    add_flag(ap, "pmc-dispatch-hz", 500.0, "counter READ rate in a dispatch-bound stream (--pmc-cp-only-min): a "
                                            "µs-kernel stream pays +0.5 %% at 1 kHz, +4 %% at 8 kHz (profiles/r4/ r4d)")
    add_flag(ap, "pmc-quiet-release-s", 30.0, "release the counter session (STOP, READ queue destroyed) after the "
                                               "GPU has been quiet this long, and bill it from the PMFW until the PMFW "
                                               "shows GFX busy again: the session costs an idle MI355X ≈32 W "
                                               "(bench phase P, r6h / r6i).  0 = never; ignored with --sm-util-source "
                                               "counters and in profiling mode")
    add_flag(ap, "pmc-cp-only-min", 0.3, "dispatch-bound READ rate: while the command processor dispatches with no "
                                         "wave in flight for at least this share of the clocks (a stream of µs "
                                         "kernels, which each READ packet slows by a fixed CP cost), READ at "
                                         "--pmc-dispatch-hz (0 = off; ignored in profiling mode)")
    add_flag(ap, "pmc-dispatch-hold-ms", 10.0, "dispatch-bound READ intervals in a row, in ms, before that rate applies "
                                              "(a few ms of small kernels inside a training step keep the full rate)")
    add_flag(ap, "pmc-batch", 8, choices=range(1, 17), help="counter READs per L2 writeback: a READ's results sit in the GPU's L2 until "
                                 "written back, and that writeback is half of what a READ costs a training step; "
                                 "with B > 1 at most every B-th READ writes back (at 8 kHz samples arrive B-2B ticks "
                                 "late; 1 = every READ).  Trade-off: batching cuts the cost to long kernels and "
                                 "training steps, but a stream of µs kernels pays +0.2-0.3 points more at 8 kHz "
                                 "than unbatched (profiles/r3/README.md r3ab)")
    add_flag(ap, "pmc-publish-us", 1000, "longest a batched counter READ waits for its L2 writeback: a READ writes "
                                         "back early when the next tick would be later (at <= 1 kHz every READ does)")
    add_flag(ap, "pmc-lite", True, "lite READs: a batch's non-publishing READs skip the per-SE counters (MFMA busy, "
                                    "TA): a compacted READ without the 32 per-SE copies of the base set's 56, which "
                                    "a µs-kernel stream pays for; "
                                    "MFMA and per-XCD values then update at the publish rate (1 kHz at 8 kHz ticks), "
                                    "their integrals stay exact")
    add_flag(ap, "pmc-timeout-ms", 250, "bound of every wait on the command processor (counter READ, START, STOP, "
                                        "queue slot): a wedged CP costs one timeout, never a hang")
    add_flag(ap, "pmc-breaker-k", 3, "consecutive failed counter drains that open the counter tier's circuit breaker "
                                     "(kgs_pmc_failed = 1: READs stop, the reader's queue is recreated)")
    add_flag(ap, "pmc-retry-s", 1.0, "first retry (reset + re-START) after the breaker opened; doubles per failed retry")
    add_flag(ap, "pmc-retry-max-s", 60.0, "longest retry interval of the counter tier's breaker")
    add_flag(ap, "tick-dither", 0.25, "counter-tick dither: each READ deadline random-walks off the fixed grid by up "
                                     "to this share of a period per tick (within half a period), so the READ phase "
                                     "does not lock onto a periodic workload; the rate stays exact (0 = fixed grid)")
    add_flag(ap, "stop-timeout", 1.0, "shutdown waits this long for the sampler threads, then abandons any stuck in a "
                                      "device call (the exporter still exits on SIGTERM during a GPU hang)")
    add_flag(ap, "listen", "0.0.0.0:9400", "HTTP listen address (port 0 = ephemeral)")
    add_flag(ap, "node-name", os.environ.get("NODE_NAME", ""), "kubernetes_io_hostname label (downward API NODE_NAME)")
    add_flag(ap, "gpu-type", "", "override the nvidia_gpu_type / gpu_type label value")
    add_flag(ap, "window", 15.0, "gauge averaging window in seconds (default: one typical scrape interval, so "
                                 "successive scrapes' gauges tile time; exact per-pod accounting uses the "
                                 "container_gpu_busy_seconds_total counter)")
    add_flag(ap, "stale-after", 5.0, "drop a device's window gauges when its last good read / counter drain is "
                                     "older than this (seconds)")
    add_flag(ap, "hbm-full-bw", 8.41e12, "HBM bytes/s at 100%% UMC activity (MI355X calibration, profiles/umc_calib.md)")
    add_flag(ap, "bdfs", "", "comma-separated PCI addresses to sample (default all)")
    add_flag(ap, "pin-numa", True, "pin each sampler thread to its GPU's NUMA node")
    add_flag(ap, "per-process", True, "export per-process HBM/CU metrics")
    add_flag(ap, "compat-unallocated", False, "emit container_gpu_sm_util for GPUs no pod holds")
    add_flag(ap, "pcie-bytes-per-unit", 105.7, "bytes per unit of the PMFW PCIe bandwidth accumulator "
                                              "(MI355X calibration, profiles/r2/pcie/)")
    add_flag(ap, "xgmi-bytes-per-unit", 1024.0, "bytes per unit of the PMFW xGMI link accumulators (amdsmi.h: KB; "
                                               "correct with bench.py's N > 1 expected / measured ratio)")
    add_flag(ap, "sm-util-source", "auto", "what container_gpu_sm_util / container_gpu_busy_seconds_total / "
                                           "amdgpu_gfx_busy_* measure: auto (READ-immune: the counter tier's "
                                           "GRBM_SPI_BUSY while it runs, the firmware GFX busy otherwise) | pmfw "
                                           "(firmware GFX busy alone: a dispatch in flight, and every counter READ "
                                           "packet as ~80 us of work) | counters (GRBM_SPI_BUSY alone; needs --pmc)")
    add_flag(ap, "pod-resources-socket", "/var/lib/kubelet/pod-resources/kubelet.sock", "kubelet pod-resources socket")
    add_flag(ap, "static-owners", "", "JSON file mapping device id -> {pod,namespace,container}")
    add_flag(ap, "attribution-interval", 1.0, "attribution refresh period (s)")
    add_flag(ap, "pod-directory", "", "pod UID / container ID → pod names for per-process attribution: 'api' "
                                      "(in-cluster API server, this node's pods) or 'file:<PodList JSON>' ('' = off)")
    add_flag(ap, "pid-file", "", "write the exporter's PID here (hand-over: `kgs pmc release` signals it)")
    add_flag(ap, "control-stdin", False, "accept 'quit' on stdin")
    add_flag(ap, "control-http", False, "serve /control/pause and /control/resume (benchmarks only)")
    add_flag(ap, "gzip-level", 0, "gzip /metrics at this zlib level for clients that accept it (0 = off; level 1 "
                                  "costs ≈0.6 ms per 8-GPU page and shrinks it ≈10×)")
    add_flag(ap, "metric-allow", "", "only these /metrics families: comma-separated globs, e.g. "
                                     "'container_gpu_*,amdgpu_gfx_*,kgs_up' ('' = all)")
    add_flag(ap, "metric-deny", "", "drop these /metrics families (globs; wins over --metric-allow), e.g. "
                                    "'amdgpu_*_xcc_percent,kgs_sample_read_seconds'")
    add_flag(ap, "http-idle-s", 300.0, "close a keep-alive HTTP connection idle this long (0 = never)")
    add_flag(ap, "http-max-conns", 256, "HTTP connections held at once; past it the least recently active one is "
                                        "closed (0 = unlimited)")
    return ap


# Floors of the tick-counted AMD SMI tiers.  --proc-every / --link-every count fast
# ticks, which suits the 10 Hz DaemonSet rate; at the counter tier's kHz rates the
# defaults (10 / 100 ticks) would poll AMD SMI's process list 800 times a second and
# keep the node-wide slow thread on a core (r3q soak: 0.33-0.43 cores at 8 kHz).
# Unless --proc-period / --link-period say otherwise, the tiers run no faster than
# 10 Hz / 1 Hz.
MIN_PROC_PERIOD_S = 0.1
MIN_LINK_PERIOD_S = 1.0


def tier_periods(a) -> tuple[float, float]:
    """(per-process, link) tier periods in seconds; 0 = off."""
    proc = a.proc_period or (max(a.proc_every / a.hz, MIN_PROC_PERIOD_S) if a.proc_every > 0 and a.hz > 0 else 0.0)
    link = a.link_period or (max(a.link_every / a.hz, MIN_LINK_PERIOD_S) if a.link_every > 0 and a.hz > 0 else 0.0)
    return proc, link


def config_from_args(a) -> dict:
    host, _, port = a.listen.rpartition(":")
    proc_period, link_period = tier_periods(a)
    cfg = {
        "backend": a.backend,
        "mock": {"n_gpus": a.mock_gpus, "fail_rate": a.mock_fail_rate, "compute_partition": a.mock_partition,
                 "xgmi_swap_dev": a.mock_xgmi_swap,
                 **(MOCK_LATENCY if a.mock_latency else {})},
        "hz": a.hz,
        "pmfw_hz": a.pmfw_hz,
        "proc_every": a.proc_every,
        "link_every": a.link_every,
        "proc_period_s": proc_period,
        "link_period_s": link_period,
        "pin_numa": a.pin_numa,
        "pmc_source": a.pmc,
        "pmc_lib": a.pmc_lib or pmc_lib_path(a.pmc),
        "pmc_pipeline": a.pmc_pipeline,
        "pmc_set": a.pmc_set,
        "pmc_lean": a.pmc_lean,
        "pmc_reclaim_s": a.pmc_reclaim_s,
        "pmc_refresh_s": a.pmc_refresh_s,
        "pmc_idle_hz": a.pmc_idle_hz,
        "pmc_dispatch_hz": a.pmc_dispatch_hz,
        "pmc_quiet_release_s": 0.0 if a.sm_util_source == "counters" else a.pmc_quiet_release_s,
        "pmc_cp_only_min": a.pmc_cp_only_min,
        "pmc_dispatch_hold_s": a.pmc_dispatch_hold_ms * 1e-3,
        "pmc_timeout_ms": a.pmc_timeout_ms,
        "pmc_batch": a.pmc_batch,
        "pmc_publish_us": a.pmc_publish_us,
        "pmc_lite": a.pmc_lite,
        "pmc_breaker_k": a.pmc_breaker_k,
        "pmc_retry_s": a.pmc_retry_s,
        "pmc_retry_max_s": a.pmc_retry_max_s,
        "stop_timeout_s": a.stop_timeout,
        "tick_dither": a.tick_dither,
        "listen_addr": host or "0.0.0.0",
        "port": int(port),
        "node_name": a.node_name,
        "gpu_type_override": a.gpu_type,
        "window_s": a.window,
        "stale_s": a.stale_after,
        "hbm_bytes_per_s_at_full_umc": a.hbm_full_bw,
        "per_process": a.per_process,
        "compat_unallocated": a.compat_unallocated,
        "sm_util_source": a.sm_util_source,
        "pcie_bytes_per_acc_unit": a.pcie_bytes_per_unit,
        "xgmi_bytes_per_acc_unit": a.xgmi_bytes_per_unit,
        "control_http": a.control_http,
        "gzip_level": a.gzip_level,
        "http_idle_s": a.http_idle_s,
        "http_max_conns": a.http_max_conns,
        "metric_allow": a.metric_allow,
        "metric_deny": a.metric_deny,
        "bdfs": [b for b in (a.bdfs.split(",") if isinstance(a.bdfs, str) else a.bdfs) if b],
    }
    return cfg


def run(a) -> int:
    if a.pmc == "rocprofiler" and os.environ.get("KGS_PMC_CROSSCHECK") != "1":
        L.error("--pmc rocprofiler is a test-only cross-check reader (set KGS_PMC_CROSSCHECK=1 in tests)")
        print(json.dumps({"event": "error", "error": "--pmc rocprofiler is test-only"}), flush=True)
        return 2
    if a.sm_util_source == "counters" and a.pmc == "none":
        msg = "--sm-util-source counters needs the counter tier (--pmc aqlprofile)"
        print(json.dumps({"event": "error", "error": msg}), flush=True)
        L.error(msg)
        return 2
    if a.pmc not in ("none", "aqlprofile", "mock", "rocprofiler"):
        print(json.dumps({"event": "error", "error": f"unknown --pmc {a.pmc!r}"}), flush=True)
        return 2
    N = load_native()
    cfg = config_from_args(a)
    try:
        ex = N.Exporter(cfg)
    except RuntimeError as e:
        L.error("%s", e)
        print(json.dumps({"event": "error", "error": str(e)}), flush=True)
        return 2
    if a.pmc != "none" and ex.pmc_name == "none":
        L.warning("hardware counters unavailable (%s); continuing without the PMC tier", ex.pmc_error)
    ex.start()
    if ex.port < 0 and cfg["port"] >= 0:
        L.error("HTTP server failed: %s", ex.error)
        ex.stop()
        return 2
    from ..attribution.attributor import Attributor

    from ..attribution.poddir import PodDirectory

    pdir = PodDirectory(a.pod_directory, node=a.node_name) if a.pod_directory else None
    attr = Attributor(ex, a.pod_resources_socket, a.static_owners or None,
                      interval_s=a.attribution_interval, pod_directory=pdir).start()
    if a.pid_file:
        with open(a.pid_file, "w") as f:
            f.write(f"{os.getpid()}\n")
    print(json.dumps({"event": "ready", "port": ex.port, "pid": os.getpid(), "backend": ex.backend_name,
                      "pmc": ex.pmc_name, "pmc_error": ex.pmc_error, "devices": ex.devices(),
                      "pmc_info": [ex.pmc_info(i) for i in range(ex.device_count)],
                      "hz": a.hz}), flush=True)
    done = threading.Event()

    def _sig(*_):
        done.set()

    signal.signal(signal.SIGTERM, _sig)
    signal.signal(signal.SIGINT, _sig)

    # Counter hand-over, like a profiling pause: SIGUSR1 gives the hardware counters
    # to another profiler, SIGUSR2 takes them back; the PMFW / per-process tiers keep
    # going.  In the DaemonSet (hostPID) PID 1 is the host's init, so signal the
    # exporter's own PID — `kubectl exec <pod> -- kgs pmc release` does that through
    # the loopback-only /control/pmc/* endpoints (or the --pid-file).
    def _pmc(signum, _frame):
        on = signum == signal.SIGUSR2
        ex.set_pmc_enabled(on)
        L.warning("hardware counters %s", "re-acquired" if on else "released to other profilers")

    signal.signal(signal.SIGUSR1, _pmc)
    signal.signal(signal.SIGUSR2, _pmc)
    if a.control_stdin:
        def _stdin():
            for line in sys.stdin:
                if line.strip().lower() in ("quit", "exit", "stop"):
                    break
            done.set()
        threading.Thread(target=_stdin, daemon=True).start()
    while not done.wait(0.5):
        pass
    attr.stop()
    ex.stop()
    print(json.dumps({"event": "stopped", "integrals": [ex.integrals(i) for i in range(ex.device_count)],
                      "pmc_info": [ex.pmc_info(i) for i in range(ex.device_count)],
                      "abandoned_threads": ex.abandoned_threads}), flush=True)
    if ex.abandoned_threads:
        # A sampler thread is stuck in a device call (a hung GPU): leave without
        # running the runtime's static destructors under it.
        L.warning("%d sampler thread(s) stuck in a device call; exiting without teardown", ex.abandoned_threads)
        sys.stderr.flush()
        os._exit(0)
    return 0


def main(argv=None) -> int:
    return run(build_parser().parse_args(argv))


if __name__ == "__main__":
    sys.exit(main())
