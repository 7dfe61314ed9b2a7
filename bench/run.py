"""One rank's run: phases A (no exporter), B (the timed region), R, Q, U, I, S, K, X, C, and the result."""
from __future__ import annotations

import os
import time

from kube_gpu_stats_amd.parallel import dist as D
from kube_gpu_stats_amd.utils.scrape import Scraper

from .common import METRIC, PHASES, REPO, calibrate_reps, pct, progress, scrape_at, tiers, timed
from .exporter import AttachedExporter, ExporterProc, Rates, proc_cpu_seconds, thread_cpu_seconds
from .loads import GpuLoad, MockLoad, TrainLoad
from .observe import allreduce_GBps, allreduce_ratio, observed, throttled, wake_lateness, xgmi_rates
from .phase_i import interleaved
from .phase_k import component_rates
from .phase_q import idle_power, quiet_gpu
from .phase_r import burst_train
from .phase_s import capacity
from .phase_u import util_accuracy
from .phase_x import xgmi_link_check


def run(a, ctx) -> dict | None:
    n = ctx.world
    hzs = tiers(a)
    a.hz = hzs[-1]  # the fastest tier is the primary (phase B)
    if ctx.local_rank == 0 and not a.attach:
        # The exporter child runs with KGS_NO_BUILD=1: make sure its artefacts exist
        # (incremental no-op when the in-tree .so files are current).
        from kube_gpu_stats_amd.native import build as B

        B.build_native()
        if not a.mock:
            B.build_pmc_aql()
    if a.mock:
        load = MockLoad(a, ctx.local_rank)
    elif a.load == "train":
        load = TrainLoad(a, ctx.local_rank, ctx)
    else:
        load = GpuLoad(a, ctx.local_rank, ctx)

    progress(ctx, f"load {type(load).__name__}: calibrating")
    calib = load.calibrate()
    load.reps, unit_s = calibrate_reps(ctx, load, a.step_ms)
    for _ in range(a.warmup):
        load.step()
    load.sync()

    # phase A: no exporter (an attached exporter is paused: process up, no reads)
    attached = None
    if a.attach and ctx.local_rank == 0:
        attached = AttachedExporter(a.attach)
        attached.pause()
    progress(ctx, f"phase A: {a.steps} steps, no exporter")
    t_a = timed(ctx, load, a.steps, "A_off")

    # start the node exporter over every local rank's GPU
    bdfs = D.all_gather_object(ctx, (ctx.local_rank, load.pci_bdf(ctx.local_rank)))
    bdfs = [b for _, b in sorted(set(bdfs))]
    exp = None
    err = ""
    if ctx.local_rank == 0:
        logdir = os.path.dirname(os.path.abspath(a.out)) if a.out else os.path.join(REPO, "gpurun_out")
        os.makedirs(logdir, exist_ok=True)
        try:
            if attached is not None:
                attached.set_rate(a.hz)
                attached.resume()
                exp = attached
            else:
                exp = ExporterProc(a, bdfs, os.path.join(logdir, f"bench_exporter_r{ctx.rank}.log"))
        except Exception as e:  # noqa: BLE001
            err = str(e)
    err = D.broadcast_object(ctx, err)
    if err:
        return {"metric": METRIC, "value": None, "error": err}
    time.sleep(a.settle)

    # phase B: exporter on at the primary rate, scraped (THE timed region)
    sc_b = None
    before = after = {}
    win = 0.0
    exp_pid = int(exp.ready.get("pid", 0) or 0) if exp is not None else 0
    cpu0 = cpu1 = 0.0
    cpu_win = 0.0
    thr0: dict = {}
    thr1: dict = {}
    if exp is not None:
        sc_b = Scraper("127.0.0.1", exp.port)
        cpu0, thr0, c_t0 = proc_cpu_seconds(exp_pid), thread_cpu_seconds(exp_pid), time.perf_counter()
        before, w0 = scrape_at(sc_b)  # counts as of the render, timed at the request
        sc_b.start(a.scrape_hz)
    progress(ctx, f"phase B: {a.steps} steps, exporter at {a.hz:g} Hz")
    t_b = timed(ctx, load, a.steps, "B_on")
    if exp is not None:
        sc_b.stop()
        after, w1 = scrape_at(sc_b)
        win = w1 - w0
        cpu1, thr1 = proc_cpu_seconds(exp_pid), thread_cpu_seconds(exp_pid)
        cpu_win = time.perf_counter() - c_t0

    progress(ctx, "phase R: burst resolution")
    resolution = burst_train(ctx, load, exp, a)
    progress(ctx, "phase Q: idle GPU")
    quiet = quiet_gpu(ctx, load, exp, a)
    if quiet is not None:
        progress(ctx, "phase P: idle-GPU power, session / released / parked")
        power = idle_power(ctx, load, exp, a)
        if power:
            quiet["idle_power"] = power
    progress(ctx, "phase U: utilisation accuracy")
    util = util_accuracy(ctx, load, exp, a)
    progress(ctx, f"phase I: {a.rounds} interleaved rounds")
    inter = interleaved(ctx, load, exp, a, hzs)
    progress(ctx, "phase S: capacity")
    cap = capacity(ctx, load, exp, a)
    progress(ctx, "phase K: per-component delivery")
    comp_rates = component_rates(ctx, load, exp, a)
    progress(ctx, "phase X: xGMI link map")
    xlink = xgmi_link_check(ctx, load, exp, a)
    stopped = exp.stop() if exp is not None else {}

    # phase C: exporter off again
    progress(ctx, "phase C: exporter stopped")
    t_c = timed(ctx, load, a.steps, "C_off")
    if exp is None:
        return None

    pmc_on = exp.ready.get("pmc", "none") != "none"
    rb = Rates()
    rb.add(before, after, win)
    per_gpu, source = rb.per_gpu(pmc_on)
    total = sum(per_gpu.values())
    lat_primary = list(sc_b.latencies_s)
    tier_out = {}
    for h, t in inter.get("tiers", {}).items():
        r: Rates = t.pop("_rates")
        lat: list = t.pop("_lat")
        pg, src = r.per_gpu(pmc_on)
        if float(h) == a.hz:
            lat_primary += lat
        tier_out[h] = {"samples_per_sec_per_gpu": {g: round(v, 2) for g, v in pg.items()},
                       "aggregate_samples_per_sec": round(sum(pg.values()), 2), "sample_source": src,
                       "p50_scrape_ms": (pct(lat, 0.5) or 0) * 1e3, "p99_scrape_ms": (pct(lat, 0.99) or 0) * 1e3,
                       "scrapes": len(lat), **{k: v for k, v in t.items()}}
    inter["tiers"] = tier_out
    prim = tier_out.get(f"{a.hz:g}", {})
    step_s = t_b / a.steps
    integrals = stopped.get("integrals") or []
    return {
        "metric": METRIC,
        "value": total,
        "unit": f"samples/s (sum over the {n} GPU{'s' if n > 1 else ''})",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": ("synthetic mock provider (CPU plumbing)" if a.mock
                 else f"synthetic tokens, random-init {a.train_layers}-layer d={a.train_dim} bf16 decoder "
                 "training step (fwd + bwd + AdamW) as the GPU load" if a.load == "train"
                 else "synthetic (gfx950 MFMA bf16 + HBM triad + HIP-graph tiny-kernel load; random-init operands)"),
        "config": {"model": "node exporter: PMFW table + HBM + per-PID + xGMI + hardware counters "
                            f"({exp.ready.get('pmc')}), {a.hz:g} Hz/GPU, /metrics scraped at {a.scrape_hz:g} Hz",
                   "global_batch": n, "seq_len": int(round(a.hz * step_s)), "parallelism": f"dp{n}",
                   "batch_meaning": "GPUs sampled per tick (one counter drain each)",
                   "seq_len_meaning": "sampler ticks per GPU per timed step",
                   "hz": a.hz, "hz_tiers": hzs, "sample_source": source,
                   "pmc_dispatch_hz": a.pmc_dispatch_hz,
                   "pmc_batch": a.pmc_batch, "pmc_publish_us": a.pmc_publish_us,
                   "exporter": "attached" if a.attach else "spawned", "load": "mock" if a.mock else a.load,
                   "units_per_step": load.reps, "unit_ms": unit_s * 1e3},
        "value_semantics": "aggregate over all GPUs (driver contract); per-GPU in samples_per_sec_per_gpu",
        "samples_per_sec_per_gpu": total / max(1, len(per_gpu)),
        "aggregate_samples_per_sec": total,
        "pmc_samples_per_sec_per_gpu": {g: round((rb.pmc.get(g, 0) / win) if win > 0 else 0, 2) for g in per_gpu},
        "pmfw_distinct_samples_per_sec_per_gpu": {g: round((rb.pmfw.get(g, 0) / win) if win > 0 else 0, 2)
                                                  for g in per_gpu},
        "p50_scrape_ms": (pct(lat_primary, 0.5) or 0) * 1e3,
        "p99_scrape_ms": (pct(lat_primary, 0.99) or 0) * 1e3,
        "scrapes": len(lat_primary),
        "scrape_errors": sc_b.errors,
        "scrape_bytes_avg": sc_b.bytes / max(1, len(sc_b.latencies_s)),
        # headline overhead: paired interleaved rounds at the primary rate (mean ± 95 % CI)
        "overhead_pct": prim.get("overhead_pct"),
        "overhead_ci95_pct": prim.get("overhead_ci95_pct"),
        "overhead_abc_pct": 100.0 * (t_b / (0.5 * (t_a + t_c)) - 1.0),
        "t_off_a_s": t_a,
        "t_on_s": t_b,
        "t_off_c_s": t_c,
        "interleaved": inter,
        "burst_resolution": resolution,
        "quiet_gpu": quiet,
        "util_accuracy": util,
        "capacity": cap,
        "delivered_by_component": comp_rates,
        "exporter_cpu_cores": round((cpu1 - cpu0) / cpu_win, 4) if cpu_win > 0 and exp_pid else None,
        "exporter_cpu_cores_by_thread": {k: round((v - thr0.get(k, 0.0)) / cpu_win, 4) for k, v in thr1.items()
                                         if cpu_win > 0 and v - thr0.get(k, 0.0) > 0.005 * cpu_win},
        "pmc_source": exp.ready.get("pmc"),
        "pmc_error": exp.ready.get("pmc_error"),
        "load": calib,
        "observed_during_load": observed(after),
        "sampler_wake_lateness": wake_lateness(before, after),
        "throttled_pct_during_load": throttled(before, after, win),
        "xgmi_GBps_per_gpu": xgmi_rates(before, after, win),
        # what the phase-B all-reduces must have moved per GPU (read + write, bandwidth-optimal
        # 2(N-1)/N each way): the measured / expected ratio pins the PMFW xGMI accumulator unit
        "xgmi_allreduce_GBps_per_gpu_expected": allreduce_GBps(load, a, n, win),
        # measured ÷ expected per GPU: 1.0 if the link counters' unit is right and the
        # all-reduces ran on xGMI (phase X pins the unit link by link)
        "xgmi_allreduce_ratio_per_gpu": allreduce_ratio(xgmi_rates(before, after, win), allreduce_GBps(load, a, n, win)),
        "xgmi_link_check": xlink,
        "xgmi_link_map_ok": xlink.get("xgmi_link_map_ok"),
        "xgmi_links_ok": xlink.get("xgmi_links_ok"),
        "xgmi_unit_ratio": xlink.get("xgmi_unit_ratio"),
        "xgmi_unit_ratio_min_max": xlink.get("xgmi_unit_ratio_min_max"),
        "phases_wall": PHASES,
        "pmc_read_us_mean": 1e6 * sum(i.get("pmc_read_seconds", 0) for i in integrals)
        / max(1, sum(i.get("pmc_samples", 0) for i in integrals)),
        "pmfw_read_us_mean": 1e6 * sum(i.get("read_seconds", 0) for i in integrals)
        / max(1, sum(i.get("reads", 0) for i in integrals)),
        "exporter_integrals": integrals,
        "pmc_reader_info": stopped.get("pmc_info") if isinstance(stopped, dict) else None,
    }
