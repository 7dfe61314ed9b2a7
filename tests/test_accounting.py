"""Exact per-pod accounting (VERDICT r1 missing #3).

The reference's daily report averages ``container_gpu_sm_util`` samples
(gpu_util_stats.py:62-94,159).  A gauge averaged over the exporter's window sees
that window only: with the window shorter than the scrape interval, a bursty job
whose bursts fall between scrapes reads ~0.  The exporter's
``container_gpu_busy_seconds_total`` integrates the PMFW busy accumulators since
the pod got the GPU, and the fixed-mode report takes ``100 * rate()`` of it per
step, so every burst counts.  Time is scaled 1:20 against production (a 0.75 s
"scrape interval", 0.1 s bursts = 2 s on / 13 s off at 15 s scrapes; the
gauge window 0.05 s = 1 s at 15 s).
"""
import time

import pytest

from fakeprom import FakeProm
from kube_gpu_stats_amd.reports import gpu_util_stats as G
from kube_gpu_stats_amd.reports.promql import PromClient
from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

PERIOD, DUTY = 0.75, 2.0 / 15.0


@pytest.mark.slow
def test_bursty_pod_counter_report_is_exact_gauge_misses(mock_exporter):
    ex = mock_exporter(n_gpus=1, hz=400, window_s=0.05, node_name="node-a",
                       mock={"square_duty": DUTY, "util_period_s": PERIOD, "util_base": 50, "util_amp": 50,
                             "fw_period_s": 0.005})
    ex.set_device_owners(0, [{"pod": "bursty", "namespace": "ml", "container": "main"}])
    time.sleep(0.2)
    # Mock time of the firmware table ↔ wall clock, to scrape mid-way through the idle part
    # of every cycle (the phase a 15 s scrape keeps relative to a 15 s job cycle).
    s = ex.snapshot(0)
    t_mock = (s["fw_ts"] - 1000) / 1e8
    offset = time.time() - t_mock
    k0 = int(t_mock / PERIOD) + 1
    phase = 0.55 * PERIOD  # bursts occupy [0, 0.1) of each cycle
    sc = Scraper("127.0.0.1", ex.port)
    fp = FakeProm()
    url = fp.start()
    stamps = []
    try:
        # 17 scrapes = 12 s of data for a 6 s report window at a 3 s step: the first step's
        # range (end-9, end-6] lies inside the data (the client sends whole seconds), so
        # rate() never extrapolates from the series start (a true Prometheus artefact)
        for k in range(k0, k0 + 17):
            at = offset + k * PERIOD + phase
            time.sleep(max(0.0, at - time.time()))
            ts = time.time()
            fp.ingest(parse_text(sc.get()), ts)
            stamps.append(ts)
        # direct check on the counter: busy seconds between the first and last scrape
        series = fp.series["container_gpu_busy_seconds_total"]
        (key, pts), = series.items()
        assert dict(key)["pod_name"] == "bursty"
        cycles = len(stamps) - 1
        assert pts[-1][1] - pts[0][1] == pytest.approx(cycles * DUTY * PERIOD, rel=0.01)
        end = int(stamps[-1])
        window, step = 6, 3
        end_f = stamps[-1]
        q_cnt = G.Queries.amd("ml", step)
        q_gauge = G.Queries.amd("ml", step, util_metric="container_gpu_sm_util")
        for q in (q_cnt, q_gauge):
            fp.add_instant(q.total, [{"metric": {"node": "node-a", q.type_label: "MI355X"}, "value": [end, "8"]}])
            fp.add_instant(q.used, [{"metric": {"node": "node-a"}, "value": [end, "1"]}])
            fp.add_instant(q.live, [{"metric": {"namespace": "ml", "pod": "bursty"}, "value": [end, "1"]}])
            fp.add_range(q.req, [{"metric": {"node": "node-a", "namespace": "ml", "pod": "bursty"},
                                  "values": [[end, "1"]]}])
        exact = 100.0 * DUTY
        rows = G.run_report(PromClient(url), q_cnt, end_f, window, step, compat=False)
        assert [r[:4] for r in rows] == [["node-a", "ml", "bursty", 1]]
        assert rows[0][4] == pytest.approx(exact, rel=0.01), rows
        gauge = G.run_report(PromClient(url), q_gauge, end_f, window, step, compat=False)
        assert abs(gauge[0][4] - exact) > 10, gauge  # the gauge only saw idle windows
    finally:
        fp.stop()


def test_busy_counter_starts_at_allocation_and_survives_owner_refresh(mock_exporter):
    ex = mock_exporter(n_gpus=1, hz=200, mock={"util_base": 60, "util_amp": 0.0001, "fw_period_s": 0.005})
    time.sleep(0.3)
    owner = [{"pod": "late", "namespace": "ml", "container": "c"}]
    ex.set_device_owners(0, owner)
    v0 = parse_text(ex.render())["container_gpu_busy_seconds_total"][0][1]
    assert v0 < 0.05  # counts from the allocation, not from exporter start
    time.sleep(0.5)
    ex.set_device_owners(0, owner)  # the attributor re-pushes an unchanged table every pass
    m = parse_text(ex.render())
    v1 = m["container_gpu_busy_seconds_total"][0][1]
    assert v1 == pytest.approx(0.6 * 0.5, abs=0.06)
    own = m["kgs_gpu_owner"]
    assert [(lb["pod_name"], lb["gpu"], v) for lb, v in own] == [("late", "0", 1.0)]
    ex.set_device_owners(0, [])
    assert "container_gpu_busy_seconds_total" not in parse_text(ex.render()) or \
        not parse_text(ex.render())["container_gpu_busy_seconds_total"]


def test_sm_util_from_counters(N, mock_exporter):
    """--sm-util-source counters: the reference-contract gauge and the per-pod busy
    counter come from the counter tier's GPU-active (GRBM_SPI_BUSY, blind to the
    exporter's own READs) instead of the PMFW GFX busy."""
    ex = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", window_s=0.5, sm_util_source="counters",
                       mock={"util_base": 60, "util_amp": 0.0001, "fw_period_s": 0.005})
    time.sleep(0.3)
    ex.set_device_owners(0, [{"pod": "p", "namespace": "ml", "container": "c"}])
    time.sleep(0.6)
    m = parse_text(ex.render())
    (lb, sm), = m["container_gpu_sm_util"]
    assert lb["pod_name"] == "p" and sm == pytest.approx(60, abs=3)
    busy = m["container_gpu_busy_seconds_total"][0][1]
    assert busy == pytest.approx(0.6 * 0.6, abs=0.08)              # from the allocation, counter integral
    act = m["amdgpu_gpu_active_seconds_total"][0][1]
    assert act > busy and act == pytest.approx(ex.integrals(0)["active_seconds"], rel=0.05)
    with pytest.raises(RuntimeError, match="sm_util_source"):
        N.Exporter({"backend": "mock", "sm_util_source": "bogus"})


def test_pod_energy_counter_starts_at_allocation(mock_exporter):
    """container_gpu_energy_joules_total: the GPU's socket energy since the pod got it."""
    ex = mock_exporter(n_gpus=1, hz=200, mock={"util_base": 60, "util_amp": 0.0001, "fw_period_s": 0.005})
    time.sleep(0.3)
    e0 = parse_text(ex.render())["amdgpu_energy_joules_total"][0][1]
    ex.set_device_owners(0, [{"pod": "p", "namespace": "ml", "container": "c"}])
    time.sleep(0.5)
    m = parse_text(ex.render())
    (lb, e_pod), = m["container_gpu_energy_joules_total"]
    e1 = m["amdgpu_energy_joules_total"][0][1]
    assert lb["pod_name"] == "p" and e_pod > 0
    assert e_pod == pytest.approx(e1 - e0, rel=0.05, abs=1.0)  # counted from the allocation, not exporter start
    assert e_pod < e1


def test_report_energy_column_tiles_the_window(mock_exporter):
    """gpu-util-stats --energy: the per-step increase() of the per-pod energy counter,
    first range point (the step before the window) left out, adds up to the energy the
    pod's GPU drew over the window."""
    ex = mock_exporter(n_gpus=2, hz=200, node_name="node-a",
                       mock={"util_base": 60, "util_amp": 0.0001, "fw_period_s": 0.005})
    ex.set_device_owners(0, [{"pod": "two", "namespace": "ml", "container": "c"}])
    ex.set_device_owners(1, [{"pod": "two", "namespace": "ml", "container": "c"}])
    sc = Scraper("127.0.0.1", ex.port)
    fp = FakeProm()
    url = fp.start()
    try:
        stamps = []
        t0 = time.time()
        for k in range(18):  # every 0.25 s for 4.25 s
            time.sleep(max(0.0, t0 + 0.25 * k - time.time()))
            ts = time.time()
            fp.ingest(parse_text(sc.get()), ts)
            stamps.append(ts)
        end, window, step = stamps[-1], 3, 1
        kwh = G.pod_energy_kwh(PromClient(url), end - window, end, step)
        assert list(kwh) == [("node-a", "ml", "two")]

        def joules_at(t):  # both GPUs' counters, linear between scrapes
            tot = 0.0
            for key, pts in fp.series[G.ENERGY_METRIC].items():
                for (ta, va), (tb, vb) in zip(pts, pts[1:]):
                    if ta <= t <= tb:
                        tot += va + (vb - va) * (t - ta) / (tb - ta)
            return tot
        # the range query runs on whole seconds (to_unix, like the reference): compare over
        # the same window, so an energy transient near the first scrapes cannot sit in one
        # window and not the other
        e_int = float(int(end))
        want = joules_at(e_int) - joules_at(e_int - window)
        gaps = [round(b - a, 3) for a, b in zip(stamps, stamps[1:])]
        assert want > 0 and kwh[("node-a", "ml", "two")] * 3.6e6 == pytest.approx(want, rel=0.05), \
            {"got_j": kwh[("node-a", "ml", "two")] * 3.6e6, "want_j": want, "end": end, "scrape_gaps_s": gaps}
        rows = G.add_energy([["node-a", "ml", "two", 2, 60.0], ["node-a", "ml", "gone (finished)", 0, 0.0]], kwh)
        assert rows[0][5] == kwh[("node-a", "ml", "two")] and rows[1][5] == 0.0
        table = G.format_rows(rows, "pod", "table", compat=False, extras=["Energy kWh"])
        assert "Energy kWh" in table and "TOTAL" in table
    finally:
        fp.stop()


def test_shared_gpu_pods_billed_by_own_compute_share(mock_exporter):
    """two pods share GPU 0; their processes hold 60 % and 0 % of its CUs.
    container_gpu_busy_seconds_total bills each the whole GPU's busy time;
    container_gpu_cu_seconds_total bills each its own processes' CU-occupancy share
    (reference per-pod accounting: gpu_util_stats.py:62-94)."""
    ex = mock_exporter(n_gpus=1, hz=100, proc_period_s=0.05, link_every=0,
                       mock={"util_base": 70, "util_amp": 1e-4, "fw_period_s": 0.005, "proc_cu_share": [0.6, 0.0]})
    ex.set_device_owners(0, [{"pod": "big", "namespace": "ml", "container": "c"},
                             {"pod": "idle", "namespace": "dev", "container": "c"}])
    # mock PIDs 100000 + 10·gpu + k: process 0 → big, process 1 → idle
    ex.set_pid_owners({(0, 100000): {"pod": "big", "namespace": "ml", "container": "c"},
                       (0, 100001): {"pod": "idle", "namespace": "dev", "container": "c"}})
    time.sleep(0.3)

    def per_pod(m, fam):
        return {lb["pod_name"]: v for lb, v in m[fam]}

    m0, t0 = parse_text(ex.render()), time.time()
    time.sleep(1.5)
    m1, dt = parse_text(ex.render()), time.time() - t0
    cu = {p: 100 * (per_pod(m1, "container_gpu_cu_seconds_total")[p] - per_pod(m0, "container_gpu_cu_seconds_total")[p]) / dt
          for p in ("big", "idle")}
    busy = {p: 100 * (per_pod(m1, "container_gpu_busy_seconds_total")[p] -
                      per_pod(m0, "container_gpu_busy_seconds_total")[p]) / dt for p in ("big", "idle")}
    assert cu["big"] == pytest.approx(60, abs=4) and cu["idle"] == pytest.approx(0, abs=0.5), cu
    assert busy["big"] == pytest.approx(70, abs=4) and busy["idle"] == pytest.approx(70, abs=4), busy  # whole GPU each
    # The pod's integral keeps its exited processes' share: drop the PID table entry
    # (process gone) and the counter holds its value.
    before = per_pod(parse_text(ex.render()), "container_gpu_cu_seconds_total")["big"]
    ex.set_pid_owners({})
    time.sleep(0.3)
    after = per_pod(parse_text(ex.render()), "container_gpu_cu_seconds_total")["big"]
    assert after >= before > 0.5


def test_report_util_metric_cu_seconds_splits_a_shared_gpu(mock_exporter):
    """`gpu-util-stats --util-metric container_gpu_cu_seconds_total`: per-pod util from
    the pods' own compute share on a shared GPU (60 / 0) instead of 70 / 70."""
    ex = mock_exporter(n_gpus=1, hz=100, proc_period_s=0.05, link_every=0, node_name="node-a",
                       mock={"util_base": 70, "util_amp": 1e-4, "fw_period_s": 0.005, "proc_cu_share": [0.6, 0.0]})
    owners = [{"pod": "big", "namespace": "ml", "container": "c"}, {"pod": "idle", "namespace": "dev", "container": "c"}]
    ex.set_device_owners(0, owners)
    ex.set_pid_owners({(0, 100000): owners[0], (0, 100001): owners[1]})
    sc = Scraper("127.0.0.1", ex.port)
    fp = FakeProm()
    url = fp.start()
    try:
        time.sleep(0.2)
        stamps = []
        t0 = time.time()
        for k in range(22):
            time.sleep(max(0.0, t0 + 0.25 * k - time.time()))
            ts = time.time()
            fp.ingest(parse_text(sc.get()), ts)
            stamps.append(ts)
        end = stamps[-1]
        for metric, want in (("container_gpu_cu_seconds_total", {"big": 60, "idle": 0}),
                             ("container_gpu_busy_seconds_total", {"big": 70, "idle": 70})):
            q = G.Queries.amd("", 2, util_metric=metric)
            fp.add_instant(q.total, [{"metric": {"node": "node-a", q.type_label: "MI355X"}, "value": [end, "1"]}])
            fp.add_instant(q.used, [{"metric": {"node": "node-a"}, "value": [end, "1"]}])
            fp.add_instant(q.live, [{"metric": {"namespace": o["namespace"], "pod": o["pod"]}, "value": [end, "1"]}
                                    for o in owners])
            fp.add_range(q.req, [{"metric": {"node": "node-a", "namespace": o["namespace"], "pod": o["pod"]},
                                  "values": [[end, "1"]]} for o in owners])
            # 2 s rate() steps: the per-process tier books CU-seconds at each 50 ms read,
            # so a 1 s step on a loaded test host is off by the read jitter
            rows = G.run_report(PromClient(url), q, end, 2, 2, compat=False)
            got = {r[2]: r[4] for r in rows}
            assert got["big"] == pytest.approx(want["big"], abs=5) and got["idle"] == pytest.approx(want["idle"], abs=5), \
                (metric, rows)
    finally:
        fp.stop()


def test_partitions_split_socket_energy(N):
    """compute partitions read one socket energy accumulator.  Each partition
    is billed its XCCs' share of the chip's GFX busy, so the partitions' energy adds up
    to the socket's instead of counting it once per partition."""
    cfg = {"backend": "mock", "hz": 200, "port": -1, "pin_numa": False, "proc_every": 0, "link_every": 0,
           "mock": {"n_gpus": 1, "compute_partition": "CPX", "fw_period_s": 0.005, "util_base": 50, "util_amp": 40,
                    "util_period_s": 0.5}}
    cpx = N.Exporter(cfg)
    cpx.start()
    try:
        time.sleep(0.3)
        e0 = [cpx.integrals(d)["energy_joules"] for d in range(8)]
        b0 = [cpx.integrals(d)["gfx_busy_seconds"] for d in range(8)]
        time.sleep(1.2)
        e1 = [cpx.integrals(d)["energy_joules"] for d in range(8)]
        b1 = [cpx.integrals(d)["gfx_busy_seconds"] for d in range(8)]
        parts = [b - a for a, b in zip(e0, e1)]
        # the socket draws 200 W + 8 W per % of chip busy ≈ 600 W here: 1.2 s ≈ 720 J in total
        assert 500 < sum(parts) < 950, parts
        socket_w = sum(parts) / 1.2
        chip = cpx.snapshot(0)
        assert socket_w == pytest.approx(chip["power_w"], rel=0.35)
        # each partition's share follows its XCC's busy share (the mock's XCC curves differ in phase)
        busy = [b - a for a, b in zip(b0, b1)]
        share_e = [p / sum(parts) for p in parts]
        share_b = [x / sum(busy) for x in busy]
        for se, sb in zip(share_e, share_b):
            assert se == pytest.approx(sb, abs=0.03)
        assert max(parts) < 0.5 * sum(parts)  # no partition is billed the whole socket
    finally:
        cpx.stop()


def test_sm_util_auto_does_not_count_the_exporters_reads(mock_exporter):
    """at kHz counter rates the PMFW GFX busy counts every counter READ
    as ≈80 µs of work, so a bursty GPU read ≈100 % (modelled here by the mock's
    pmfw_busy_floor 99).  The default --sm-util-source auto bills the pod the counter
    tier's GPU-active while that tier runs — the true 25 % duty of a square load — and
    falls back to the PMFW busy when the counters are handed over, without the
    per-pod counter ever running backwards."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", window_s=0.8, pmc_idle_hz=0,
                       mock={"square_duty": 0.25, "util_base": 50, "util_amp": 50, "util_period_s": 0.2,
                             "pmfw_busy_floor": 99})
    ex.set_device_owners(0, [{"pod": "p", "namespace": "n", "container": "c"}])
    one = lambda m, f, **kw: [v for lb, v in m[f] if all(lb.get(k) == w for k, w in kw.items())][0]  # noqa: E731

    def window(secs):
        m0 = parse_text(ex.render())
        time.sleep(secs)
        m1 = parse_text(ex.render())
        d = lambda f, **kw: one(m1, f, **kw) - one(m0, f, **kw)  # noqa: E731
        dt = d("kgs_sampled_seconds_total")
        return m1, {"busy": 100 * d("container_gpu_busy_seconds_total") / dt,
                    "gfx": 100 * d("amdgpu_gfx_busy_seconds_total") / dt,
                    "pmfw": 100 * d("amdgpu_pmfw_gfx_busy_seconds_total") / dt,
                    "from_counters": d("kgs_util_source_seconds_total", source="counters") / dt,
                    "pod_busy": one(m1, "container_gpu_busy_seconds_total")}

    time.sleep(0.3)
    m, on = window(1.6)
    assert on["busy"] == pytest.approx(25, abs=3) and on["gfx"] == pytest.approx(25, abs=3), on
    assert on["pmfw"] > 98 and on["from_counters"] > 0.95, on
    assert one(m, "container_gpu_sm_util") == pytest.approx(25, abs=6)
    ex.set_pmc_enabled(False)                     # counters handed over: PMFW is all there is
    time.sleep(0.3)
    _, off = window(1.0)
    assert off["busy"] > 98 and off["from_counters"] < 0.05, off
    ex.set_pmc_enabled(True)
    time.sleep(0.3)
    _, back = window(1.6)
    assert back["busy"] == pytest.approx(25, abs=3) and back["from_counters"] > 0.95, back
    assert on["pod_busy"] <= off["pod_busy"] <= back["pod_busy"]


def test_sm_util_pmfw_source_keeps_the_firmware_busy(mock_exporter):
    """--sm-util-source pmfw: the reference-contract series is the PMFW GFX busy,
    READs included (the mock's floor), exactly as before round 4."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", window_s=0.8, pmc_idle_hz=0, sm_util_source="pmfw",
                       mock={"square_duty": 0.25, "util_base": 50, "util_amp": 50, "util_period_s": 0.2,
                             "pmfw_busy_floor": 99})
    ex.set_device_owners(0, [{"pod": "p", "namespace": "n", "container": "c"}])
    time.sleep(1.2)
    m = parse_text(ex.render())
    (_, sm), = m["container_gpu_sm_util"]
    assert sm > 98


def test_dispatch_busy_learns_and_removes_the_reads_cp_time(mock_exporter):
    """The dispatch-in-flight integral behind --sm-util-source auto: CPC busy counts a
    dispatch in flight and, for a short fixed time, every counter READ packet (the
    mock: 20 µs per READ, 4 % of the time at 2 kHz).  The sampler learns that time on
    intervals without waves (kgs_pmc_read_cp_seconds) and subtracts it, so a 25 %-duty
    square load integrates to 25 %, not 29-ish."""
    ex = mock_exporter(n_gpus=1, hz=2000, pmc_source="mock", pmc_idle_hz=0, window_s=1.0,
                       mock={"square_duty": 0.25, "util_base": 50, "util_amp": 50, "util_period_s": 0.2},
                       mock_pmc={"cpc_read_us": 20.0})
    time.sleep(0.5)
    a, t0 = ex.integrals(0), time.time()
    time.sleep(1.6)
    b, dt = ex.integrals(0), time.time() - t0
    assert b["dispatch_drains"] > 1000
    assert (b["dispatch_seconds"] - a["dispatch_seconds"]) / dt == pytest.approx(0.25, abs=0.02)
    m = parse_text(ex.render())
    (_, cp), = m["kgs_pmc_read_cp_seconds"]
    assert cp == pytest.approx(20e-6, rel=0.1)
    raw = {lb["counter"]: v for lb, v in m["amdgpu_pmc_total"]}
    assert raw["CPC_CPC_STAT_BUSY"] > raw["GRBM_SPI_BUSY"]  # the READs' own CP time is in the raw count


def test_unreadable_cu_occupancy_is_withheld_not_billed_zero(mock_exporter):
    """a process whose CU occupancy cannot be read (its KFD stats gone —
    AMD SMI printed "Unable to open queues directory" and reported 0) used to bill its
    pod 0 CU-seconds, indistinguishable from "no compute".  Now: nothing is integrated
    for it, its amdgpu_process_cu_occupancy line is withheld, kgs_process_cu_unavailable
    counts it, and a pod whose processes are all unreadable gets no
    container_gpu_cu_seconds_total line (the other pod on the GPU keeps its own)."""
    ex = mock_exporter(n_gpus=1, hz=100, proc_period_s=0.05, link_every=0,
                       mock={"util_base": 70, "util_amp": 1e-4, "proc_cu_share": [0.6, 0.3], "proc_cu_fail": 0})
    ex.set_device_owners(0, [{"pod": "lost", "namespace": "ml", "container": "c"},
                             {"pod": "seen", "namespace": "dev", "container": "c"}])
    ex.set_pid_owners({(0, 100000): {"pod": "lost", "namespace": "ml", "container": "c"},
                       (0, 100001): {"pod": "seen", "namespace": "dev", "container": "c"}})
    time.sleep(0.6)
    m = parse_text(ex.render())
    cu = {lb["pod_name"]: v for lb, v in m["container_gpu_cu_seconds_total"]}
    assert "lost" not in cu and cu["seen"] > 0.05, cu
    occ = {lb["pid"]: v for lb, v in m["amdgpu_process_cu_occupancy"]}
    assert occ == {"100001": pytest.approx(0.3 * 256, abs=1)}, occ
    assert [v for lb, v in m["kgs_process_cu_unavailable"]] == [1.0]
    procs = {p["pid"]: p for p in ex.procs(0)}
    assert procs[100000]["cu_valid"] is False and procs[100000]["cu_seconds"] == 0.0
    assert procs[100001]["cu_valid"] is True and procs[100001]["cu_seconds"] > 0.05


def test_kfd_sysfs_process_reader(N, tmp_path):
    """The KFD-sysfs process reader (native/src/kfd_procs.cpp) on a fake tree laid out as
    MI355X's (profiles/r6/r6b/kfd_proc.json): processes on this GPU only (vram_<gpu_id>),
    CU occupancy from stats_<gpu_id>/ (unreadable → cu_valid False, not 0), the name from
    /proc/<pid>/comm, GTT / CPU bytes and gfx ns from the fdinfo of this GPU's DRM client
    (dup'd fds counted once)."""
    import os as _os

    kfd, proc = tmp_path / "kfd", tmp_path / "proc"
    gid, other = 36622, 23660

    def kproc(pid, gpu, vram, cu=None, evicted=0):
        d = kfd / str(pid)
        d.mkdir(parents=True, exist_ok=True)
        (d / f"vram_{gpu}").write_text(f"{vram}\n")
        if cu is not None:
            (d / f"stats_{gpu}").mkdir()
            (d / f"stats_{gpu}" / "cu_occupancy").write_text(f"{cu}\n")
            (d / f"stats_{gpu}" / "evicted_ms").write_text(f"{evicted}\n")

    kproc(101, gid, 534769664, cu=128, evicted=7)   # a tenant on our GPU
    kproc(102, gid, 0, cu=None)                      # tearing down: stats gone
    kproc(103, other, 1 << 30, cu=64)                # another GPU's tenant
    (kfd / "not-a-pid").mkdir()
    p101 = proc / "101"
    (p101 / "fd").mkdir(parents=True)
    (p101 / "fdinfo").mkdir()
    (p101 / "comm").write_text("python3\n")
    for fd in ("5", "9"):  # a dup'd render-node fd: one DRM client
        _os.symlink("/dev/dri/renderD128", p101 / "fd" / fd)
        (p101 / "fdinfo" / fd).write_text("pos:\t0\ndrm-driver:\tamdgpu\ndrm-client-id:\t9\ndrm-pdev:\t0000:75:00.0\n"
                                          "drm-memory-vram:\t1464 KiB\ndrm-memory-gtt: \t6896 KiB\n"
                                          "drm-memory-cpu: \t2 MiB\ndrm-engine-gfx:\t15483 ns\n")
    _os.symlink("/dev/dri/renderD136", p101 / "fd" / "11")  # another GPU's render node
    (p101 / "fdinfo" / "11").write_text("drm-client-id:\t12\ndrm-pdev:\t0000:05:00.0\ndrm-memory-gtt:\t99 KiB\n")
    _os.symlink("/tmp/log.txt", p101 / "fd" / "1")
    got = {p["pid"]: p for p in N.read_kfd_procs(str(kfd), str(proc), gid, "0000:75:00.0")}
    assert set(got) == {101, 102}
    a, b = got[101], got[102]
    assert a["vram_bytes"] == 534769664 and a["cu_occupancy"] == 128 and a["cu_valid"] and a["evicted_ms"] == 7
    assert a["name"] == "python3" and a["gtt_bytes"] == 6896 << 10 and a["cpu_bytes"] == 2 << 20
    assert a["gfx_ns"] == 15483
    assert b["cu_valid"] is False and b["cu_occupancy"] == 0 and b["name"] == "" and b["gtt_bytes"] == 0
    assert N.read_kfd_procs(str(tmp_path / "absent"), str(proc), gid, "0000:75:00.0") is None


def test_kfd_reader_walks_a_process_fd_directory_at_most_every_10s(N, tmp_path):
    """A process holding thousands of fds cost the per-process tier one readlink each per
    poll (5.6 ms at 2000 fds).  With the slow thread's DrmFdCache the /proc/<pid>/fd walk
    repeats only every DRM_RESCAN_S; in between the remembered DRM fds' fdinfo are read
    (values still current), a remembered fd that stopped being a DRM link forces a walk,
    and a process that left the GPU is forgotten."""
    import os as _os

    kfd, proc = tmp_path / "kfd", tmp_path / "proc"
    gid = 7
    (kfd / "201").mkdir(parents=True)
    (kfd / "201" / f"vram_{gid}").write_text("4096\n")
    p = proc / "201"
    (p / "fd").mkdir(parents=True)
    (p / "fdinfo").mkdir()
    for i in range(50):
        _os.symlink("/tmp/data.bin", p / "fd" / str(100 + i))
    _os.symlink("/dev/dri/renderD128", p / "fd" / "5")

    def info(ns):
        (p / "fdinfo" / "5").write_text(f"drm-client-id:\t3\ndrm-pdev:\t0000:75:00.0\ndrm-engine-gfx:\t{ns} ns\n")

    info(100)
    c = N.DrmFdCache()
    read = lambda t: N.read_kfd_procs(str(kfd), str(proc), gid, "0000:75:00.0", c, t)[0]  # noqa: E731
    assert read(1.0)["gfx_ns"] == 100 and c.walks == 1
    info(250)
    assert read(2.0)["gfx_ns"] == 250 and c.walks == 1          # fdinfo re-read, no walk
    assert read(1.0 + N.DRM_RESCAN_S)["gfx_ns"] == 250 and c.walks == 2  # the periodic walk
    (p / "fd" / "5").unlink()                                     # fd 5 closed and reused for a file
    _os.symlink("/tmp/other.bin", p / "fd" / "5")
    _os.symlink("/dev/dri/renderD128", p / "fd" / "7")
    (p / "fdinfo" / "7").write_text("drm-client-id:\t4\ndrm-pdev:\t0000:75:00.0\ndrm-engine-gfx:\t9 ns\n")
    assert read(12.0)["gfx_ns"] == 9 and c.walks == 3              # stale entry: walked again at once
    (kfd / "201" / f"vram_{gid}").unlink()                         # the process left this GPU
    assert N.read_kfd_procs(str(kfd), str(proc), gid, "0000:75:00.0", c, 13.0) == [] and c.pids == 0
