"""Exporter on the mock N-GPU provider (BASELINE.json config 1): sampling tiers,
exact integrals, Prometheus exposition, HTTP endpoints, fault isolation."""
import http.client
import json
import math
import os
import time
import urllib.error
import urllib.request

import pytest
from prometheus_client.parser import text_string_to_metric_families

from kube_gpu_stats_amd.utils.scrape import parse_text

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def get(port, path):
    return urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5)


def test_distinct_samples_follow_firmware_cadence(mock_exporter):
    ex = mock_exporter(hz=200, pmfw_hz=0, mock={"fw_period_s": 0.02})
    time.sleep(1.0)
    I = ex.integrals(0)
    # 200 reads/s but only ~50 distinct PMFW tables/s
    assert 150 <= I["reads"] <= 260
    assert 40 <= I["distinct_samples"] <= 60
    s = ex.samples(0, 10)
    seqs = [x["seq"] for x in s]
    assert seqs == sorted(seqs) and len(set(x["fw_ts"] for x in s)) == len(s)


def test_integral_matches_analytic_mean(mock_exporter):
    ex = mock_exporter(hz=100, mock={"util_base": 50, "util_amp": 40, "util_period_s": 2.0, "fw_period_s": 0.01})
    time.sleep(2.2)
    I = ex.integrals(1)
    # over ~one full period the sine averages out → ~50 % busy
    mean = I["gfx_busy_seconds"] / I["sampled_seconds"]
    assert I["sampled_seconds"] > 1.8
    assert abs(mean - 0.5) < 0.12
    w = ex.window(1, 0.2)
    snap = ex.snapshot(1)
    assert abs(w["gfx_busy_pct"] - snap["gfx_busy_pct"]) < 25
    assert I["energy_joules"] > 0


def test_prometheus_exposition_is_valid(mock_exporter):
    ex = mock_exporter(n_gpus=2, pmc_source="mock", proc_every=1, link_every=1)
    ex.set_device_owners(0, [{"pod": "train-0", "namespace": "ml", "container": "main"}])
    ex.set_pid_owners({(0, 100000): {"pod": "train-0", "namespace": "ml", "container": "main", "pod_uid": "u-1"}})
    time.sleep(0.5)
    body = ex.render()
    fams = {f.name: f for f in text_string_to_metric_families(body)}
    for name in ["container_gpu_sm_util", "amdgpu_gfx_busy_percent", "amdgpu_hbm_used_bytes", "amdgpu_power_watts",
                 "amdgpu_temperature_celsius", "amdgpu_energy_joules", "amdgpu_xgmi_read_bytes",
                 "amdgpu_mfma_util_percent", "amdgpu_vmem_busy_percent", "amdgpu_process_hbm_bytes",
                 "kgs_samples", "kgs_sample_read_seconds", "amdgpu_topology_link", "amdgpu_device_info"]:
        assert name in fams, name
    compat = fams["container_gpu_sm_util"].samples
    assert len(compat) == 1  # only GPU 0 is allocated
    lb = compat[0].labels
    assert lb["kubernetes_io_hostname"] == "node-a" and lb["nvidia_gpu_type"] == "MI355X"
    assert lb["pod_name"] == "train-0" and lb["namespace"] == "ml" and lb["gpu"] == "0"
    procs = [s for s in fams["amdgpu_process_hbm_bytes"].samples if s.labels["pid"] == "100000"]
    assert procs and procs[0].labels["pod"] == "train-0" and procs[0].labels["pod_uid"] == "u-1"
    hist = [s for s in fams["kgs_sample_read_seconds"].samples if s.name.endswith("_count")]
    assert len(hist) == 2 and all(s.value > 0 for s in hist)
    m = parse_text(body)
    mfma = [v for _, v in m["amdgpu_mfma_util_percent"]]
    assert all(abs(v - 60.0) < 1 for v in mfma)  # mock mfma_frac 0.6


def test_unallocated_compat_and_owner_removal(mock_exporter):
    ex = mock_exporter(n_gpus=2, compat_unallocated=True)
    time.sleep(0.3)
    m = parse_text(ex.render())
    assert {lb["pod_name"] for lb, _ in m["container_gpu_sm_util"]} == {""}
    ex.set_device_owners(1, [{"pod": "a", "namespace": "x"}, {"pod": "b", "namespace": "x"}])
    m = parse_text(ex.render())
    assert sorted(lb["pod_name"] for lb, _ in m["container_gpu_sm_util"]) == ["", "a", "b"]
    ex.set_device_owners(1, [])
    m = parse_text(ex.render())
    assert len(m["container_gpu_sm_util"]) == 2


def test_http_endpoints_keepalive_and_errors(mock_exporter):
    ex = mock_exporter(n_gpus=3, link_every=1)
    time.sleep(0.3)
    c = http.client.HTTPConnection("127.0.0.1", ex.port, timeout=5)
    for _ in range(5):  # keep-alive: same connection
        c.request("GET", "/metrics")
        r = c.getresponse()
        assert r.status == 200 and r.getheader("Content-Type").startswith("text/plain; version=0.0.4")
        assert b"kgs_up" in r.read()
    c.request("HEAD", "/metrics")
    r = c.getresponse()
    assert r.status == 200 and r.read() == b""
    c.request("GET", "/nope")
    r = c.getresponse()
    assert r.status == 404
    r.read()
    c.close()
    assert get(ex.port, "/healthz").status == 200
    topo = json.load(get(ex.port, "/topology"))
    assert len(topo["devices"]) == 3 and len(topo["edges"]) == 6
    assert all(e["link_type"] == 2 for e in topo["edges"])
    devs = json.load(get(ex.port, "/devices"))
    assert devs[0]["gfx_target"] == "gfx950"
    samples = json.load(get(ex.port, "/samples?gpu=2&n=5"))
    assert 1 <= len(samples) <= 5 and samples[-1]["seq"] >= samples[0]["seq"]
    assert ex.stats()["http_requests"] >= 10


def test_fault_isolation_vanishing_device(mock_exporter):
    ex = mock_exporter(n_gpus=3, hz=200, max_backoff_ms=50, mock={"vanish_dev": 1, "vanish_after_s": 0.2,
                                                                  "fail_rate": 0.05})
    time.sleep(0.8)
    ups = {lb["gpu"]: v for lb, v in parse_text(ex.render())["kgs_up"]}
    assert ups == {"0": 1.0, "1": 0.0, "2": 1.0}
    assert ex.healthy()
    I0, I1 = ex.integrals(0), ex.integrals(1)
    assert I0["read_errors"] > 0 and I0["up"] == 1  # transient errors do not take a device down
    assert I1["reads"] < I0["reads"] / 2             # failing device backs off
    age = {lb["gpu"]: v for lb, v in parse_text(ex.render())["kgs_last_sample_age_seconds"]}
    assert age["1"] > 0.3 and age["0"] < 0.1


def test_device_recovers_after_reset(mock_exporter):
    """A GPU that drops out (reset) comes back once the backend re-opens it; its
    firmware clock and accumulators restart at zero, and the sampler re-baselines
    instead of reading a wrap: counters stay monotonic, the window stays sane."""
    ex = mock_exporter(n_gpus=2, hz=200, max_backoff_ms=40,
                       mock={"vanish_dev": 1, "vanish_after_s": 0.3, "vanish_for_s": 0.3, "util_amp": 0.0001,
                             "util_base": 60, "fw_period_s": 0.01})
    time.sleep(0.25)
    e0 = ex.integrals(1)["energy_joules"]
    busy0 = ex.integrals(1)["gfx_busy_seconds"]
    time.sleep(0.2)
    assert ex.integrals(1)["up"] == 0
    time.sleep(0.8)
    I = ex.integrals(1)
    assert I["up"] == 1 and I["recoveries"] == 1 and I["recover_attempts"] >= 1, I
    assert I["energy_joules"] > e0 and I["gfx_busy_seconds"] > busy0
    w = ex.window(1, 0.2)
    assert w["gfx_busy_pct"] == pytest.approx(60, abs=2), w
    m = parse_text(ex.render())
    rec = {lb["gpu"]: v for lb, v in m["kgs_device_recoveries_total"]}
    assert rec == {"0": 0.0, "1": 1.0}


def test_process_cu_seconds_integral(mock_exporter):
    ex = mock_exporter(n_gpus=2, hz=100, proc_every=2)
    time.sleep(0.2)
    a = {p["pid"]: p["cu_seconds"] for p in ex.procs(1)}
    time.sleep(1.0)
    b = {p["pid"]: p["cu_seconds"] for p in ex.procs(1)}
    # mock processes occupy 128 of 256 CUs → half a CU-share-second per second
    for pid in b:
        assert (b[pid] - a[pid]) == pytest.approx(0.5, abs=0.06)


def test_energy_counter_survives_accumulator_wrap(mock_exporter):
    # accumulator wraps every ~0.4 J·2^16 units → many wraps per second
    ex = mock_exporter(n_gpus=1, hz=100, mock={"energy_wrap_at": 1 << 26, "fw_period_s": 0.01})
    vals = []
    for _ in range(5):
        time.sleep(0.2)
        vals.append(ex.integrals(0)["energy_joules"])
    assert vals == sorted(vals) and vals[-1] > vals[0]


def test_bdf_filter_samples_subset(N):
    ex = N.Exporter({"backend": "mock", "mock": {"n_gpus": 4}, "port": -1, "hz": 100, "pin_numa": False,
                     "bdfs": ["0000:21:00.0", "0000:41:00.0"]})
    ex.start()
    time.sleep(0.3)
    body = ex.render()
    ex.stop()
    gpus = {lb["gpu"] for lb, _ in parse_text(body)["kgs_samples_total"]}
    assert gpus == {"1", "3"}
    with pytest.raises(RuntimeError):
        N.Exporter({"backend": "mock", "port": -1, "bdfs": ["ffff:00:00.0"]})


def test_unknown_backend_and_pmc_errors(N):
    with pytest.raises(RuntimeError, match="unknown backend"):
        N.Exporter({"backend": "nvml"})
    with pytest.raises(RuntimeError, match="unknown pmc_source"):
        N.Exporter({"backend": "mock", "pmc_source": "dcgm"})
    ex = N.Exporter({"backend": "mock", "port": -1, "pmc_source": "rocprofiler", "pmc_lib": "/nonexistent.so"})
    assert ex.pmc_name == "none" and "dlopen" in ex.pmc_error


def test_render_latency_8_gpus(mock_exporter):
    ex = mock_exporter(n_gpus=8, hz=100, pmc_source="mock", proc_every=10, link_every=10)
    time.sleep(0.5)
    for _ in range(20):
        ex.render()
    st = ex.stats()
    mean_ms = st["render_ns_total"] / st["scrapes"] / 1e6
    assert mean_ms < 20, mean_ms  # generous for CI; bench reports the real p50
    assert not math.isnan(mean_ms)


def test_counter_stream_endpoint_is_gapless(mock_exporter):
    """/counters: full-rate counter drains, oldest first; polling with ``since``
    returns every drain exactly once (no gaps, no repeats) while the ring holds it."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0,
                       mock={"util_base": 50, "util_amp": 0.0001})
    time.sleep(0.3)
    body = json.load(get(ex.port, "/counters?gpu=0&n=50"))
    assert body["counters"][:3] == ["GRBM_COUNT", "GRBM_SPI_BUSY", "SQ_VALU_MFMA_BUSY_CYCLES"]
    s = body["samples"]
    assert len(s) == 50
    seqs = [x["seq"] for x in s]
    assert seqs == list(range(seqs[0], seqs[0] + 50))
    assert all("mfma_util_pct" in x for x in s)  # the extra base sample gives the first one its rates
    # mock: 50 % busy, MFMA busy 60 % of active time
    assert abs(sum(x["gpu_active_pct"] for x in s) / len(s) - 50) < 5
    assert abs(sum(x["mfma_util_pct"] for x in s) / len(s) - 60) < 6
    assert all(0 < x["dt_us"] < 100000 for x in s)  # ≈1000 µs; overrun catch-up ticks come sooner
    last = seqs[-1]
    got = []
    for _ in range(5):
        time.sleep(0.1)
        b = json.load(get(ex.port, f"/counters?gpu=0&since={last}"))
        new = [x["seq"] for x in b["samples"]]
        if new:
            assert new[0] == last + 1, (last, new[:3])
            last = new[-1]
        got += new
    assert got == list(range(seqs[-1] + 1, last + 1)) and len(got) > 300
    assert json.load(get(ex.port, "/counters?gpu=7"))["samples"] == []


def test_counter_window_covers_full_window_at_high_rate(mock_exporter):
    """At 8 kHz the 1024-deep full-rate ring spans 128 ms; the window gauges use the
    decimated ring, so a 1 s window really covers ≈1 s."""
    ex = mock_exporter(n_gpus=1, hz=8000, pmc_source="mock", proc_every=0, link_every=0, window_s=1.0)
    time.sleep(1.5)
    w = ex.window(0, 1.0)
    assert 0.95 <= w["pmc_dt_s"] <= 1.05, w
    w = ex.window(0, 0.2)
    assert 0.19 <= w["pmc_dt_s"] <= 0.21, w


def test_pmc_counter_sets(N, mock_exporter):
    """base set (default): GRBM clocks + SPI busy + MFMA busy + CPC busy (the dispatch-in-flight
    signal, round 4) — no TA, so no vmem gauge; full adds TA."""
    base = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0)
    full = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0, pmc_set="full")
    time.sleep(0.4)
    mb, mf = parse_text(base.render()), parse_text(full.render())
    assert {lb["counter"] for lb, _ in mb["amdgpu_pmc_total"]} == {"GRBM_COUNT", "GRBM_SPI_BUSY",
                                                                   "SQ_VALU_MFMA_BUSY_CYCLES", "CPC_CPC_STAT_BUSY"}
    assert "TA_TA_BUSY" in {lb["counter"] for lb, _ in mf["amdgpu_pmc_total"]}
    assert "amdgpu_vmem_busy_percent" not in mb and abs(mf["amdgpu_vmem_busy_percent"][0][1] - 30) < 3
    assert abs(mb["amdgpu_mfma_util_percent"][0][1] - 60) < 3
    assert "vmem_busy_pct" not in base.window(0, 0.2) and "vmem_busy_pct" in full.window(0, 0.2)
    s = json.load(get(base.port, "/counters?gpu=0&n=2"))["samples"][-1]
    assert s["v"][3] is None and "vmem_busy_pct" not in s
    with pytest.raises(RuntimeError, match="unknown pmc_set"):
        N.Exporter({"backend": "mock", "pmc_source": "mock", "pmc_set": "everything"})


def test_per_xcd_counter_breakdown(mock_exporter):
    """Per-XCD GUI-active and MFMA busy: XCD x of the mock is active (1 - 0.05·x) of
    XCD 0's cycles and holds that share of the MFMA cycles, so its MFMA busy per
    active SIMD cycle is 0.6 · 8 / Σ(1 - 0.05·x) for every x."""
    ex = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0,
                       mock={"util_base": 50, "util_amp": 0.0001}, mock_pmc={"xcd_skew": 0.05})
    time.sleep(0.5)
    w = ex.window(0, 0.3)
    wsum = sum(1 - 0.05 * x for x in range(8))
    assert len(w["xcd_active_pct"]) == 8
    for x in range(8):
        assert w["xcd_active_pct"][x] == pytest.approx(50 * (1 - 0.05 * x), abs=2.5)
        assert w["xcd_mfma_util_pct"][x] == pytest.approx(100 * 0.6 * 8 / wsum, abs=3)
    m = parse_text(ex.render())
    got = {lb["xcc"]: v for lb, v in m["amdgpu_mfma_util_xcc_percent"]}
    assert sorted(got) == [str(x) for x in range(8)]
    assert {lb["xcc"] for lb, _ in m["amdgpu_gpu_active_xcc_percent"]} == set(got)
    p = ex.pmc(0)
    assert len(p["xcd_mfma"]) == 8 and sum(p["xcd_mfma"]) <= p["values"]["SQ_VALU_MFMA_BUSY_CYCLES"]
    s = json.load(get(ex.port, "/counters?gpu=0&n=2"))["samples"][-1]
    assert len(s["xcd_mfma_util_pct"]) == 8
    # a reader without the breakdown emits no per-XCD families
    flat = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0, mock_pmc={"n_xcd": 0})
    time.sleep(0.3)
    mf = parse_text(flat.render())
    assert "amdgpu_mfma_util_xcc_percent" not in mf and "amdgpu_mfma_util_percent" in mf
    assert "xcd_mfma_util_pct" not in flat.window(0, 0.2)


def test_per_pod_mfma_series_follows_compat_labels(mock_exporter):
    """container_gpu_mfma_util: the counter tier's MFMA busy under the reference
    series' labels, so the per-pod report can run on it unchanged."""
    ex = mock_exporter(n_gpus=2, hz=500, pmc_source="mock", proc_every=0, link_every=0, compat_unallocated=True,
                       mock={"util_base": 50, "util_amp": 0.0001})
    ex.set_device_owners(0, [{"pod": "train-0", "namespace": "ml", "container": "main"}])
    time.sleep(0.4)
    m = parse_text(ex.render())
    sm = {lb["gpu"]: lb for lb, _ in m["container_gpu_sm_util"]}
    mf = {lb["gpu"]: (lb, v) for lb, v in m["container_gpu_mfma_util"]}
    assert set(mf) == set(sm) == {"0", "1"}
    assert mf["0"][0] == sm["0"] and mf["0"][0]["pod_name"] == "train-0"
    assert mf["0"][1] == pytest.approx(60, abs=3)  # mock: MFMA busy 60 % of active cycles
    plain = mock_exporter(n_gpus=1, hz=100, proc_every=0, link_every=0, compat_unallocated=True)
    time.sleep(0.3)
    assert "container_gpu_mfma_util" not in parse_text(plain.render())  # no counter tier, no series


def test_metrics_gzip_negotiation(mock_exporter):
    """--gzip-level: gzip only for clients that send Accept-Encoding: gzip; the
    decompressed page is a normal exposition.  Off by default."""
    import gzip

    ex = mock_exporter(n_gpus=2, hz=100, gzip_level=1)
    off = mock_exporter(n_gpus=1, hz=100)
    time.sleep(0.3)
    c = http.client.HTTPConnection("127.0.0.1", ex.port, timeout=5)
    for _ in range(2):  # keep-alive, deflate state reused
        c.request("GET", "/metrics", headers={"Accept-Encoding": "gzip, deflate"})
        r = c.getresponse()
        raw = r.read()
        assert r.getheader("Content-Encoding") == "gzip" and r.getheader("Vary") == "Accept-Encoding"
        body = gzip.decompress(raw).decode()
        assert "kgs_up" in body and len(raw) < len(body) / 3
        assert len(list(text_string_to_metric_families(body))) > 10
    c.request("GET", "/metrics")
    r = c.getresponse()
    assert r.getheader("Content-Encoding") is None and b"kgs_up" in r.read()
    c.close()
    c = http.client.HTTPConnection("127.0.0.1", off.port, timeout=5)
    c.request("GET", "/metrics", headers={"accept-encoding": "gzip"})
    r = c.getresponse()
    assert r.getheader("Content-Encoding") is None and b"kgs_up" in r.read()
    c.close()


def test_counter_handover_keeps_totals_monotonic(mock_exporter):
    """set_pmc_enabled(False): the sampler STOPs its counters (another profiler may
    program them) and skips the PMC tier; True re-STARTs them.  Exported totals carry
    over the restart, so counters stay monotonic."""
    ex = mock_exporter(n_gpus=2, hz=500, pmc_source="mock", proc_every=0, link_every=0,
                       mock={"util_base": 50, "util_amp": 0.0001})
    time.sleep(0.3)
    tot = lambda m: {lb["gpu"]: v for lb, v in m["amdgpu_pmc_total"] if lb["counter"] == "GRBM_COUNT"}  # noqa: E731
    m0 = parse_text(ex.render())
    assert {lb["gpu"]: v for lb, v in m0["kgs_pmc_enabled"]} == {"0": 1.0, "1": 1.0}
    ex.set_pmc_enabled(False)
    assert ex.pmc_enabled is False
    time.sleep(0.1)
    m1 = parse_text(ex.render())
    n1 = ex.integrals(0)["pmc_samples"]
    time.sleep(0.3)
    m2 = parse_text(ex.render())
    assert ex.integrals(0)["pmc_samples"] == n1                      # no READs while released
    assert {lb["gpu"]: v for lb, v in m2["kgs_pmc_enabled"]} == {"0": 0.0, "1": 0.0}
    assert {lb["gpu"]: v for lb, v in m2["kgs_pmc_releases_total"]} == {"0": 1.0, "1": 1.0}
    assert ex.integrals(1)["reads"] > 0                              # PMFW tier keeps sampling
    # while released, no rate gauge may keep its last pre-hand-over value
    assert not m2.get("amdgpu_mfma_util_percent") and not m2.get("container_gpu_mfma_util")
    assert m2["amdgpu_gfx_busy_percent"]                              # the PMFW gauges stay
    ex.set_pmc_enabled(True)
    time.sleep(0.4)
    m3 = parse_text(ex.render())
    assert ex.integrals(0)["pmc_samples"] > n1 + 50
    assert {lb["gpu"]: v for lb, v in m3["kgs_pmc_enabled"]} == {"0": 1.0, "1": 1.0}
    for g in ("0", "1"):
        assert tot(m0)[g] <= tot(m1)[g] <= tot(m2)[g] < tot(m3)[g]   # monotonic across the re-START
    w = ex.window(0, 0.2)
    assert w["gpu_active_pct"] == pytest.approx(50, abs=3) and w["mfma_util_pct"] == pytest.approx(60, abs=3)


def test_exporter_process_counter_handover_signals(tmp_path):
    """`kgs exporter`: SIGUSR1 releases the counters, SIGUSR2 takes them back."""
    import os
    import signal
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--backend", "mock",
                          "--mock-gpus", "1", "--pmc", "mock", "--hz", "200", "--listen", "127.0.0.1:0",
                          "--control-stdin", "--no-pin-numa"], cwd=repo, stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        ready = json.loads(p.stdout.readline())
        port = ready["port"]
        en = lambda: parse_text(get(port, "/metrics").read().decode())["kgs_pmc_enabled"][0][1]  # noqa: E731
        assert en() == 1.0
        p.send_signal(signal.SIGUSR1)
        time.sleep(0.3)
        assert en() == 0.0
        p.send_signal(signal.SIGUSR2)
        time.sleep(0.3)
        assert en() == 1.0
    finally:
        p.stdin.write("quit\n")
        p.stdin.flush()
        p.communicate(timeout=30)


def test_stalled_counters_are_withheld_then_reclaimed(mock_exporter):
    """A foreign profiler that STOPs the counters leaves GRBM_COUNT frozen (run r44).
    The exporter flags kgs_pmc_stalled, withholds the counter-tier gauges instead of
    publishing zeros, and re-STARTs its session after --pmc-reclaim-s."""
    ex = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0, window_s=0.2,
                       pmc_reclaim_s=1.2, mock={"util_base": 50, "util_amp": 0.0001},
                       mock_pmc={"freeze_after_s": 0.3})
    time.sleep(0.25)
    m = parse_text(ex.render())
    assert m["kgs_pmc_stalled"][0][1] == 0 and "amdgpu_mfma_util_percent" in m
    time.sleep(0.75)  # frozen since 0.3 s: stalled after another 0.5 s
    m = parse_text(ex.render())
    assert m["kgs_pmc_stalled"][0][1] == 1
    assert "amdgpu_mfma_util_percent" not in m and "amdgpu_gpu_clock_effective_mhz" not in m
    grbm = lambda mm: [v for lb, v in mm["amdgpu_pmc_total"] if lb["counter"] == "GRBM_COUNT"][0]  # noqa: E731
    before = grbm(m)
    t0 = time.time()
    while time.time() - t0 < 3 and parse_text(ex.render())["kgs_pmc_reclaims_total"][0][1] < 1:
        time.sleep(0.05)
    time.sleep(0.15)  # counting again for 0.3 s after the re-START
    m = parse_text(ex.render())
    assert m["kgs_pmc_reclaims_total"][0][1] >= 1 and m["kgs_pmc_stalled"][0][1] == 0
    assert grbm(m) > before                      # totals continue monotonically after the re-START
    assert m["amdgpu_mfma_util_percent"][0][1] == pytest.approx(60, abs=5)
    off = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0, pmc_reclaim_s=0,
                        mock_pmc={"freeze_after_s": 0.2})
    time.sleep(1.0)
    m = parse_text(off.render())
    assert m["kgs_pmc_stalled"][0][1] == 1 and m["kgs_pmc_reclaims_total"][0][1] == 0  # reclaim disabled


def test_periodic_counter_refresh(mock_exporter):
    """--pmc-refresh-s re-STARTs the session on a schedule (selects reprogrammed);
    totals and rates are continuous across it."""
    ex = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0, window_s=0.2,
                       pmc_refresh_s=0.3, mock={"util_base": 50, "util_amp": 0.0001})
    time.sleep(1.1)
    m = parse_text(ex.render())
    assert 2 <= m["kgs_pmc_refreshes_total"][0][1] <= 4 and m["kgs_pmc_reclaims_total"][0][1] == 0
    assert m["kgs_pmc_stalled"][0][1] == 0
    assert m["amdgpu_gpu_active_percent"][0][1] == pytest.approx(50, abs=5)
    g = [v for lb, v in m["amdgpu_pmc_total"] if lb["counter"] == "GRBM_COUNT"][0]
    assert g == pytest.approx(2100e6 * 1.1, rel=0.1)  # 2100 MHz mock clock × ≈1.1 s, refreshes included


def test_per_xcd_vmem_busy_full_set(mock_exporter):
    """--pmc-set full adds TA busy per XCD (mean over the XCD's CUs): the mock keeps
    the TA units busy 30 % of every XCD's active cycles."""
    ex = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0, pmc_set="full",
                       mock={"util_base": 50, "util_amp": 0.0001}, mock_pmc={"xcd_skew": 0.05})
    base = mock_exporter(n_gpus=1, hz=500, pmc_source="mock", proc_every=0, link_every=0)
    time.sleep(0.5)
    w = ex.window(0, 0.3)
    assert w["xcd_vmem_busy_pct"] == pytest.approx([30.0] * 8, abs=1.5)
    m = parse_text(ex.render())
    assert len(m["amdgpu_vmem_busy_xcc_percent"]) == 8
    assert "amdgpu_vmem_busy_xcc_percent" not in parse_text(base.render())  # base set: no TA block


def test_stale_devices_export_no_window_gauges(mock_exporter):
    """a device whose reads keep failing drops its busy gauges (and its
    container_gpu_sm_util, which feeds the per-pod report) after stale_s instead of
    repeating its last value; counters and kgs_up stay."""
    ex = mock_exporter(n_gpus=2, hz=200, window_s=0.2, stale_s=0.3, max_backoff_ms=50,
                       mock={"vanish_dev": 1, "vanish_after_s": 0.4})
    for g in (0, 1):
        ex.set_device_owners(g, [{"pod": f"p{g}", "namespace": "n", "container": "c"}])
    time.sleep(0.3)
    m = parse_text(ex.render())
    assert sorted(lb["gpu"] for lb, _ in m["amdgpu_gfx_busy_percent"]) == ["0", "1"]
    time.sleep(0.8)  # device 1 has failed for ≥ 0.4 s > stale_s
    m = parse_text(ex.render())
    assert sorted(lb["gpu"] for lb, _ in m["amdgpu_gfx_busy_percent"]) == ["0"]
    assert sorted(lb["pod_name"] for lb, _ in m["container_gpu_sm_util"]) == ["p0"]
    assert sorted(lb["gpu"] for lb, _ in m["amdgpu_gfx_busy_seconds_total"]) == ["0", "1"]
    assert {lb["gpu"]: v for lb, v in m["kgs_up"]} == {"0": 1.0, "1": 0.0}
    # paused sampling: everything goes stale, nothing frozen is exported
    ex.pause()
    time.sleep(0.5)
    assert not parse_text(ex.render()).get("amdgpu_gfx_busy_percent")
    ex.resume()


def test_slow_tiers_never_stall_the_counter_threads(mock_exporter):
    """the per-process / link / RAS reads go through one
    process-wide AMD SMI lock and take milliseconds.  With the mock's latency
    model (2 ms process list, 0.5 ms link table and RAS, all under one lock; 0.1 ms
    table read) and those tiers at 50 / 20 Hz on 8 GPUs — the slow thread holds
    the lock ~90 % of the time — every GPU's counter tier still delivers its rate."""
    hz = 2000
    lat = {"proc_latency_s": 2e-3, "link_latency_s": 5e-4, "health_latency_s": 5e-4, "metrics_latency_s": 1e-4}

    def rates(ex):
        time.sleep(0.3)
        n0 = [ex.integrals(g)["pmc_samples"] for g in range(8)]
        t0 = time.time()
        time.sleep(1.5)
        n1 = [ex.integrals(g)["pmc_samples"] for g in range(8)]
        dt = time.time() - t0
        return [(b - a) / dt for a, b in zip(n0, n1)]

    ex = mock_exporter(n_gpus=8, hz=hz, pmc_source="mock", proc_period_s=0.02, link_period_s=0.05, mock=lat)
    on = rates(ex)
    ex.stop()
    # control: the same 8 counter threads with no slow tier at all, on the same (shared,
    # possibly busy) CPUs — the slow tiers may cost nothing beyond what the host costs both
    ctl = mock_exporter(n_gpus=8, hz=hz, pmc_source="mock", proc_period_s=0, link_period_s=0, proc_every=0,
                        link_every=0, mock=lat)
    off = rates(ctl)
    ctl.stop()
    # 0.9: the two runs are seconds apart on an 8-CPU host that other work shares
    assert min(on) > 0.9 * min(hz, sum(off) / len(off)), (on, off)
    assert min(on) > 0.85 * hz, (on, off)
    I = [ex.integrals(g) for g in range(8)]
    assert all(i["proc_reads"] > 10 and i["link_reads"] > 5 for i in I), I
    # the locked calls happened on the slow thread: its time per pass ≈ 8 × (2 + 0.5 + 0.5) ms
    slow = sum(i["slow_read_seconds"] for i in I)
    assert slow > 0.5, slow
    assert ex.slow_passes > 10


def test_rocprofiler_reader_is_test_only():
    """one counter reader in the product; the rocprofiler-sdk
    reader is a cross-check that only tests can select."""
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k != "KGS_PMC_CROSSCHECK"}
    r = subprocess.run([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--backend", "mock",
                        "--listen", "127.0.0.1:0", "--pmc", "rocprofiler"],
                       cwd=REPO, capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 2 and "test-only" in r.stdout


def test_quiet_gpu_counter_reads_drop_to_idle_rate(mock_exporter):
    """Adaptive READ rate (profiles/r2/idle_busy/): every counter READ is a packet the
    GPU's busy gauges count as work, so while the READ-immune SPI-busy / MFMA counters
    show nothing the sampler READs at pmc_idle_hz, and on every tick again as soon
    as work shows up.  Integrals stay exact: the duty cycle of a square load is
    read the same with or without the idle rate."""
    def rate(ex, secs=1.0):
        n0 = ex.integrals(0)["pmc_samples"]
        time.sleep(secs)
        return (ex.integrals(0)["pmc_samples"] - n0) / secs

    idle = mock_exporter(n_gpus=1, hz=2000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=50,
                         mock={"util_base": 0, "util_amp": 0})
    time.sleep(0.2)
    r_idle = rate(idle)
    m = parse_text(idle.render())
    assert 30 <= r_idle <= 80, r_idle                       # ≈ pmc_idle_hz, not 2000
    assert m["kgs_pmc_quiet"][0][1] == 1 and m["kgs_pmc_quiet_skips_total"][0][1] > 1000
    idle.pmc_idle_hz = 0                                   # profiling mode: every tick
    time.sleep(0.05)
    assert rate(idle, 0.5) > 1400                          # (2000 less timer slack on a shared CPU)
    assert json.load(get(idle.port, "/control/pmc/idle?hz=25"))["pmc_idle_hz"] == 25
    time.sleep(0.05)
    assert 10 <= rate(idle, 1.0) <= 45
    idle.stop()

    # square load: 100 % for 0.1 s of every 0.4 s → every tick while busy, idle rate otherwise
    sq = mock_exporter(n_gpus=1, hz=2000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=50,
                       window_s=1.2, mock={"square_duty": 0.25, "util_period_s": 0.4, "util_base": 50, "util_amp": 50})
    time.sleep(0.3)
    r_sq = rate(sq, 1.2)
    assert 0.25 * 2000 * 0.6 <= r_sq <= 0.25 * 2000 + 0.75 * 50 + 150, r_sq
    w = sq.window(0, 1.2)
    assert w["gpu_active_pct"] == pytest.approx(25, abs=4), w      # the integral is exact at any READ rate


def test_learned_shader_clocks_are_exported(mock_exporter):
    """kgs_pmc_shader_clock_hz: the clocks the dispatch estimator learned (idle on READ-only
    intervals, busy on fully busy ones) — what the time split of long intervals prices idle
    cycles at.  The mock counts GRBM_COUNT at its 2100 MHz throughout."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=0,
                       mock={"square_duty": 0.5, "util_period_s": 0.2, "util_base": 50, "util_amp": 50})
    time.sleep(1.0)
    m = parse_text(ex.render())
    clk = {lb["kind"]: v for lb, v in m["kgs_pmc_shader_clock_hz"]}
    assert set(clk) == {"idle", "busy"}, clk
    assert clk["idle"] == pytest.approx(2.1e9, rel=0.02) and clk["busy"] == pytest.approx(2.1e9, rel=0.02), clk
    i = ex.integrals(0)
    assert i["pmc_clk_idle_hz"] == pytest.approx(clk["idle"], rel=0.05)
    # one clock everywhere: the time split, the cycle share and their blend agree, so the
    # square wave bills its duty
    w = ex.window(0, 0.8)
    assert w["util_pct"] == pytest.approx(50, abs=6), w


def test_counter_tick_dither_keeps_the_rate(mock_exporter):
    """--tick-dither: each counter tick's deadline random-walks off the fixed grid (≤ a
    quarter period per tick, within half a period; native TickDither, test_core.cpp), so
    the READ phase does not lock onto a periodic workload (tools/phase_probe.py, r5t: the
    window-to-window spread of a 0.2 ms / 1 ms train at 8 kHz fell from 0.60 to 0.08
    points); the grid keeps the delivered rate the configured one."""
    for dither in (0.25, 0.0):
        ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=0,
                           tick_dither=dither, mock={"util_base": 50, "util_amp": 0})
        time.sleep(0.3)
        n0, t0 = ex.integrals(0)["pmc_samples"], time.monotonic()
        time.sleep(1.5)
        rate = (ex.integrals(0)["pmc_samples"] - n0) / (time.monotonic() - t0)
        ex.stop()
        assert 0.9 * 1000 <= rate <= 1.01 * 1000, (dither, rate)


def test_dispatch_bound_reads_drop_to_dispatch_rate(mock_exporter):
    """Dispatch-bound READ rate (--pmc-cp-only-min, on by default): a stream of µs
    kernels keeps the CP busy while waves are present only part of the time (on
    MI355X: CPC ≈100 %, SPI ≈41 %), and that stream pays each READ packet (+3.8 % at
    8 kHz, profiles/r4/ r4c).  The mock's wave_frac 0.4 models it: after the hold,
    READs drop to the dispatch rate and the dispatch integral stays exact (100 %); long
    kernels (wave_frac 1) and --pmc-cp-only-min 0 keep every tick.  The rate is
    settable in place (Python property, loopback /control/pmc/dispatch)."""
    def rate(ex, secs=0.6):
        n0 = ex.integrals(0)["pmc_samples"]
        time.sleep(secs)
        return (ex.integrals(0)["pmc_samples"] - n0) / secs

    kw = dict(n_gpus=1, hz=4000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=100, window_s=1.0,
              pmc_dispatch_hz=500)
    ex = mock_exporter(mock={"util_base": 100, "util_amp": 0}, mock_pmc={"wave_frac": 0.4}, **kw)
    time.sleep(0.3)
    a, t0 = ex.integrals(0), time.time()
    r = rate(ex)
    b, dt = ex.integrals(0), time.time() - t0
    assert 350 <= r <= 750, r                                           # ≈ the dispatch rate, not 4000
    assert b["pmc_dispatch_bound"] == 1 and b["pmc_quiet"] == 0 and "pmc_gap" not in b, b
    assert (b["dispatch_seconds"] - a["dispatch_seconds"]) / dt == pytest.approx(1.0, abs=0.03)
    assert (b["active_seconds"] - a["active_seconds"]) / dt == pytest.approx(0.4, abs=0.03)
    m = parse_text(ex.render())
    assert m["kgs_pmc_dispatch_bound"][0][1] == 1 and m["kgs_pmc_dispatch_skips_total"][0][1] > 1000
    assert "kgs_pmc_gap" not in m and "kgs_pmc_gap_skips_total" not in m
    ex.pmc_dispatch_hz = 200
    time.sleep(0.05)
    assert 150 <= rate(ex) <= 300
    with urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/control/pmc/dispatch?hz=1000", timeout=5) as resp:
        assert json.load(resp) == {"pmc_dispatch_hz": 1000.0}
    time.sleep(0.05)
    assert 700 <= rate(ex) <= 1300
    for bad in ("hz=0", "hz=-5", "hz=200000"):
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/control/pmc/dispatch?{bad}", timeout=5)
        assert e.value.code == 400, bad
    with pytest.raises(ValueError):
        ex.pmc_dispatch_hz = 0
    assert ex.pmc_dispatch_hz == 1000
    ex.stop()

    for extra in ({"mock_pmc": {"wave_frac": 1.0}}, {"mock_pmc": {"wave_frac": 0.4}, "pmc_cp_only_min": 0.0}):
        ex = mock_exporter(mock={"util_base": 100, "util_amp": 0}, **extra, **kw)
        time.sleep(0.3)
        assert rate(ex) > 3000, extra
        assert ex.integrals(0)["pmc_dispatch_bound"] == 0
        ex.stop()


def test_batched_counter_source_is_not_a_failure(mock_exporter):
    """--pmc-batch: a reader that publishes every B-th READ returns kPmcPending for its
    first B samples after each (re)START and then every sample B calls late.  The
    sampler must neither count that as an error nor trip the breaker, and the
    integrals stay exact (each sample carries its own CP time)."""
    ex = mock_exporter(n_gpus=2, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=0,
                       window_s=1.0, mock={"util_base": 40, "util_amp": 0}, mock_pmc={"batch": 8},
                       pmc_refresh_s=0.3)                       # a re-START every 0.3 s: pending again each time
    time.sleep(1.3)
    for g in (0, 1):
        i = ex.integrals(g)
        assert i["pmc_errors"] == 0 and i["pmc_breaker_trips"] == 0 and i["pmc_failed"] == 0, i
        assert i["pmc_samples"] > 900, i
    w = ex.window(0, 1.0)
    assert w["gpu_active_pct"] == pytest.approx(40, abs=3), w
    m = parse_text(ex.render())
    assert m["kgs_pmc_refreshes_total"][0][1] >= 3
    # one L2 writeback per 8 READs, every result landed
    reads = ex.integrals(0)["pmc_samples"]
    pub = m["kgs_pmc_publishes_total"][0][1]
    assert 0.9 * reads / 8 <= pub <= 1.3 * reads / 8 + 10, (pub, reads)
    assert [v for _, v in m["kgs_pmc_unlanded_total"]] == [0, 0]


def test_throttle_seconds_by_reason(mock_exporter):
    """amdgpu_throttle_seconds_total{reason}: per distinct PMFW table, Δresidency /
    Δaccumulation_counter of each throttler times the interval (amdsmi PVIOL/TVIOL),
    so 100 * rate() is the violation percent."""
    ex = mock_exporter(n_gpus=1, hz=200, mock={"ppt_frac": 0.25, "fw_period_s": 0.005})
    time.sleep(0.3)
    i0, t0 = ex.integrals(0), time.time()
    time.sleep(1.0)
    i1, dt = ex.integrals(0), time.time() - t0
    ppt = (i1["throttle_seconds"]["ppt"] - i0["throttle_seconds"]["ppt"]) / dt
    assert ppt == pytest.approx(0.25, abs=0.03)
    assert i1["throttle_seconds"]["socket_thermal"] == 0
    m = parse_text(ex.render())
    rs = {lb["reason"]: v for lb, v in m["amdgpu_throttle_seconds_total"]}
    assert set(rs) == {"prochot", "ppt", "socket_thermal", "vr_thermal", "hbm_thermal"} and rs["ppt"] > 0.2


def test_http_connection_cap_and_idle_timeout(mock_exporter):
    """Clients that connect and never send cannot hold the exporter's fds: past
    http_max_conns the least recently active connection is closed, and an idle
    keep-alive connection is closed after http_idle_s; scrapes keep working."""
    import socket

    ex = mock_exporter(n_gpus=1, http_max_conns=4, http_idle_s=1.0)
    port = ex.port
    socks = []
    for _ in range(6):
        s = socket.create_connection(("127.0.0.1", port), timeout=5)
        socks.append(s)
        time.sleep(0.05)  # distinct activity times: eviction order is defined
    # the two oldest were evicted to admit the 5th and 6th: they read EOF
    for s in socks[:2]:
        assert s.recv(1) == b""
    socks[-1].sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
    head = socks[-1].recv(65536)
    assert head.startswith(b"HTTP/1.1 200"), head[:64]
    m = parse_text(get(port, "/metrics").read().decode())  # a 7th connection: evicts one more
    closed = {lb["reason"]: v for lb, v in m["kgs_http_connections_closed_total"]}
    assert closed["limit"] == 3 and closed["idle"] == 0
    assert m["kgs_http_connections"][0][1] == 4
    time.sleep(2.2)  # idle timeout 1 s, sweep every 0.5 s
    for s in socks[2:]:
        assert s.recv(1) == b""  # every silent connection was closed
        s.close()
    m = parse_text(get(port, "/metrics").read().decode())
    closed = {lb["reason"]: v for lb, v in m["kgs_http_connections_closed_total"]}
    assert closed["idle"] >= 3 and closed["limit"] == 3
    st = ex.stats()
    assert st["http_closed_idle"] >= 3 and st["http_closed_limit"] == 3


def test_ecc_totals_and_per_block_counts(mock_exporter):
    """RAS tier (node-wide slow thread): device totals by type and per-block counts for
    the blocks with ECC enabled; on the mock the HBM controller (umc) carries the
    correctable errors and gfx / xgmi_wafl are enabled and clean."""
    ex = mock_exporter(n_gpus=2, link_period_s=0.05, mock={"ecc_correctable_per_s": 1000})
    time.sleep(0.4)
    m = parse_text(ex.render())
    tot = {(lb["gpu"], lb["type"]): v for lb, v in m["amdgpu_ecc_errors_total"]}
    blk = {(lb["gpu"], lb["block"], lb["type"]): v for lb, v in m["amdgpu_ecc_block_errors_total"]}
    for g in ("0", "1"):
        assert {b for (gg, b, _) in blk if gg == g} == {"umc", "gfx", "xgmi_wafl"}
        assert tot[(g, "correctable")] > 0
        assert blk[(g, "umc", "correctable")] == tot[(g, "correctable")]
        assert blk[(g, "gfx", "uncorrectable")] == 0 and blk[(g, "xgmi_wafl", "deferred")] == 0


def test_kgs_ps_lists_processes_with_pods_and_compute_share(mock_exporter):
    """`kgs ps`: one row per (GPU, process) from the exporter's per-process families,
    with its pod and its compute share over the interval (rate of the CU-seconds
    counter; the mock's processes occupy 128 of 256 CUs = 50 %)."""
    import argparse
    import io

    from kube_gpu_stats_amd.reports import ps

    ex = mock_exporter(n_gpus=2, proc_period_s=0.05)
    ex.set_pid_owners({(0, 100000): {"pod": "train-0", "namespace": "ml", "container": "main", "pod_uid": "u0"},
                       (1, 100010): {"pod": "a", "namespace": "ml", "container": "c", "pod_uid": "ua"},
                       (1, 100011): {"pod": "b", "namespace": "dev", "container": "c", "pod_uid": "ub"}})
    time.sleep(0.3)
    args = lambda **kw: argparse.Namespace(**{"url": f"127.0.0.1:{ex.port}", "interval": 0.6, "gpu": "",  # noqa: E731
                                              "pod": "", "format": "json", **kw})
    buf = io.StringIO()
    assert ps.run(args(), out=buf) == 0
    rows = json.loads(buf.getvalue())
    by = {(r["gpu"], r["pid"]): r for r in rows}
    assert set(by) == {("0", 100000), ("1", 100010), ("1", 100011)}
    assert by[("0", 100000)]["pod"] == "train-0" and by[("1", 100011)]["namespace"] == "dev"
    assert abs(by[("1", 100011)]["hbm_gib"] - 2.0) < 1e-6
    for r in rows:
        assert abs(r["cu_share_pct"] - 50.0) < 8, r
    buf = io.StringIO()
    ps.run(args(format="table", pod="b", interval=0), out=buf)
    table = buf.getvalue()
    assert "| GPU |" in table.replace("  ", " ") or "GPU" in table.splitlines()[1]
    assert " b " in table and "train-0" not in table and table.count("\n") == 5  # rule, header, rule, 1 row, rule


def test_metric_allow_deny_filters_families(mock_exporter):
    """--metric-allow / --metric-deny trim /metrics by family (globs; deny wins; a
    histogram's _bucket/_sum/_count follow it; the control plane's text block too)."""
    full = mock_exporter(n_gpus=2, pmc_source="mock", proc_every=1, link_every=1)
    deny = mock_exporter(n_gpus=2, pmc_source="mock", proc_every=1, link_every=1,
                         metric_deny="amdgpu_*_xcc_percent, kgs_sample_read_seconds,amdgpu_xgmi_link_info,"
                                     "amdgpu_device_info,kgs_attribution_*")
    allow = mock_exporter(n_gpus=2, pmc_source="mock", proc_every=1, link_every=1,
                          metric_allow="container_gpu_*,amdgpu_gfx_busy_percent,kgs_up,kgs_attribution_updates_total",
                          metric_deny="container_gpu_mfma_*")
    for ex in (full, deny, allow):
        ex.set_device_owners(0, [{"pod": "train-0", "namespace": "ml", "container": "main"}])
        ex.set_extra_metrics("# HELP kgs_attribution_updates_total x\n# TYPE kgs_attribution_updates_total counter\n"
                             "kgs_attribution_updates_total 3\n# HELP kgs_attribution_errors_total y\n"
                             "# TYPE kgs_attribution_errors_total counter\nkgs_attribution_errors_total 0\n")
    time.sleep(0.5)
    fams = {}
    for name, ex in (("full", full), ("deny", deny), ("allow", allow)):
        body = ex.render()
        fams[name] = {f.name for f in text_string_to_metric_families(body)}  # still valid exposition
    dropped = fams["full"] - fams["deny"]
    assert {"amdgpu_gfx_busy_xcc_percent", "amdgpu_mfma_util_xcc_percent", "kgs_sample_read_seconds",
            "amdgpu_xgmi_link_info", "amdgpu_device_info", "kgs_attribution_updates", "kgs_attribution_errors"} <= dropped
    assert all(f.startswith(("amdgpu_", "kgs_sample_read", "kgs_attribution")) for f in dropped), dropped
    assert "container_gpu_sm_util" in fams["deny"] and "amdgpu_topology_link" in fams["deny"]
    assert fams["allow"] == {"container_gpu_sm_util", "container_gpu_busy_seconds", "container_gpu_energy_joules",
                             "container_gpu_cu_seconds", "amdgpu_gfx_busy_percent", "kgs_up",
                             "kgs_attribution_updates"}, fams["allow"]
    assert len(fams["deny"]) < len(fams["full"])


def test_xgmi_bytes_unit_is_configurable(mock_exporter):
    """amdgpu_xgmi_*_bytes_total = PMFW accumulator units × --xgmi-bytes-per-unit
    (amdsmi.h: KB; a multi-GPU bench run's expected / measured ratio corrects it)."""
    ex = mock_exporter(n_gpus=2, hz=200)
    time.sleep(0.4)
    ex.pause()
    m = parse_text(ex.render())
    kb = ex.samples(0, 1)[-1]["xgmi_read_kb"]
    got = {lb["link"]: v for lb, v in m["amdgpu_xgmi_read_bytes_total"] if lb["gpu"] == "0"}
    assert got and all(got[k] == kb[int(k)] * 1024 for k in got), (got, kb)
    ex2 = mock_exporter(n_gpus=2, hz=200, xgmi_bytes_per_acc_unit=1000.0)
    time.sleep(0.4)
    ex2.pause()
    kb2 = ex2.samples(0, 1)[-1]["xgmi_read_kb"]
    m2 = parse_text(ex2.render())
    got2 = {lb["link"]: v for lb, v in m2["amdgpu_xgmi_read_bytes_total"] if lb["gpu"] == "0"}
    assert got2 and all(got2[k] == kb2[int(k)] * 1000 for k in got2), (got2, kb2)


def test_short_idle_gaps_do_not_drop_to_the_idle_rate(mock_exporter):
    """Quiet hysteresis (r2be): a busy GPU whose kernels are separated by short gaps
    (here 2 ms idle in every 20 ms) stays on every tick — a device counts as quiet
    only after 5 ms of quiet READ intervals; a 25 ms gap still drops to the idle rate."""
    def skips_per_s(ex, secs=1.0):
        k0 = ex.integrals(0)["pmc_quiet_skips"]
        time.sleep(secs)
        return (ex.integrals(0)["pmc_quiet_skips"] - k0) / secs

    short = mock_exporter(n_gpus=1, hz=2000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=50,
                          mock={"square_duty": 0.9, "util_period_s": 0.02, "util_base": 50, "util_amp": 50})
    time.sleep(0.3)
    assert skips_per_s(short) == 0                       # 2 ms gaps: never quiet
    short.stop()
    long_gap = mock_exporter(n_gpus=1, hz=2000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=50,
                             mock={"square_duty": 0.5, "util_period_s": 0.05, "util_base": 50, "util_amp": 50})
    time.sleep(0.3)
    assert skips_per_s(long_gap) > 200                   # 25 ms gaps: ≈20 ms of each at the idle rate


def test_mock_peer_copy_lands_on_the_link_to_that_peer(mock_exporter):
    """a simulated GPU 0 → GPU 3 copy must move exactly the link whose
    /topology peer_bdf is GPU 3 on the source (write) and the link back to GPU 0 on
    the destination (read), by the copied bytes (default unit: KB accumulators)."""
    ex = mock_exporter(n_gpus=8, pmfw_hz=200, link_every=1, mock={"xgmi_bg": False, "fw_period_s": 0.005})
    time.sleep(0.2)
    bdf = {int(d["gpu"]): d["bdf"] for d in json.load(get(ex.port, "/devices"))}
    peer = {(int(x["gpu"]), int(x["link"])): x.get("peer_bdf", "") for x in json.load(get(ex.port, "/topology"))["links"]}

    def links(fam):
        return {(int(lb["gpu"]), int(lb["link"])): v for lb, v in parse_text(ex.render()).get(fam, [])}

    w0, r0 = links("amdgpu_xgmi_write_bytes_total"), links("amdgpu_xgmi_read_bytes_total")
    nbytes = 256 << 20
    assert ex.inject_xgmi(0, 3, nbytes) == 0
    assert ex.inject_xgmi(0, 0, nbytes) != 0  # no link to itself
    time.sleep(0.2)
    w1, r1 = links("amdgpu_xgmi_write_bytes_total"), links("amdgpu_xgmi_read_bytes_total")
    dw = {k: w1[k] - w0.get(k, 0.0) for k in w1 if w1[k] != w0.get(k, 0.0)}
    dr = {k: r1[k] - r0.get(k, 0.0) for k in r1 if r1[k] != r0.get(k, 0.0)}
    assert len(dw) == 1 and len(dr) == 1, (dw, dr)
    (src_key, src_b), = dw.items()
    (dst_key, dst_b), = dr.items()
    assert src_key[0] == 0 and peer[src_key] == bdf[3]
    assert dst_key[0] == 3 and peer[dst_key] == bdf[0]
    assert src_b == pytest.approx(nbytes, rel=1e-3) and dst_b == pytest.approx(nbytes, rel=1e-3)


def test_wake_lateness_histogram(mock_exporter):
    """kgs_sampler_wake_lateness_seconds: one observation per counter-thread tick,
    cumulative buckets, a sum of the positive lateness."""
    ex = mock_exporter(n_gpus=2, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=0)
    time.sleep(0.6)
    m = parse_text(ex.render())
    for g in ("0", "1"):
        b = [(float("inf") if lb["le"] == "+Inf" else float(lb["le"]), v)
             for lb, v in m["kgs_sampler_wake_lateness_seconds_bucket"] if lb["gpu"] == g]
        counts = [v for _, v in sorted(b)]
        n = [v for lb, v in m["kgs_sampler_wake_lateness_seconds_count"] if lb["gpu"] == g][0]
        assert counts == sorted(counts) and counts[-1] == n and n > 300, (g, b, n)
        assert [v for lb, v in m["kgs_sampler_wake_lateness_seconds_sum"] if lb["gpu"] == g][0] >= 0


def test_util_counter_set_exports_the_utilisation_only(mock_exporter):
    """--pmc-set util: GRBM count, SPI busy and CPC busy only (24 register reads per
    READ instead of 56), enough for the dispatch integral behind the reference-contract
    utilisation.  No MFMA or per-XCD series are exported, rather than zeros."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", pmc_set="util", pmc_idle_hz=0, window_s=1.0,
                       mock={"square_duty": 0.25, "util_base": 50, "util_amp": 50, "util_period_s": 0.2,
                             "pmfw_busy_floor": 99})
    ex.set_device_owners(0, [{"pod": "p", "namespace": "n", "container": "c"}])
    time.sleep(0.3)
    a, t0 = ex.integrals(0), time.time()
    time.sleep(1.2)
    b, dt = ex.integrals(0), time.time() - t0
    assert (b["dispatch_seconds"] - a["dispatch_seconds"]) / dt == pytest.approx(0.25, abs=0.03)
    assert b["mfma_busy_seconds"] == 0
    m = parse_text(ex.render())
    for fam in ("amdgpu_mfma_busy_seconds_total", "amdgpu_mfma_util_percent", "amdgpu_mfma_util_xcc_percent",
                "container_gpu_mfma_util", "container_gpu_mfma_busy_seconds_total"):
        assert not m.get(fam), fam
    assert {lb["counter"] for lb, _ in m["amdgpu_pmc_total"]} == {"GRBM_COUNT", "GRBM_SPI_BUSY", "CPC_CPC_STAT_BUSY"}
    (_, sm), = m["container_gpu_sm_util"]
    assert sm == pytest.approx(25, abs=6)                     # from the counters, not the PMFW floor of 99
    assert m["amdgpu_gpu_active_percent"][0][1] == pytest.approx(25, abs=6)


def test_lite_reads_keep_the_mfma_integral_exact(mock_exporter):
    """--pmc-lite: a batch's non-publishing READs skip the per-SE counters (MFMA busy:
    32 of the base set's 56 register copies), so they carry the last values read.  The
    MFMA integral spans fresh drains only and the window gauges use fresh drains, so
    both stay what every-READ reading gives (mock: 50 % busy × mfma_frac 0.6)."""
    kw = dict(n_gpus=1, hz=2000, pmc_source="mock", pmc_idle_hz=0, window_s=0.5, proc_every=0, link_every=0,
              mock={"util_base": 50, "util_amp": 0})
    rates = {}
    for lite in (0, 8):
        ex = mock_exporter(mock_pmc={"lite_every": lite}, **kw)
        time.sleep(0.3)
        a, t0 = ex.integrals(0), time.time()
        time.sleep(1.0)
        b, dt = ex.integrals(0), time.time() - t0
        rates[lite] = (b["mfma_busy_seconds"] - a["mfma_busy_seconds"]) / dt
        m = parse_text(ex.render())
        assert m["amdgpu_mfma_util_percent"][0][1] == pytest.approx(60, abs=2), lite
        assert (b["active_seconds"] - a["active_seconds"]) / dt == pytest.approx(0.5, abs=0.03)
        ex.stop()
    assert rates[0] == pytest.approx(0.3, abs=0.02) and rates[8] == pytest.approx(rates[0], abs=0.02), rates


def test_counter_stream_marks_stale_drains_and_rates_mfma_between_fresh_ones(mock_exporter):
    """with lite READs (lite_every 8) seven of every eight drains carry
    the last MFMA / TA values read.  /counters says which (se_fresh) and gives MFMA and
    vmem rates only on fresh drains, measured from the previous fresh one — so their
    per-sample mean is the load's 60 %, not a 0 / 100 sawtooth."""
    ex = mock_exporter(n_gpus=1, hz=2000, pmc_source="mock", pmc_idle_hz=0, proc_every=0, link_every=0,
                       mock={"util_base": 50, "util_amp": 0}, mock_pmc={"lite_every": 8})
    time.sleep(0.4)
    s = json.load(get(ex.port, "/counters?gpu=0&n=400"))["samples"]
    assert len(s) == 400
    fresh = [x for x in s if x["se_fresh"]]
    stale = [x for x in s if not x["se_fresh"]]
    assert 40 <= len(fresh) <= 60 and len(stale) > 300, (len(fresh), len(stale))
    assert not any("mfma_util_pct" in x or "vmem_busy_pct" in x for x in stale)
    assert all("gpu_active_pct" in x for x in s)  # device-wide counters: every drain
    mf = [x["mfma_util_pct"] for x in fresh if "mfma_util_pct" in x]
    assert len(mf) >= len(fresh) - 1  # the first one has its base: the ring is read past it
    assert sum(mf) / len(mf) == pytest.approx(60, abs=3) and min(mf) > 40 and max(mf) < 80, mf


def test_quiet_release_parks_the_session_and_bills_continuously(mock_exporter):
    """a programmed counter session keeps an idle MI355X ≈32 W above its
    released state (bench phase P, profiles/r6/r6b).  With --pmc-quiet-release-s the
    counter thread releases the session (STOP + READ queue destroyed) once the GPU has
    been quiet that long, bills from the PMFW meanwhile, and re-acquires once the PMFW
    shows a load starting (one table ≥ 10 % busy).  A 50 % square wave (1.5 s at 100 %, 1.5 s
    idle): every idle half parks, every busy half unparks, and the billed integral over
    whole periods is the wave's 50 % — as without parking."""
    import urllib.request

    kw = dict(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=100,
              mock={"util_base": 50, "util_amp": 50, "square_duty": 0.5, "util_period_s": 3.0, "fw_period_s": 0.02})
    ex = mock_exporter(pmc_quiet_release_s=0.3, **kw)
    ref = mock_exporter(pmc_quiet_release_s=0.0, **kw)
    time.sleep(0.5)
    a, r0, t0 = ex.integrals(0), ref.integrals(0), time.monotonic()
    parked_seen = on_seen = 0
    parked_s = []  # kgs_pmc_parked_seconds_total as scraped: monotonic through every park / unpark
    while time.monotonic() - t0 < 6.0:
        i = ex.integrals(0)
        parked_seen |= i["pmc_parked"]
        on_seen |= i["pmc_on"] and not i["pmc_parked"]
        parked_s.append(parse_text(ex.render())["kgs_pmc_parked_seconds_total"][0][1])
        time.sleep(0.05)
    assert all(y >= x for x, y in zip(parked_s, parked_s[1:])), parked_s
    assert 1.5 < parked_s[-1] - parked_s[0] < 4.5, parked_s  # most of each 1.5 s idle half
    b, r1 = ex.integrals(0), ref.integrals(0)
    assert parked_seen and on_seen
    assert b["pmc_parks"] - a["pmc_parks"] >= 2, b          # one per idle half
    assert b["pmc_unpark_lag_s"] is not None and b["pmc_unpark_lag_s"] < 0.05, b  # ≤ one 20 ms table + a poll
    billed = (b["util_seconds"] - a["util_seconds"]) / (b["sampled_seconds"] - a["sampled_seconds"])
    billed_ref = (r1["util_seconds"] - r0["util_seconds"]) / (r1["sampled_seconds"] - r0["sampled_seconds"])
    assert billed == pytest.approx(billed_ref, abs=0.02) and billed == pytest.approx(0.5, abs=0.05), (billed, billed_ref)
    assert ref.integrals(0)["pmc_parks"] == 0
    m = parse_text(ex.render())
    assert m["kgs_pmc_parks_total"][0][1] >= 2 and "kgs_pmc_parked" in m
    # the control plane: read / set the delay; an acquire ends a park at once
    with urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/control/pmc/quiet_release?s=0.1", timeout=5) as resp:
        assert json.load(resp) == {"pmc_quiet_release_s": 0.1}
    for bad in ("s=-5", "s=1e9"):
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/control/pmc/quiet_release?{bad}", timeout=5)
        assert e.value.code == 400, bad
    with pytest.raises(ValueError):
        ex.pmc_quiet_release_s = -2
    assert ex.pmc_quiet_release_s == pytest.approx(0.1)


def test_a_stray_blip_does_not_unpark(mock_exporter):
    """r6g phase P: a parked GPU un- and re-parked in 2 of 6 idle blocks — one 20 ms PMFW
    table ≥ 1 % busy (a 0.2 ms packet) was enough to re-acquire.  The wake-up now needs
    ≥ 10 % in one table (a load starting) or ≥ 1 % over 100 ms of table time (a trickle):
    0.2 ms blips every 0.5 s leave the device parked."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=100,
                       pmc_quiet_release_s=0.2,
                       mock={"util_base": 50, "util_amp": 50, "square_duty": 0.0004, "util_period_s": 0.5,
                             "fw_period_s": 0.02})
    t0 = time.monotonic()
    while time.monotonic() - t0 < 3 and not ex.integrals(0)["pmc_parked"]:
        time.sleep(0.02)
    a = ex.integrals(0)
    assert a["pmc_parked"] == 1, a
    time.sleep(2.5)  # five blips
    b = ex.integrals(0)
    assert b["pmc_parked"] == 1 and b["pmc_parks"] == a["pmc_parks"], (a, b)
    assert b["pmc_parked_s"] - a["pmc_parked_s"] == pytest.approx(2.5, abs=0.2), (a, b)  # kgs_pmc_parked_seconds_total


@pytest.mark.parametrize("floor,wakes", [(2.0, True), (0.5, False)])
def test_a_trickle_unparks_over_100ms(mock_exporter, floor, wakes):
    """The parked tier's slow wake-up path: no PMFW table reaches 10 %, but a steady
    trickle of GFX busy (the mock PMFW reads `floor` % while the counters see no wave)
    re-acquires once 100 ms of table time average ≥ 1 % — and the GPU, still quiet to the
    counters, parks again; below 1 % it stays parked."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=100,
                       pmc_quiet_release_s=0.2,
                       mock={"util_base": 0, "util_amp": 0, "square_duty": 0.5, "util_period_s": 1.0,
                             "pmfw_busy_floor": floor, "fw_period_s": 0.02})
    t0 = time.monotonic()
    while time.monotonic() - t0 < 3 and not ex.integrals(0)["pmc_parks"]:
        time.sleep(0.02)
    a = ex.integrals(0)
    assert a["pmc_parks"] >= 1, a
    time.sleep(1.5)
    b = ex.integrals(0)
    if wakes:
        assert b["pmc_parks"] - a["pmc_parks"] >= 2, (a, b)  # woke (≈0.1 s) and parked again (0.2 s quiet), repeatedly
    else:
        assert b["pmc_parks"] == a["pmc_parks"] and b["pmc_parked"] == 1, (a, b)


def test_a_parked_tier_wakes_when_the_pmfw_goes_silent(mock_exporter):
    """While parked only the PMFW bills the GPU: with no PMFW table for 1 s (every read
    failing here) the counter tier re-acquires rather than leave the GPU unbilled — and,
    the mock GPU still quiet, parks again; with the PMFW reading, one park holds."""
    kw = dict(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=100,
              pmc_quiet_release_s=0.2)
    silent = mock_exporter(mock={"util_base": 0, "util_amp": 0, "fail_rate": 1.0}, **kw)
    ok = mock_exporter(mock={"util_base": 0, "util_amp": 0}, **kw)
    time.sleep(3.5)
    assert silent.integrals(0)["pmc_parks"] >= 2, silent.integrals(0)
    assert ok.integrals(0)["pmc_parks"] == 1, ok.integrals(0)


def test_hand_over_while_parked_and_back(mock_exporter):
    """A device parked by the quiet release can be handed over (kgs pmc release: nothing is
    held, the hand-over stands) and acquired back at once by the control plane, whatever
    the load (an explicit acquire ends a park without waiting for PMFW busy); switching
    parking off while parked (quiet release 0, or profiling mode) re-acquires too."""
    ex = mock_exporter(n_gpus=1, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=100,
                       pmc_quiet_release_s=0.2, mock={"util_base": 0, "util_amp": 0})
    t0 = time.monotonic()
    while time.monotonic() - t0 < 3 and not ex.integrals(0)["pmc_parked"]:
        time.sleep(0.02)
    i = ex.integrals(0)
    assert i["pmc_parked"] == 1 and i["pmc_on"] == 0, i
    ex.set_pmc_enabled(False)
    time.sleep(0.1)
    i = ex.integrals(0)
    assert i["pmc_parked"] == 0 and i["pmc_on"] == 0 and not ex.pmc_enabled, i
    ex.pmc_quiet_release_s = 0          # stay acquired on the idle mock GPU this time
    ex.set_pmc_enabled(True)
    time.sleep(0.2)
    i = ex.integrals(0)
    assert i["pmc_on"] == 1 and i["pmc_parked"] == 0, i
    n = i["pmc_samples"]
    time.sleep(0.3)
    assert ex.integrals(0)["pmc_samples"] > n  # drains again (at the idle rate)
    # parking switched off while parked — the quiet release set to 0, or profiling mode
    # on — re-acquires at once, whatever the load
    for switch_off in (lambda: setattr(ex, "pmc_quiet_release_s", 0), lambda: setattr(ex, "pmc_idle_hz", 0)):
        ex.pmc_idle_hz = 100
        ex.pmc_quiet_release_s = 0.2
        t0 = time.monotonic()
        while time.monotonic() - t0 < 3 and not ex.integrals(0)["pmc_parked"]:
            time.sleep(0.02)
        assert ex.integrals(0)["pmc_parked"] == 1
        switch_off()
        time.sleep(0.2)
        i = ex.integrals(0)
        assert i["pmc_parked"] == 0 and i["pmc_on"] == 1, i
