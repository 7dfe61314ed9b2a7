"""Renderer ↔ metric catalogue consistency, and the ``kgs`` CLI subcommands."""
import json
import os
import subprocess
import sys
import time

import pytest

from prometheus_client.parser import text_string_to_metric_families

from kube_gpu_stats_amd.models.schema import BY_NAME, CATALOG

from fixtures import reference_podlist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rendered_families_match_catalog(mock_exporter):
    from kube_gpu_stats_amd.attribution.attributor import Attributor

    ex = mock_exporter(n_gpus=3, pmc_source="mock", pmc_set="full", proc_every=1, link_every=1)
    ex.set_device_owners(0, [{"pod": "p", "namespace": "n", "container": "c"}])
    time.sleep(0.4)
    Attributor(ex, socket_path=None).publish()
    fams = list(text_string_to_metric_families(ex.render()))
    names = {f.name for f in fams}
    # prometheus_client strips _total from counter family names
    catalog = {f.name[:-6] if f.type == "counter" and f.name.endswith("_total") else f.name for f in CATALOG}
    assert names == catalog, (names ^ catalog)
    for fam in fams:
        cat = BY_NAME.get(fam.name) or BY_NAME.get(fam.name + "_total")
        assert cat.type == fam.type, fam.name
        for s in fam.samples:
            allowed = set(cat.labels) | set(cat.extra)
            assert set(s.labels) <= allowed, (fam.name, set(s.labels) - allowed)


@pytest.mark.parametrize("mode", ["auto", "counters", "pmfw"])
def test_rendered_help_is_the_catalogue_text(N, mode):
    """every HELP line /metrics serves is the catalogue's text for the
    exporter's --sm-util-source mode (the renderer reads it from the header generated
    from models/schema.py), and every family the renderer emits is in the catalogue."""
    from kube_gpu_stats_amd.attribution.attributor import Attributor

    ex = N.Exporter({"backend": "mock", "mock": {"n_gpus": 2}, "hz": 200, "port": 0, "node_name": "n",
                     "pin_numa": False, "pmc_source": "mock", "pmc_set": "full", "proc_every": 1, "link_every": 1,
                     "sm_util_source": mode})
    ex.start()
    try:
        ex.set_device_owners(0, [{"pod": "p", "namespace": "n", "container": "c"}])
        time.sleep(0.4)
        Attributor(ex, socket_path=None).publish()
        body = ex.render()
    finally:
        ex.stop()
    seen = 0
    for line in body.splitlines():
        if line.startswith("# HELP "):
            name, text = line[7:].split(" ", 1)
            assert name in BY_NAME, name
            assert text == BY_NAME[name].help_for("" if mode == "auto" else mode), name
            seen += 1
        elif line.startswith("# TYPE "):
            name, typ = line[7:].split(" ", 1)
            assert typ == BY_NAME[name].type, name
    assert seen >= 90, seen


def test_metric_help_header_is_generated_from_the_catalogue():
    from kube_gpu_stats_amd.models.schema import cpp_header

    path = os.path.join(REPO, "kube_gpu_stats_amd", "native", "include", "kgs", "metric_help.h")
    assert open(path).read() == cpp_header(), "run: python -m kube_gpu_stats_amd.models.schema --cpp-header"
    assert all("\n" not in f.help and "\\" not in f.help for f in CATALOG)


def test_utilisation_help_names_the_shipped_estimator():
    """The default (auto) text of the utilisation families describes what the sampler
    computes: CP busy less the learned READ cost, floored at SPI busy, PMFW otherwise.
    GRBM_SPI_BUSY alone is the source only of --sm-util-source counters and the
    amdgpu_gpu_active_* families."""
    for name in ("container_gpu_sm_util", "container_gpu_busy_seconds_total", "kgs_util_source_seconds_total",
                 "amdgpu_dispatch_busy_seconds_total"):
        h = BY_NAME[name].help
        assert "CPC_CPC_STAT_BUSY" in h and "READ" in h and "GRBM_SPI_BUSY" in h, name
    for f in CATALOG:
        if "GRBM_SPI_BUSY" in f.help and "CPC_CPC_STAT_BUSY" not in f.help:
            assert "active" in f.name, f.name  # amdgpu_gpu_active_*: SPI really is the source
    for name in ("container_gpu_sm_util", "container_gpu_busy_seconds_total"):
        assert "GRBM_SPI_BUSY" in BY_NAME[name].help_for("counters")
        assert "PMFW" in BY_NAME[name].help_for("pmfw")
    doc = open(os.path.join(REPO, "docs", "METRICS.md")).read()
    from kube_gpu_stats_amd.models.schema import PREAMBLE, markdown
    assert doc.strip() == (PREAMBLE + markdown()).strip(), "regenerate docs/METRICS.md"


def _kgs(*args, **kw):
    return subprocess.run([sys.executable, "-m", "kube_gpu_stats_amd.cli", *args], cwd=REPO, capture_output=True,
                          text=True, timeout=120, **kw)


def test_cli_who_use_gpu_compat_from_file(tmp_path):
    p = tmp_path / "pods.json"
    p.write_text(json.dumps(reference_podlist()))
    r = _kgs("who-use-gpu", "--compat", "--source", "file", "--pods-json", str(p))
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "'nodeName'"
    assert lines[-3:] == ["Total GPU: 7", "tesla-v100\t6", "<unspecified>\t1"]


def test_cli_who_use_gpu_json_and_env_override(tmp_path):
    p = tmp_path / "pods.json"
    p.write_text(json.dumps(reference_podlist()))
    env = dict(os.environ, KGS_RESOURCE="nvidia.com/gpu", KGS_FORMAT="json")
    r = _kgs("who-use-gpu", "--source", "file", "--pods-json", str(p), env=env)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["total"] == 8 and out["pods"][0]["pod"] == "new-style"


def test_cli_topo_mock():
    r = _kgs("topo", "--backend", "mock", "--mock-gpus", "4")
    assert r.returncode == 0, r.stderr
    topo = json.loads(r.stdout)
    assert len(topo["devices"]) == 4 and len(topo["edges"]) == 12
    assert all(len([x for x in topo["links"] if x["gpu"] == g]) == 3 for g in range(4))


def test_topology_ring_order():
    from kube_gpu_stats_amd.parallel.topology import discover, node_graph, prometheus_lines, ring_order

    topo = discover("mock", 8)
    g = node_graph(topo)
    assert all(len(v) == 7 for v in g.values())  # MI355X: all-to-all xGMI
    ring = ring_order(g)
    assert len(ring) == 8 and all(ring[(i + 1) % 8] in g[ring[i]] for i in range(8))
    assert len(prometheus_lines(topo, "n")) == 56


def test_cli_exporter_mock_process():
    p = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--backend", "mock",
                          "--mock-gpus", "2", "--listen", "127.0.0.1:0", "--control-stdin", "--hz", "50"],
                         cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        ready = json.loads(p.stdout.readline())
        assert ready["event"] == "ready" and ready["backend"] == "mock" and len(ready["devices"]) == 2
        time.sleep(0.3)
        r = _kgs("scrape", f"http://127.0.0.1:{ready['port']}/metrics", "--match", "kgs_up{")
        assert r.stdout.count("kgs_up{") == 2
    finally:
        p.stdin.write("quit\n")
        p.stdin.flush()
        out, _ = p.communicate(timeout=30)
    stopped = json.loads(out.splitlines()[-1])
    assert stopped["event"] == "stopped" and stopped["integrals"][0]["reads"] > 0


def test_dmon_segments_resolve_bursts_with_hysteresis():
    """segments(): a 200 Hz train of 1 ms bursts sampled every 125 µs (8 kHz) gives
    one segment per burst — a burst split across drain boundaries, or dipping to
    50 % inside, stays one — and the exact busy integral / duty of 20 %."""
    from kube_gpu_stats_amd.reports.dmon import segments

    dt_ns = 125_000
    samples, t = [], 10_000_000
    for k in range(1600):  # 0.2 s
        t += dt_ns
        phase = (t - dt_ns - 10_000_000) % 5_000_000  # interval start within the 5 ms period
        v = 100.0 if phase < 1_000_000 else 0.0
        if phase == 500_000:
            v = 50.0  # a dip inside a burst: above the low threshold, no new segment
        samples.append({"seq": k, "mono_ns": t, "dt_us": dt_ns / 1e3, "gpu_active_pct": v})
    segs, busy, span = segments(samples)
    assert len(segs) == 40
    assert all(e - s == 1_000_000 for s, e in segs)
    assert all(b[0] - a[0] == 5_000_000 for a, b in zip(segs, segs[1:]))
    assert span == pytest.approx(0.2) and busy / span == pytest.approx(0.2 - 0.5 * 40 * 125e-6 / 0.2, rel=1e-6)
    # an open burst at the end closes at the last sample; entries without rates are skipped
    segs2, _, _ = segments([{"seq": 0, "mono_ns": 5}] + samples[:4])
    assert segs2 == [(samples[0]["mono_ns"] - dt_ns, samples[3]["mono_ns"])]


def test_cli_dmon_rows_and_counter_bursts(mock_exporter):
    """`kgs dmon` against a live (mock) exporter: one row per GPU per poll, rates
    from counter deltas, and min/max MFMA from the full-rate /counters stream."""
    import io

    from kube_gpu_stats_amd.reports import dmon

    ex = mock_exporter(n_gpus=2, hz=1000, pmc_source="mock", proc_every=100, link_every=1000,
                       mock={"util_base": 50, "util_amp": 30, "util_period_s": 0.5})
    time.sleep(0.3)
    buf = io.StringIO()
    a = dmon.build_parser().parse_args([f"127.0.0.1:{ex.port}", "--interval", "0.2", "--count", "3", "--counters",
                                        "--json"])
    assert dmon.run(a, out=buf) == 0
    rows = [json.loads(x) for x in buf.getvalue().splitlines()]
    assert [r["gpu"] for r in rows] == ["0", "1"] * 3
    last = rows[-2:]
    for r in last:
        assert 0 <= r["gfx"] <= 100 and r["hbm_gb"] > 0 and r["power_w"] > 0
        assert r["energy_w"] is not None and r["energy_w"] > 0      # rate from the energy counter
        assert r["drains"] >= 100                                    # ≈200 drains per 0.2 s at 1 kHz
        assert 55 <= r["mfma_min"] <= r["mfma_max"] <= 65             # mock: MFMA busy 60 % of active cycles
        assert [55 <= float(x) <= 65 for x in r["xcd_mfma"].split("/")] == [True] * 8  # per-XCD split
        assert 15 <= r["duty"] <= 85 and r["bursts"] is not None     # mock GPU active 50 ± 30 %
        assert r["pmc"] == "on"                                      # the counter tier, one word
    buf = io.StringIO()
    a = dmon.build_parser().parse_args([f"http://127.0.0.1:{ex.port}", "--interval", "0.1", "--count", "2"])
    dmon.run(a, out=buf)
    lines = buf.getvalue().splitlines()
    assert lines[0].split()[:4] == ["GPU", "POD", "GFX%", "MFMA%"] and len(lines) == 1 + 2 * 2


def test_cli_record_chrome_trace(mock_exporter, tmp_path):
    """`kgs record`: drain the full-rate /counters stream of every GPU into a Chrome
    trace (counter tracks + busy segments); no drain is lost at 1 kHz with 100 ms polls,
    and --profiling switches the exporter to READ every tick only for the capture."""
    from kube_gpu_stats_amd.reports import record

    ex = mock_exporter(n_gpus=2, hz=1000, pmc_source="mock", proc_every=0, link_every=0, pmc_idle_hz=50,
                       mock={"square_duty": 0.5, "util_period_s": 0.2, "util_base": 50, "util_amp": 50})
    time.sleep(0.3)
    out = tmp_path / "t.json"
    a = record.build_parser().parse_args([f"127.0.0.1:{ex.port}", "--seconds", "1.0", "--poll-ms", "100",
                                          "--profiling", "--out", str(out)])
    import io

    buf = io.StringIO()
    assert record.run(a, out=buf) == 0
    res = json.loads(buf.getvalue())
    assert ex.pmc_idle_hz == 50                                    # restored after the capture
    for g in ("0", "1"):
        s = res["gpus"][g]
        assert s["lost"] == 0 and s["drains"] >= 700, s            # every tick, square load or not
        assert 35 <= s["duty_pct"] <= 65 and 3 <= s["busy_segments"] <= 7, s  # 0.1 s on / 0.1 s off
    tr = json.loads(out.read_text())
    ev = tr["traceEvents"]
    names = {e["args"]["name"] for e in ev if e["ph"] == "M" and e["name"] == "process_name"}
    assert names == {"GPU 0 (0000:11:00.0)", "GPU 1 (0000:21:00.0)"}
    assert sum(1 for e in ev if e["ph"] == "C" and e["name"] == "GPU active %" and e["pid"] == 0) == \
        res["gpus"]["0"]["drains"]
    busy = [e for e in ev if e["ph"] == "X" and e["pid"] == 0]
    assert busy and all(80_000 <= e["dur"] <= 120_000 for e in busy[1:-1])   # µs: 0.1 s blocks


def test_amd_smi_tiers_are_floored_at_khz_tick_rates():
    """--proc-every / --link-every count fast ticks; at the counter tier's 8 kHz the
    defaults would poll AMD SMI's process list 800×/s (r3q soak: the slow thread on
    0.33-0.43 cores).  Unless a period is given, the tiers run at ≤ 10 Hz / ≤ 1 Hz."""
    from kube_gpu_stats_amd.exporter.main import build_parser, config_from_args

    def periods(*argv):
        c = config_from_args(build_parser().parse_args(list(argv)))
        return c["proc_period_s"], c["link_period_s"]

    assert periods("--hz", "8000") == (0.1, 1.0)
    assert periods("--hz", "10") == (1.0, 10.0)                     # the DaemonSet rate: as before
    assert periods("--hz", "8000", "--proc-every", "0", "--link-every", "0") == (0.0, 0.0)
    assert periods("--hz", "8000", "--proc-period", "0.02", "--link-period", "0.5") == (0.02, 0.5)  # explicit wins


@pytest.mark.parametrize("sub", ["exporter", "who-use-gpu", "gpu-util-stats", "ps", "dmon", "record", "topo", "pmc",
                                 "scrape"])
def test_every_subcommand_help_renders(sub):
    """argparse formats every help string with %: a bare % in one flag's help breaks
    `--help` for the whole subcommand."""
    r = subprocess.run([sys.executable, "-m", "kube_gpu_stats_amd.cli", sub, "--help"], cwd=REPO,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "usage:" in r.stdout


def test_dmon_pmc_state_word():
    """`kgs dmon`'s PMC column: the counter tier per GPU in one word, the breaker first."""
    from kube_gpu_stats_amd.reports.dmon import pmc_state

    def fam(*vals):
        return [({"gpu": str(i)}, v) for i, v in enumerate(vals)]

    m = {"kgs_pmc_enabled": fam(1, 1, 1, 0, 0, 0), "kgs_pmc_quiet": fam(0, 1, 0, 0, 0, 0),
         "kgs_pmc_dispatch_bound": fam(0, 0, 1, 0, 0, 0), "kgs_pmc_parked": fam(0, 0, 0, 1, 0, 0),
         "kgs_pmc_failed": fam(0, 0, 0, 0, 0, 1)}
    assert pmc_state(m) == {"0": "on", "1": "quiet", "2": "dbnd", "3": "park", "4": "off", "5": "fail"}
    assert pmc_state({}) == {}
