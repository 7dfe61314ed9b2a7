"""bench.py driver contract (CPU, mock provider; 1 process and torchrun gloo ×2)
and the minimum end-to-end slice of SURVEY.md §7.3: exporter → (fake) Prometheus
TSDB fed by scrapes → ``gpu-util-stats`` per-pod report."""
import json
import os
import subprocess
import sys
import time

import pytest

from kube_gpu_stats_amd.attribution import proto
from kube_gpu_stats_amd.attribution.attributor import Attributor
from fakekubelet import FakeKubelet
from kube_gpu_stats_amd.reports import gpu_util_stats as G
from fakeprom import FakeProm
from kube_gpu_stats_amd.reports.promql import PromClient
from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


SUMMARY_KEYS = {"value", "samples_per_sec_per_gpu", "p50_scrape_ms", "p99_scrape_ms", "scrapes", "overhead_pct",
                "overhead_by_tier", "overhead_median_by_tier", "overhead_by_component", "overhead_by_rank",
                "released", "delivered_by_component", "util_accuracy", "xgmi_link_map_ok", "xgmi_links_ok", "xgmi_unit_ratio"}


def _result(out: str) -> tuple[dict, dict]:
    """(the stdout result line, the full result it points to).  VERDICT r3 #2: the
    driver keeps only the last few KB of stdout, so the line itself must fit in the
    last 3000 characters, with every headline number in its last key, ``summary``."""
    tail = out.rstrip("\n")[-3000:]
    line = json.loads(tail[tail.index("{"):]) if tail.count("\n") == 0 else _last_json(tail)
    assert len(json.dumps(line)) <= 3000, len(json.dumps(line))
    assert list(line)[-1] == "summary" and len(json.dumps(line["summary"])) <= 1800, len(json.dumps(line["summary"]))
    assert SUMMARY_KEYS <= set(line["summary"]), SUMMARY_KEYS - set(line["summary"])
    with open(os.path.join(REPO, line["full_result"])) as f:
        full = json.load(f)
    assert full["value"] == line["value"] and full["ms_per_step"] == line["ms_per_step"]
    return line, full


# Counter-tier delivery floor for the 8 kHz mock runs.  This build VM is noisy: a bare
# clock_nanosleep loop at 125 µs misses ≈11 % of its deadlines here (4.6 k of 40 k ticks,
# worst stall 12 ms, host steal time), so the mock exporter delivers 72–99 % depending on
# the neighbours.  On MI355X the same tier delivers 99.6 % (profiles/r2/r2ae/bench.json);
# these tests check the plumbing, not this VM's scheduler.
MIN_8K = 0.6


def _rate_ok(v: float, hz: float) -> bool:
    return MIN_8K * hz < v <= 1.02 * hz


# The mock runs at bench.py's default 8 kHz, stated here so that the tests do not follow a
# change of the default: this 8-CPU VM cannot hold 16 kHz for several mock GPUs at once.
FAST = ["--hz", "8000", "--pmc-batch", "8", "--step-ms", "60", "--rounds", "4", "--block-steps", "1", "--settle",
        "0.3", "--util-hz", "", "--idle-power-s", "0"]
# phase P's orchestration on the mock (constant synthetic power: the plumbing, not a number)
POWER = ["--idle-power-s", "1.2", "--idle-power-rounds", "2"]


@pytest.mark.slow
def test_bench_contract_single_process(tmp_path):
    r = subprocess.run([sys.executable, "bench.py", "--mock", "--steps", "10", "--warmup", "1", *FAST,
                        "--util-hz", "1000,10", *POWER, "--out", str(tmp_path / "bench.json")],
                       cwd=REPO, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    line, res = _result(r.stdout)
    assert KEYS <= set(line) and KEYS <= set(res)
    assert res["n_gpus"] == 1 and res["steps"] == 10 and res["higher_is_better"] is True
    assert res["scaling"] == "weak" and res["dtype"] == "bf16"
    cfg = res["config"]
    assert cfg["parallelism"] == "dp1" and cfg["global_batch"] == 1
    # a step is ≥ --step-ms of load (whole 20 ms mock units), and seq_len = ticks per GPU per step
    assert cfg["units_per_step"] == 3 and res["ms_per_step"] == pytest.approx(60, abs=15)
    assert cfg["seq_len"] == pytest.approx(cfg["hz"] * res["ms_per_step"] / 1e3, rel=0.01)
    assert cfg["hz_tiers"] == [100.0, 8000.0]
    # mock counters at the 8 kHz primary tier; on a shared 8-CPU container the mock
    # sampler's timer slack and overrun catch-up cost it up to ~15 % (MI355X: 99.98 %)
    assert _rate_ok(res["value"], 8000.0)
    assert res["p50_scrape_ms"] < 50 and res["scrapes"] > 10
    inter = res["interleaved"]
    # rounds cycle through every order of (paused, 100 Hz, 8 kHz): each condition in
    # each block position; paused blocks really do not read
    # (a fourth condition, "released" — counter session STOPped and the
    # READ queue destroyed for the block)
    order = [c for c, _ in inter["block_seconds"]]
    assert order[:12] == ["0", "released", "100", "8000", "0", "released", "8000", "100", "0", "100", "released",
                          "8000"]
    assert inter["order_design"]["kind"] == "all permutations in turn" and len(inter["order_design"]["orders"]) == 4
    assert set(inter["position_means"]["all"]) == {"0", "1", "2", "3"}
    assert set(inter["position_means"]["by_condition"]) == {"0", "released", "100", "8000"}
    pa = inter["position_adjusted"]
    assert set(pa) >= {"released", "100", "8000", "position_effect_pct"} and abs(pa["8000"]["overhead_pct"]) < 50
    rel = inter["released"]
    assert set(rel) == {"paused_vs_released_pct", "paused_vs_released_ci95_pct", "100_vs_released_pct",
                        "100_vs_released_ci95_pct", "8000_vs_released_pct", "8000_vs_released_ci95_pct"}
    assert line["summary"]["released"]["paused_vs_released"][0] == pytest.approx(rel["paused_vs_released_pct"], abs=1e-3)
    # per component against "released" too
    for hz in ("100", "8000"):
        vr = inter["tiers"][hz]["overhead_by_component_vs_released"]
        assert set(vr) == set(inter["tiers"][hz]["overhead_by_component"])
        row = line["summary"]["overhead_by_component"][hz]["mock"]  # [vs paused, ci, vs released, ci]
        assert len(row) == 4 and row[2] == pytest.approx(vr["mock"]["overhead_pct"], abs=1e-3)
    # phase U plumbing: every load at the primary rate, at 1 kHz and at
    # the DaemonSet's 10 Hz, the exported busy counter next to the GPU-timed duty
    ua = res["util_accuracy"]
    assert set(ua["per_rate"]) == {"8000", "1000", "10"}
    for per in ua["per_rate"].values():
        assert set(per) == {"idle", "burst_1ms_every_5ms", "burst_0.2ms_every_1ms", "triad_1ms_every_5ms",
                            "mfma_saturating", "random_kernels", "two_stream_random", "train_step"}
        row = per["burst_1ms_every_5ms"]["0"]
        assert set(row) >= {"duty_gpu_pct", "duty_host_pct", "busy_counter_pct", "sm_util_gauge", "pmfw_gfx_busy_pct",
                            "from_counters_pct", "error_pts"}
        assert 10 < row["duty_gpu_pct"] < 30 and row["from_counters_pct"] > 90, row  # mock bursts: sleeps
    assert set(ua["worst_error_pts"]) == {"idle", "burst_1ms_every_5ms", "burst_0.2ms_every_1ms", "triad_1ms_every_5ms",
                                          "mfma_saturating", "random_kernels", "two_stream_random", "train_step"}
    assert inter["paused_reads"] == 0
    assert res["xgmi_link_check"] == {"skipped": "N=1: no peer GPU to copy to"} and res["xgmi_link_map_ok"] is None
    for hz in ("100", "8000"):
        t = inter["tiers"][hz]
        assert len(t["overhead_per_round_pct"]) == 4
        assert t["overhead_ci95_pct"] > 0 and abs(t["overhead_pct"]) < 50
        # the mock load's one component, timed per block; the one rank's own overhead
        comp = t["overhead_by_component"]["mock"]
        assert abs(comp["overhead_pct"]) < 50 and comp["share_of_block_time"] == pytest.approx(1.0, abs=0.2)
        assert [r["rank"] for r in t["overhead_by_rank"]] == [0]
        # 4 blocks of ~60 ms: at 100 Hz that is ~25 ticks, so whole-tick quantisation at
        # each block edge alone is ±4 per cent; 8 kHz (~2000 ticks) loses up to ~15 % to
        # timer slack on a shared CPU container
        if hz == "100":
            assert t["samples_per_sec_per_gpu"]["0"] == pytest.approx(100.0, rel=0.15)
        else:
            assert _rate_ok(t["samples_per_sec_per_gpu"]["0"], 8000.0)
    assert res["overhead_pct"] == inter["tiers"]["8000"]["overhead_pct"]
    # phase R plumbing: the burst train was launched and the full-rate stream read back
    # for it (the mock's counters do not follow the host, so no segment count is checked)
    br = res["burst_resolution"]["per_gpu"]["0"]
    assert br["launched"] >= 100 and _rate_ok(br["drains_per_s"], 8000.0)
    # phase Q plumbing: both exporter modes measured, the default idle rate restored after
    q = res["quiet_gpu"]
    assert q["adaptive"]["pmc_idle_hz"] == 100 and q["profiling"]["pmc_idle_hz"] == 0
    ip = q["idle_power"]  # phase P ran every condition on the mock, in rounds of every order
    assert ip["rounds"] == 2 and [b["cond"] for b in ip["blocks"]][:3] == ["session", "released", "parked"], ip
    assert ip["per_rank"][0]["session_minus_released_w"][0] == pytest.approx(0.0, abs=1.0), ip
    assert set(ip["exporter_by_condition"]) == {"session", "released", "parked"}
    assert ip["exporter_by_condition"]["released"]["reads_per_s"] == 0, ip
    assert set(q["adaptive"]["per_gpu"]["0"]) == {"reads_per_s", "pmfw_gfx_busy_pct", "gpu_active_pct"}
    # phase S plumbing: the primary rate and each capacity rate got a block, rate restored after
    cap = res["capacity"]
    assert list(cap["rates"]) == ["8000", "16000", "24000", "32000"]
    for row in cap["rates"].values():
        assert row["sample_source"] == "pmc" and row["samples_per_sec_per_gpu"]["0"] > 0
        assert row["host_us_per_drain"] > 0
    assert cap["rates"]["16000"]["samples_per_sec_per_gpu"]["0"] > cap["rates"]["8000"]["samples_per_sec_per_gpu"]["0"]


@pytest.mark.slow
def test_bench_contract_torchrun_gloo_world2(tmp_path):
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", "--mock",
                        "--steps", "6", "--warmup", "1", *FAST, "--out", str(tmp_path / "bench.json")],
                       cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    _, res = _result(r.stdout)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    # both ranks' GPUs sampled by the one node exporter → aggregate ≈ 2 × per-GPU
    assert len(res["pmc_samples_per_sec_per_gpu"]) == 2
    assert res["value"] == pytest.approx(sum(res["pmc_samples_per_sec_per_gpu"].values()), rel=0.01)


@pytest.mark.slow
def test_bench_8_ranks_xgmi_link_map_and_per_rank_overheads(tmp_path):
    """The 8-GPU driver run must validate itself unattended: phase X
    books a GPU 0 → GPU k peer copy per peer (the mock backend puts it on the link to
    k) and finds each copy on the link whose peer_bdf is k's, at unit ratio 1; the
    interleaved overheads come per rank and per component, power per rank."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--mock", "--gpus", "8", "--steps", "4", "--warmup", "1",
                        *FAST, "--hz", "2000", "--capacity-hz", "", "--burst-s", "0", "--quiet-s", "0", *POWER,
                        "--idle-power-absent", "1", "--out", str(tmp_path / "bench.json")],
                       cwd=REPO, capture_output=True, text=True, timeout=420, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line, res = _result(r.stdout)
    assert res["n_gpus"] == 8
    s = line["summary"]                        # the headline survives the driver's stdout tail
    assert s["xgmi_link_map_ok"] is True and s["xgmi_unit_ratio"] == pytest.approx(1.0, abs=0.02)
    assert len(s["overhead_by_rank"]) == 8 and set(s["overhead_by_component"]) == {"100", "2000"}
    x = res["xgmi_link_check"]
    assert res["xgmi_link_map_ok"] is True and x["xgmi_link_map_ok"] is True, x
    assert res["xgmi_unit_ratio"] == pytest.approx(1.0, abs=0.02) and x["xgmi_unit_ok"] is True, x
    assert x["xgmi_links_ok"] == [56, 56] and s["xgmi_links_ok"] == [56, 56], x["xgmi_links_ok"]
    assert sorted((p["src_gpu"], p["peer_gpu"]) for p in x["per_copy"]) == [(i, j) for i in range(8) for j in range(8)
                                                                            if i != j]
    for p in x["per_copy"]:
        assert p["src"]["link_peer_bdf"] == p["peer_bdf"] and p["dst"]["ok"], p
    ip = res["quiet_gpu"]["idle_power"]
    assert len(ip["per_rank"]) == 8  # phase P: every rank's own probe
    # the fourth condition, "absent" (every tier paused), in a Williams square
    assert [b["cond"] for b in ip["blocks"]] == ["session", "released", "absent", "parked",
                                                 "released", "parked", "session", "absent"], ip["blocks"]
    assert ip["exporter_by_condition"]["absent"]["reads_per_s"] == 0 and "absent_minus_released_w" in ip
    for hz in ("100", "2000"):
        t = res["interleaved"]["tiers"][hz]
        assert [q["rank"] for q in t["overhead_by_rank"]] == list(range(8))
        assert len(t["overhead_by_component"]["mock"]["per_rank_overhead_pct"]) == 8


@pytest.mark.slow
def test_bench_self_spawns_ranks_without_torchrun(tmp_path):
    """`python bench.py --gpus 4` (no torchrun env) launches 4 ranks itself, so a plain
    invocation — the driver's scaling runs included — measures N GPUs, not 1."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--mock", "--gpus", "4", "--steps", "6", "--warmup", "1", *FAST,
                        "--out", str(tmp_path / "bench.json")],
                       cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    _, res = _result(r.stdout)
    assert res["n_gpus"] == 4 and res["config"]["parallelism"] == "dp4" and res["config"]["global_batch"] == 4
    assert sorted(res["pmc_samples_per_sec_per_gpu"]) == ["0", "1", "2", "3"]
    # weak scaling: value is the node aggregate, the per-GPU rate stays at the tick rate
    assert _rate_ok(res["samples_per_sec_per_gpu"], 8000.0)
    assert res["value"] == pytest.approx(4 * res["samples_per_sec_per_gpu"], rel=1e-6)


def test_end_to_end_exporter_to_report(mock_exporter, tmp_path):
    """Native sampler → /metrics → TSDB → gpu-util-stats report rows (§7.3)."""
    ex = mock_exporter(n_gpus=2, hz=100, window_s=0.2,
                       mock={"util_base": 60, "util_amp": 0.0001, "fw_period_s": 0.01})
    sock = str(tmp_path / "kubelet.sock")
    resp = proto.ListPodResourcesResponse([proto.PodResources("train-0", "ml", [proto.ContainerResources(
        "main", [proto.ContainerDevices("amd.com/gpu", ["0000:11:00.0", "0000:21:00.0"])])])])
    fp = FakeProm()
    url = fp.start()
    try:
        with FakeKubelet(sock, resp):
            Attributor(ex, sock).update_once()
            sc = Scraper("127.0.0.1", ex.port)
            time.sleep(0.3)
            t0 = 1_700_000_000.0
            for i in range(6):  # six "scrapes", 10 s apart in TSDB time
                fp.ingest(parse_text(sc.scrape_once()), t0 + 10 * i)
                time.sleep(0.05)
        q = G.Queries.amd("ml", 10, util_metric="container_gpu_sm_util")  # gauge path; counters: test_accounting
        fp.add_instant(q.total, [{"metric": {"node": "node-a", q.type_label: "MI355X"}, "value": [t0, "8"]}])
        fp.add_instant(q.used, [{"metric": {"node": "node-a"}, "value": [t0, "2"]}])
        fp.add_instant(q.live, [{"metric": {"namespace": "ml", "pod": "train-0"}, "value": [t0, "1"]}])
        fp.add_range(q.req, [{"metric": {"node": "node-a", "namespace": "ml", "pod": "train-0"},
                              "values": [[t0, "2"]]}])
        rows = G.run_report(PromClient(url), q, t0 + 50, 50, 10, compat=False)
        assert len(rows) == 1
        node, ns, pod, cards, util = rows[0]
        assert (node, ns, pod, cards) == ("node-a", "ml", "train-0", 2)
        assert util == pytest.approx(60.0, abs=1.0)
        # the reference's own M1 query shape works unchanged against the exporter's series
        body = fp.eval_instant(G.REF_Q_UTIL, t0 + 50)
        assert body[0]["metric"] == {"kubernetes_io_hostname": "node-a", "nvidia_gpu_type": "MI355X",
                                     "pod_name": "train-0"}
    finally:
        fp.stop()


def test_multi_node_exporters_to_reports(mock_exporter):
    """"Multi-node" without a cluster: two exporters with their own
    --node-name feed one (fake) Prometheus; the per-pod report (F3), the per-node
    report (F4) and the per-pod MFMA report all span both nodes."""
    a = mock_exporter(n_gpus=2, hz=200, window_s=0.2, node_name="node-a", pmc_source="mock",
                      mock={"util_base": 60, "util_amp": 0.0001, "fw_period_s": 0.01}, mock_pmc={"mfma_frac": 0.6})
    b = mock_exporter(n_gpus=2, hz=200, window_s=0.2, node_name="node-b", pmc_source="mock",
                      mock={"util_base": 30, "util_amp": 0.0001, "fw_period_s": 0.01}, mock_pmc={"mfma_frac": 0.3})
    a.set_device_owners(0, [{"pod": "train-0", "namespace": "ml", "container": "main"}])
    a.set_device_owners(1, [{"pod": "train-0", "namespace": "ml", "container": "main"}])
    b.set_device_owners(1, [{"pod": "infer-1", "namespace": "ml", "container": "srv"}])
    fp = FakeProm()
    url = fp.start()
    try:
        time.sleep(0.4)
        sa, sb = Scraper("127.0.0.1", a.port), Scraper("127.0.0.1", b.port)
        t0 = 1_700_000_000.0
        for i in range(6):
            fp.ingest(parse_text(sa.scrape_once()), t0 + 10 * i, {"instance": "node-a:9400"})
            fp.ingest(parse_text(sb.scrape_once()), t0 + 10 * i, {"instance": "node-b:9400"})
            time.sleep(0.05)
        for metric in ("container_gpu_sm_util", "container_gpu_mfma_util"):
            q = G.Queries.amd("ml", 10, util_metric=metric)
            fp.add_instant(q.total, [{"metric": {"node": n, q.type_label: "MI355X"}, "value": [t0, "8"]}
                                     for n in ("node-a", "node-b")])
            fp.add_instant(q.used, [{"metric": {"node": "node-a"}, "value": [t0, "2"]},
                                    {"metric": {"node": "node-b"}, "value": [t0, "1"]}])
            fp.add_instant(q.live, [{"metric": {"namespace": "ml", "pod": p}, "value": [t0, "1"]}
                                    for p in ("train-0", "infer-1")])
            fp.add_range(q.req, [{"metric": {"node": "node-a", "namespace": "ml", "pod": "train-0"},
                                  "values": [[t0, "2"]]},
                                 {"metric": {"node": "node-b", "namespace": "ml", "pod": "infer-1"},
                                  "values": [[t0, "1"]]}])
            rows = sorted(G.run_report(PromClient(url), q, t0 + 50, 50, 10, compat=False))
            want = (60.0, 30.0)  # mock: GFX busy 60 / 30 %, MFMA busy 60 / 30 % of active cycles
            assert [r[:4] for r in rows] == [["node-a", "ml", "train-0", 2], ["node-b", "ml", "infer-1", 1]], rows
            assert rows[0][4] == pytest.approx(want[0], abs=2) and rows[1][4] == pytest.approx(want[1], abs=2), rows
            if metric == "container_gpu_sm_util":
                nodes = G.run_report(PromClient(url), q, t0 + 50, 50, 10, compat=False, mode="node")
                assert [(r[0], r[1], r[3], r[4]) for r in nodes] == [("node-a", "MI355X", 2, 8),
                                                                    ("node-b", "MI355X", 1, 8)], nodes
                assert nodes[0][2] == pytest.approx(60, abs=2) and nodes[1][2] == pytest.approx(30, abs=2), nodes
    finally:
        fp.stop()


def test_train_load_steps_on_cpu():
    """bench.py --load train: the decoder step runs, learns (loss falls on a fixed batch),
    and calibrate() reports the step's rate.  Tiny dims; CPU stands in for cuda:0."""
    import torch

    import bench

    a = bench.parse_args(["--load", "train", "--train-dim", "128", "--train-layers", "2",
                          "--train-batch", "2", "--train-seq", "32", "--train-vocab", "512"])
    ld = bench.TrainLoad(a, -1, None)
    # loss on the fixed batch before / after a few steps
    F = torch.nn.functional

    def loss():
        with torch.no_grad():
            lg = ld.model(ld.tok[:, :-1])
            return F.cross_entropy(lg.float().view(-1, lg.shape[-1]), ld.tok[:, 1:].reshape(-1)).item()

    l0 = loss()
    for _ in range(5):
        ld.step()
    assert loss() < l0
    assert ld.params > 0


def test_allreduce_expected_xgmi_rate():
    """Phase B's all-reduces imply 2·2(N-1)/N·size bytes per GPU per call (read + write):
    the figure the 8-GPU run's measured xgmi_GBps_per_gpu is checked against."""
    import types

    sys.path.insert(0, REPO)
    import bench

    ar = types.SimpleNamespace(numel=lambda: 64 << 20, element_size=lambda: 4)  # 256 MiB
    load = types.SimpleNamespace(ar=ar, reps=11)
    a = types.SimpleNamespace(steps=20)
    want = 2 * 2 * 7 / 8 * (256 << 20) * 20 * 11 / 10.0 / 1e9
    assert bench.allreduce_GBps(load, a, 8, 10.0) == pytest.approx(want, abs=1e-3)
    assert bench.allreduce_GBps(load, a, 1, 10.0) is None
    assert bench.allreduce_GBps(types.SimpleNamespace(reps=1), a, 8, 10.0) is None


@pytest.mark.parametrize("swap", [-1, 5])
def test_phase_x_checks_every_directed_link_and_names_a_wrong_one(N, swap):
    """phase X copies between every ordered pair of an 8-GPU node (in
    parallel rounds of disjoint pairs) and checks both ends of each copy, so all 56
    directed link ends are validated: [56, 56] on a right map.  A mock GPU 5 whose link
    table swaps two ports' peers fails exactly the copies over those two links, and
    the report names GPU 5's links."""
    import types

    import bench as B

    ex = N.Exporter({"backend": "mock", "mock": {"n_gpus": 8, "xgmi_swap_dev": swap}, "hz": 100, "port": 0,
                     "node_name": "n", "pin_numa": False, "control_http": True, "link_every": 1, "proc_every": 0})
    ex.start()
    try:
        time.sleep(0.5)
        exp = B.AttachedExporter(f"127.0.0.1:{ex.port}")
        bdfs = [d["bdf"] for d in exp.json("/devices")]
        a = types.SimpleNamespace(xgmi_check_mib=64, mock=True, xgmi_check_settle=0.15, xgmi_check_budget_s=60)
        out = B._xgmi_rank0(a, exp, bdfs)
    finally:
        ex.stop()
    assert out["xgmi_unit_ratio_min_max"] == [1.0, 1.0]
    if swap < 0:
        assert out["xgmi_links_ok"] == [56, 56] and out["xgmi_link_map_ok"] and not out["bad_links"], out["bad_links"]
    else:
        ok, total = out["xgmi_links_ok"]
        assert total == 56 and ok == 52 and not out["xgmi_link_map_ok"]  # 5↔peer0, 5↔peer1, both directions
        assert all("gpu5 link 1" in b or "gpu5 link 2" in b for b in out["bad_links"]), out["bad_links"]
        assert {(r["src_gpu"], r["peer_gpu"]) for r in out["per_copy"] if not r["ok"]} == {(0, 5), (5, 0), (1, 5), (5, 1)}


def test_pair_rounds_cover_every_ordered_pair_once():
    import bench as B

    for n in (2, 3, 4, 7, 8):
        rounds = B._pair_rounds(n)
        flat = [p for r in rounds for p in r]
        assert sorted(flat) == [(i, j) for i in range(n) for j in range(n) if i != j], n
        for r in rounds:  # a GPU is in at most one copy per round
            used = [g for p in r for g in p]
            assert len(used) == len(set(used)), (n, r)


def test_phase_x_failure_does_not_take_the_run_down(monkeypatch):
    """Phase X runs on local rank 0 between two collectives: an exception there (a
    failed peer copy, an exporter endpoint error) must end in the result, not in a
    crashed rank 0 that leaves the other ranks waiting at the barrier."""
    import types

    import bench as b
    calls = []
    monkeypatch.setattr(b.D, "cpu_barrier", lambda ctx: calls.append("barrier"))
    monkeypatch.setattr(b.D, "all_gather_object", lambda ctx, obj: [(0, "0000:01:00.0"), (1, "0000:02:00.0")])

    class Exp:  # an exporter that went away: nothing listens on its port
        port = b.free_port()

    ctx = types.SimpleNamespace(world=2, rank=0, local_rank=0)
    a = types.SimpleNamespace(xgmi_check_mib=64, mock=True, xgmi_check_settle=0.0)
    load = types.SimpleNamespace(pci_bdf=lambda r: f"0000:0{r + 1}:00.0")
    out = b.xgmi_link_check(ctx, load, Exp(), a)
    assert out["xgmi_link_map_ok"] is False and "Error" in out["error"], out
    assert calls == ["barrier", "barrier"]  # both collectives still reached
