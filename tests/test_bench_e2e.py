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
from kube_gpu_stats_amd.attribution.podresources import FakeKubelet
from kube_gpu_stats_amd.reports import gpu_util_stats as G
from kube_gpu_stats_amd.reports.fakeprom import FakeProm
from kube_gpu_stats_amd.reports.promql import PromClient
from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.slow
def test_bench_contract_single_process():
    r = subprocess.run([sys.executable, "bench.py", "--mock", "--steps", "20", "--warmup", "1", "--settle", "0.5"],
                       cwd=REPO, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _last_json(r.stdout)
    assert KEYS <= set(res)
    assert res["n_gpus"] == 1 and res["steps"] == 20 and res["higher_is_better"] is True
    assert res["scaling"] == "weak" and res["dtype"] == "bf16"
    assert res["config"]["parallelism"] == "dp1"
    assert res["value"] > 50  # mock PMC at 100 Hz
    assert res["p50_scrape_ms"] < 50
    assert abs(res["ms_per_step"] - 20.0) < 10


@pytest.mark.slow
def test_bench_contract_torchrun_gloo_world2():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", "--mock",
                        "--steps", "15", "--warmup", "1", "--settle", "0.5"],
                       cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    res = _last_json(r.stdout)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    # both ranks' GPUs sampled by the one node exporter → aggregate ≈ 2 × per-GPU
    assert len(res["pmc_samples_per_sec_per_gpu"]) == 2
    assert res["value"] == pytest.approx(sum(res["pmc_samples_per_sec_per_gpu"].values()), rel=0.01)


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
        q = G.Queries.amd("ml", 10)
        fp.add_instant(q.total, [{"metric": {"node": "node-a", q.type_label: "MI355X"}, "value": [t0, "8"]}])
        fp.add_instant(q.used, [{"metric": {"node": "node-a"}, "value": [t0, "2"]}])
        fp.add_instant(q.live, [{"metric": {"pod": "train-0"}, "value": [t0, "1"]}])
        fp.add_range(q.req, [{"metric": {"node": "node-a", "pod": "train-0"}, "values": [[t0, "2"]]}])
        rows = G.run_report(PromClient(url), q, t0 + 50, 50, 10, compat=False)
        assert len(rows) == 1
        node, pod, cards, util = rows[0]
        assert (node, pod, cards) == ("node-a", "train-0", 2)
        assert util == pytest.approx(60.0, abs=1.0)
        # the reference's own M1 query shape works unchanged against the exporter's series
        body = fp.eval_instant(G.REF_Q_UTIL, t0 + 50)
        assert body[0]["metric"] == {"kubernetes_io_hostname": "node-a", "nvidia_gpu_type": "MI355X",
                                     "pod_name": "train-0"}
    finally:
        fp.stop()
