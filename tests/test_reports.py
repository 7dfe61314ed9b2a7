"""Report layer (capabilities F1-F4): golden --compat outputs of SURVEY.md §2.8 and
the fixed default mode.  Reference: gpu_util_stats/gpu_util_stats.py,
who_use_gpu/who_use_gpu.py."""
import io
import json
from datetime import datetime

import pytest

from kube_gpu_stats_amd.reports import gpu_util_stats as G
from kube_gpu_stats_amd.reports import who_use_gpu as W
from fakeprom import FakeProm
from kube_gpu_stats_amd.reports.promql import PromClient, PromError
from kube_gpu_stats_amd.reports.table import render

from fixtures import STEP, T_END, WINDOW, install_reference_scenario, reference_podlist


@pytest.fixture
def prom():
    fp = FakeProm()
    url = fp.start()
    yield fp, url
    fp.stop()


def test_gpu_util_stats_compat_golden(prom):
    fp, url = prom
    q = install_reference_scenario(fp)
    out = io.StringIO()
    c = PromClient(url)
    rows = G.run_report(c, q, datetime.fromtimestamp(T_END), WINDOW, STEP, compat=True, out=out)
    text = out.getvalue() + G.format_rows(rows, "pod", "table", compat=True) + "\n"
    assert text == ('{\n  "node-a": {\n    "pod1": "4",\n    "pod2": "2"\n  }\n}\n'
                    "['node-a', 'pod1', '4', 50.0]\n['node-a', 'pod2', '2', 0.0]\n")
    # call order M1 → M2 → M3 → M4 → M5, both range queries step 3600 over one day
    paths = [p for p, _ in c.calls]
    assert paths == ["/query_range", "/query", "/query", "/query", "/query_range"]
    assert [c.calls[i][1]["query"] for i in range(5)] == [q.util, q.total, q.used, q.live, q.req]
    for i in (0, 4):
        prm = c.calls[i][1]
        assert prm["step"] == 3600 and prm["end"] - prm["start"] == 86400


def test_compat_reproduces_reference_proxy_pattern(prom, monkeypatch):
    """the reference proxies M1-M3 and M5 but not the instant
    query M4 (gpu_util_stats.py:32 vs :24,107,119): pattern T,T,T,F,T.  --compat keeps
    it; the fixed mode proxies every call.  The fake Prometheus doubles as the proxy
    and sees absolute-URL request lines for proxied calls."""
    for k in ("NO_PROXY", "no_proxy", "HTTP_PROXY", "http_proxy"):
        monkeypatch.delenv(k, raising=False)
    fp, url = prom
    q = install_reference_scenario(fp)
    proxy = url.rsplit("/api/v1", 1)[0]
    c = PromClient(url, proxy=proxy)
    G.run_report(c, q, datetime.fromtimestamp(T_END), WINDOW, STEP, compat=True, out=io.StringIO())
    assert c.proxied == [True, True, True, False, True]
    assert fp.via_proxy[-5:] == [True, True, True, False, True]
    c2 = PromClient(url, proxy=proxy)
    G.run_report(c2, q, datetime.fromtimestamp(T_END), WINDOW, STEP, compat=False, out=io.StringIO())
    assert all(c2.proxied) and all(fp.via_proxy[-5:])


def test_node_report_compat_golden(prom):
    fp, url = prom
    q = install_reference_scenario(fp)
    c = PromClient(url)
    rows = G.run_report(c, q, datetime.fromtimestamp(T_END), WINDOW, STEP, compat=True, mode="node")
    assert rows == [["node-a", "v100", 11.25, "6", "8"], ["node-b", "p4", 10.416666666666666, 0, "4"]]


def test_node_report_fixed_mode_fixes_q1_q2():
    util = {"data": {"result": [
        {"metric": {"kubernetes_io_hostname": "n", "namespace": "ml", "pod_name": "a"}, "values": [[0, "50"], [3600, "50"]]},
        {"metric": {"kubernetes_io_hostname": "n", "namespace": "ml", "pod_name": "b"}, "values": [[0, "90"], [3600, "90"]]},
    ]}}
    servers = {"n": (8, 6, "MI355X")}
    # card-weighted: a holds 6 cards, b holds 2 → (6*50 + 2*90)/8 = 60
    rows = G.stats_server_results(util, servers, 7200, 3600, compat=False,
                                  weights={"n": {("ml", "a"): 6, ("ml", "b"): 2}})
    assert rows == [["n", "MI355X", 60.0, 6, 8]]
    rows = G.stats_server_results(util, servers, 4 * 3600, 3600, compat=False, missing="zero",
                                  weights={"n": {("ml", "a"): 1, ("ml", "b"): 1}})
    assert rows[0][2] == pytest.approx(70.0 * 2 / 4)


def test_pod_report_fixed_mode_ints_and_max_cards(prom):
    fp, url = prom
    q = G.Queries.amd("ml", STEP)
    fp.add_range(q.util, [{"metric": {"kubernetes_io_hostname": "n1", "namespace": "ml", "pod_name": "p"},
                           "values": [[T_END - 3600, "40"], [T_END, "60"]]}])
    fp.add_instant(q.total, [{"metric": {"node": "n1", q.type_label: "MI355X"}, "value": [T_END, "8"]}])
    fp.add_instant(q.used, [{"metric": {"node": "n1"}, "value": [T_END, "4"]}])
    fp.add_instant(q.live, [{"metric": {"namespace": "ml", "pod": "p"}, "value": [T_END, "1"]}])
    fp.add_range(q.req, [{"metric": {"node": "n1", "namespace": "ml", "pod": "p"},
                          "values": [[T_END - 3600, "2"], [T_END, "4"]]}])
    out = io.StringIO()
    rows = G.run_report(PromClient(url), q, T_END, 7200, STEP, compat=False, out=out)
    assert rows == [["n1", "ml", "p", 4, 50.0]]
    assert out.getvalue() == ""  # no debug dump on stdout (Q8)
    table = G.format_rows(rows, "pod", "table", compat=False)
    assert "| n1   | p   |  4   | 50.00  |" in table or "50.00" in table
    assert json.loads(G.format_rows(rows, "pod", "json", False))[0]["GPUs"] == 4


def test_amd_queries_mention_amd_resource():
    q = G.Queries.amd("ml", 3600)
    assert 'resource="amd_com_gpu"' in q.total and 'resource="amd_com_gpu"' in q.req
    assert q.util == ("100 * avg(rate(container_gpu_busy_seconds_total[3600s])) "
                      "by (kubernetes_io_hostname, nvidia_gpu_type, namespace, pod_name)")
    assert q.live.endswith("by (namespace, pod) > 0") and q.req.endswith("by (node, namespace, pod)")
    assert "avg_over_time(container_gpu_sm_util[3600s])" in G.Queries.amd("ml", 3600, util_metric="container_gpu_sm_util").util
    assert 'namespace="ml"' in q.live
    assert 'namespace=' not in G.Queries.amd("", 60).live


def test_prom_errors_are_typed(prom):
    fp, url = prom
    c = PromClient(url)
    with pytest.raises(PromError):
        c.query("rate(nonsense[5m])")  # fake answers 400 bad_data
    with pytest.raises(PromError):
        PromClient("http://127.0.0.1:9/api/v1", timeout_s=0.5).query("up")


def test_who_use_gpu_compat_golden():
    out = io.StringIO()
    rows, total, per_type = W.census(reference_podlist(), compat=True, resources=(W.REF_GPU_RESOURCE,), out=out)
    assert out.getvalue() == "'nodeName'\n"
    assert [r.as_list() for r in rows] == [["ava", "node-a", "train-1", "tesla-v100", 6],
                                            ["dev", "node-b", "no-aff", "<unspecified>", 1]]
    assert total == 7 and per_type == {"tesla-v100": 6, "<unspecified>": 1}
    text = W.format_report(rows, total, per_type)
    assert text.splitlines()[-3:] == ["Total GPU: 7", "tesla-v100\t6", "<unspecified>\t1"]
    assert "| Namespace |  Node  |   Pod   |    GPU Type   | GPU Cores |" in text
    # Q16: the column counts devices, so fixed mode names it "GPUs"
    fixed = W.format_report(rows, total, per_type, compat=False)
    assert "GPU Cores" not in fixed and "GPUs |" in fixed


def test_who_use_gpu_fixed_mode():
    from fixtures import ctr, pod

    R = "amd.com/gpu"
    pods = {"items": [
        pod("a", "ml", "n1", [ctr("x", {R: "2"}), ctr("y", requests={R: "1"})]),
        pod("init-heavy", "ml", "n1", [ctr("x", {R: "1"})], init=[ctr("i", {R: "4"})]),
        pod("done", "ml", "n1", [ctr("x", {R: "8"})], phase="Succeeded"),
        pod("queued", "ml", None, [ctr("x", {R: "1"})], phase="Pending"),
    ]}
    nodes = {"n1": {"metadata": {"name": "n1", "labels": {"amd.com/gpu.product-name": "MI355X"}}}}
    rows, total, per_type = W.census(pods, compat=False, resources=(R,), nodes=nodes)
    got = {r.pod: (r.node, r.gpu_type, r.gpus) for r in rows}
    assert got == {"a": ("n1", "MI355X", 3), "init-heavy": ("n1", "MI355X", 4),
                   "queued": ("<unscheduled>", "<unspecified>", 1)}
    assert total == 8
    rows2, total2, _ = W.census(pods, compat=False, resources=(R,), nodes=nodes, include_finished=True)
    assert total2 == 16


def test_table_matches_prettytable_centering():
    t = render(["A", "Long header"], [["xy", 1], ["odd", 22]])
    assert t.splitlines() == [
        "+-----+-------------+",
        "|  A  | Long header |",
        "+-----+-------------+",
        "|  xy |      1      |",
        "| odd |      22     |",
        "+-----+-------------+",
    ]


def test_idle_gpu_hours_column_and_total():
    """--idle-hours: cards × window hours × (1 − util) per pod, plus a total row."""
    rows = G.idle_gpu_hours([["n1", "ml", "a", 4, 25.0], ["n1", "ml", "b", 2, 100.0], ["n2", "dev", "c", 1, 0.0]],
                            86400)
    assert [r[5] for r in rows] == [72.0, 0.0, 24.0]
    table = G.format_rows(rows, "pod", "table", compat=False, idle_hours=True)
    assert "Idle GPU-h" in table and "TOTAL" in table and "96.00" in table
    js = json.loads(G.format_rows(rows, "pod", "json", False, idle_hours=True))
    assert js[0]["Idle GPU-h"] == 72.0 and len(js) == 3


def test_api_pod_list_follows_continue_tokens():
    """`--source api` lists pods in pages (limit + metadata.continue) like kubectl."""
    from kube_gpu_stats_amd.reports.who_use_gpu import api_list

    pages = {"": (["a", "b"], "t1"), "t1": (["c", "d"], "t/2=="), "t/2==": (["e"], "")}
    seen = []

    def get(path, timeout):
        seen.append(path)
        tok = ""
        if "continue=" in path:
            import urllib.parse

            tok = urllib.parse.unquote(path.split("continue=")[1])
        names, nxt = pages[tok]
        return {"kind": "PodList", "metadata": {"continue": nxt} if nxt else {},
                "items": [{"metadata": {"name": n}} for n in names]}

    out = api_list("/api/v1/pods?fieldSelector=spec.nodeName%3Dn1", 5.0, limit=2, get=get)
    assert [p["metadata"]["name"] for p in out["items"]] == ["a", "b", "c", "d", "e"]
    assert "continue" not in out["metadata"] and out["kind"] == "PodList"
    assert seen[0] == "/api/v1/pods?fieldSelector=spec.nodeName%3Dn1&limit=2"
    assert seen[2].endswith("&limit=2&continue=t%2F2%3D%3D")


def test_util_report_rolls_up_per_namespace():
    """gpu-util-stats --group-by namespace: GPU-hours held / busy / idle and util per
    namespace from the pod rows' own Namespace column (+ extras' totals)."""
    from kube_gpu_stats_amd.reports import gpu_util_stats as G

    rows = [["n1", "ml", "a", 4, 50.0, 1.5], ["n1", "ml", "b", 2, 100.0, 0.5], ["n2", "vision", "c", 8, 25.0, 2.0],
            ["n2", "vision", "d (finished)", 1, 10.0, 0.1]]
    header, out = G.by_namespace(rows, 86400, ["Energy kWh"])
    assert header == G.NS_HEADER + ["Energy kWh"]
    by = {r[0]: r for r in out}
    # vision: 9 cards × 24 h = 216 GPU-h; busy 8·24·0.25 + 1·24·0.10 = 50.4
    assert by["vision"][1:3] == [2, 9.0] and by["vision"][3] == 216.0
    assert abs(by["vision"][4] - 50.4) < 1e-9 and abs(by["vision"][6] - 165.6) < 1e-9
    assert abs(by["vision"][7] - 2.1) < 1e-9
    # ml: 6 cards = 144 GPU-h, busy 4·24·0.5 + 2·24 = 96 → 66.7 %
    assert abs(by["ml"][5] - 100 * 96 / 144) < 1e-9
    assert [r[0] for r in out] == ["vision", "ml", "TOTAL"]  # most GPU-hours first
    tot = by["TOTAL"]
    assert tot[1] == 4 and tot[3] == 360.0 and abs(tot[5] - 100 * (96 + 50.4) / 360) < 1e-9
    text = G.format_namespace_rows(header, out, "table")
    assert "vision" in text and "TOTAL" in text
    # idle-hours as an extra is not double counted (it is a column already)
    h2, _ = G.by_namespace([r[:5] + [0.0, r[5]] for r in rows], 86400, ["Idle GPU-h", "Energy kWh"])
    assert h2 == G.NS_HEADER + ["Energy kWh"]


def install_two_namespaces(fp, q):
    """train-0 in namespaces a and b on one node: 2 and 4 cards, 30 % and 80 % util."""
    fp.add_range(q.util, [{"metric": {"kubernetes_io_hostname": "n1", "nvidia_gpu_type": "MI355X", "namespace": ns,
                                      "pod_name": "train-0"}, "values": [[T_END - 3600, u], [T_END, u]]}
                          for ns, u in (("a", "30"), ("b", "80"))])
    fp.add_instant(q.total, [{"metric": {"node": "n1", q.type_label: "MI355X"}, "value": [T_END, "8"]}])
    fp.add_instant(q.used, [{"metric": {"node": "n1"}, "value": [T_END, "6"]}])
    fp.add_instant(q.live, [{"metric": {"namespace": ns, "pod": "train-0"}, "value": [T_END, "1"]} for ns in "ab"])
    fp.add_range(q.req, [{"metric": {"node": "n1", "namespace": ns, "pod": "train-0"}, "values": [[T_END, c]]}
                         for ns, c in (("a", "2"), ("b", "4"))])


def test_fixed_mode_keeps_equal_pod_names_in_two_namespaces_apart(prom):
    """VERDICT r2 #5 / SURVEY §2.6: the reference's live filter is namespaced but its
    request and util series are not (gpu_util_stats.py:133 vs :137, :159), so two
    train-0 pods merge.  The fixed mode joins on (namespace, pod)."""
    fp, url = prom
    q = G.Queries.amd("", STEP)
    install_two_namespaces(fp, q)
    rows = G.run_report(PromClient(url), q, T_END, 7200, STEP, compat=False)
    assert rows == [["n1", "a", "train-0", 2, 30.0], ["n1", "b", "train-0", 4, 80.0]]
    table = G.format_rows(rows, "pod", "table", compat=False)
    assert "Namespace" in table.splitlines()[1] or "Namespace" in table
    idle = G.idle_gpu_hours(rows, 7200)
    assert [round(r[5], 6) for r in idle] == [2 * 2 * 0.7, 4 * 2 * 0.2]
    header, ns_rows = G.by_namespace(idle, 7200, ["Idle GPU-h"])
    assert {r[0]: r[2] for r in ns_rows} == {"a": 2.0, "b": 4.0, "TOTAL": 6.0}
    # only namespace b
    qb = G.Queries.amd("b", STEP)
    assert 'namespace="b"' in qb.live


def test_compat_mode_still_merges_across_namespaces(prom):
    """--compat reproduces the reference's join on pod name: the two train-0 series
    and requests collapse into one row (the collision SURVEY §2.6 names)."""
    fp, url = prom
    q = G.Queries.compat("a")
    fp.add_range(q.util, [{"metric": {"kubernetes_io_hostname": "n1", "nvidia_gpu_type": "MI355X",
                                      "pod_name": "train-0"}, "values": [[T_END - 3600, "55"], [T_END, "55"]]}])
    fp.add_instant(q.total, [{"metric": {"node": "n1", "label_nvidia_gpu_type": "MI355X"}, "value": [T_END, "8"]}])
    fp.add_instant(q.used, [{"metric": {"node": "n1"}, "value": [T_END, "6"]}])
    fp.add_instant(q.live, [{"metric": {"pod": "train-0"}, "value": [T_END, "1"]}])
    fp.add_range(q.req, [{"metric": {"node": "n1", "pod": "train-0"}, "values": [[T_END, "2"]]}])
    rows = G.run_report(PromClient(url), q, datetime.fromtimestamp(T_END), 7200, STEP, compat=True,
                        out=io.StringIO())
    assert rows == [["n1", "train-0", "2", 55.0]]


def test_cli_namespace_default_all_in_fixed_mode_ava_in_compat():
    a = G.build_parser().parse_args([])
    assert a.namespace == ""
    ap = G.build_parser().parse_args(["--compat"])
    assert ap.compat and ap.namespace == ""  # resolved to the reference's 'ava' in run()


def test_cli_group_by_namespace_end_to_end(prom, capsys):
    """`kgs gpu-util-stats --group-by namespace --format json` over the fake Prometheus.
    The r series carries no namespace label (an older exporter): it joins the node's
    only allocation named r."""
    fp, url = prom
    q = G.Queries.amd("", STEP)
    fp.add_range(q.util, [{"metric": {"kubernetes_io_hostname": "n1", "namespace": "ml", "pod_name": "p"},
                           "values": [[T_END - 3600, "40"], [T_END, "60"]]},
                          {"metric": {"kubernetes_io_hostname": "n1", "pod_name": "r"},
                           "values": [[T_END - 3600, "100"], [T_END, "100"]]}])
    fp.add_instant(q.total, [{"metric": {"node": "n1", q.type_label: "MI355X"}, "value": [T_END, "8"]}])
    fp.add_instant(q.used, [{"metric": {"node": "n1"}, "value": [T_END, "6"]}])
    fp.add_instant(q.live, [{"metric": {"namespace": "ml", "pod": "p"}, "value": [T_END, "1"]},
                            {"metric": {"namespace": "infer", "pod": "r"}, "value": [T_END, "1"]}])
    fp.add_range(q.req, [{"metric": {"node": "n1", "namespace": "ml", "pod": "p"}, "values": [[T_END, "4"]]},
                         {"metric": {"node": "n1", "namespace": "infer", "pod": "r"}, "values": [[T_END, "2"]]}])
    G.main(["--prom-url", url, "--window", "7200", "--step", str(STEP), "--end", str(T_END),
            "--group-by", "namespace", "--format", "json"])
    got = {r["Namespace"]: r for r in json.loads(capsys.readouterr().out)}
    assert got["ml"]["GPU-h"] == 8.0 and got["ml"]["Util %"] == 50.0 and got["ml"]["Idle GPU-h"] == 4.0
    assert got["infer"]["GPU-h"] == 4.0 and got["infer"]["Busy GPU-h"] == 4.0
    assert got["TOTAL"]["Pods"] == 2 and abs(got["TOTAL"]["Util %"] - 100 * 8 / 12) < 1e-9


def _shared_scenario(fp):
    q = G.Queries.amd("", STEP)
    fp.add_range(q.util, [{"metric": {"kubernetes_io_hostname": "n1", "namespace": "ml", "pod_name": p},
                           "values": [[T_END, "90"]]} for p in ("a", "b")])
    fp.add_instant(q.total, [{"metric": {"node": "n1", q.type_label: "MI355X"}, "value": [T_END, "8"]}])
    fp.add_instant(q.used, [{"metric": {"node": "n1"}, "value": [T_END, "1"]}])
    fp.add_instant(q.live, [{"metric": {"namespace": "ml", "pod": p}, "value": [T_END, "1"]} for p in ("a", "b")])
    fp.add_range(q.req, [{"metric": {"node": "n1", "namespace": "ml", "pod": p}, "values": [[T_END, "1"]]}
                         for p in ("a", "b")])
    return q


def test_fixed_mode_warns_when_the_busy_counter_bills_a_shared_gpu_twice(prom, capsys):
    """pods a and b share GPU 3 of n1; the default util metric
    (container_gpu_busy_seconds_total) bills both the whole GPU, so the report says so
    on stderr and names container_gpu_cu_seconds_total — stdout stays the table."""
    fp, url = prom
    _shared_scenario(fp)
    fp.add_instant(G.shared_query(7200, STEP), [{"metric": {"kubernetes_io_hostname": "n1", "gpu": "3", "uuid": "u3"},
                                                "value": [T_END, "2"]}])
    G.main(["--prom-url", url, "--window", "7200", "--step", str(STEP), "--end", str(T_END), "--format", "json"])
    cap = capsys.readouterr()
    assert len(json.loads(cap.out)) == 2
    assert "n1/gpu3" in cap.err and "container_gpu_cu_seconds_total" in cap.err
    # per-pod compute share asked for: no warning; a Prometheus that cannot evaluate the check: no warning
    G.main(["--prom-url", url, "--window", "7200", "--step", str(STEP), "--end", str(T_END), "--format", "json",
            "--util-metric", "container_gpu_cu_seconds_total"])
    assert "warning" not in capsys.readouterr().err


def test_shared_gpu_check_is_best_effort(prom, capsys):
    fp, url = prom
    _shared_scenario(fp)  # no canned answer: the fake Prometheus rejects the subquery (400)
    G.main(["--prom-url", url, "--window", "7200", "--step", str(STEP), "--end", str(T_END), "--format", "json"])
    cap = capsys.readouterr()
    assert len(json.loads(cap.out)) == 2 and "warning" not in cap.err
