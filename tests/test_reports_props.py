"""Property tests (hypothesis) for the report aggregation, chunked range queries,
and a multi-node rehearsal: several exporters with different node names feeding
one (fake) Prometheus, reported by ``gpu-util-stats``."""
import time

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from kube_gpu_stats_amd.reports import gpu_util_stats as G
from fakeprom import FakeProm
from kube_gpu_stats_amd.reports.promql import PromClient
from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

nodes = st.sampled_from(["n1", "n2", "n3"])
namespaces = st.sampled_from(["ml", "dev"])
pods = st.sampled_from(["a", "b", "c", "d"])
vals = st.lists(st.floats(min_value=0, max_value=100, allow_nan=False), min_size=0, max_size=30)


@settings(max_examples=150, deadline=None)
@given(series=st.lists(st.tuples(nodes, namespaces, pods, vals), max_size=12),
       alloc=st.dictionaries(st.tuples(nodes, namespaces, pods), st.integers(1, 8), max_size=8),
       inventory=st.sets(nodes, min_size=1))
def test_pod_report_properties(series, alloc, inventory):
    util = {"data": {"result": [{"metric": {"kubernetes_io_hostname": n, "namespace": ns, "pod_name": p},
                                 "values": [[i, str(v)] for i, v in enumerate(vs)]} for n, ns, p, vs in series]}}
    servers = {n: (8, 0, "MI355X") for n in inventory}
    server_pods: dict = {}
    for (n, ns, p), c in alloc.items():
        server_pods.setdefault(n, {})[(ns, p)] = c
    rows = G.stats_pod_results(util, servers, server_pods, compat=False)
    # only inventoried nodes, sorted; only allocated (namespace, pod)s; util within [0, 100]
    assert [r[0] for r in rows] == sorted(r[0] for r in rows)
    for node, ns, pod, cards, u in rows:
        assert node in inventory
        assert server_pods[node][(ns, pod)] == cards
        assert 0.0 <= u <= 100.0 + 1e-9
        # the util of (ns, pod) comes from that namespace's series only (last one wins per key)
        own = [vs for n, s_ns, p, vs in series if (n, s_ns, p) == (node, ns, pod)]
        if own and own[-1]:
            assert u == pytest.approx(sum(own[-1]) / len(own[-1]))
    expected = {k for k in alloc if k[0] in inventory}
    assert {(r[0], r[1], r[2]) for r in rows} == expected


def test_show_finished_lists_unallocated_pods():
    """Q7: the reference silently drops pods that have utilisation but no live
    allocation; ``show_finished`` lists them as finished with 0 cards."""
    util = {"data": {"result": [
        {"metric": {"kubernetes_io_hostname": "n1", "namespace": "ml", "pod_name": "live"},
         "values": [[0, "40"], [1, "60"]]},
        {"metric": {"kubernetes_io_hostname": "n1", "namespace": "ml", "pod_name": "gone"}, "values": [[0, "10"]]}]}}
    servers = {"n1": (8, 1, "MI355X")}
    alloc = {"n1": {("ml", "live"): 2}}
    assert [r[2] for r in G.stats_pod_results(util, servers, alloc, compat=False)] == ["live"]
    rows = G.stats_pod_results(util, servers, alloc, compat=False, show_finished=True)
    assert sorted((r[2], r[3], round(r[4])) for r in rows) == [("gone (finished)", 0, 10), ("live", 2, 50)]
    # compat keeps the reference behaviour regardless (pod-name keys)
    assert [r[1] for r in G.stats_pod_results(util, servers, {"n1": {"live": 2}}, compat=True,
                                              show_finished=True)] == ["live"]


@settings(max_examples=60, deadline=None)
@given(series=st.lists(st.tuples(pods, st.lists(st.floats(0, 100, allow_nan=False), min_size=1, max_size=10)),
                       min_size=1, max_size=5))
def test_node_report_weighted_mean_is_bounded(series):
    util = {"data": {"result": [{"metric": {"kubernetes_io_hostname": "n", "pod_name": p},
                                 "values": [[i * 60, str(v)] for i, v in enumerate(vs)]} for p, vs in series]}}
    rows = G.stats_server_results(util, {"n": (8, 1, "MI355X")}, 600, 60, compat=False)
    allv = [v for _, vs in series for v in vs]
    assert min(allv) - 1e-9 <= rows[0][2] <= max(allv) + 1e-9


def test_chunked_range_query_merges_series():
    fp = FakeProm()
    url = fp.start()
    try:
        for t in range(0, 100):
            fp.ingest({"m": [({"kubernetes_io_hostname": "n", "pod_name": "p"}, float(t))]}, float(t))
        c = PromClient(url)
        body = c.query_range("avg(m) by (kubernetes_io_hostname, pod_name)", 0, 99, 1, max_points=17)
        vs = body["data"]["result"][0]["values"]
        assert [int(v[0]) for v in vs] == list(range(100))
        assert len([p for p, _ in c.calls if p == "/query_range"]) == 6  # ceil(100/17)
    finally:
        fp.stop()


@pytest.mark.slow
def test_multi_node_rehearsal(N):
    """Three node exporters (mock) → one TSDB → per-pod report across nodes."""
    exs = []
    fp = FakeProm()
    url = fp.start()
    try:
        for i, util in enumerate((20.0, 50.0, 80.0)):
            ex = N.Exporter({"backend": "mock", "mock": {"n_gpus": 2, "util_base": util, "util_amp": 0.0001},
                             "hz": 100, "port": 0, "node_name": f"node-{i}", "pin_numa": False, "window_s": 0.2})
            ex.start()
            ex.set_device_owners(0, [{"pod": f"job-{i}", "namespace": "ml", "container": "c"}])
            exs.append(ex)
        time.sleep(0.4)
        t0 = 1_700_000_000.0
        for k in range(4):
            for ex in exs:
                fp.ingest(parse_text(Scraper("127.0.0.1", ex.port).get()), t0 + 15 * k)
        q = G.Queries.amd("ml", 15, util_metric="container_gpu_sm_util")
        fp.add_instant(q.total, [{"metric": {"node": f"node-{i}", q.type_label: "MI355X"}, "value": [t0, "2"]}
                                 for i in range(3)])
        fp.add_instant(q.used, [{"metric": {"node": f"node-{i}"}, "value": [t0, "1"]} for i in range(3)])
        fp.add_instant(q.live, [{"metric": {"namespace": "ml", "pod": f"job-{i}"}, "value": [t0, "1"]}
                                for i in range(3)])
        fp.add_range(q.req, [{"metric": {"node": f"node-{i}", "namespace": "ml", "pod": f"job-{i}"},
                              "values": [[t0, "1"]]} for i in range(3)])
        rows = G.run_report(PromClient(url), q, t0 + 45, 45, 15, compat=False)
        assert [tuple(r[:4]) for r in rows] == [("node-0", "ml", "job-0", 1), ("node-1", "ml", "job-1", 1),
                                                ("node-2", "ml", "job-2", 1)]
        assert [round(r[4]) for r in rows] == [20, 50, 80]
        node_rows = G.run_report(PromClient(url), q, t0 + 45, 45, 15, compat=False, mode="node")
        assert [round(r[2]) for r in node_rows] == [20, 50, 80]
    finally:
        for ex in exs:
            ex.stop()
        fp.stop()
