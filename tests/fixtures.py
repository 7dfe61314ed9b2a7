"""Shared fixtures: the SURVEY.md §2.8 golden scenarios (reproduced there with a
fake-Prometheus harness around Python-3 copies of the reference)."""
from __future__ import annotations

from kube_gpu_stats_amd.reports import gpu_util_stats as G

T_END = 1_700_000_000
STEP = 3600
WINDOW = 86400


def util_series(host, gpu_type, pod, values, t0=T_END - WINDOW):
    return {"metric": {"kubernetes_io_hostname": host, "nvidia_gpu_type": gpu_type, "pod_name": pod},
            "values": [[t0 + i * STEP, str(v)] for i, v in enumerate(values)]}


def install_reference_scenario(fp, namespace="ava"):
    """node-a: 8× v100, 6 used; node-b: 4× p4; live pods pod1, pod2."""
    q = G.Queries.compat(namespace)
    fp.add_range(q.util, [
        util_series("node-a", "v100", "pod1", [50.0] * 25),
        util_series("node-a", "v100", "pod-ended", [90.0] * 3),
        util_series("node-b", "p4", "pod3", [10.0] * 25),
        util_series("node-c", "v100", "pod4", [70.0] * 25),
    ])
    fp.add_instant(q.total, [
        {"metric": {"node": "node-a", "label_nvidia_gpu_type": "v100"}, "value": [T_END, "8"]},
        {"metric": {"node": "node-b", "label_nvidia_gpu_type": "p4"}, "value": [T_END, "4"]},
    ])
    fp.add_instant(q.used, [{"metric": {"node": "node-a"}, "value": [T_END, "6"]}])
    fp.add_instant(q.live, [{"metric": {"pod": "pod1"}, "value": [T_END, "1"]},
                            {"metric": {"pod": "pod2"}, "value": [T_END, "1"]}])
    fp.add_range(q.req, [
        {"metric": {"node": "node-a", "pod": "pod1"}, "values": [[T_END - WINDOW, "4"], [T_END, "4"]]},
        {"metric": {"node": "node-a", "pod": "pod2"}, "values": [[T_END - 7200, "2"], [T_END, "2"]]},
        {"metric": {"node": "node-b", "pod": "pod-x"}, "values": [[T_END, "1"]]},
    ])
    return q


def pod(name, ns, node=None, containers=(), init=(), phase="Running", affinity=None):
    spec = {"containers": list(containers)}
    if init:
        spec["initContainers"] = list(init)
    if node is not None:
        spec["nodeName"] = node
    if affinity is not None:
        spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": [{"matchExpressions": [{"key": "gpu-type", "operator": "In",
                                                          "values": [affinity]}]}]}}}
    return {"metadata": {"name": name, "namespace": ns}, "spec": spec, "status": {"phase": phase}}


def ctr(name, limits=None, requests=None):
    c = {"name": name}
    if limits is not None or requests is not None:
        c["resources"] = {}
        if limits is not None:
            c["resources"]["limits"] = limits
        if requests is not None:
            c["resources"]["requests"] = requests
    return c


REF_RES = "alpha.kubernetes.io/nvidia-gpu"


def reference_podlist():
    return {"items": [
        pod("train-1", "ava", "node-a", [ctr("a", {REF_RES: "4"}), ctr("b", {REF_RES: 2}), ctr("sidecar")],
            affinity="tesla-v100"),
        pod("no-aff", "dev", "node-b", [ctr("a", {REF_RES: "1"})], phase="Succeeded"),
        pod("pending", "dev", None, [ctr("a", {REF_RES: "1"})], phase="Pending"),
        pod("cpu-only", "dev", "node-b", [ctr("a", {"cpu": "2"})]),
        pod("new-style", "dev", "node-c", [ctr("a", {"nvidia.com/gpu": "8"})]),
    ]}
