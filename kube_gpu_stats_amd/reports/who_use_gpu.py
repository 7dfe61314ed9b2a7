"""``kgs who-use-gpu`` — per-pod GPU allocation census (capability F1).

Reference: who_use_gpu/who_use_gpu.py.  Pods come from ``kubectl get pods
--all-namespaces -o json`` (reference :8-10), a JSON file, or the API server.
For every pod with GPUs: ``[namespace, node, pod, gpu type, gpu count]``
(:27-49), then ``Total GPU: N`` (:23) and one ``<type>\\t<n>`` line per type (:24-25).

``--compat`` reproduces the reference exactly (SURVEY.md §2.8 golden output):
only ``resources.limits["alpha.kubernetes.io/nvidia-gpu"]`` of ``spec.containers``
(:35-41), no phase filter (Q12), an unscheduled pod prints the KeyError
``'nodeName'`` and is dropped (:33,46-48), the GPU type is the first nodeAffinity
expression's first value whatever its key (:51-58, Q13), header "GPU Cores" (Q16).

The default mode fixes Q12-Q15: resource ``amd.com/gpu`` (configurable), limits
*or* requests, init containers by the Kubernetes effective-request rule
(max(max(init), sum(containers))), Succeeded/Failed pods excluded, unscheduled
pods shown as ``<unscheduled>``, the GPU type taken from the node's labels when
node objects are available, kubectl's return code checked and a timeout applied.
"""
from __future__ import annotations

import argparse
import json
import shlex
import subprocess
import sys
from dataclasses import dataclass

from ..utils.config import AMD_GPU_RESOURCE, REF_GPU_RESOURCE, REF_KUBECTL, add_flag
from .table import render, render_csv

NODE_TYPE_LABELS = ("amd.com/gpu.product-name", "amd.com/gpu.family", "nvidia_gpu_type", "gpu-type")


@dataclass
class Row:
    namespace: str
    node: str
    pod: str
    gpu_type: str
    gpus: int

    def as_list(self):
        return [self.namespace, self.node, self.pod, self.gpu_type, self.gpus]


# ----------------------------------------------------------------------------- reference semantics
def gpu_type_from_affinity(pod: dict) -> str:
    """Reference getGPUType (who_use_gpu.py:51-58)."""
    try:
        return pod["spec"]["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][
            "nodeSelectorTerms"][0]["matchExpressions"][0]["values"][0]
    except Exception:  # noqa: BLE001 - reference swallows every error here
        return "<unspecified>"


def check_pod_compat(pod: dict, resource: str = REF_GPU_RESOURCE, out=sys.stdout) -> list:
    """Reference checkPod (who_use_gpu.py:27-49), including its printed exceptions."""
    try:
        metadata = pod["metadata"]
        name = metadata["name"]
        namespace = metadata["namespace"]
        containers = pod["spec"]["containers"]
        node = pod["spec"]["nodeName"]
        total = 0
        for c in containers:
            if "resources" not in c or "limits" not in c["resources"]:
                continue
            total += int(c["resources"]["limits"].get(resource, 0))
        if total > 0:
            return [namespace, node, name, gpu_type_from_affinity(pod), total]
    except Exception as e:  # noqa: BLE001
        print(e if not isinstance(e, KeyError) else repr(e.args[0]), file=out)
        return []
    return []


# ----------------------------------------------------------------------------- fixed semantics
def _qty(v) -> int:
    try:
        return int(str(v))
    except ValueError:
        return 0


def container_gpus(c: dict, resources: tuple[str, ...]) -> int:
    res = c.get("resources") or {}
    lim = res.get("limits") or {}
    req = res.get("requests") or {}
    n = 0
    for r in resources:
        n += _qty(lim.get(r, req.get(r, 0)))
    return n


def pod_gpus(pod: dict, resources: tuple[str, ...]) -> int:
    spec = pod.get("spec") or {}
    main = sum(container_gpus(c, resources) for c in spec.get("containers") or [])
    init = max([container_gpus(c, resources) for c in spec.get("initContainers") or []] or [0])
    return max(main, init)


def node_gpu_type(node_obj: dict | None, labels=NODE_TYPE_LABELS) -> str | None:
    if not node_obj:
        return None
    lab = (node_obj.get("metadata") or {}).get("labels") or {}
    for k in labels:
        if lab.get(k):
            return lab[k]
    return None


def check_pod(pod: dict, resources: tuple[str, ...], nodes: dict[str, dict], include_finished: bool) -> Row | None:
    md = pod.get("metadata") or {}
    phase = (pod.get("status") or {}).get("phase", "")
    if not include_finished and phase in ("Succeeded", "Failed"):
        return None
    n = pod_gpus(pod, resources)
    if n <= 0:
        return None
    node = (pod.get("spec") or {}).get("nodeName") or "<unscheduled>"
    gtype = node_gpu_type(nodes.get(node)) or gpu_type_from_affinity(pod)
    return Row(md.get("namespace", ""), node, md.get("name", ""), gtype, n)


# ----------------------------------------------------------------------------- sources
def load_pods(source: str, kubectl: str, path: str, timeout: float) -> dict:
    if source == "file":
        if path == "-":
            return json.load(sys.stdin)
        with open(path) as f:
            return json.load(f)
    if source == "kubectl":
        r = subprocess.run(shlex.split(kubectl), capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"kubectl failed ({r.returncode}): {r.stderr.strip()}")
        return json.loads(r.stdout)
    if source == "api":
        return api_list("/api/v1/pods", timeout)
    raise ValueError(source)


def api_list(path: str, timeout: float, limit: int = 500, get=None) -> dict:
    """A LIST over the API server in pages of ``limit`` (``metadata.continue``), as
    kubectl does: a cluster of tens of thousands of pods is never one response."""
    import urllib.parse

    get = get or _api_get
    sep = "&" if "?" in path else "?"
    items: list = []
    token = ""
    while True:
        q = f"{path}{sep}limit={limit}" + (f"&continue={urllib.parse.quote(token, safe='')}" if token else "")
        page = get(q, timeout)
        items.extend(page.get("items") or [])
        token = (page.get("metadata") or {}).get("continue") or ""
        if not token:
            page["items"] = items
            page.setdefault("metadata", {}).pop("continue", None)
            return page


def _api_get(path: str, timeout: float) -> dict:
    """In-cluster API server GET with the pod's service-account token."""
    import os

    import requests

    host = os.environ.get("KUBERNETES_SERVICE_HOST")
    port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
    sa = "/var/run/secrets/kubernetes.io/serviceaccount"
    if not host:
        raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
    with open(f"{sa}/token") as f:
        token = f.read().strip()
    r = requests.get(f"https://{host}:{port}{path}", headers={"Authorization": f"Bearer {token}"},
                     verify=f"{sa}/ca.crt", timeout=timeout)
    r.raise_for_status()
    return r.json()


# ----------------------------------------------------------------------------- report
def census(pods: dict, compat: bool, resources: tuple[str, ...] = (AMD_GPU_RESOURCE,), nodes: dict | None = None,
           include_finished: bool = False, out=sys.stdout) -> tuple[list[Row], int, dict[str, int]]:
    rows: list[Row] = []
    total = 0
    per_type: dict[str, int] = {}
    for pod in pods.get("items", []):
        if compat:
            r = check_pod_compat(pod, resources[0], out)
            if not r:
                continue
            row = Row(*r)
        else:
            row = check_pod(pod, resources, nodes or {}, include_finished)
            if row is None:
                continue
        total += row.gpus
        per_type[row.gpu_type] = per_type.get(row.gpu_type, 0) + row.gpus
        rows.append(row)
    return rows, total, per_type


HEADER = ["Namespace", "Node", "Pod", "GPU Type", "GPU Cores"]  # reference header (who:11); counts devices (Q16)
HEADER_FIXED = ["Namespace", "Node", "Pod", "GPU Type", "GPUs"]


def format_report(rows: list[Row], total: int, per_type: dict[str, int], fmt: str = "table",
                  compat: bool = True) -> str:
    header = HEADER if compat else HEADER_FIXED
    if fmt == "json":
        return json.dumps({"pods": [r.__dict__ for r in rows], "total": total, "per_type": per_type}, indent=2)
    if fmt == "csv":
        return render_csv(header, [r.as_list() for r in rows])
    lines = [render(header, [r.as_list() for r in rows]), "Total GPU: %d" % total]
    lines += ["%s\t%d" % (t, n) for t, n in per_type.items()]
    return "\n".join(lines)


def build_parser(ap: argparse.ArgumentParser | None = None) -> argparse.ArgumentParser:
    ap = ap or argparse.ArgumentParser(prog="kgs who-use-gpu", description=__doc__.splitlines()[0])
    add_flag(ap, "compat", False, "reproduce the reference output and quirks exactly")
    add_flag(ap, "source", "kubectl", "pod source: kubectl | file | api")
    add_flag(ap, "pods-json", "-", "PodList JSON file for --source file ('-' = stdin)")
    add_flag(ap, "nodes-json", "", "optional NodeList JSON (GPU type from node labels)")
    add_flag(ap, "kubectl", REF_KUBECTL, "kubectl command line")
    add_flag(ap, "resource", "", f"GPU resource names, comma separated (default {AMD_GPU_RESOURCE}; "
                                 f"--compat: {REF_GPU_RESOURCE})")
    add_flag(ap, "include-finished", False, "count Succeeded/Failed pods too")
    add_flag(ap, "format", "table", "table | json | csv")
    add_flag(ap, "timeout", 30.0, "kubectl / API timeout seconds")
    return ap


def run(a) -> int:
    pods = load_pods(a.source, a.kubectl, a.pods_json, a.timeout)
    if a.resource:
        resources = tuple(r for r in a.resource.split(",") if r)
    else:
        resources = (REF_GPU_RESOURCE,) if a.compat else (AMD_GPU_RESOURCE,)
    nodes = {}
    if a.nodes_json:
        with open(a.nodes_json) as f:
            nodes = {n["metadata"]["name"]: n for n in json.load(f).get("items", [])}
    rows, total, per_type = census(pods, a.compat, resources, nodes, a.include_finished)
    print(format_report(rows, total, per_type, "table" if a.compat else a.format, compat=a.compat))
    return 0


def main(argv=None) -> int:
    return run(build_parser().parse_args(argv))


if __name__ == "__main__":
    sys.exit(main())
