"""xGMI topology discovery and export (BASELINE.json config 5).

MI355X platforms connect the 8 GPUs of a node all-to-all: 7 point-to-point xGMI
links per GPU.  Two sources are merged:

* pairwise ``amdsmi_topo_get_link_type/weight`` between *visible* devices;
* per-link ``amdsmi_get_link_metrics`` peer PCI addresses — available even when
  the peers are not visible to this process (a 1-GPU container still learns its
  7 neighbours).

``discover()`` returns a JSON-able dict; ``node_graph()`` turns it into an
adjacency map keyed by PCI address, which ``ring_order()`` uses to pick a ring
for xGMI benchmarking (per-link bound ring collectives).
"""
from __future__ import annotations

import json
import time


def discover(backend: str = "amdsmi", mock_gpus: int = 8, wait_links_s: float = 2.0) -> dict:
    from ..native import load

    N = load()
    ex = N.Exporter({"backend": backend, "mock": {"n_gpus": mock_gpus}, "port": -1, "hz": 10,
                     "link_every": 1, "proc_every": 0, "pin_numa": False})
    ex.start()
    end = time.time() + wait_links_s
    while time.time() < end and not all(ex.links(i) for i in range(ex.device_count)):
        time.sleep(0.05)
    topo = json.loads(ex.topology_json())
    ex.stop()
    return topo


def node_graph(topo: dict) -> dict[str, set[str]]:
    """Undirected adjacency {bdf: {peer bdf}} over xGMI links (pairwise edges + link peers)."""
    bdf_of = {d["gpu"]: d["bdf"] for d in topo.get("devices", [])}
    g: dict[str, set[str]] = {b: set() for b in bdf_of.values()}
    for e in topo.get("edges", []):
        if e.get("link_type") == 2:
            a, b = bdf_of.get(e["src"]), bdf_of.get(e["dst"])
            if a and b:
                g.setdefault(a, set()).add(b)
                g.setdefault(b, set()).add(a)
    for link in topo.get("links", []):
        if link.get("link_type") != 2 or not link.get("peer_bdf"):
            continue
        a = bdf_of.get(link["gpu"])
        if a:
            g.setdefault(a, set()).add(link["peer_bdf"])
            g.setdefault(link["peer_bdf"], set()).add(a)
    return g


def ring_order(graph: dict[str, set[str]], nodes: list[str] | None = None) -> list[str]:
    """A Hamiltonian ring over ``nodes`` using only direct xGMI hops (DFS; tiny n)."""
    nodes = sorted(nodes or graph)
    if len(nodes) <= 2:
        return nodes
    want = set(nodes)

    def dfs(path: list[str]) -> list[str] | None:
        if len(path) == len(nodes):
            return path if path[0] in graph.get(path[-1], set()) else None
        for nxt in sorted(graph.get(path[-1], set()) & want):
            if nxt not in path:
                r = dfs(path + [nxt])
                if r:
                    return r
        return None

    return dfs([nodes[0]]) or nodes


def prometheus_lines(topo: dict, node: str) -> list[str]:
    """``amdgpu_xgmi_neighbor{...} 1`` lines for a static topology export (DaemonSet init)."""
    out = []
    g = node_graph(topo)
    for a in sorted(g):
        for b in sorted(g[a]):
            out.append(f'amdgpu_xgmi_neighbor{{kubernetes_io_hostname="{node}",bdf="{a}",peer_bdf="{b}"}} 1')
    return out
