"""``kgs gpu-util-stats`` — daily GPU utilisation accounting (capabilities F2-F4).

Reference: gpu_util_stats/gpu_util_stats.py.

* F2 node inventory (``get_gpu_servers`` :96-127): allocatable cards ⋈ node GPU
  type label, and cards requested by Running pods, per node.
* F3 per-pod report (``stats_pod_results`` :62-94 + ``get_pod_by_servers``
  :129-151 + ``main`` :154-163): mean ``container_gpu_sm_util`` per (node, pod)
  over the window joined with the pod's card count, for live (Running/Pending)
  pods of one namespace.
* F4 per-node report (``stats_server_results`` :36-60, dead code in the
  reference): time-weighted node utilisation + type + used + total.

``--compat`` issues the reference's five PromQL queries verbatim (M1-M5, in the
order M1 → M2 → M3 → M4 → M5) and reproduces its arithmetic and
output exactly, quirks included (Q1 overwrite, Q2 divide-by-range, Q5 first
sample, Q6 string counts, Q7 finished pods dropped, Q8 JSON dump on stdout), and
the reference's cross-namespace join: only the live-pod filter is namespaced
(:133), the request and util series are not (:137, :159), so two pods of one name
in two namespaces merge.

The default mode joins on (namespace, pod) throughout — the util series grouped
``by (kubernetes_io_hostname, nvidia_gpu_type, namespace, pod_name)``, requests
``by (node, namespace, pod)``, live pods ``by (namespace, pod)`` — and reports a
Namespace column; its ``--namespace`` defaults to every namespace.
The default mode keeps the join semantics but fixes the quirks: exact per-step
means (Q4) from the exporter's per-pod counter
``100 * avg(rate(container_gpu_busy_seconds_total[step])) by (...)`` — the
integral of the PMFW busy accumulators since the pod got the GPU, so bursts
between scrapes count; a gauge (``--util-metric container_gpu_sm_util``) gets
``avg_over_time`` instead, which only sees what the exporter's window saw at each
scrape — max card count (Q5), ints (Q6), series of one node combined
card-weighted (Q1), time-weighted means with ``--missing`` (Q2/Q3), AMD
resource/label names, debug output on stderr (Q8).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from dataclasses import dataclass
from datetime import datetime, timedelta

from ..utils import log
from ..utils.config import (REF_NAMESPACE, REF_PROM_URL, REF_PROXY, REF_STEP_S, REF_TIMEOUT_S, REF_WINDOW_S,
                            add_flag)
from .promql import PromClient, result, to_unix
from .table import render, render_csv

L = log.get("gpu_util_stats")

# --------------------------------------------------------------------------- queries
REF_Q_UTIL = "avg(container_gpu_sm_util) by (kubernetes_io_hostname, nvidia_gpu_type, pod_name)"  # :159
REF_Q_TOTAL = ("max(kube_node_status_allocatable_nvidia_gpu_cards * on (instance, node) "
               "group_left(label_nvidia_gpu_type) kube_node_labels) by (node,label_nvidia_gpu_type)")  # :105
REF_Q_USED = ('(sum(max(kube_pod_container_resource_requests_nvidia_gpu_devices{node!=""} * on (instance,pod)  '
              'group_right(node) kube_pod_status_phase{phase="Running"}) by (node,pod)) by (node) > 0) '
              '* on (node) group_right kube_node_labels')  # :117
REF_Q_LIVE = 'max(kube_pod_status_phase{namespace="%s",phase=~"Running|Pending"}) by (pod) > 0'  # :133
REF_Q_REQ = "max(kube_pod_container_resource_requests_nvidia_gpu_devices) by (node, pod)"  # :137


@dataclass
class Queries:
    util: str
    total: str
    used: str
    live: str
    req: str
    type_label: str
    util_host: str = "kubernetes_io_hostname"
    util_pod: str = "pod_name"

    @classmethod
    def compat(cls, namespace: str = REF_NAMESPACE) -> "Queries":
        return cls(REF_Q_UTIL, REF_Q_TOTAL, REF_Q_USED, REF_Q_LIVE % namespace, REF_Q_REQ, "label_nvidia_gpu_type")

    @classmethod
    def amd(cls, namespace: str, step_s: int, resource: str = "amd_com_gpu",
            type_label: str = "label_amd_com_gpu_product_name",
            util_metric: str = "container_gpu_busy_seconds_total") -> "Queries":
        ns = f'namespace="{namespace}",' if namespace else ""
        return cls(
            util=util_query(util_metric, step_s),
            total=(f'max(kube_node_status_allocatable{{resource="{resource}"}} * on (node) '
                   f"group_left({type_label}) max(kube_node_labels) by (node, {type_label})) by (node, {type_label})"),
            used=(f'sum(max(kube_pod_container_resource_requests{{resource="{resource}",node!=""}} '
                  f'* on (namespace, pod) group_left() max(kube_pod_status_phase{{phase="Running"}}) '
                  f"by (namespace, pod)) by (node, namespace, pod)) by (node) > 0"),
            live=f'max(kube_pod_status_phase{{{ns}phase=~"Running|Pending"}}) by (namespace, pod) > 0',
            req=f'max(kube_pod_container_resource_requests{{resource="{resource}"}}) by (node, namespace, pod)',
            type_label=type_label,
        )


def util_query(metric: str, step_s: int) -> str:
    """Per-(node, type, namespace, pod) utilisation percent per step.  A
    ``*_seconds_total`` counter (busy seconds since allocation) gives the exact mean
    over each step, ``100 * rate``; a gauge can only be averaged at the scrapes."""
    by = "by (kubernetes_io_hostname, nvidia_gpu_type, namespace, pod_name)"
    if metric.endswith("_seconds_total"):
        return f"100 * avg(rate({metric}[{step_s}s])) {by}"
    return f"avg(avg_over_time({metric}[{step_s}s])) {by}"


# --------------------------------------------------------------------------- collectors (L2)
def get_gpu_servers(c: PromClient, q: Queries, compat: bool) -> dict[str, tuple]:
    """{node: (total, used, type)} — reference get_gpu_servers :96-127 (M2, M3)."""
    server_card, server_total, server_used = {}, {}, {}
    for res in result(c.query(q.total)):
        node = res["metric"]["node"]
        server_card[node] = res["metric"].get(q.type_label, "")
        server_total[node] = res["value"][1]
    for res in result(c.query(q.used)):
        server_used[res["metric"]["node"]] = res["value"][1]
    out = {}
    for node in server_total:
        if compat:  # strings, used defaults to int 0 (:126, Q6)
            out[node] = (server_total[node], server_used.get(node, 0), server_card.get(node, ""))
        else:
            out[node] = (int(float(server_total[node])), int(float(server_used.get(node, 0))),
                         server_card.get(node, ""))
    return out


def get_pod_by_servers(c: PromClient, q: Queries, start, end, step_s: int, compat: bool,
                       out=sys.stdout) -> dict[str, dict]:
    """Live pods' cards per node — reference get_pod_by_servers :129-151 (M4, M5).
    compat: {node: {pod: cards}}, joined on pod name only (:143-145); fixed:
    {node: {(namespace, pod): cards}}."""
    # M4 is the reference's query_prom_instant, which sends no proxy (:32, Q9)
    live_rows = result(c.query(q.live, proxied=not compat))
    live = ({m["metric"]["pod"] for m in live_rows} if compat
            else {(m["metric"].get("namespace", ""), m["metric"]["pod"]) for m in live_rows})
    res = {}
    for m in result(c.query_range(q.req, start, end, step_s)):
        node = m["metric"].get("node", "<unknown>")
        pod = m["metric"].get("pod", "<unknown>")
        if not m.get("values"):
            continue
        if compat:
            val = m["values"][0][1]  # first sample, string (Q5, Q6)
            key = pod
        else:
            val = int(max(float(v[1]) for v in m["values"]))
            key = (m["metric"].get("namespace", ""), pod)
        if key not in live:
            continue
        res.setdefault(node, {})[key] = val
    if compat:
        print(json.dumps(res, indent=2), file=out)  # :150 (Q8)
    else:
        L.debug("live GPU pods: %s", {n: {"/".join(k): v for k, v in p.items()} for n, p in res.items()})
    return res


# --------------------------------------------------------------------------- aggregation (L3)
# Pod rows: compat [node, pod, cards, util] (the reference's, :92); fixed
# [node, namespace, pod, cards, util, *extras].
F_NODE, F_NS, F_POD, F_CARDS, F_UTIL, F_EXTRA = range(6)


def _series_key(metric: dict, allocated: dict) -> tuple[str, str]:
    """(namespace, pod) of a util series.  A series without a namespace label (an
    exporter that predates it) joins the node's one allocation of that pod name,
    when there is exactly one."""
    pod = metric.get("pod_name", "")
    ns = metric.get("namespace")
    if ns is not None and ns != "":
        return ns, pod
    same = [k for k in allocated if k[1] == pod]
    return same[0] if len(same) == 1 else ("", pod)


def stats_pod_results(util_body: dict, servers: dict, server_pods: dict, compat: bool,
                      show_finished: bool = False) -> list[list]:
    """Reference stats_pod_results :62-94 (F3).  compat joins util and allocations on
    the pod name (the reference's cross-namespace merge); fixed on (namespace, pod)."""
    vals: dict[str, dict] = {}
    for res in result(util_body):
        server = res["metric"].get("kubernetes_io_hostname", "")
        key = (res["metric"].get("pod_name", "") if compat
               else _series_key(res["metric"], server_pods.get(server, {})))
        v = [float(x[1]) for x in res.get("values", [])]
        vals.setdefault(server, {})[key] = sum(v) / len(v) if v else 0.0
    lines = []
    for server in sorted(servers):
        if server not in server_pods and server not in vals:
            continue
        pods = set(server_pods.get(server, {})) | set(vals.get(server, {}))
        for key in sorted(pods):  # the reference iterates a set (unspecified order); sorted is stable
            cards = server_pods.get(server, {}).get(key)
            u = vals.get(server, {}).get(key, 0.0)
            if compat:
                if cards is not None:  # finished pod with util but no allocation dropped (:87-90, Q7)
                    lines.append([server, key, cards, u])
                continue
            ns, pod = key
            if cards is None:
                if show_finished:
                    lines.append([server, ns, pod + " (finished)", 0, u])
                continue
            lines.append([server, ns, pod, cards, u])
    return lines


def stats_server_results(util_body: dict, servers: dict, time_range_s: float, step_s: int, compat: bool,
                         missing: str = "skip", weights: dict | None = None) -> list[list]:
    """Per-node report (F4).  Reference stats_server_results :36-60 in compat mode."""
    if compat:
        sv = {}
        for res in result(util_body):
            sv[res["metric"]["kubernetes_io_hostname"]] = [float(x[1]) for x in res.get("values", [])]  # Q1
        avg = {s: sum(v) * step_s / time_range_s for s, v in sv.items()}  # Q2/Q3
        lines = []
        for server in sorted(servers):
            total, used, card = servers[server]
            lines.append([server, card, avg.get(server, 0), used, total])
        return lines
    # fixed: combine every series of a node card-weighted per timestamp, then average over time
    per_node: dict[str, dict[float, list[tuple[float, float]]]] = {}
    for res in result(util_body):
        node = res["metric"].get("kubernetes_io_hostname", "")
        alloc = (weights or {}).get(node, {})
        w = float(alloc.get(_series_key(res["metric"], alloc), 1) or 1)
        for ts, v in res.get("values", []):
            per_node.setdefault(node, {}).setdefault(float(ts), []).append((float(v), w))
    n_steps = max(1, int(round(time_range_s / step_s)))
    lines = []
    for server in sorted(servers):
        total, used, card = servers[server]
        pts = per_node.get(server, {})
        series = [sum(v * w for v, w in vs) / sum(w for _, w in vs) for vs in pts.values()]
        if not series:
            u = 0.0
        elif missing == "zero":
            u = sum(series) / max(n_steps, len(series))
        else:
            u = sum(series) / len(series)
        lines.append([server, card, u, used, total])
    return lines


# --------------------------------------------------------------------------- report (L4)
def run_report(c: PromClient, q: Queries, end: datetime | float, window_s: float, step_s: int, compat: bool,
               mode: str = "pod", missing: str = "skip", out=sys.stdout, show_finished: bool = False) -> list[list]:
    if isinstance(end, (int, float)):
        end = datetime.fromtimestamp(end)
    start = end - timedelta(seconds=window_s)
    util = c.query_range(q.util, start, end, step_s)                     # M1
    servers = get_gpu_servers(c, q, compat)                              # M2, M3
    if mode == "node":
        pods = None if compat else get_pod_by_servers(c, q, start, end, step_s, compat, out)
        return stats_server_results(util, servers, window_s, step_s, compat, missing, pods)
    pods = get_pod_by_servers(c, q, start, end, step_s, compat, out)     # M4, M5
    return stats_pod_results(util, servers, pods, compat, show_finished)


def idle_gpu_hours(rows: list[list], window_s: float) -> list[list]:
    """Pod rows (fixed layout) + the GPU-hours each pod held but left idle over the
    window: cards × hours × (1 − util/100) — the waste figure an accounting report is for."""
    h = window_s / 3600.0
    return [[*r, float(r[F_CARDS]) * h * (1.0 - min(100.0, max(0.0, r[F_UTIL])) / 100.0)] for r in rows]


ENERGY_METRIC = "container_gpu_energy_joules_total"


def energy_query(step_s: int, metric: str = ENERGY_METRIC) -> str:
    """Joules per (node, namespace, pod) per step: the exporter's per-pod energy
    counter (socket energy of the pod's GPUs since allocation), summed over its GPUs."""
    return f"sum(increase({metric}[{step_s}s])) by (kubernetes_io_hostname, namespace, pod_name)"


def pod_energy_kwh(c: PromClient, start, end, step_s: int) -> dict[tuple[str, str, str], float]:
    """{(node, namespace, pod): kWh} over (start, end].  The range query's first point
    covers the step *before* ``start``, so it is left out: the kept points tile the window."""
    t0 = to_unix(start)  # the start the range query is evaluated from (whole seconds)
    out: dict[tuple[str, str, str], float] = {}
    for r in result(c.query_range(energy_query(step_s), start, end, step_s)):
        m = r["metric"]
        key = (m.get("kubernetes_io_hostname", ""), m.get("namespace", ""), m.get("pod_name", ""))
        j = sum(float(v) for ts, v in r.get("values", []) if float(ts) > t0 + 0.5)
        out[key] = out.get(key, 0.0) + j / 3.6e6
    return out


def add_energy(rows: list[list], kwh: dict[tuple[str, str, str], float]) -> list[list]:
    """Pod rows (fixed layout) + the kWh their GPUs drew over the window (0 for a pod with no series)."""
    return [[*r, kwh.get((r[F_NODE], r[F_NS], str(r[F_POD]).removesuffix(" (finished)")), 0.0)] for r in rows]


NS_HEADER = ["Namespace", "Pods", "GPUs", "GPU-h", "Busy GPU-h", "Util %", "Idle GPU-h"]


def by_namespace(rows: list[list], window_s: float,
                 extras: list[str] | None = None) -> tuple[list[str], list[list]]:
    """Roll pod rows ([node, namespace, pod, cards, util %, *extras]) up per
    namespace — the team-level view of the same accounting: GPU-hours held (cards ×
    window, as the pod report assumes), busy GPU-hours (× util), their ratio, the
    idle rest, and the extras' totals (e.g. Energy kWh; "Idle GPU-h" is a column
    already).  Sorted by GPU-hours held, with a total."""
    extras = list(extras or [])
    keep = [k for k, e in enumerate(extras) if e != "Idle GPU-h"]
    h = window_s / 3600.0
    agg: dict[str, dict] = {}
    for r in rows:
        node, ns, pod = r[F_NODE], r[F_NS], str(r[F_POD]).removesuffix(" (finished)")
        cards, util = float(r[F_CARDS]), float(r[F_UTIL])
        a = agg.setdefault(ns or "<unknown>",
                           {"pods": set(), "gpus": 0.0, "gpu_h": 0.0, "busy_h": 0.0, "extra": [0.0] * len(keep)})
        a["pods"].add((node, ns, pod))
        a["gpus"] += cards
        a["gpu_h"] += cards * h
        a["busy_h"] += cards * h * min(100.0, max(0.0, util)) / 100.0
        for j, k in enumerate(keep):
            a["extra"][j] += float(r[F_EXTRA + k])
    header = NS_HEADER + [extras[k] for k in keep]
    out = []
    for ns, a in sorted(agg.items(), key=lambda kv: (-kv[1]["gpu_h"], kv[0])):
        util = 100.0 * a["busy_h"] / a["gpu_h"] if a["gpu_h"] > 0 else 0.0
        out.append([ns, len(a["pods"]), a["gpus"], a["gpu_h"], a["busy_h"], util, a["gpu_h"] - a["busy_h"], *a["extra"]])
    if out:
        tot = [sum(r[i] for r in out) for i in range(1, len(header))]
        tot[4] = 100.0 * tot[3] / tot[2] if tot[2] > 0 else 0.0  # util of the totals, not a sum of percents
        out.append(["TOTAL", *tot])
    return header, out


def format_namespace_rows(header: list[str], rows: list[list], fmt: str) -> str:
    if fmt == "json":
        return json.dumps([dict(zip(header, r)) for r in rows], indent=2)
    disp = [[r[0], r[1], f"{r[2]:g}", *(f"{x:.2f}" for x in r[3:])] for r in rows]
    return render_csv(header, disp) if fmt == "csv" else render(header, disp)


def format_rows(rows: list[list], mode: str, fmt: str, compat: bool, idle_hours: bool = False,
                extras: list[str] | None = None) -> str:
    """Table / JSON / CSV.  Pod mode may carry extra numeric columns after Util %
    (``extras`` headers; ``idle_hours`` is the "Idle GPU-h" one), totalled in a last row."""
    if compat:
        return "\n".join(str(r) for r in rows)  # :162-163 prints each row's repr
    extras = list(extras or [])
    if idle_hours and "Idle GPU-h" not in extras:
        extras.insert(0, "Idle GPU-h")
    header = (["Node", "Namespace", "Pod", "GPUs", "Util %"] if mode == "pod"
              else ["Node", "GPU Type", "Util %", "Used", "Total"])
    if mode == "pod":
        header = header + extras
        n = len(extras)
        disp = [[r[F_NODE], r[F_NS], r[F_POD], r[F_CARDS], f"{r[F_UTIL]:.2f}",
                 *(f"{x:.2f}" for x in r[F_EXTRA:F_EXTRA + n])] for r in rows]
        if rows and extras:
            disp.append(["TOTAL", "", "", sum(int(r[F_CARDS]) for r in rows), "",
                         *(f"{sum(r[F_EXTRA + k] for r in rows):.2f}" for k in range(n))])
    else:
        disp = [[r[0], r[1], f"{r[2]:.2f}", r[3], r[4]] for r in rows]
    if fmt == "json":
        return json.dumps([dict(zip(header, r)) for r in rows], indent=2)
    if fmt == "csv":
        return render_csv(header, disp)
    return render(header, disp)


def build_parser(ap: argparse.ArgumentParser | None = None) -> argparse.ArgumentParser:
    ap = ap or argparse.ArgumentParser(prog="kgs gpu-util-stats", description=__doc__.splitlines()[0])
    add_flag(ap, "compat", False, "reference queries, arithmetic and output, quirks included")
    add_flag(ap, "prom-url", REF_PROM_URL, "Prometheus HTTP API base URL (…/api/v1)")
    add_flag(ap, "proxy", "", f"HTTP proxy for every call (reference used {REF_PROXY})")
    add_flag(ap, "timeout", REF_TIMEOUT_S, "per-request timeout seconds")
    add_flag(ap, "retries", 0, "retries per request")
    add_flag(ap, "namespace", "", f"namespace of the live-pod filter ('' = all; --compat: {REF_NAMESPACE!r}, the "
                                  "reference's)")
    add_flag(ap, "window", float(REF_WINDOW_S), "report window seconds (reference: 1 day)")
    add_flag(ap, "step", REF_STEP_S, "query_range step seconds (reference: 3600)")
    add_flag(ap, "end", 0.0, "window end as unix seconds (default now)")
    add_flag(ap, "mode", "pod", "pod (F3) | node (F4)")
    add_flag(ap, "missing", "skip", "node mode: treat missing samples as skip | zero")
    add_flag(ap, "resource", "amd_com_gpu", "KSM resource label value of the GPU resource")
    add_flag(ap, "type-label", "label_amd_com_gpu_product_name", "kube_node_labels label holding the GPU type")
    add_flag(ap, "util-metric", "container_gpu_busy_seconds_total",
             "utilisation series: a *_seconds_total busy counter (exact, rate() per step; default) or a percent "
             "gauge such as container_gpu_sm_util / container_gpu_mfma_util (avg_over_time of the scrapes)")
    add_flag(ap, "format", "table", "table | json | csv")
    add_flag(ap, "show-finished", False, "also list pods with utilisation but no live allocation (reference drops them)")
    add_flag(ap, "idle-hours", False, "pod mode: add the GPU-hours each pod held but left idle (cards × window × "
                                      "(1 − util)), and a total")
    add_flag(ap, "energy", False, "pod mode: add the kWh each pod's GPUs drew over the window "
                                  f"({ENERGY_METRIC}), and a total")
    add_flag(ap, "group-by", "pod", "pod mode: pod (one row per pod) | namespace (per-namespace GPU-hours held, "
                                    "busy and idle, util, + the extras' totals)")
    return ap


def shared_query(window_s: float, step_s: int) -> str:
    """GPUs that had more than one owner at the same time somewhere in the window
    (kgs_gpu_owner: one series per (GPU, pod, container) allocation)."""
    return (f"max_over_time((count by (kubernetes_io_hostname, gpu, uuid) (kgs_gpu_owner))"
            f"[{int(window_s)}s:{int(step_s)}s]) > 1")


def warn_shared_gpus(c: PromClient, end_unix: float, window_s: float, step_s: int, err=None) -> list[dict]:
    """the default busy counter bills every tenant of a shared GPU
    the whole GPU's busy time.  When any GPU had several owners in the window, say so
    on stderr and name the per-pod alternative.  Best effort: a Prometheus that cannot
    evaluate the query only costs the warning."""
    try:
        shared = [r["metric"] for r in result(c.query(shared_query(window_s, step_s), end_unix))]
    except Exception as e:  # noqa: BLE001
        L.debug("shared-GPU check skipped: %s", e)
        return []
    if shared:
        gpus = ", ".join(f'{m.get("kubernetes_io_hostname", "?")}/gpu{m.get("gpu", "?")}' for m in shared[:8])
        print(f"warning: {len(shared)} GPU(s) had more than one pod at once ({gpus}{', ...' if len(shared) > 8 else ''}); "
              "container_gpu_busy_seconds_total bills each of them the whole GPU — "
              "use --util-metric container_gpu_cu_seconds_total for each pod's own compute share",
              file=err or sys.stderr)
    return shared


def run(a) -> int:
    c = PromClient(a.prom_url, a.proxy, a.timeout, a.retries)
    if a.compat and not a.namespace:
        a.namespace = REF_NAMESPACE  # gpu_util_stats.py:133
    q = (Queries.compat(a.namespace) if a.compat else
         Queries.amd(a.namespace, a.step, a.resource, a.type_label, a.util_metric))
    end = a.end if a.end else (datetime.now() if a.compat else time.time())
    rows = run_report(c, q, end, a.window, a.step, a.compat, a.mode, a.missing, show_finished=a.show_finished)
    if not a.compat and a.util_metric == "container_gpu_busy_seconds_total":
        warn_shared_gpus(c, end if isinstance(end, (int, float)) else end.timestamp(), a.window, a.step)
    extras: list[str] = []
    if a.mode == "pod" and not a.compat:
        if a.idle_hours:
            rows = idle_gpu_hours(rows, a.window)
            extras.append("Idle GPU-h")
        if a.energy:
            e = end if isinstance(end, (int, float)) else end.timestamp()
            rows = add_energy(rows, pod_energy_kwh(c, e - a.window, e, a.step))
            extras.append("Energy kWh")
        if a.group_by == "namespace":
            header, ns_rows = by_namespace(rows, a.window, extras)
            print(format_namespace_rows(header, ns_rows, a.format))
            return 0
    elif a.group_by != "pod":
        raise SystemExit("--group-by namespace needs pod mode without --compat")
    print(format_rows(rows, a.mode, a.format, a.compat, extras=extras))
    return 0


def main(argv=None) -> int:
    return run(build_parser().parse_args(argv))


if __name__ == "__main__":
    sys.exit(main())
