"""Kubernetes manifests parse and wire the exporter the way the code expects."""
import os

import yaml

from kube_gpu_stats_amd.exporter.main import build_parser

DEPLOY = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "deploy")


def load(name):
    with open(os.path.join(DEPLOY, name)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def test_daemonset_args_are_valid_exporter_flags():
    docs = load("daemonset.yaml")
    ds = next(d for d in docs if d["kind"] == "DaemonSet")
    spec = ds["spec"]["template"]["spec"]
    assert spec["hostPID"] is True
    c = spec["containers"][0]
    a = build_parser().parse_args(c["args"])
    assert a.pmc == "aqlprofile" and a.hz == 10.0 and a.listen == "0.0.0.0:9400"
    env = {e["name"]: e for e in c["env"]}
    assert env["NODE_NAME"]["valueFrom"]["fieldRef"]["fieldPath"] == "spec.nodeName"
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert "/var/lib/kubelet/pod-resources" in mounts and "/dev/kfd" in mounts
    assert c["readinessProbe"]["httpGet"]["path"] == "/healthz"
    assert a.pod_directory == "api" and a.window == 15.0
    # the pod directory lists pods: the exporter's service account must be allowed to
    sa = spec["serviceAccountName"]
    role = next(d for d in docs if d["kind"] == "ClusterRole")
    binding = next(d for d in docs if d["kind"] == "ClusterRoleBinding")
    assert any("pods" in r["resources"] and "list" in r["verbs"] for r in role["rules"])
    assert binding["subjects"][0]["name"] == sa and binding["roleRef"]["name"] == role["metadata"]["name"]


def test_daemonset_handover_does_not_signal_pid1():
    """hostPID: PID 1 in the pod is the host's init."""
    with open(os.path.join(DEPLOY, "daemonset.yaml")) as f:
        text = f.read()
    assert "kill -USR1 1" not in text.replace("Never `kill -USR1 1`", "")
    assert "kgs pmc release" in text


PROMQL_WORDS = {"avg", "sum", "max", "min", "count", "rate", "increase", "avg_over_time", "label_values", "by", "or",
                "and", "on", "without", "group_left", "group_right", "histogram_quantile"}
LABELS = {"kubernetes_io_hostname", "nvidia_gpu_type", "pod_name", "namespace", "gpu", "instance", "sensor", "pod",
          "pid", "xcc", "block", "type", "reason"}


def unknown_series(exprs: str) -> set:
    """Series names used in PromQL that the exporter does not emit (catalogue check)."""
    import re

    from kube_gpu_stats_amd.models.schema import BY_NAME

    bare = re.sub(r"\{[^}]*\}|\[[^]]*\]|\"[^\"]*\"", "", exprs)
    names = {n for n in re.findall(r"[a-zA-Z_:][a-zA-Z0-9_:]*", bare) if ":" not in n}
    def known(n: str) -> bool:  # a histogram's series carry _bucket / _sum / _count
        base = re.sub(r"_(bucket|sum|count)$", "", n)
        return n in BY_NAME or (base in BY_NAME and BY_NAME[base].type == "histogram")

    return {n for n in names - PROMQL_WORDS - LABELS if not known(n)}


def test_monitoring_rules_reference_exported_families():
    from kube_gpu_stats_amd.models.schema import BY_NAME

    docs = load("monitoring.yaml")
    rule = next(d for d in docs if d["kind"] == "PrometheusRule")
    exprs = " ".join(r["expr"] for g in rule["spec"]["groups"] for r in g["rules"])
    for fam in ("container_gpu_sm_util", "amdgpu_gfx_busy_seconds_total", "amdgpu_hbm_used_bytes", "kgs_up",
                "amdgpu_xgmi_read_bytes_total"):
        assert fam in exprs and fam in BY_NAME
    assert not unknown_series(exprs)


def _alert_not_from_counters(pmfw_rate: float, enabled: int, failed: int) -> bool:
    """KgsUtilisationNotFromCounters for one (instance, gpu), evaluated by hand on the
    exact expression shape the rule uses: ``A > 0.5 and on (instance, gpu) (B == 1 or
    C == 1)`` (PromQL ``and`` keeps the left sample where the right side has a series)."""
    right = enabled == 1 or failed == 1
    return pmfw_rate > 0.5 and right


def test_pmfw_billing_alert_fires_while_the_breaker_is_open():
    """trip() sets kgs_pmc_enabled 0 while the counter tier's breaker is open,
    so a rule gated on kgs_pmc_enabled == 1 alone never fired for the case it names.
    Gated on the exporter *wanting* the counters: an open breaker (enabled 0, failed 1)
    and stale drains (enabled 1) fire; a hand-over to another profiler (enabled 0,
    failed 0) does not."""
    docs = load("monitoring.yaml")
    rule = next(d for d in docs if d["kind"] == "PrometheusRule")
    r = next(r for g in rule["spec"]["groups"] for r in g["rules"] if r.get("alert") == "KgsUtilisationNotFromCounters")
    expr = " ".join(r["expr"].split())
    assert expr.endswith("and on (instance, gpu) (kgs_pmc_enabled == 1 or kgs_pmc_failed == 1)"), expr
    assert expr.startswith('rate(kgs_util_source_seconds_total{source="pmfw"}[15m]) > 0.5'), expr
    assert _alert_not_from_counters(1.0, enabled=0, failed=1)       # breaker open between retries
    assert _alert_not_from_counters(1.0, enabled=1, failed=0)       # counters held, drains stale
    assert not _alert_not_from_counters(1.0, enabled=0, failed=0)   # handed over (SIGUSR1): expected
    assert not _alert_not_from_counters(0.1, enabled=0, failed=1)   # mostly billed from counters


def test_report_cronjob_has_rbac():
    docs = load("reports-cronjob.yaml")
    kinds = {d["kind"] for d in docs}
    assert {"ServiceAccount", "ClusterRole", "ClusterRoleBinding", "CronJob"} <= kinds


def test_grafana_dashboard_is_current_and_uses_exported_families():
    from kube_gpu_stats_amd.models import dashboard

    with open(os.path.join(DEPLOY, "grafana-dashboard.json")) as f:
        assert f.read() == dashboard.render(), "regenerate: python -m kube_gpu_stats_amd.models.dashboard"
    ex = dashboard.exprs()
    assert len(ex) >= 15
    assert not unknown_series(" ".join(ex))
    assert any("container_gpu_sm_util" in e for e in ex)


def _mib(q: str) -> float:
    units = {"Ki": 1 / 1024, "Mi": 1, "Gi": 1024}
    for u, f in units.items():
        if q.endswith(u):
            return float(q[:-2]) * f
    return float(q) / 2**20


def test_daemonset_memory_fits_the_counter_tier_on_8_gpus():
    """Each GPU's private AQL READ queue pins ≈350 MiB of host memory on MI355X (the
    KFD context save/restore area of a compute queue for 256 CUs + per-agent runtime
    state; profiles/r3/README.md r3s-r3v): with --pmc=aqlprofile an 8-GPU node needs
    ≈2.9 GiB, so a 512Mi limit (rounds 1-2) would OOM-kill the exporter."""
    ds = next(d for d in load("daemonset.yaml") if d["kind"] == "DaemonSet")
    c = ds["spec"]["template"]["spec"]["containers"][0]
    a = build_parser().parse_args(c["args"])
    need = 40 + (8 * 350 if a.pmc == "aqlprofile" else 0)
    res = c["resources"]
    assert _mib(res["requests"]["memory"]) >= need and _mib(res["limits"]["memory"]) >= need, res
