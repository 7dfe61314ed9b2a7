"""1 Hz attribution loop: pushes GPU→pod and PID→pod tables into the native exporter.

* GPU → (pod, namespace, container): kubelet pod-resources ``List`` (device-plugin
  allocations), resolved to exporter GPU indices.  Fills the labels of the
  reference-contract series ``container_gpu_sm_util{pod_name,...}``
  (reference gpu_util_stats.py:159).
* PID → pod, per (GPU, PID): the process's own cgroup names its pod UID and
  container ID; a pod directory (poddir.py: the node's PodList) turns those into
  pod / namespace / container, so processes of different pods sharing one GPU are
  told apart.  Without a directory entry, a process inherits its GPU's owner only
  when the GPU has exactly one owner AND the process's cgroup names a pod that is
  not the exporter's own (the exporter's counter queues make it show up in every
  GPU's process list; host processes have no pod UID) — ADVICE r1.
* Optional static mapping file (JSON ``{"<device id>": {"pod":..,"namespace":..,
  "container":..}}``) for nodes without a kubelet socket (and the 1-GPU box).

Failure handling: the kubelet socket may not exist yet when the
DaemonSet pod starts and disappears while kubelet restarts.  The client is
created lazily once the socket shows up and re-created after a failed call; the
last good GPU→pod table is kept for ``stale_after_s`` so a kubelet restart does
not strip the pod labels from every series, then dropped.  The loop's own health
is exported as ``kgs_attribution_*`` on /metrics.
"""
from __future__ import annotations

import json
import os
import threading
import time

from ..models.schema import BY_NAME
from ..utils import log
from .cgroup import pid_cgroup
from .poddir import PodDirectory
from .podresources import GPU_RESOURCES, DeviceIndex, PodResourcesClient

L = log.get("attribution")


class Attributor:
    def __init__(self, exporter, socket_path: str | None = None, static_map: str | None = None,
                 resources=GPU_RESOURCES, interval_s: float = 1.0, proc_root: str = "/proc",
                 stale_after_s: float = 30.0, sysfs_root: str | None = "/sys",
                 pod_directory: PodDirectory | None = None, self_pid: int | None = None):
        self.ex = exporter
        self.interval_s = interval_s
        self.proc_root = proc_root
        self.resources = tuple(resources)
        self.index = DeviceIndex(exporter.devices(), sysfs_root)
        self.poddir = pod_directory
        self.own_pod_uid = pid_cgroup(self_pid if self_pid is not None else os.getpid(), proc_root).pod_uid
        self.socket_path = socket_path
        self.client: PodResourcesClient | None = None
        self.static_map = static_map
        self.stale_after_s = stale_after_s
        self.owners: dict[int, list[dict]] = {}
        self.kubelet_owners: dict[int, list[dict]] = {}
        self.last_kubelet_ok = 0.0
        self.errors = 0
        self.reconnects = 0
        self.updates = 0
        self._stop = threading.Event()
        self._th: threading.Thread | None = None
        self._connect()

    # ------------------------------------------------------------------ kubelet
    def _connect(self) -> bool:
        if self.client is None and self.socket_path and os.path.exists(self.socket_path):
            self.client = PodResourcesClient(self.socket_path)
            return True
        return self.client is not None

    def _drop_client(self) -> None:
        if self.client is not None:
            try:
                self.client.close()
            except Exception:  # noqa: BLE001
                pass
            self.client = None
            self.reconnects += 1

    def _kubelet_owners(self) -> dict[int, list[dict]]:
        """Allocations from kubelet, or the last good table while it is briefly away."""
        if self.socket_path and self._connect():
            try:
                owners: dict[int, list[dict]] = {}
                for a in self.client.gpu_allocations(self.resources):
                    i = self.index.resolve(a.device_id)
                    if i is None:
                        continue
                    o = {"pod": a.pod, "namespace": a.namespace, "container": a.container}
                    if o not in owners.setdefault(i, []):
                        owners[i].append(o)
                self.kubelet_owners = owners
                self.last_kubelet_ok = time.monotonic()
                return owners
            except Exception as e:  # noqa: BLE001 - grpc.RpcError and decode errors alike
                self.errors += 1
                L.warning("kubelet pod-resources List failed: %s", e)
                self._drop_client()
        if self.kubelet_owners and time.monotonic() - self.last_kubelet_ok > self.stale_after_s:
            L.warning("kubelet unreachable for %.0fs: dropping pod attribution", self.stale_after_s)
            self.kubelet_owners = {}
        return self.kubelet_owners

    # ------------------------------------------------------------------ one pass
    def device_owners(self) -> dict[int, list[dict]]:
        owners: dict[int, list[dict]] = {}
        if self.static_map and os.path.exists(self.static_map):
            with open(self.static_map) as f:
                for dev_id, o in json.load(f).items():
                    i = self.index.resolve(dev_id)
                    if i is not None:
                        owners.setdefault(i, []).append(
                            {"pod": o.get("pod", ""), "namespace": o.get("namespace", ""),
                             "container": o.get("container", "")})
        for i, lst in self._kubelet_owners().items():
            for o in lst:
                if o not in owners.setdefault(i, []):
                    owners[i].append(o)
        return owners

    def pid_owners(self, owners: dict[int, list[dict]]) -> dict[tuple[int, int], dict]:
        """{(gpu, pid): {pod, namespace, container, pod_uid}} for every process the
        exporter's process tier sees on every GPU."""
        out: dict[tuple[int, int], dict] = {}
        if self.poddir is not None:
            self.poddir.refresh()
        cgroups: dict[int, object] = {}
        for gpu in range(self.ex.device_count):
            gpu_owners = owners.get(gpu, [])
            for p in self.ex.procs(gpu):
                pid = int(p["pid"])
                cg = cgroups.get(pid)
                if cg is None:
                    cg = cgroups[pid] = pid_cgroup(pid, self.proc_root)
                o = {"pod": "", "namespace": "", "container": "", "pod_uid": cg.pod_uid}
                ref = self.poddir.lookup(cg.pod_uid, cg.container_id) if self.poddir is not None else None
                if ref is not None:
                    o.update(pod=ref.pod, namespace=ref.namespace, container=ref.container)
                elif cg.pod_uid and cg.pod_uid != self.own_pod_uid and len(gpu_owners) == 1:
                    o.update(pod=gpu_owners[0]["pod"], namespace=gpu_owners[0]["namespace"],
                             container=gpu_owners[0]["container"])
                out[(gpu, pid)] = o
        return out

    def update_once(self) -> None:
        owners = self.device_owners()
        for gpu in range(self.ex.device_count):
            new = owners.get(gpu, [])
            if self.owners.get(gpu, []) != new:
                self.ex.set_device_owners(gpu, new)
        self.owners = owners
        self.ex.set_pid_owners(self.pid_owners(owners))
        self.updates += 1
        self.publish()

    def self_metrics(self) -> str:
        age = time.monotonic() - self.last_kubelet_ok if self.last_kubelet_ok else -1.0
        connected = 1 if self.client is not None else 0
        values = {"kgs_attribution_updates_total": self.updates,
                  "kgs_attribution_errors_total": self.errors,
                  "kgs_attribution_kubelet_reconnects_total": self.reconnects,
                  "kgs_attribution_kubelet_connected": connected,
                  "kgs_attribution_kubelet_age_seconds": f"{age:.3f}",
                  "kgs_attribution_allocated_gpus": sum(1 for v in self.owners.values() if v)}
        lines = []
        for name, v in values.items():  # HELP / TYPE from the metric catalogue, like the native families
            fam = BY_NAME[name]
            lines += [f"# HELP {name} {fam.help}", f"# TYPE {name} {fam.type}", f"{name} {v}"]
        return "\n".join(lines) + "\n"

    def publish(self) -> None:
        setter = getattr(self.ex, "set_extra_metrics", None)
        if setter is not None:
            setter(self.self_metrics())

    # ------------------------------------------------------------------ thread
    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                self.update_once()
            except Exception as e:  # noqa: BLE001 - keep attributing; kubelet restarts are normal
                self.errors += 1
                L.warning("attribution pass failed: %s", e)
                self.publish()
            self._stop.wait(self.interval_s)

    def start(self) -> "Attributor":
        self._th = threading.Thread(target=self._run, name="kgs-attrib", daemon=True)
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._th:
            self._th.join(timeout=5)
        self._drop_client()
