"""1 Hz attribution loop: pushes GPU→pod and PID→pod tables into the native exporter.

* GPU → (pod, namespace, container): kubelet pod-resources ``List`` (device-plugin
  allocations), resolved to exporter GPU indices.  Fills the labels of the
  reference-contract series ``container_gpu_sm_util{pod_name,...}``
  (reference gpu_util_stats.py:159).
* PID → pod: a process found on a GPU inherits that GPU's owner when the GPU is
  held by exactly one container; its pod UID always comes from its cgroup.
* Optional static mapping file (JSON ``{"<device id>": {"pod":..,"namespace":..,
  "container":..}}``) for nodes without a kubelet socket (and the 1-GPU box).
"""
from __future__ import annotations

import json
import os
import threading
import time

from ..utils import log
from .cgroup import pid_cgroup
from .podresources import GPU_RESOURCES, DeviceIndex, PodResourcesClient

L = log.get("attribution")


class Attributor:
    def __init__(self, exporter, socket_path: str | None = None, static_map: str | None = None,
                 resources=GPU_RESOURCES, interval_s: float = 1.0, proc_root: str = "/proc"):
        self.ex = exporter
        self.interval_s = interval_s
        self.proc_root = proc_root
        self.resources = tuple(resources)
        self.index = DeviceIndex(exporter.devices())
        self.client = PodResourcesClient(socket_path) if socket_path and os.path.exists(socket_path) else None
        self.static_map = static_map
        self.owners: dict[int, list[dict]] = {}
        self.errors = 0
        self.updates = 0
        self._stop = threading.Event()
        self._th: threading.Thread | None = None

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
        if self.client is not None:
            for a in self.client.gpu_allocations(self.resources):
                i = self.index.resolve(a.device_id)
                if i is None:
                    continue
                o = {"pod": a.pod, "namespace": a.namespace, "container": a.container}
                if o not in owners.setdefault(i, []):
                    owners[i].append(o)
        return owners

    def pid_owners(self, owners: dict[int, list[dict]]) -> dict[int, dict]:
        out: dict[int, dict] = {}
        for gpu in range(self.ex.device_count):
            single = owners.get(gpu, [])
            for p in self.ex.procs(gpu):
                pid = int(p["pid"])
                cg = pid_cgroup(pid, self.proc_root)
                o = dict(single[0]) if len(single) == 1 else {"pod": "", "namespace": "", "container": ""}
                o["pod_uid"] = cg.pod_uid
                out[pid] = o
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

    # ------------------------------------------------------------------ thread
    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                self.update_once()
            except Exception as e:  # noqa: BLE001 - keep attributing; kubelet restarts are normal
                self.errors += 1
                L.warning("attribution pass failed: %s", e)
            self._stop.wait(self.interval_s)

    def start(self) -> "Attributor":
        self._th = threading.Thread(target=self._run, name="kgs-attrib", daemon=True)
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._th:
            self._th.join(timeout=5)
        if self.client:
            self.client.close()
