"""PID → pod UID / container ID from ``/proc/<pid>/cgroup``.

Handles the layouts kubelet produces:

* cgroup v1/v2, cgroupfs driver:   ``/kubepods/burstable/pod<uid>/<container-id>``
* systemd driver:                  ``/kubepods.slice/kubepods-burstable.slice/
                                     kubepods-burstable-pod<uid_with_underscores>.slice/
                                     cri-containerd-<container-id>.scope``
  (also ``docker-<id>.scope`` and ``crio-<id>.scope``)
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass

_POD_RE = re.compile(r"pod([0-9a-fA-F]{8}[-_][0-9a-fA-F]{4}[-_][0-9a-fA-F]{4}[-_][0-9a-fA-F]{4}[-_][0-9a-fA-F]{12})")
_CID_RE = re.compile(r"(?:cri-containerd-|docker-|crio-|containerd-)?([0-9a-f]{64})(?:\.scope)?$")


@dataclass(frozen=True)
class CgroupInfo:
    pod_uid: str = ""
    container_id: str = ""
    qos: str = ""


def parse_cgroup_text(text: str) -> CgroupInfo:
    pod_uid = cid = qos = ""
    for line in text.splitlines():
        parts = line.split(":", 2)
        if len(parts) != 3:
            continue
        path = parts[2]
        m = _POD_RE.search(path)
        if not m:
            continue
        pod_uid = m.group(1).replace("_", "-").lower()
        if "burstable" in path:
            qos = "burstable"
        elif "besteffort" in path:
            qos = "besteffort"
        else:
            qos = "guaranteed"
        last = path.rstrip("/").rsplit("/", 1)[-1]
        mc = _CID_RE.search(last)
        if mc:
            cid = mc.group(1)
        if cid:
            break
    return CgroupInfo(pod_uid, cid, qos)


def pid_cgroup(pid: int, proc_root: str = "/proc") -> CgroupInfo:
    try:
        with open(os.path.join(proc_root, str(pid), "cgroup")) as f:
            return parse_cgroup_text(f.read())
    except OSError:
        return CgroupInfo()
