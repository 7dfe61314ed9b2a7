"""kubelet pod-resources gRPC client (GPU → pod/namespace/container).

The reference learns which pod holds GPUs from ``kubectl get pods -o json``
(who_use_gpu.py:8-10) and from kube-state-metrics request series
(gpu_util_stats.py:117,137).  A node exporter needs the *device-level* answer —
which physical GPU a container was given — and the kubelet exposes exactly that
on ``/var/lib/kubelet/pod-resources/kubelet.sock`` (``v1.PodResourcesLister``).

Device IDs reported by the AMD device plugin are PCI addresses; node-local
indices, UUIDs, serials and DRM card names are accepted too (``DeviceIndex``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Iterable

from . import proto

DEFAULT_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
LIST_METHOD = "/v1.PodResourcesLister/List"
ALLOCATABLE_METHOD = "/v1.PodResourcesLister/GetAllocatableResources"
GPU_RESOURCES = ("amd.com/gpu", "amd.com/gpu-partition")


@dataclass(frozen=True)
class Allocation:
    pod: str
    namespace: str
    container: str
    resource: str
    device_id: str


def _identity(b: bytes) -> bytes:
    return b


class PodResourcesClient:
    """Unary calls over a unix-socket gRPC channel with raw-bytes (de)serialisers."""

    def __init__(self, socket_path: str = DEFAULT_SOCKET, timeout_s: float = 2.0):
        import grpc

        self.socket_path = socket_path
        self.timeout_s = timeout_s
        self._channel = grpc.insecure_channel(f"unix://{socket_path}")
        self._list = self._channel.unary_unary(LIST_METHOD, request_serializer=_identity,
                                               response_deserializer=_identity)
        self._alloc = self._channel.unary_unary(ALLOCATABLE_METHOD, request_serializer=_identity,
                                                response_deserializer=_identity)

    def available(self) -> bool:
        return os.path.exists(self.socket_path)

    def list(self) -> proto.ListPodResourcesResponse:
        return proto.ListPodResourcesResponse.decode(self._list(b"", timeout=self.timeout_s))

    def allocatable(self) -> proto.AllocatableResourcesResponse:
        return proto.AllocatableResourcesResponse.decode(self._alloc(b"", timeout=self.timeout_s))

    def gpu_allocations(self, resources: Iterable[str] = GPU_RESOURCES) -> list[Allocation]:
        res = set(resources)
        out = []
        for p in self.list().pod_resources:
            for c in p.containers:
                for d in c.devices:
                    if d.resource_name not in res:
                        continue
                    for dev in d.device_ids:
                        out.append(Allocation(p.name, p.namespace, c.name, d.resource_name, dev))
        return out

    def close(self) -> None:
        self._channel.close()


class DeviceIndex:
    """Resolve a device-plugin device ID to the exporter's device index.

    Every key is exact (case-insensitive); an ID that matches nothing, or matches
    more than one exporter device, resolves to ``None`` — a wrong pod label is
    worse than none.  Accepted:

    * PCI address (``0000:72:00.0`` / ``72:00.0``).  Under compute partitioning
      (DPX/QPX/CPX) every partition of a GPU shares its PCI function; the address
      then names the function's own partition, partition 0 (the other partitions
      are ``amdgpu_xcp_*`` platform devices).
    * UUID; serial when unique (partitions share their GPU's serial).
    * DRM names ``card<N>`` / ``renderD<128+N>`` and KFD node ``kfd<N>``.
    * ``amdgpu_xcp_<n>``: the partition platform device, resolved through sysfs
      (``<sysfs>/devices/platform/amdgpu_xcp_<n>/drm/card<M>`` → the device whose
      DRM card is M).  Never by the number alone: XCP numbers are node-global and
      do not follow exporter indices.
    * The exporter index itself, as the whole ID (``"3"``).
    * Prefixed forms (``gpu-0000:72:00.0``): the tail after the last ``-``/``_``
      only when that tail is a PCI address or UUID key, never a bare number.
    """

    def __init__(self, devices: list[dict], sysfs_root: str | None = "/sys"):
        self._map: dict[str, set[int]] = {}
        self._strong: set[str] = set()  # keys a prefixed ID may resolve through
        by_bdf: dict[str, list[dict]] = {}
        card_to_idx: dict[int, int] = {}
        for d in devices:
            i = int(d["index"])
            self._add(str(i), i)
            if d.get("uuid"):
                self._add(d["uuid"], i, strong=True)
            if d.get("serial"):
                self._add(d["serial"], i)
            card = int(d.get("drm_card", -1) if d.get("drm_card") is not None else -1)
            if card >= 0:
                self._add(f"card{card}", i)
                self._add(f"renderD{128 + card}", i)
                card_to_idx[card] = i
            if int(d.get("kfd_node", -1) if d.get("kfd_node") is not None else -1) >= 0:
                self._add(f"kfd{int(d['kfd_node'])}", i)
            if d.get("bdf"):
                by_bdf.setdefault(d["bdf"].lower(), []).append(d)
        for bdf, ds in by_bdf.items():
            if len(ds) > 1:  # partitions: the PCI function is partition 0
                ds = [d for d in ds if int(d.get("partition_id", -1)) == 0] or ds
            for d in ds:
                self._add(bdf, int(d["index"]), strong=True)
                if bdf.startswith("0000:"):
                    self._add(bdf[5:], int(d["index"]), strong=True)
        for xcp, card in _xcp_cards(sysfs_root).items():
            if card in card_to_idx:
                self._add(xcp, card_to_idx[card], strong=True)

    def _add(self, key: str, i: int, strong: bool = False) -> None:
        k = str(key).lower()
        self._map.setdefault(k, set()).add(i)
        if strong:
            self._strong.add(k)

    def _one(self, k: str) -> int | None:
        s = self._map.get(k)
        return next(iter(s)) if s and len(s) == 1 else None

    def resolve(self, device_id: str) -> int | None:
        k = device_id.strip().lower()
        if k in self._map:
            return self._one(k)
        for sep in ("-", "_"):
            tail = k.rsplit(sep, 1)[-1]
            if tail != k and tail in self._strong:
                return self._one(tail)
        return None


def _xcp_cards(sysfs_root: str | None) -> dict[str, int]:
    """``amdgpu_xcp_<n>`` platform devices → their DRM card number."""
    out: dict[str, int] = {}
    if not sysfs_root:
        return out
    base = os.path.join(sysfs_root, "devices", "platform")
    try:
        names = os.listdir(base)
    except OSError:
        return out
    for name in names:
        if not name.startswith("amdgpu_xcp"):
            continue
        try:
            for e in os.listdir(os.path.join(base, name, "drm")):
                if e.startswith("card") and e[4:].isdigit():
                    out[name.replace(".", "_").lower()] = int(e[4:])
        except OSError:
            continue
    return out
