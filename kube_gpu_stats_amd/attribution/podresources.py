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
    """Resolve a device-plugin device ID to the exporter's GPU index."""

    def __init__(self, devices: list[dict]):
        self._map: dict[str, int] = {}
        for d in devices:
            i = int(d["index"])
            for key in (d.get("bdf"), d.get("uuid"), d.get("serial"), str(i)):
                if key:
                    self._map[str(key).lower()] = i
            bdf = (d.get("bdf") or "").lower()
            if bdf.startswith("0000:"):
                self._map[bdf[5:]] = i          # "72:00.0"
            if d.get("drm_card", -1) is not None and int(d.get("drm_card", -1)) >= 0:
                self._map[f"card{int(d['drm_card'])}"] = i

    def resolve(self, device_id: str) -> int | None:
        k = device_id.strip().lower()
        if k in self._map:
            return self._map[k]
        # "gpu-0000:72:00.0" / "amdgpu_xcp_3"-style prefixes
        for sep in ("-", "_"):
            tail = k.rsplit(sep, 1)[-1]
            if tail in self._map:
                return self._map[tail]
        return None


# --------------------------------------------------------------------------- fake kubelet
class FakeKubelet:
    """In-process kubelet pod-resources server on a unix socket (tests, BASELINE config 5 rehearsal)."""

    def __init__(self, socket_path: str, response: proto.ListPodResourcesResponse,
                 allocatable: proto.AllocatableResourcesResponse | None = None):
        import grpc
        from concurrent import futures

        self.socket_path = socket_path
        self.response = response
        self.allocatable = allocatable or proto.AllocatableResourcesResponse()
        self.calls = 0
        outer = self

        class Handler(grpc.GenericRpcHandler):
            def service(self, details):
                if details.method == LIST_METHOD:
                    def list_(req, ctx):
                        outer.calls += 1
                        return outer.response.encode()
                    return grpc.unary_unary_rpc_method_handler(list_, request_deserializer=_identity,
                                                               response_serializer=_identity)
                if details.method == ALLOCATABLE_METHOD:
                    return grpc.unary_unary_rpc_method_handler(lambda r, c: outer.allocatable.encode(),
                                                               request_deserializer=_identity,
                                                               response_serializer=_identity)
                return None

        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self._server.add_generic_rpc_handlers((Handler(),))
        if os.path.exists(socket_path):
            os.unlink(socket_path)
        self._server.add_insecure_port(f"unix://{socket_path}")

    def __enter__(self):
        self._server.start()
        return self

    def __exit__(self, *exc):
        self._server.stop(0)
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
