"""In-process kubelet pod-resources server on a unix socket (tests only).

Speaks ``v1.PodResourcesLister`` List / GetAllocatableResources with the same
hand-encoded protobuf the product client decodes
(kube_gpu_stats_amd/attribution/proto.py); BASELINE config 5 rehearsal.
"""
from __future__ import annotations

import os

from kube_gpu_stats_amd.attribution import proto
from kube_gpu_stats_amd.attribution.podresources import ALLOCATABLE_METHOD, LIST_METHOD


def _identity(b: bytes) -> bytes:
    return b


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
        try:
            os.unlink(socket_path)
        except FileNotFoundError:
            pass
        self._server.add_insecure_port(f"unix://{socket_path}")

    def __enter__(self):
        self._server.start()
        return self

    def __exit__(self, *exc):
        # grpc removes the socket file asynchronously after stop(): unlink without a
        # separate exists() check (that was a TOCTOU race).
        self._server.stop(0).wait(5)
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
