"""Minimal protobuf wire-format codec for the kubelet pod-resources v1 API.

``grpc_tools`` is not available in the image, so the handful
of messages the exporter needs are encoded/decoded by hand.  Field numbers follow
``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto``:

    ListPodResourcesResponse { repeated PodResources pod_resources = 1; }
    PodResources     { string name = 1; string namespace = 2; repeated ContainerResources containers = 3; }
    ContainerResources { string name = 1; repeated ContainerDevices devices = 2; repeated int64 cpu_ids = 3; ... }
    ContainerDevices { string resource_name = 1; repeated string device_ids = 2; TopologyInfo topology = 3; }
    TopologyInfo     { repeated NUMANode nodes = 1; }   NUMANode { int64 ID = 1; }
    AllocatableResourcesResponse { repeated ContainerDevices devices = 1; repeated int64 cpu_ids = 2; ... }
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Iterator


# --------------------------------------------------------------------------- wire
def _varint(n: int) -> bytes:
    if n < 0:
        n += 1 << 64
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> tuple[int, int]:
    shift = 0
    val = 0
    while True:
        if i >= len(buf):
            raise ValueError("truncated varint")
        b = buf[i]
        i += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val, i
        shift += 7
        if shift > 70:
            raise ValueError("varint too long")


def fields(buf: bytes) -> Iterator[tuple[int, int, object]]:
    """Yield (field_number, wire_type, value) for every field of a message."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            v, i = int.from_bytes(buf[i:i + 8], "little"), i + 8
        elif wt == 2:
            n, i = _read_varint(buf, i)
            v, i = buf[i:i + n], i + n
            if i > len(buf):
                raise ValueError("truncated length-delimited field")
        elif wt == 5:
            v, i = int.from_bytes(buf[i:i + 4], "little"), i + 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fno, wt, v


def enc_str(fno: int, s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else s
    return _varint((fno << 3) | 2) + _varint(len(b)) + b


def enc_int(fno: int, v: int) -> bytes:
    return _varint(fno << 3) + _varint(v)


def enc_packed_ints(fno: int, vs: list[int]) -> bytes:
    body = b"".join(_varint(v) for v in vs)
    return enc_str(fno, body) if vs else b""


def _ints(wt: int, v) -> list[int]:
    if wt == 0:
        return [v]
    out, i = [], 0
    while i < len(v):
        x, i = _read_varint(v, i)
        out.append(x)
    return out


# --------------------------------------------------------------------------- messages
@dataclass
class ContainerDevices:
    resource_name: str = ""
    device_ids: list[str] = field(default_factory=list)
    numa_nodes: list[int] = field(default_factory=list)

    def encode(self) -> bytes:
        out = enc_str(1, self.resource_name) + b"".join(enc_str(2, d) for d in self.device_ids)
        if self.numa_nodes:
            topo = b"".join(enc_str(1, enc_int(1, n)) for n in self.numa_nodes)
            out += enc_str(3, topo)
        return out

    @classmethod
    def decode(cls, buf: bytes) -> "ContainerDevices":
        m = cls()
        for fno, wt, v in fields(buf):
            if fno == 1 and wt == 2:
                m.resource_name = v.decode()
            elif fno == 2 and wt == 2:
                m.device_ids.append(v.decode())
            elif fno == 3 and wt == 2:
                for f2, w2, node in fields(v):
                    if f2 == 1 and w2 == 2:
                        for f3, w3, nid in fields(node):
                            if f3 == 1 and w3 == 0:
                                m.numa_nodes.append(nid)
        return m


@dataclass
class ContainerResources:
    name: str = ""
    devices: list[ContainerDevices] = field(default_factory=list)
    cpu_ids: list[int] = field(default_factory=list)

    def encode(self) -> bytes:
        return (enc_str(1, self.name) + b"".join(enc_str(2, d.encode()) for d in self.devices)
                + enc_packed_ints(3, self.cpu_ids))

    @classmethod
    def decode(cls, buf: bytes) -> "ContainerResources":
        m = cls()
        for fno, wt, v in fields(buf):
            if fno == 1 and wt == 2:
                m.name = v.decode()
            elif fno == 2 and wt == 2:
                m.devices.append(ContainerDevices.decode(v))
            elif fno == 3:
                m.cpu_ids.extend(_ints(wt, v))
        return m


@dataclass
class PodResources:
    name: str = ""
    namespace: str = ""
    containers: list[ContainerResources] = field(default_factory=list)

    def encode(self) -> bytes:
        return enc_str(1, self.name) + enc_str(2, self.namespace) + b"".join(
            enc_str(3, c.encode()) for c in self.containers)

    @classmethod
    def decode(cls, buf: bytes) -> "PodResources":
        m = cls()
        for fno, wt, v in fields(buf):
            if fno == 1 and wt == 2:
                m.name = v.decode()
            elif fno == 2 and wt == 2:
                m.namespace = v.decode()
            elif fno == 3 and wt == 2:
                m.containers.append(ContainerResources.decode(v))
        return m


@dataclass
class ListPodResourcesResponse:
    pod_resources: list[PodResources] = field(default_factory=list)

    def encode(self) -> bytes:
        return b"".join(enc_str(1, p.encode()) for p in self.pod_resources)

    @classmethod
    def decode(cls, buf: bytes) -> "ListPodResourcesResponse":
        m = cls()
        for fno, wt, v in fields(buf):
            if fno == 1 and wt == 2:
                m.pod_resources.append(PodResources.decode(v))
        return m


@dataclass
class AllocatableResourcesResponse:
    devices: list[ContainerDevices] = field(default_factory=list)
    cpu_ids: list[int] = field(default_factory=list)

    def encode(self) -> bytes:
        return b"".join(enc_str(1, d.encode()) for d in self.devices) + enc_packed_ints(2, self.cpu_ids)

    @classmethod
    def decode(cls, buf: bytes) -> "AllocatableResourcesResponse":
        m = cls()
        for fno, wt, v in fields(buf):
            if fno == 1 and wt == 2:
                m.devices.append(ContainerDevices.decode(v))
            elif fno == 2:
                m.cpu_ids.extend(_ints(wt, v))
        return m
