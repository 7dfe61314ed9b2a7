"""GPU/PID → pod attribution: hand-encoded pod-resources protobuf, a fake kubelet
gRPC server on a unix socket, device-id resolution, cgroup parsing, and the
attribution loop feeding the exporter's reference-contract series."""
import json
import os
import tempfile
import time

import pytest

from kube_gpu_stats_amd.attribution import proto
from kube_gpu_stats_amd.attribution.attributor import Attributor
from kube_gpu_stats_amd.attribution.cgroup import parse_cgroup_text
from kube_gpu_stats_amd.attribution.podresources import DeviceIndex, FakeKubelet, PodResourcesClient
from kube_gpu_stats_amd.utils.scrape import parse_text


def sample_response():
    return proto.ListPodResourcesResponse([
        proto.PodResources("train-0", "ml", [proto.ContainerResources("main", [
            proto.ContainerDevices("amd.com/gpu", ["0000:11:00.0", "0000:21:00.0"], [0])], [1, 2, 3])]),
        proto.PodResources("infer-1", "serve", [proto.ContainerResources("srv", [
            proto.ContainerDevices("amd.com/gpu", ["0000:31:00.0"]),
            proto.ContainerDevices("example.com/nic", ["eth1"])])]),
        proto.PodResources("cpu-pod", "default", [proto.ContainerResources("c", [], [5])]),
    ])


def test_proto_roundtrip_and_wire_compat():
    r = sample_response()
    b = r.encode()
    back = proto.ListPodResourcesResponse.decode(b)
    assert back == r
    # hand-checked wire bytes for a minimal message: field 1 (LEN) "a"
    assert proto.enc_str(1, "a") == b"\x0a\x01a"
    assert proto.enc_int(1, 300) == b"\x08\xac\x02"
    # unknown fields are skipped
    extra = r.pod_resources[0].encode() + proto.enc_int(9, 7)
    assert proto.PodResources.decode(extra).name == "train-0"
    alloc = proto.AllocatableResourcesResponse([proto.ContainerDevices("amd.com/gpu", ["a", "b"])], [0, 1])
    assert proto.AllocatableResourcesResponse.decode(alloc.encode()) == alloc


def test_fake_kubelet_client_roundtrip():
    with tempfile.TemporaryDirectory() as d:
        sock = os.path.join(d, "kubelet.sock")
        with FakeKubelet(sock, sample_response()) as fk:
            c = PodResourcesClient(sock)
            allocs = c.gpu_allocations()
            assert [(a.pod, a.container, a.device_id) for a in allocs] == [
                ("train-0", "main", "0000:11:00.0"), ("train-0", "main", "0000:21:00.0"),
                ("infer-1", "srv", "0000:31:00.0")]
            assert c.allocatable().devices == []
            c.close()
            assert fk.calls == 1


def test_device_index_resolution():
    idx = DeviceIndex([{"index": 0, "bdf": "0000:72:00.0", "uuid": "dfff75a3-x", "serial": "0xABC", "drm_card": 8},
                       {"index": 1, "bdf": "0000:8B:00.0", "uuid": "1eff", "serial": "", "drm_card": 16}])
    assert idx.resolve("0000:72:00.0") == 0
    assert idx.resolve("72:00.0") == 0
    assert idx.resolve("0000:8b:00.0") == 1
    assert idx.resolve("DFFF75A3-X") == 0
    assert idx.resolve("card16") == 1
    assert idx.resolve("1") == 1
    assert idx.resolve("gpu-0000:72:00.0") == 0
    assert idx.resolve("nope") is None


@pytest.mark.parametrize("text,uid,cid,qos", [
    ("0::/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod0a1b2c3d_1111_2222_3333_444455556666.slice/"
     "cri-containerd-" + "a" * 64 + ".scope\n", "0a1b2c3d-1111-2222-3333-444455556666", "a" * 64, "burstable"),
    ("12:memory:/kubepods/besteffort/pod0a1b2c3d-1111-2222-3333-444455556666/" + "b" * 64 + "\n",
     "0a1b2c3d-1111-2222-3333-444455556666", "b" * 64, "besteffort"),
    ("0::/kubepods.slice/kubepods-pod0a1b2c3d_1111_2222_3333_444455556666.slice/crio-" + "c" * 64 + ".scope",
     "0a1b2c3d-1111-2222-3333-444455556666", "c" * 64, "guaranteed"),
    ("0::/user.slice/user-1000.slice/session-2.scope\n", "", "", ""),
])
def test_cgroup_parsing(text, uid, cid, qos):
    info = parse_cgroup_text(text)
    assert (info.pod_uid, info.container_id, info.qos) == (uid, cid, qos)


def test_attributor_end_to_end(mock_exporter, tmp_path):
    ex = mock_exporter(n_gpus=4, proc_every=1)
    sock = str(tmp_path / "kubelet.sock")
    proc_root = tmp_path / "proc"
    # mock backend PIDs: 100000 + 10*gpu + k
    for pid in (100000, 100010, 100011):
        (proc_root / str(pid)).mkdir(parents=True)
        (proc_root / str(pid) / "cgroup").write_text(
            f"0::/kubepods/pod0a1b2c3d-1111-2222-3333-44445555{pid % 10000:04d}/" + "d" * 64 + "\n")
    static = tmp_path / "owners.json"
    static.write_text(json.dumps({"3": {"pod": "static-pod", "namespace": "ops", "container": "x"}}))
    with FakeKubelet(sock, sample_response()):
        time.sleep(0.3)
        a = Attributor(ex, sock, str(static), proc_root=str(proc_root))
        a.update_once()
        body = ex.render()
    m = parse_text(body)
    compat = sorted((lb["gpu"], lb["pod_name"], lb["namespace"], lb["container_name"])
                    for lb, _ in m["container_gpu_sm_util"])
    assert compat == [("0", "train-0", "ml", "main"), ("1", "train-0", "ml", "main"),
                      ("2", "infer-1", "serve", "srv"), ("3", "static-pod", "ops", "x")]
    procs = {lb["pid"]: lb for lb, _ in m["amdgpu_process_hbm_bytes"]}
    assert procs["100000"]["pod"] == "train-0"
    assert procs["100000"]["pod_uid"] == "0a1b2c3d-1111-2222-3333-444455550000"
    assert procs["100010"]["pod"] == "train-0"  # GPU 1 held by one container
    assert a.updates == 1 and a.errors == 0


def test_attributor_survives_kubelet_outage(mock_exporter, tmp_path):
    ex = mock_exporter(n_gpus=2)
    sock = str(tmp_path / "kubelet.sock")
    with FakeKubelet(sock, sample_response()):
        a = Attributor(ex, sock, interval_s=0.05).start()
        time.sleep(0.3)
    time.sleep(0.3)  # kubelet gone: passes fail, thread keeps running
    a.stop()
    assert a.updates >= 1 and a.errors >= 1


def test_attributor_late_kubelet_reconnect_and_stale_drop(mock_exporter, tmp_path):
    """Socket absent at start → connects when it appears; a kubelet restart keeps
    the last table for stale_after_s, reconnects, and drops it only past that."""
    ex = mock_exporter(n_gpus=2)
    sock = str(tmp_path / "kubelet.sock")
    a = Attributor(ex, sock, stale_after_s=0.5)
    a.update_once()
    assert a.client is None and a.owners == {}
    with FakeKubelet(sock, sample_response()):
        a.update_once()
        assert a.client is not None and sorted(a.owners) == [0, 1]
    a.update_once()  # kubelet gone: the call fails, the last table is kept
    assert a.errors == 1 and a.reconnects == 1 and sorted(a.owners) == [0, 1]
    m = parse_text(ex.render())
    assert {lb["pod_name"] for lb, _ in m["container_gpu_sm_util"]} == {"train-0"}
    assert m["kgs_attribution_errors_total"][0][1] == 1
    assert m["kgs_attribution_kubelet_connected"][0][1] == 0
    with FakeKubelet(sock, sample_response()):  # kubelet back: new client
        a.update_once()
        assert a.client is not None and a.errors == 1
    a.update_once()
    assert sorted(a.owners) == [0, 1] and a.errors == 2  # gone again, table still fresh
    time.sleep(0.6)
    a.update_once()
    assert a.owners == {}  # past stale_after_s: pod labels dropped
    assert "container_gpu_sm_util" not in parse_text(ex.render())
    a.stop()
