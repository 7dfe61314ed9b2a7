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
from fakekubelet import FakeKubelet
from kube_gpu_stats_amd.attribution.podresources import DeviceIndex, PodResourcesClient
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


def _cpx_devices(n_gpus=1):
    return [{"index": g * 8 + p, "bdf": f"0000:{0x11 + 0x10 * g:02x}:00.0", "uuid": f"u-{g}-{p}",
             "serial": f"MOCK{g}", "drm_card": 8 * g + p, "kfd_node": 2 + 8 * g + p, "partition_id": p}
            for g in range(n_gpus) for p in range(8)]


def _fake_xcp_sysfs(root, xcp_to_card: dict[int, int]):
    for n, card in xcp_to_card.items():
        d = root / "devices" / "platform" / f"amdgpu_xcp.{n}" / "drm" / f"card{card}"
        d.mkdir(parents=True)


def test_device_index_partitions_resolve_explicitly(tmp_path):
    """CPX: 8 devices share one BDF.  XCP IDs resolve through sysfs to the device
    owning that DRM card — never by their number (amdgpu_xcp_3 is not GPU 3)."""
    devs = _cpx_devices(2)  # GPU 0 → devices 0..7 (cards 0..7), GPU 1 → 8..15 (cards 8..15)
    # node-global XCP numbering: the secondary partitions of both GPUs, 7 each
    xcp = {n: (n // 7) * 8 + 1 + n % 7 for n in range(14)}
    _fake_xcp_sysfs(tmp_path, xcp)
    idx = DeviceIndex(devs, str(tmp_path))
    assert idx.resolve("amdgpu_xcp_3") == 4          # xcp 3 → card 4 → GPU 0 partition 4
    assert idx.resolve("amdgpu_xcp_10") == 12        # xcp 10 → card 12 → GPU 1 partition 4
    assert idx.resolve("amdgpu_xcp_99") is None      # unknown XCP: no guess
    assert idx.resolve("0000:11:00.0") == 0          # the PCI function is partition 0
    assert idx.resolve("0000:21:00.0") == 8
    assert idx.resolve("MOCK0") is None              # serial shared by 8 partitions: ambiguous
    assert idx.resolve("gpu-3") is None              # bare-number tails never resolve
    assert idx.resolve("card13") == 13 and idx.resolve("renderD133") == 5
    assert idx.resolve("3") == 3                     # the whole ID as an exporter index is exact
    assert DeviceIndex(devs, None).resolve("amdgpu_xcp_3") is None  # no sysfs, no XCP map


def test_cpx_partitions_each_carry_their_own_xcc(mock_exporter, tmp_path):
    """1 MI355X in CPX mode = 8 devices; 8 pods each get their partition's XCC busy
    (mock XCC x runs 50 + 40·sin(0.7·x) over a 1000 s period: ≈ constant here)."""
    import math

    ex = mock_exporter(n_gpus=1, hz=200, window_s=0.2,
                       mock={"compute_partition": "CPX", "util_period_s": 1000.0, "fw_period_s": 0.005})
    devs = ex.devices()
    assert len(devs) == 8 and {d["bdf"] for d in devs} == {"0000:11:00.0"}
    assert [d["partition_id"] for d in devs] == list(range(8)) and all(d["num_xcc"] == 1 for d in devs)
    assert [d["xcc_first"] for d in devs] == list(range(8)) and devs[0]["compute_partition"] == "CPX"
    _fake_xcp_sysfs(tmp_path / "sys", {n: n + 1 for n in range(7)})  # xcp n → card n+1 → partition n+1
    sock = str(tmp_path / "kubelet.sock")
    ids = ["0000:11:00.0"] + [f"amdgpu_xcp_{n}" for n in range(7)]
    resp = proto.ListPodResourcesResponse([
        proto.PodResources(f"job-{p}", "ml", [proto.ContainerResources("main", [
            proto.ContainerDevices("amd.com/gpu", [ids[p]])])]) for p in range(8)])
    with FakeKubelet(sock, resp):
        time.sleep(0.3)
        Attributor(ex, sock, sysfs_root=str(tmp_path / "sys")).update_once()
        m = parse_text(ex.render())
    got = {lb["pod_name"]: (int(lb["gpu"]), v) for lb, v in m["container_gpu_sm_util"]}
    assert sorted(got) == [f"job-{p}" for p in range(8)]
    for p in range(8):
        gpu, v = got[f"job-{p}"]
        assert gpu == p
        assert v == pytest.approx(50 + 40 * math.sin(0.7 * p), abs=1.0), (p, v)
    assert len({round(v) for _, v in got.values()}) == 8  # eight distinct series


class _StubExporter:
    """Duck-typed exporter for the PID→pod logic: fixed process lists per GPU."""

    def __init__(self, procs: dict[int, list[int]]):
        self._procs = procs
        self.device_count = len(procs)

    def devices(self):
        return [{"index": g, "bdf": f"0000:{0x11 + 0x10 * g:02x}:00.0"} for g in self._procs]

    def procs(self, gpu):
        return [{"pid": p} for p in self._procs[gpu]]


def test_pid_owners_keyed_by_gpu_and_pid(tmp_path):
    """one PID on two GPUs of different pods gets each GPU's owner on that
    GPU's line; a host process (no pod UID) and the exporter's own pod inherit nothing;
    with a pod directory every process gets its own pod, shared GPU or not."""
    from kube_gpu_stats_amd.attribution.poddir import PodDirectory

    proc_root = tmp_path / "proc"
    uid = {42: "0a1b2c3d-1111-2222-3333-444455550042", 99: "0a1b2c3d-1111-2222-3333-444455550099",
           51: "0a1b2c3d-1111-2222-3333-444455550051"}
    for pid in (42, 99, 51, 7, 1000):
        (proc_root / str(pid)).mkdir(parents=True)
        text = (f"0::/kubepods/pod{uid[pid]}/" + f"{pid:064x}\n") if pid in uid else "0::/user.slice/session-2.scope\n"
        (proc_root / str(pid) / "cgroup").write_text(text)
    (proc_root / "1000" / "cgroup").write_text(f"0::/kubepods/pod{uid[99]}/" + "e" * 64 + "\n")  # exporter = pod 99
    ex = _StubExporter({0: [42, 7, 1000], 1: [42, 51, 1000]})
    owners = {0: [{"pod": "a", "namespace": "ml", "container": "c"}],
              1: [{"pod": "b", "namespace": "ml", "container": "c"}]}
    a = Attributor(ex, None, proc_root=str(proc_root), self_pid=1000)
    out = a.pid_owners(owners)
    assert out[(0, 42)]["pod"] == "a" and out[(1, 42)]["pod"] == "b"   # each GPU's own owner
    assert out[(0, 7)]["pod"] == "" and out[(0, 7)]["pod_uid"] == ""     # host process
    assert out[(0, 1000)]["pod"] == "" and out[(1, 1000)]["pod"] == ""  # the exporter itself
    # pod directory: UID / container ID → the process's real pod
    pl = {"items": [
        {"metadata": {"name": "real-42", "namespace": "team", "uid": uid[42]},
         "status": {"containerStatuses": [{"name": "w", "containerID": "containerd://" + f"{42:064x}"}]}},
        {"metadata": {"name": "real-51", "namespace": "team", "uid": uid[51]}}]}
    f = tmp_path / "pods.json"
    f.write_text(json.dumps(pl))
    a2 = Attributor(ex, None, proc_root=str(proc_root), self_pid=1000, pod_directory=PodDirectory(f"file:{f}"))
    out2 = a2.pid_owners(owners)
    assert (out2[(0, 42)]["pod"], out2[(0, 42)]["container"]) == ("real-42", "w")
    assert out2[(1, 42)]["pod"] == "real-42" and out2[(1, 51)]["pod"] == "real-51"
    assert out2[(0, 7)]["pod"] == ""


def test_pid_owner_labels_per_gpu_line(mock_exporter):
    ex = mock_exporter(n_gpus=2, proc_every=1)
    time.sleep(0.3)
    pid0 = ex.procs(0)[0]["pid"]
    pid1 = ex.procs(1)[0]["pid"]
    ex.set_pid_owners({(0, pid0): {"pod": "p0", "namespace": "n", "container": "c", "pod_uid": "u0"},
                       (1, pid0): {"pod": "WRONG", "namespace": "n", "container": "c", "pod_uid": "u0"},
                       (1, pid1): {"pod": "p1", "namespace": "n", "container": "c", "pod_uid": "u1"}})
    m = parse_text(ex.render())
    lines = {(lb["gpu"], lb["pid"]): lb["pod"] for lb, _ in m["amdgpu_process_hbm_bytes"]}
    assert lines[("0", str(pid0))] == "p0" and lines[("1", str(pid1))] == "p1"
