"""Real-hardware tests (MI355X).  Run on a GPU box: ``pytest -m gpu``.

Every test here exercises native code: the C++ amdsmi/PMFW backend, the gfx950
HIP load kernels (numerics vs a torch fp32 reference), and the rocprofiler-sdk
counter reader (in its own exporter process — HSA must come up under the tool
before any HIP runtime, and this pytest process initialises HIP).
"""
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


def test_amdsmi_backend_inventory(N):
    ex = N.Exporter({"backend": "amdsmi", "port": -1, "hz": 50, "pin_numa": True})
    devs = ex.devices()
    assert len(devs) >= 1
    d = devs[0]
    assert d["gfx_target"] == "gfx950", d
    assert d["gpu_type"].startswith("MI3"), d
    assert d["num_cu"] == 256 and d["num_xcc"] == 8, d
    assert d["vram_total_bytes"] > 250e9, d  # 288 GB HBM3E
    assert d["sysfs_dir"].endswith("/device"), d
    assert d["compute_partition"] in ("SPX", "DPX", "QPX", "CPX"), d  # MI355X compute partition modes
    assert d["memory_partition"].startswith("NPS"), d
    ex.start()
    time.sleep(0.5)
    s = ex.snapshot(0)
    ex.stop()
    assert s is not None and s["fw_ts"] > 0
    assert 0 <= s["gfx_busy_pct"] <= 100
    assert s["vram_used_bytes"] > 0 and s["power_w"] > 50
    assert s["temp_hotspot_c"] > 10
    assert len(s["gfx_busy_xcc"]) == 8


def test_pmfw_table_parser_matches_amdsmi(N):
    """Our direct v1.8 table parse equals amdsmi's parse of the same firmware tick."""
    import amdsmi as A

    ex = N.Exporter({"backend": "amdsmi", "port": -1})
    sysfs = ex.devices()[0]["sysfs_dir"]
    A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
    try:
        h = A.amdsmi_get_processor_handles()[0]
        for _ in range(20):
            with open(os.path.join(sysfs, "gpu_metrics"), "rb") as f:
                raw0 = f.read()
            m = A.amdsmi_get_gpu_metrics_info(h)
            with open(os.path.join(sysfs, "gpu_metrics"), "rb") as f:
                raw1 = f.read()
            p0, p1 = N.parse_gpu_metrics_v1_8(raw0), N.parse_gpu_metrics_v1_8(raw1)
            if p0["fw_ts"] == p1["fw_ts"] == m["firmware_timestamp"]:
                break
        else:
            pytest.fail("could not catch one firmware tick in 20 tries")
    finally:
        A.amdsmi_shut_down()
    assert p0["energy_acc"] == m["energy_accumulator"]
    assert p0["temp_hotspot_c"] == m["temperature_hotspot"]
    assert p0["gfx_busy_pct"] == m["average_gfx_activity"]
    assert p0["gfx_activity_acc"] == m["gfx_activity_acc"]
    assert p0["xgmi_read_kb"][1] == m["xgmi_read_data_acc"][1]
    assert p0["pcie_bw_acc_gb"] == m["pcie_bandwidth_acc"]
    assert p0["uclk_mhz"] == m["current_uclk"]


def test_mfma_kernel_numerics(torch_dev):
    import torch

    from kube_gpu_stats_amd.ops import load

    g = torch.Generator().manual_seed(7)
    # exact small integers: bf16-exact inputs, fp32-exact accumulation
    A = torch.randint(-3, 4, (16, 32), generator=g).to(torch.bfloat16).to(torch_dev)
    B = torch.randint(-3, 4, (32, 64), generator=g).float()
    B[0, 5] = 3.0  # asymmetric B (guide: catch row/col swaps)
    B = B.to(torch.bfloat16).to(torch_dev)
    blocks, iters = 8, 5
    C = torch.full((blocks * 4 * 16 * 64,), float("nan"), device=torch_dev)
    load.mfma_bf16(A, B, C, blocks, iters)
    torch.cuda.synchronize()
    ref = (A.float() @ B.float()) * iters
    got = C.view(blocks * 4, 16, 64)
    assert torch.equal(got, ref.expand_as(got)), (got[0] - ref).abs().max()

    Ar = torch.randn(16, 32, generator=g).to(torch.bfloat16).to(torch_dev)
    Br = torch.randn(32, 64, generator=g).to(torch.bfloat16).to(torch_dev)
    load.mfma_bf16(Ar, Br, C, blocks, 3)
    torch.cuda.synchronize()
    ref = (Ar.float() @ Br.float()) * 3
    torch.testing.assert_close(C.view(-1, 16, 64)[-1], ref, rtol=1e-5, atol=1e-4)


def test_stream_kernels_numerics(torch_dev):
    import torch

    from kube_gpu_stats_amd.ops import load

    n = (1 << 22) + 4
    a = torch.rand(n, device=torch_dev)
    b = torch.rand(n, device=torch_dev)
    c = torch.empty(n, device=torch_dev)
    load.triad_f32(a, b, c, 2.5)
    torch.cuda.synchronize()
    torch.testing.assert_close(c, a + 2.5 * b, rtol=1e-6, atol=1e-6)
    d = torch.empty(n, device=torch_dev)
    load.copy_f32(a, d)
    torch.cuda.synchronize()
    assert torch.equal(a, d)


def test_load_throughput_and_util_accumulators(N, torch_dev):
    """Under a saturating MFMA load the PMFW-accumulator window mean reads ~100 %."""
    import torch

    from kube_gpu_stats_amd.ops.load import LoadStep

    ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=3 << 30)
    ls()
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    ls.run_mfma()
    e1.record()
    ls.run_stream()
    e2.record()
    torch.cuda.synchronize()
    tflops = ls.flops / (e0.elapsed_time(e1) * 1e-3) / 1e12
    tbps = ls.bytes / (e1.elapsed_time(e2) * 1e-3) / 1e12
    print(json.dumps({"mfma_tflops": tflops, "triad_tbps": tbps}))
    assert tflops > 500, tflops      # dense bf16 MFMA peak ≈2500
    assert tbps > 3.0, tbps          # HBM3E ≈6.3 measured achievable

    ex = N.Exporter({"backend": "amdsmi", "port": -1, "hz": 100})
    ex.start()
    t0 = time.time()
    while time.time() - t0 < 2.0:
        ls.run_mfma()
        torch.cuda.synchronize()  # keep the queue short: the window below must see *this* load
    w = ex.window(0, 1.0)
    integ = ex.integrals(0)
    snap = ex.snapshot(0)
    procs = ex.procs(0)
    wall = time.time() - t0
    ex.stop()
    print(json.dumps({"procs": procs}))
    # this process' waves occupy CUs; the occupancy integral grows (PIDs are host-namespace).
    # The instantaneous cu_occupancy of the last list can already be 0 (the loop ended
    # with a synchronize), so the integral is the check.
    assert any(p["cu_seconds"] > 0.2 for p in procs), procs
    # per-XCC accumulators: every one of the 8 dies is busy under a full-grid MFMA load
    assert len(snap["gfx_busy_xcc_window"]) == 8 and min(snap["gfx_busy_xcc_window"]) > 90, snap
    print(json.dumps({"window": w, "integrals": integ, "wall_s": wall}))
    assert w["gfx_busy_pct"] > 90, w
    # PMFW cadence ≈ 50 Hz of distinct tables
    assert 30 <= integ["distinct_samples"] / wall <= 120, integ


def _proc_cpu_seconds(pid: int) -> float:
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")


@pytest.mark.parametrize("mode", ["aqlprofile", "aqlprofile-full", "aqlprofile-sync", "rocprofiler"])
def test_counter_reader_exporter_process(torch_dev, mode):
    """Exporter process with --pmc <reader> sees MFMA busy + HBM traffic of *this* process' kernels.

    aqlprofile (direct CP reads, the default) must also stay cheap on the host:
    the rocprofiler-sdk path keeps one HSA helper thread spinning (≈1 core).
    ``aqlprofile`` runs pipelined READs of the base set (the default),
    ``aqlprofile-full`` adds the TA block (vector-memory busy), ``aqlprofile-sync``
    submits and waits per sample; the rocprofiler-sdk reader runs the full set."""
    import torch

    from kube_gpu_stats_amd.ops.load import LoadStep
    from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

    reader = mode.split("-")[0]
    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0", "--hz", "100",
           "--pmc", reader, "--control-stdin", "--bdfs", bdf]
    if mode == "aqlprofile-sync":
        cmd.append("--no-pmc-pipeline")
    full = mode in ("aqlprofile-full", "rocprofiler")
    cmd += ["--pmc-set", "full" if full else "base"]
    proc = subprocess.Popen(cmd, cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                            text=True)
    try:
        ready = json.loads(proc.stdout.readline())
        print(json.dumps(ready)[:2000])
        assert ready["event"] == "ready", ready
        if ready["pmc"] != reader:
            pytest.fail(f"{reader} counters unavailable: " + ready.get("pmc_error", ""))
        sc = Scraper("127.0.0.1", ready["port"])
        ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=3 << 30)
        cpu0, w0 = _proc_cpu_seconds(proc.pid), time.time()
        t0 = time.time()
        while time.time() - t0 < 2.0:
            ls.run_mfma()
            torch.cuda.synchronize()
        m1 = parse_text(sc.get())
        mfma = [v for lb, v in m1["amdgpu_mfma_util_percent"]]
        t0 = time.time()
        while time.time() - t0 < 2.0:
            ls.run_stream()
            torch.cuda.synchronize()
        m2 = parse_text(sc.get())
        vmem = [v for lb, v in m2.get("amdgpu_vmem_busy_percent", [])]
        clk = [v for lb, v in m2["amdgpu_gpu_clock_effective_mhz"]]
        pmc_n = [v for lb, v in m2["kgs_pmc_samples_total"]]
        cores = (_proc_cpu_seconds(proc.pid) - cpu0) / (time.time() - w0)
        print(json.dumps({"mode": mode, "mfma_util": mfma, "vmem_busy": vmem, "clock_mhz": clk,
                          "pmc_samples": pmc_n, "exporter_cpu_cores": cores, "pmc_info": ready.get("pmc_info")}))
        assert mfma[0] > 50, mfma
        if full:
            assert vmem[0] > 30, vmem     # triad keeps the TA units busy
        else:
            assert not vmem, vmem         # base set: no TA block read
        assert 1000 < clk[0] < 2600, clk
        assert pmc_n[0] > 200
        if reader == "aqlprofile":
            assert cores < 0.5, cores  # no spinning helper thread (rocprofiler path: ≈1.0)
            want = "pipelined=0" if mode.endswith("-sync") else "pipelined=1"
            assert want in ready["pmc_info"][0], ready["pmc_info"]
    finally:
        out = err = ""
        try:
            proc.stdin.write("quit\n")
            proc.stdin.flush()
            out, err = proc.communicate(timeout=30)
        except Exception:  # noqa: BLE001
            proc.kill()
            out, err = proc.communicate()
        print(out[-3000:])  # "stopped" event: integrals + the reader's final pmc_info
        if err:
            print(err[-4000:])


def test_per_xcd_counters_follow_xcc_gated_load(torch_dev):
    """Per-XCD MFMA busy / GUI-active from the aqlprofile reader land on the XCDs the
    load really ran on.  The gated MFMA kernel reads its XCC id from the hardware
    (HW_REG_XCC_ID) and works only on XCDs 0 and 2, so the reader's XCD coordinate
    must match the hardware id (an order swap would light up other XCDs)."""
    import torch

    from kube_gpu_stats_amd.ops import load
    from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

    g = torch.Generator().manual_seed(3)
    A = torch.randn(16, 32, generator=g).to(torch.bfloat16).to(torch_dev)
    B = torch.randn(32, 64, generator=g).to(torch.bfloat16).to(torch_dev)
    blocks = 2048
    C = torch.empty(blocks * 4 * 16 * 64, device=torch_dev)
    ids = torch.full((blocks,), -1, dtype=torch.int32, device=torch_dev)
    load.mfma_bf16_xcc(A, B, C, blocks, 2, 0xFF, ids)
    torch.cuda.synchronize()
    hist = torch.bincount(ids.cpu().long(), minlength=8).tolist()
    first = ids[:16].cpu().tolist()
    print(json.dumps({"xcc_histogram": hist, "first_16_workgroups": first}))
    assert len(hist) == 8 and min(hist) > 0, hist  # SPX: all 8 XCDs take workgroups
    # gated numerics: a workgroup on an XCD outside the mask writes zeros
    load.mfma_bf16_xcc(A, B, C, blocks, 3, 0b101, ids)
    torch.cuda.synchronize()
    ref = (A.float() @ B.float()) * 3
    got = C.view(blocks, 4, 16, 64)
    on = (ids == 0) | (ids == 2)
    torch.testing.assert_close(got[on][0, 0], ref, rtol=1e-5, atol=1e-4)
    assert torch.count_nonzero(got[~on]).item() == 0

    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0", "--hz", "200",
           "--pmc", "aqlprofile", "--control-stdin", "--bdfs", bdf, "--proc-every", "0", "--link-every", "0"]
    # KGS_AQL_DUMP_RESULTS: the reader logs every result of its 250th READ (≈1.2 s
    # into the load) with aqlprofile's event coordinates — the raw layout evidence
    # (profiles/r1/xcd/).
    proc = subprocess.Popen(cmd, cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                            text=True, env=dict(os.environ, KGS_AQL_DUMP_RESULTS="250"))
    try:
        ready = json.loads(proc.stdout.readline())
        assert ready["event"] == "ready" and ready["pmc"] == "aqlprofile", ready
        sc = Scraper("127.0.0.1", ready["port"])
        t0 = time.time()
        while time.time() - t0 < 1.6:
            load.mfma_bf16_xcc(A, B, C, blocks, 20000, 0b101)
            torch.cuda.synchronize()
        m = parse_text(sc.get())
        mfma = {int(lb["xcc"]): v for lb, v in m.get("amdgpu_mfma_util_xcc_percent", [])}
        act = {int(lb["xcc"]): v for lb, v in m.get("amdgpu_gpu_active_xcc_percent", [])}
        gfx = {int(lb["xcc"]): v for lb, v in m.get("amdgpu_gfx_busy_xcc_percent", [])}
        print(json.dumps({"mfma_util_xcc": mfma, "gpu_active_xcc": act, "pmfw_gfx_busy_xcc": gfx,
                          "pmc_info": ready.get("pmc_info")}))
        assert sorted(mfma) == list(range(8)), mfma
        assert mfma[0] > 50 and mfma[2] > 50, mfma
        assert max(mfma[x] for x in (1, 3, 4, 5, 6, 7)) < 5, mfma
        # GUI-active is "a dispatch in flight", not "waves resident": the idle XCDs
        # read ~100 % too while the chip-wide kernel runs (profiles/r1/xcd/README.md).
        assert act[0] > 80 and act[2] > 80, act
        assert "xcd=8:" in ready["pmc_info"][0], ready["pmc_info"]  # all 8 XCDs placed
    finally:
        try:
            proc.stdin.write("quit\n")
            proc.stdin.flush()
            out, err = proc.communicate(timeout=30)
        except Exception:  # noqa: BLE001
            proc.kill()
            out, err = proc.communicate()
        print("\n".join(ln for ln in err.splitlines() if ln.startswith("[aql-res]")))
        print(out[-1500:])


def test_per_xcd_vmem_follows_xcc_gated_stream(torch_dev):
    """--pmc-set full: TA (vector-memory) busy per XCD lands on the XCDs a gated HBM
    triad runs on ({1, 6}, chosen by HW_REG_XCC_ID), and the gated triad computes
    exactly the elements of those XCDs' workgroups."""
    import torch

    from kube_gpu_stats_amd.ops import load
    from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

    n = 1 << 28  # 1 GiB per array
    a = torch.rand(n, device=torch_dev)
    b = torch.rand(n, device=torch_dev)
    c = torch.zeros(n, device=torch_dev)
    nb = load.default_stream_blocks(n)
    load.triad_f32_xcc(a, b, c, 2.0, 0b01000010, nblocks=nb)
    torch.cuda.synchronize()
    per = (n // 4 + nb - 1) // nb * 4  # elements per workgroup
    blk = torch.arange(n, device=torch_dev) // per
    on = ((blk % 8) == 1) | ((blk % 8) == 6)  # round-robin XCD placement (profiles/r1/xcd)
    torch.testing.assert_close(c[on], (a + 2.0 * b)[on])
    assert torch.count_nonzero(c[~on]).item() == 0
    del blk, on

    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    proc = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
                             "--hz", "200", "--pmc", "aqlprofile", "--pmc-set", "full", "--control-stdin", "--bdfs", bdf,
                             "--proc-every", "0", "--link-every", "0"],
                            cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        ready = json.loads(proc.stdout.readline())
        assert ready["event"] == "ready" and ready["pmc"] == "aqlprofile", ready
        sc = Scraper("127.0.0.1", ready["port"])
        t0 = time.time()
        while time.time() - t0 < 1.6:
            load.triad_f32_xcc(a, b, c, 2.0, 0b01000010, nblocks=nb)
            torch.cuda.synchronize()
        m = parse_text(sc.get())
        vm = {int(lb["xcc"]): v for lb, v in m.get("amdgpu_vmem_busy_xcc_percent", [])}
        print(json.dumps({"vmem_busy_xcc": vm, "pmc_info": ready.get("pmc_info")}))
        assert sorted(vm) == list(range(8)), vm
        assert vm[1] > 20 and vm[6] > 20, vm
        assert max(vm[x] for x in (0, 2, 3, 4, 5, 7)) < 0.25 * min(vm[1], vm[6]), vm
    finally:
        try:
            proc.stdin.write("quit\n")
            proc.stdin.flush()
            proc.communicate(timeout=30)
        except Exception:  # noqa: BLE001
            proc.kill()
            proc.communicate()


def test_counter_handover_stop_and_restart(torch_dev):
    """SIGUSR1 makes the aqlprofile reader STOP its counting session (another
    profiler may program the counters); SIGUSR2 re-STARTs it.  Counters read right
    after the re-START, and the exported totals stay monotonic."""
    import signal

    import torch

    from kube_gpu_stats_amd.ops.load import LoadStep
    from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    proc = subprocess.Popen([sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
                             "--hz", "1000", "--pmc", "aqlprofile", "--control-stdin", "--bdfs", bdf,
                             "--proc-every", "0", "--link-every", "0"],
                            cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=1 << 30)

    def load(secs):
        t0 = time.time()
        while time.time() - t0 < secs:
            ls.run_mfma()
            torch.cuda.synchronize()

    try:
        ready = json.loads(proc.stdout.readline())
        assert ready["event"] == "ready" and ready["pmc"] == "aqlprofile", ready
        sc = Scraper("127.0.0.1", ready["port"])
        one = lambda m, f: m[f][0][1]  # noqa: E731
        load(1.2)
        m0 = parse_text(sc.get())
        proc.send_signal(signal.SIGUSR1)
        time.sleep(0.3)
        m1 = parse_text(sc.get())
        time.sleep(0.5)
        m2 = parse_text(sc.get())
        proc.send_signal(signal.SIGUSR2)
        load(1.5)
        m3 = parse_text(sc.get())
        print(json.dumps({k: [one(m, "amdgpu_mfma_util_percent"), one(m, "kgs_pmc_enabled"),
                              one(m, "kgs_pmc_samples_total")] for k, m in (("m0", m0), ("m1", m1), ("m2", m2),
                                                                           ("m3", m3))}))
        assert one(m0, "amdgpu_mfma_util_percent") > 50 and one(m0, "kgs_pmc_enabled") == 1
        assert one(m2, "kgs_pmc_enabled") == 0 and one(m2, "kgs_pmc_samples_total") == one(m1, "kgs_pmc_samples_total")
        assert one(m3, "kgs_pmc_enabled") == 1 and one(m3, "kgs_pmc_releases_total") == 1
        assert one(m3, "amdgpu_mfma_util_percent") > 50                    # counters read right after re-START
        grbm = lambda m: [v for lb, v in m["amdgpu_pmc_total"] if lb["counter"] == "GRBM_COUNT"][0]  # noqa: E731
        assert grbm(m0) <= grbm(m2) < grbm(m3)
    finally:
        out = err = ""
        try:
            proc.stdin.write("quit\n")
            proc.stdin.flush()
            out, err = proc.communicate(timeout=30)
        except Exception:  # noqa: BLE001
            proc.kill()
            out, err = proc.communicate()
        print(out[-1500:])
        print(err[-1500:])


def test_hbm_bandwidth_estimate_tracks_stream_kernels(N, torch_dev):
    """amdgpu_hbm_bandwidth_bytes_per_second (UMC activity × MI355X calibration)
    agrees with the bytes a triad loop moves, and reads ~0 under a pure MFMA load."""
    import torch

    from kube_gpu_stats_amd.ops.load import LoadStep
    from kube_gpu_stats_amd.utils.scrape import parse_text

    ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=6 << 30)
    ls()
    torch.cuda.synchronize()
    ex = N.Exporter({"backend": "amdsmi", "port": -1, "hz": 100, "proc_every": 0, "link_every": 0,
                     "window_s": 1.0})
    ex.start()
    try:
        t0 = time.time()
        k = 0
        while time.time() - t0 < 1.6:
            ls.run_stream()
            torch.cuda.synchronize()
            k += 1
        measured = ls.bytes * k / (time.time() - t0)
        est = parse_text(ex.render())["amdgpu_hbm_bandwidth_bytes_per_second"][0][1]
        t0 = time.time()
        while time.time() - t0 < 1.6:
            ls.run_mfma()
            torch.cuda.synchronize()
        idle_est = parse_text(ex.render())["amdgpu_hbm_bandwidth_bytes_per_second"][0][1]
    finally:
        ex.stop()
    print(json.dumps({"measured_Bps": measured, "estimate_Bps": est, "mfma_estimate_Bps": idle_est}))
    assert measured > 3e12, measured
    assert abs(est / measured - 1) < 0.10, (est, measured)
    assert idle_est < 0.05e12, idle_est
