"""Native core: PMFW v1.8 table parser against a captured MI355X table, and the
TSAN build of the seqlock / ring / sampler concurrency test."""
import os
import subprocess

import pytest

DATA = os.path.join(os.path.dirname(__file__), "data", "gpu_metrics_mi355x_v1_8.bin")


def test_parse_captured_mi355x_table(N):
    blob = open(DATA, "rb").read()
    assert len(blob) == 3872 and blob[2:4] == b"\x01\x08"
    s = N.parse_gpu_metrics_v1_8(blob)
    # values decoded from the table captured on the gpurun box (tools/probe_gpu.py)
    assert s["temp_hotspot_c"] == 49 and s["temp_mem_c"] == 34 and s["temp_vrsoc_c"] == 45
    assert s["power_w"] == 255
    assert s["energy_acc"] == 4079392858440
    assert s["fw_ts"] == 23294450932196
    assert s["accumulation_counter"] == 232672000
    assert s["gfx_activity_acc"] == 1142341926
    assert s["xgmi_read_kb"][:3] == [0, 12840266, 12849075]
    assert s["xgmi_write_kb"][1] == 12826071
    assert s["xgmi_link_up"][0] == 0xFFFF and s["xgmi_link_up"][1] == 1
    assert s["xgmi_link_speed_gbps"] == 38
    assert s["pcie_bw_acc_gb"] == 333115936218
    assert s["pcie_link_width"] == 16 and s["pcie_link_speed_01gts"] == 320
    assert s["gfxclk_mhz"] == [157] * 7 + [158]
    assert s["uclk_mhz"] == 2000 and s["socclk_mhz"] == 38
    assert s["num_xcc"] == 8 and s["gfx_busy_xcc"] == [0.0] * 8
    assert s["gfx_busy_acc_xcc"][:2] == [1144238836, 1143176127]  # xcp_stats[0].gfx_busy_acc
    assert s["valid"] & (1 << 17)


def test_parser_rejects_other_revisions(N):
    blob = bytearray(open(DATA, "rb").read())
    blob[3] = 7
    with pytest.raises(RuntimeError):
        N.parse_gpu_metrics_v1_8(bytes(blob))
    with pytest.raises(RuntimeError):
        N.parse_gpu_metrics_v1_8(bytes(blob[:100]))


def test_gpu_type_label(N):
    assert N.gpu_type_from_market_name("AMD Instinct MI355 OAM") == "MI355X"
    assert N.gpu_type_from_market_name("AMD Instinct MI300X") == "MI300X"
    assert N.gpu_type_from_market_name("AMD Instinct MI325X OAM") == "MI325X"
    assert N.gpu_type_from_market_name("") == "unknown"


@pytest.mark.slow
@pytest.mark.parametrize("sanitizer,marker", [("thread", "ThreadSanitizer"),
                                              ("address,undefined", "runtime error")])
def test_sanitized_seqlock_ring_sampler(sanitizer, marker):
    from kube_gpu_stats_amd.native import build

    exe = build.build_tsan_test(sanitizer=sanitizer)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, UBSAN_OPTIONS="print_stacktrace=1", ASAN_OPTIONS="detect_leaks=1"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    assert marker not in out and "AddressSanitizer" not in out, out
    assert "ALL OK" in out


@pytest.mark.slow
def test_cmake_build_matches_python_build(tmp_path):
    """The CMake route (image builds) produces a working module from the same sources."""
    import shutil
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = tmp_path / "kube_gpu_stats_amd"
    shutil.copytree(os.path.join(repo, "kube_gpu_stats_amd"), pkg,
                    ignore=shutil.ignore_patterns("*.so", "build", "__pycache__"))
    bdir = tmp_path / "build"
    subprocess.run(["cmake", "-S", str(pkg / "native"), "-B", str(bdir), "-G", "Ninja", "-DKGS_BUILD_LOAD=OFF"],
                   check=True, capture_output=True, timeout=300)
    subprocess.run(["cmake", "--build", str(bdir), "-j", "8"], check=True, capture_output=True, timeout=900)
    assert (pkg / "lib" / "libkgs_pmc.so").exists()
    code = ("import time, kube_gpu_stats_amd.native as n; N = n.load(rebuild=False); "
            "e = N.Exporter({'backend': 'mock', 'mock': {'n_gpus': 2}, 'port': -1, 'hz': 100, 'pin_numa': False}); "
            "e.start(); time.sleep(0.2); assert 'kgs_up' in e.render(); "
            "print(N.__file__); e.stop()")
    r = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                       env={**os.environ, "KGS_NO_BUILD": "1", "PYTHONPATH": str(tmp_path)})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().startswith(str(pkg))
