"""the CPU suite must not write into ``gpurun_out/`` — the scratch
directory GPU runs merge their results into (BENCH_r05's ``full_result`` pointed at a
file the CPU suite later overwrote with a mock result).  conftest.py hashes the tree
when the session starts; this module sorts last and checks it is byte-identical."""
import pytest

import conftest


def test_cpu_suite_left_gpurun_out_byte_identical(request):
    expr = request.config.getoption("markexpr") or ""
    if "gpu" in expr and "not gpu" not in expr:
        pytest.skip("GPU runs keep their results under gpurun_out/ on purpose")
    assert conftest.gpurun_out_digest() == conftest.GPURUN_OUT_AT_START, (
        "a CPU test wrote under gpurun_out/: pass it a tmp_path (bench.py --out ...) instead")
