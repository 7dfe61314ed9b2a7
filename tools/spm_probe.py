"""GPU probe: how far does the streaming-performance-monitor (SPM) path go on this ROCm?

SPM is the RLC's counter streamer: once programmed, the RLC writes counter snapshots into
a ring at a fixed interval with no command-processor packet per sample, so it would
avoid the per-READ CP cost (profiles/r2/idle_busy/README.md, profiles/launch_overhead.md).
It has two halves:

* the data path: ROCr's ``hsa_amd_spm_acquire`` / ``hsa_amd_spm_set_dest_buffer`` /
  ``hsa_amd_spm_release`` (``hsa_ext_amd.h``), a thin wrapper over KFD's SPM ioctl;
* the programming: the PM4 packets that select the counters (RLC SPM muxsel RAM,
  per-block perfmon selects, sample interval).  rocprofiler-sdk declares
  ``rocprofiler_configure_spm_service`` (``rocprofiler-sdk/spm.h``, experimental) and
  aqlprofile carries gfx9..gfx12 SPM packet builders internally, but neither library
  exports an entry point that builds or configures SPM (``nm -D``).

This checks the first half on the box: which SPM symbols the shipped libraries export,
and whether KFD grants SPM on the GPU to an unprivileged process (acquire, then release;
no destination buffer is set, so the RLC never writes).  Prints one JSON line and
writes gpurun_out/spm_probe.json.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LIBS = ["libhsa-runtime64.so", "libhsa-amd-aqlprofile64.so", "librocprofiler-sdk.so"]
HSA_DEVICE_TYPE_GPU = 1
HSA_AGENT_INFO_DEVICE = 17
HSA_AGENT_INFO_NAME = 0


def exported_spm_symbols(path: str) -> list[str]:
    try:
        out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, timeout=60).stdout
    except (OSError, subprocess.TimeoutExpired):
        return ["<nm failed>"]
    return sorted({ln.split()[-1] for ln in out.splitlines() if "spm" in ln.lower()})


def main() -> int:
    res: dict = {"exports": {lib: exported_spm_symbols(os.path.join(ROCM, "lib", lib)) for lib in LIBS}}
    hsa = ctypes.CDLL(os.path.join(ROCM, "lib", "libhsa-runtime64.so"))
    res["hsa_init"] = hsa.hsa_init()
    gpus: list[int] = []
    CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)

    def on_agent(agent, _):
        t = ctypes.c_int(0)
        hsa.hsa_agent_get_info(ctypes.c_uint64(agent), HSA_AGENT_INFO_DEVICE, ctypes.byref(t))
        if t.value == HSA_DEVICE_TYPE_GPU:
            gpus.append(agent)
        return 0

    cb = CB(on_agent)
    hsa.hsa_iterate_agents(cb, None)
    res["gpu_agents"] = len(gpus)
    if gpus:
        agent = ctypes.c_uint64(gpus[0])
        name = ctypes.create_string_buffer(64)
        hsa.hsa_agent_get_info(agent, HSA_AGENT_INFO_NAME, name)
        res["agent"] = name.value.decode(errors="replace")
        st = hsa.hsa_amd_spm_acquire(agent)
        res["spm_acquire_status"] = hex(st)
        if st == 0:
            res["spm_release_status"] = hex(hsa.hsa_amd_spm_release(agent))
        msg = ctypes.c_char_p()
        hsa.hsa_status_string(st, ctypes.byref(msg))
        res["spm_acquire_message"] = (msg.value or b"").decode(errors="replace")
    hsa.hsa_shut_down()
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "spm_probe.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
