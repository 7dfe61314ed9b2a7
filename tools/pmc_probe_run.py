"""GPU diagnostic: which hardware counters count under device counting, and what a
read costs.  Launches native pmc_probe (its own HSA process) over candidate
counter sets, runs idle / MFMA / triad / copy phases here, and attributes each
probe interval to a phase.  Writes gpurun_out/pmc_probe.json."""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PROBE = os.path.join(REPO, "kube_gpu_stats_amd", "native", "build", "pmc_probe")
LIB = os.path.join(REPO, "kube_gpu_stats_amd", "lib", "libkgs_pmc.so")

SETS = {
    "base": ["GRBM_COUNT:max", "GRBM_GUI_ACTIVE:max", "SQ_VALU_MFMA_BUSY_CYCLES"],
    "tcc_ea": ["GRBM_COUNT:max", "TCC_EA0_RDREQ", "TCC_EA0_WRREQ"],
    "tcc_hm": ["GRBM_COUNT:max", "TCC_HIT", "TCC_MISS"],
    "tcc_req": ["GRBM_COUNT:max", "TCC_REQ", "TCC_BUBBLE"],
    "derived": ["GRBM_COUNT:max", "FETCH_SIZE", "WRITE_SIZE"],
    "sq_waves": ["GRBM_COUNT:max", "SQ_WAVES", "SQ_BUSY_CYCLES"],
    "sq_insts": ["GRBM_COUNT:max", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_MFMA"],
    "sq_cycles": ["GRBM_COUNT:max", "SQ_WAVE_CYCLES", "SQ_BUSY_CU_CYCLES", "SQ_ACTIVE_INST_VALU"],
    "grbm": ["GRBM_COUNT:max", "GRBM_TC_BUSY:max", "GRBM_EA_BUSY:max", "GRBM_SPI_BUSY:max", "GRBM_CP_BUSY:max"],
    "tcp": ["GRBM_COUNT:max", "TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum"],
    "ta": ["GRBM_COUNT:max", "TA_BUSY_avr", "TA_FLAT_READ_WAVEFRONTS_sum"],
}



def main():
    from kube_gpu_stats_amd import load_native

    N = load_native()
    ex = N.Exporter({"backend": "amdsmi", "port": -1})
    gpu_id = ex.devices()[0]["kfd_gpu_id"]
    del ex
    out = {"gpu_id": gpu_id, "sets": {}}
    import torch

    from kube_gpu_stats_amd.ops import load
    from kube_gpu_stats_amd.ops.load import LoadStep

    ls = LoadStep(device=0, mfma_blocks=2048, mfma_iters=20000, stream_bytes=6 << 30)
    ls()
    torch.cuda.synchronize()
    for name, counters in SETS.items():
        period = "50"
        p = subprocess.Popen([PROBE, LIB, str(gpu_id), "4.8", period, *counters], stdout=subprocess.PIPE, text=True,
                             env=dict(os.environ, KGS_PMC_MODE="cumulative"))
        first = p.stdout.readline()
        phases = []

        def run(ph, fn, secs=1.5):
            t0 = time.time()
            while time.time() - t0 < secs:
                fn()
                torch.cuda.synchronize()
            phases.append((ph, t0 + 0.2, time.time()))

        time.sleep(0.3)
        run("idle", lambda: time.sleep(0.02), 1.0)
        run("mfma", ls.run_mfma, 1.0)
        run("triad", lambda: load.triad_f32(ls.a, ls.b, ls.c, 1.5, nt=False), 1.0)
        run("copy", lambda: load.copy_f32(ls.a, ls.c), 1.0)
        rest, _ = p.communicate(timeout=60)
        lines = [json.loads(x) for x in (first + rest).splitlines() if x.startswith("{")]
        res = {"info": lines[0], "summary": lines[-1], "phases": {}}
        for ph, a, b in phases:
            iv = [x for x in lines if "t" in x and a <= x["t"] <= b]
            if iv:
                res["phases"][ph] = {k: sum(x[k] for x in iv) / len(iv) for k in iv[0] if k not in ("t",)}
        out["sets"][name] = res
        print(name, json.dumps(res), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "pmc_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
