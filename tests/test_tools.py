"""Offline checks of the evidence tools (no GPU): the rocprofv3 trace splitter
assigns kernels to bench segments by launch order."""
import csv
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rocprof_overhead_splits_by_condition(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import rocprof_overhead as R

    res = {"steps": 3, "warmup": 1, "config": {"units_per_step": 2},
           "burst_resolution": {"per_gpu": {"0": {"launched": 4}}},
           "interleaved": {"block_steps": 1, "block_seconds": [["0", 1], ["100", 1], ["8000", 1],
                                                               ["8000", 1], ["100", 1], ["0", 1]]},
           "capacity": {"block_steps": 1, "rates": {"8000": {}, "16000": {}}}}
    tiny, triads = 3, 2
    dur = {"A_off": 100, "B_on_8k": 102, "C_off": 100, "I_paused": 100, "I_100Hz": 100, "I_8000Hz": 101,
           "calib": 50, "calib_reps": 50, "warmup": 50, "R_bursts": 1,
           "S_8000Hz": 300, "S_16000Hz": 300}  # phase S sits between I and C: off by one would skew C
    rows, t = [], 0

    def launch(name, d):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + d})
        t += d + 10

    def unit(d):
        launch("mfma_bf16_kernel(...)", d * 1000)
        for _ in range(triads):
            launch("triad_f32_kernel(...)", d * 10)
        for _ in range(tiny):
            launch("copy_f32_kernel(...)", d)

    launch("copy_f32_kernel(...)", 50)          # eager warm-up copy before graph capture
    launch("mfma_bf16_kernel(...)", 50 * 1000)  # calibrate(): 1 mfma, 1 triad, 1 graph replay
    launch("triad_f32_kernel(...)", 500)
    for _ in range(tiny):
        launch("copy_f32_kernel(...)", 50)
    launch("elementwise_kernel<torch>", 7)      # foreign kernels are ignored
    for label, units, extra in R.segments(res, triads, tiny):
        for _ in range(units):
            unit(dur[label])
        for _ in range(extra.get("mfma", 0)):      # phase R: bare MFMA bursts
            launch("mfma_bf16_kernel(...)", dur[label] * 1000)
    d = tmp_path / "trace" / "host" / "123"
    d.mkdir(parents=True)
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    bj = tmp_path / "bench.json"
    bj.write_text(json.dumps(res) + "\n")
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "rocprof_overhead.py"), str(tmp_path / "trace"),
                          str(bj), "--triads", str(triads), "--tiny", str(tiny), "--out", str(tmp_path / "o.md")],
                         capture_output=True, text=True, check=True).stdout
    r = json.loads(out)["kernels"]
    for kind in ("mfma", "triad", "copy"):
        k = r[kind]
        assert abs(k["B_vs_AC_pct"] - 2.0) < 1e-9, k
        assert abs(k["I_8000Hz_vs_paused_pct"] - 1.0) < 1e-9 and abs(k["I_100Hz_vs_paused_pct"]) < 1e-9, k
        # paired per round (two rounds of three blocks): every round says +1 % / 0 %
        assert k["rounds"] == 2 and abs(k["I_8000Hz_vs_paused_paired_pct"] - 1.0) < 1e-9, k
        assert abs(k["I_8000Hz_vs_paused_ci95_pct"]) < 1e-9 and abs(k["I_100Hz_vs_paused_paired_pct"]) < 1e-9, k
    md = (tmp_path / "o.md").read_text()
    assert "| mfma |" in md and "+1.000 ± 0.000" in md


def test_soak_tool_on_the_mock(tmp_path):
    """tools/soak.py rehearsed on the mock GPU: windows come out, nothing fails."""
    out = tmp_path / "soak.json"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "soak.py"), "--mock", "--seconds", "11",
                    "--window", "5", "--hz", "500", "--out", str(out)], cwd=REPO, capture_output=True, text=True,
                   check=True, timeout=120)
    r = json.loads(out.read_text())
    assert r["fail"] == [] and len(r["windows"]) >= 2, r
    assert all(w["pmc_samples_per_s"] > 400 and w["pmfw_tables_per_s"] > 40 for w in r["windows"]), r


def test_util_estimator_sim_replays_a_synthetic_dump(tmp_path, capsys):
    """tools/util_estimator_sim.py on a synthetic READ stream: 8 kHz READs that each
    cost the CP 20 µs, an idle stretch, and a 1 ms-every-5 ms burst train whose bursts
    run at a lower clock (1.8 GHz) than the idle stretches (2.1 GHz).  The sampler's
    estimator (the bound C++ class) learns the 20 µs on the idle READs, reads the idle
    GPU as ≈0 and the train at its 20 % duty."""
    import json

    sys.path.insert(0, os.path.join(REPO, "tools"))
    import util_estimator_sim as U

    def stream(busy_at, secs=1.0, hz=8000.0):
        t, cnt, spi, cpc, out = 0.0, 0.0, 0.0, 0.0, []
        dt = 1.0 / hz
        step = 1e-6
        while t < secs:
            out.append([t, int(cnt), int(spi), int(cpc), 0])
            s = 0.0
            while s < dt:
                b = busy_at(t + s)
                f = 1.8e9 if b else 2.1e9
                cnt += f * step
                if b:
                    spi += f * step
                    cpc += f * step
                s += step
            cpc += 20e-6 * 2.1e9      # the READ's own CP time
            t += dt
        return out

    burst = lambda t: (t % 0.005) < 0.001  # noqa: E731
    loads = {"idle": {"t0": 0.0, "t1": 0.5, "duty_gpu_s": 0.0, "samples": stream(lambda t: False, 0.5)},
             "burst_1_5": {"t0": 0.0, "t1": 0.5, "duty_gpu_s": 0.1, "samples": stream(burst, 0.5)}}
    p = tmp_path / "dump.json"
    p.write_text(json.dumps({"counters": [], "pipelined": 1, "rates": {"8000": loads}}))
    assert U.main([str(p)]) == 0
    out = json.loads(capsys.readouterr().out)["8000"]
    assert out["read_us"] == pytest.approx(20.0, rel=0.05)
    assert out["idle"]["busy_pct"] < 0.5
    b = out["burst_1_5"]
    assert b["busy_pct"] == pytest.approx(20.0, abs=0.5), b
    # --classes: the train's busy comes from the full intervals (≈ 7 of every 8 burst
    # intervals) plus its edges; the READ-only intervals between bursts add nothing
    assert U.main([str(p), "--classes"]) == 0
    c = json.loads(capsys.readouterr().out)["8000"]["burst_1_5"]
    assert c["read_only"]["intervals"] > 1000 and c["read_only"]["busy_us_per_s"] == 0.0, c
    total = sum(c[k]["busy_us_per_s"] for k in ("full", "partial", "read_only"))
    assert total == pytest.approx(c["duty_us_per_s"], rel=0.03) and c["full"]["busy_us_per_s"] > 0.8 * total, c


@pytest.mark.parametrize("tool", sorted(f for f in os.listdir(os.path.join(REPO, "tools")) if f.endswith(".py")))
def test_every_tool_answers_help_without_a_gpu(tool):
    """Every evidence tool answers --help on a machine without a GPU (argparse, or the
    docstring of a one-off probe, before any torch / HIP call)."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", tool), "--help"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0 and len(r.stdout.strip()) > 40, (r.stdout[-300:], r.stderr[-500:])


def test_tools_readme_lists_every_remaining_file():
    """tools/ holds the probes its README cites as evidence, and the README
    lists every file that remains."""
    here = os.path.join(REPO, "tools")
    text = open(os.path.join(here, "README.md")).read()
    files = [f for f in os.listdir(here) if os.path.isfile(os.path.join(here, f)) and f != "README.md"
             and not f.endswith(".pyc")]
    missing = [f for f in files if f"`{f}`" not in text and f"`{f} " not in text]
    assert not missing, missing


def test_gpu_margins_reads_runs_in_the_order_they_were_taken():
    """The bounds in force come from the last margins.jsonl read: run tags go r6y, r6z,
    r6aa, r6ab (spreadsheet columns), rounds in order."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import gpu_margins as G

    paths = [os.path.join(G.PROFILES, *p.split("/"), "margins.jsonl")
             for p in ("r6/r6ab", "r6/r6z", "r5/r5an", "r6/r6aa", "r6/r6b", "r6/r6y")]
    got = [G.run_dir(p) for p in sorted(paths, key=G.run_order)]
    assert got == ["r5/r5an", "r6/r6b", "r6/r6y", "r6/r6z", "r6/r6aa", "r6/r6ab"], got
