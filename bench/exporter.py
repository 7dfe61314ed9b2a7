"""The exporter under test, spawned as its own process (as in production) or attached over HTTP,
and the readings taken from it: sample counts, CPU time, the rank-local PMFW probe."""
from __future__ import annotations

import json
import os
import select
import subprocess
import sys
import time

from kube_gpu_stats_amd.utils.scrape import Scraper, parse_text

from .common import PMC_READER, REPO


class ExporterCtl:
    """Control calls shared by the spawned and the attached exporter (``self.sc``)."""

    def pmc_enabled(self) -> dict:
        m = parse_text(self.sc.get())
        return {lb["gpu"]: v for lb, v in m.get("kgs_pmc_enabled", [])}

    def _wait_pmc(self, on: bool, timeout: float = 10.0) -> bool:
        end = time.time() + timeout
        while time.time() < end:
            st = self.pmc_enabled()
            if st and all((v == 1) == on for v in st.values()):
                return True
            time.sleep(0.01)
        return False

    def release(self, drop_queue: bool = True) -> bool:
        """Counter sessions STOPped on every GPU (and, with drop_queue, the reader's READ
        queues destroyed): the "released" condition.  Needs running sampler threads —
        each GPU's own counter thread acts — and waits until all have."""
        self.sc.get("/control/pmc/release" + ("?drop_queue=1" if drop_queue else ""))
        return self._wait_pmc(False)

    def acquire(self) -> bool:
        self.sc.get("/control/pmc/acquire")
        return self._wait_pmc(True)

    def set_quiet_release(self, secs: float) -> float:
        """--pmc-quiet-release-s in place (secs < 0 only reads it)."""
        q = f"?s={secs:g}" if secs >= 0 else ""
        return json.loads(self.sc.get("/control/pmc/quiet_release" + q)).get("pmc_quiet_release_s", 0.0)

    def wait_parked(self, timeout: float = 10.0) -> bool:
        """Every GPU's counter session released for quiet (kgs_pmc_parked 1)."""
        end = time.time() + timeout
        while time.time() < end:
            st = {lb["gpu"]: v for lb, v in parse_text(self.sc.get()).get("kgs_pmc_parked", [])}
            if st and all(v == 1 for v in st.values()):
                return True
            time.sleep(0.05)
        return False


class AttachedExporter(ExporterCtl):
    """An already-running exporter (``--control-http``) driven over HTTP."""

    def __init__(self, hostport: str):
        host, _, port = hostport.rpartition(":")
        self.port = int(port)
        self.sc = Scraper(host or "127.0.0.1", self.port)
        m = parse_text(self.sc.get())
        info = m.get("kgs_build_info", [({}, 0)])[0][0]
        self.ready = {"pmc": info.get("pmc_source", "none"), "pmc_error": "",
                      "hz": float(info.get("sample_hz", "0") or 0)}

    def pause(self):
        self.sc.get("/control/pause")

    def resume(self):
        self.sc.get("/control/resume")

    def set_rate(self, hz: float):
        self.sc.get(f"/control/rate?hz={hz:g}")

    def set_idle_hz(self, hz: float) -> float:
        return json.loads(self.sc.get(f"/control/pmc/idle?hz={hz:g}")).get("pmc_idle_hz", 0.0)

    def json(self, path: str):
        return json.loads(self.sc.get(path))

    def stop(self) -> dict:
        self.pause()
        m = parse_text(self.sc.get())
        fam = lambda n: {lb["gpu"]: v for lb, v in m.get(n, [])}  # noqa: E731
        reads, rs, pmc, prs = (fam("kgs_reads_total"), fam("kgs_read_seconds_total"),
                               fam("kgs_pmc_samples_total"), fam("kgs_pmc_read_seconds_total"))
        hist = fam("kgs_sample_read_seconds_sum")
        return {"integrals": [{"gpu": g, "reads": reads[g], "read_seconds": hist.get(g, rs.get(g, 0.0)),
                               "pmc_samples": pmc.get(g, 0), "pmc_read_seconds": prs.get(g, 0.0),
                               "overruns": fam("kgs_sampler_overruns_total").get(g, 0)} for g in sorted(reads)]}


class ExporterProc(ExporterCtl):
    def __init__(self, a, bdfs: list[str], log_path: str):
        # Production tiers: per-process list at 10 Hz, xGMI links + RAS at 1 Hz (node-wide
        # slow thread), gauges over a 2 s window (phase B is ~10 s).
        # --compat-unallocated: the reference-contract series (container_gpu_sm_util,
        # container_gpu_busy_seconds_total) for every GPU, pod_name="" (phase U reads them).
        cmd = [sys.executable, "-m", "kube_gpu_stats_amd.cli", "exporter", "--listen", "127.0.0.1:0",
               "--hz", str(a.hz), "--proc-period", "0.1", "--link-period", "1.0", "--window", "2",
               "--control-stdin", "--control-http", "--node-name", "bench-node", "--bdfs", ",".join(bdfs),
               "--compat-unallocated"]
        if a.mock:
            cmd += ["--backend", "mock", "--mock-gpus", str(max(8, len(bdfs))), "--pmc", "mock",
                    "--mock-xgmi-swap", str(a.mock_xgmi_swap)]
            if a.mock_latency:
                cmd += ["--mock-latency"]
        else:
            pmc = PMC_READER if a.pmc == "auto" else a.pmc
            cmd += ["--pmc", pmc, "--pmc-pipeline" if a.pmc_pipeline else "--no-pmc-pipeline", "--pmc-set", a.pmc_set,
                    "--pmc-lean", str(a.pmc_lean)]
        cmd += ["--pmc-dispatch-hz", f"{a.pmc_dispatch_hz:g}"]
        if not a.mock:
            cmd += ["--pmc-batch", str(a.pmc_batch), "--pmc-publish-us", str(a.pmc_publish_us)]
        env = dict(os.environ)
        env.setdefault("KGS_NO_BUILD", "1")
        env.setdefault("PYTHONFAULTHANDLER", "1")  # a native fault leaves a trace in the exporter log
        self.log = open(log_path, "w")
        self.p = subprocess.Popen(cmd, cwd=REPO, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=self.log,
                                  text=True, env=env)
        self.ready = self._wait_ready(120.0)
        self.port = int(self.ready["port"])
        self.sc = Scraper("127.0.0.1", self.port)

    def pause(self):
        self.sc.get("/control/pause")

    def resume(self):
        self.sc.get("/control/resume")

    def set_rate(self, hz: float):
        self.sc.get(f"/control/rate?hz={hz:g}")

    def set_idle_hz(self, hz: float) -> float:
        return json.loads(self.sc.get(f"/control/pmc/idle?hz={hz:g}")).get("pmc_idle_hz", 0.0)

    def json(self, path: str):
        return json.loads(self.sc.get(path))

    def _wait_ready(self, timeout: float) -> dict:
        end = time.time() + timeout
        while time.time() < end:
            r, _, _ = select.select([self.p.stdout], [], [], 1.0)
            if r:
                line = self.p.stdout.readline()
                if not line:
                    break
                try:
                    msg = json.loads(line)
                except ValueError:
                    continue
                if msg.get("event") == "ready":
                    return msg
                if msg.get("event") == "error":
                    raise RuntimeError("exporter failed: " + msg.get("error", ""))
            if self.p.poll() is not None:
                break
        raise RuntimeError(f"exporter did not become ready (rc={self.p.poll()}); see {self.log.name}")

    def stop(self) -> dict:
        try:
            self.p.stdin.write("quit\n")
            self.p.stdin.flush()
        except OSError:
            pass
        try:
            out, _ = self.p.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            self.p.kill()
            out, _ = self.p.communicate()
        self.log.close()
        for line in out.splitlines():
            try:
                msg = json.loads(line)
                if msg.get("event") == "stopped":
                    return msg
            except ValueError:
                pass
        return {}


def proc_cpu_seconds(pid: int) -> float:
    """utime + stime of a process (all threads), seconds; 0 if unreadable."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return 0.0


def thread_cpu_seconds(pid: int) -> dict:
    """Per-thread utime + stime, keyed ``<comm>/<tid>`` (finds spinning helper threads)."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"/proc/{pid}/task/{tid}/stat") as f:
                raw = f.read()
            comm = raw[raw.index("(") + 1:raw.rindex(")")]
            fields = raw.rsplit(")", 1)[1].split()
            out[f"{comm}/{tid}"] = (int(fields[11]) + int(fields[12])) / tck
        except (OSError, ValueError, IndexError):
            continue
    return out


def sample_counts(m: dict) -> tuple[dict, dict]:
    pmfw = {lb["gpu"]: v for lb, v in m.get("kgs_samples_total", [])}
    pmc = {lb["gpu"]: v for lb, v in m.get("kgs_pmc_samples_total", [])}
    return pmfw, pmc


class Rates:
    """Per-GPU sample counts over a set of windows, from /metrics counter deltas."""

    def __init__(self):
        self.pmc: dict[str, float] = {}
        self.pmfw: dict[str, float] = {}
        self.secs = 0.0

    def add(self, before: dict, after: dict, secs: float) -> None:
        bp, bc = sample_counts(before)
        ap_, ac = sample_counts(after)
        for g in ap_:
            self.pmfw[g] = self.pmfw.get(g, 0.0) + ap_[g] - bp.get(g, 0.0)
            self.pmc[g] = self.pmc.get(g, 0.0) + ac.get(g, 0.0) - bc.get(g, 0.0)
        self.secs += secs

    def per_gpu(self, pmc_on: bool) -> tuple[dict, str]:
        """Per GPU: its counter stream if it delivered one, else its PMFW table rate,
        so one device whose counter tier failed lowers the total by its own share only."""
        if self.secs <= 0:
            return {}, "none"
        gpus = sorted(self.pmfw, key=int)
        out, n_pmc = {}, 0
        for g in gpus:
            if pmc_on and self.pmc.get(g, 0) > 0:
                out[g] = self.pmc[g] / self.secs
                n_pmc += 1
            else:
                out[g] = self.pmfw[g] / self.secs
        src = "pmc" if n_pmc == len(gpus) else ("pmfw" if n_pmc == 0 else f"pmc on {n_pmc}/{len(gpus)} GPUs")
        return out, src


class PmfwProbe:
    """Rank-local PMFW table reads at interleaved-block edges (one ≈46 µs sysfs pread
    each), independent of the exporter — which is paused in the "off" blocks: the
    block's average socket power and package-power throttle residency, from the
    table's own energy / PPT-residency accumulators and firmware clock.  Shows
    whether a sampling rate changes the GPU's power state (profiles/r2/r2aq)."""

    def __init__(self, bdf: str):
        self.path = f"/sys/bus/pci/devices/{bdf}/gpu_metrics"
        try:
            from kube_gpu_stats_amd.native import load

            self.N = load(rebuild=False)  # built by local rank 0 long before the rounds
            self.read()
        except Exception:  # noqa: BLE001 - mock runs, other table revisions: no probe
            self.N = None

    def read(self) -> dict | None:
        if self.N is None:
            return None
        with open(self.path, "rb") as f:
            return self.N.parse_gpu_metrics_v1_8(f.read())

    @staticmethod
    def delta(a: dict | None, b: dict | None) -> dict | None:
        if not a or not b or b["fw_ts"] <= a["fw_ts"]:
            return None
        dt = (b["fw_ts"] - a["fw_ts"]) * 1e-8  # firmware clock: 10 ns
        out = {"power_w": (b["energy_acc"] - a["energy_acc"]) / 65536.0 / dt}  # 2^-16 J units
        dc = b["accumulation_counter"] - a["accumulation_counter"]
        if dc > 0 and b["ppt_residency_acc"] >= a["ppt_residency_acc"]:
            out["ppt_pct"] = 100.0 * (b["ppt_residency_acc"] - a["ppt_residency_acc"]) / dc
        if dc > 0 and b.get("gfx_activity_acc", -1) >= a.get("gfx_activity_acc", 0) >= 0:
            out["gfx_busy_pct"] = (b["gfx_activity_acc"] - a["gfx_activity_acc"]) / dc  # % per tick
        return out
