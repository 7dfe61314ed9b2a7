"""The utilisation estimators as pure units (native/include/kgs/util_estimator.h).

* DispatchEstimator: raw counter READs recorded on MI355X (profiles/r4/r4f/cp_dump.json:
  every READ of GRBM_COUNT, GRBM_SPI_BUSY and CPC busy at 8 kHz and 1 kHz under seven
  loads, with each load's event-timed kernel duty) replayed through the very class
  Sampler::run_pmc runs, with the default SamplerConfig's parameters.  Every load
  must read within 1 point of its duty; the parameter values earlier rounds rejected
  must fail that bound, so a change to a threshold shows up here.
* UtilBiller: the per-PMFW-interval billing of container_gpu_busy_seconds_total
  (reference gpu_util_stats/gpu_util_stats.py:159 reads the series, :62-94 bills each
  pod its mean) loses nothing when drains and PMFW intervals alias.
"""
from __future__ import annotations

import json
import math
import os
import random

import pytest

from tools import util_estimator_sim as sim

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(REPO, "profiles", "r4", "r4f", "cp_dump.json")


@pytest.fixture(scope="module")
def shipped():
    return sim.replay(DUMP)


def test_dump_replays_within_one_point_of_the_kernels_duty(shipped):
    for rate in ("8000", "1000"):
        rows = shipped[rate]
        assert rows["read_us"] == pytest.approx(15.5, abs=1.5)  # the READ packet's CP time (r4f: 15.5 µs)
        for load in ("idle", "mfma", "triad", "gemm", "tiny_graph", "burst_1_5", "burst_02_1"):
            r = rows[load]
            assert abs(r["err_pts"]) <= 1.0, (rate, load, r)
        # a µs-kernel graph: SPI busy sees 43 % (waves part of the time), the estimator the dispatch
        assert rows["tiny_graph"]["active_pct"] < 50 and rows["tiny_graph"]["busy_pct"] > 99, rows["tiny_graph"]


LOWRATE = os.path.join(REPO, "profiles", "r5", "r5b_cp_dump_lowrate.json")


def test_read_only_intervals_bill_nothing(shipped):
    """A READ-only interval's CP busy less the learned mean READ cost is the READ's own
    scatter: keeping its positive half billed an idle GPU 0.14 % at 8 kHz and the gaps of a
    burst train with it (sampler.h kReadOnlyBillsZero)."""
    assert abs(shipped["8000"]["idle"]["err_pts"]) <= 0.05 and abs(shipped["1000"]["idle"]["err_pts"]) <= 0.05
    old = sim.replay(DUMP, {"read_only_bills_zero": "false"})
    assert old["8000"]["idle"]["err_pts"] > 0.1, old["8000"]["idle"]


def test_one_khz_bursts_read_the_reads_cp_time_once(shipped):
    """a READ that lands inside a kernel adds no CP busy; subtracting its
    cost whole from a 1 ms interval under-read the 1 kHz trains."""
    for load in ("burst_1_5", "burst_02_1"):
        assert abs(shipped["1000"][load]["err_pts"]) < 0.8, shipped["1000"][load]
    old = sim.replay(DUMP, {"read_overlap_ns": -1})
    assert old["1000"]["burst_02_1"]["err_pts"] < shipped["1000"]["burst_02_1"]["err_pts"] - 0.2


LOWRATE_R5L = os.path.join(REPO, "profiles", "r5", "r5l_cp_dump_1k.json")
TRAINS = ("burst_1_5", "burst_02_1")


def _worst_train_error(over: dict | None = None) -> float:
    worst = 0.0
    for path in (LOWRATE, LOWRATE_R5L):
        for rows in sim.replay(path, over).values():
            worst = max(worst, *(abs(rows[t]["err_pts"]) for t in TRAINS))
    return worst


def test_low_rate_reads_in_the_exporters_read_mode_stay_within_two_points():
    """The exporter's own READ mode (batched, lite, its counter set) recorded on MI355X at
    1 kHz, 100 Hz and the DaemonSet's 10 Hz (r5b), and at 1 kHz on another box (r5l).  Long
    READ intervals mix power-capped MFMA bursts (≈2.0 GHz) with faster gaps: a cycle
    share under-reads the 1 ms / 5 ms train by 2.2-2.7 points, and at 10 Hz no fully busy
    interval ever teaches the busy clock the old clock-ratio split needs.  The time split
    (idle cycles at the learned idle clock, sampler.h kTimeSplitNs) over-reads instead
    where the gaps clock below that (r5l: the 0.2 ms / 1 ms train +2.0): the shipped blend
    of the two (kTimeSplitWeight) reads every load within 2 points and both trains within
    1.5 at every rate, the DaemonSet's 10 Hz within 0.5."""
    now = sim.replay(LOWRATE)
    for rate in ("1000", "100", "10"):
        for load in ("idle", "mfma", "triad", "gemm", "tiny_graph", "burst_1_5", "burst_02_1"):
            assert abs(now[rate][load]["err_pts"]) <= 2.0, (rate, load, now[rate][load])
    for t in TRAINS:
        assert abs(now["10"][t]["err_pts"]) <= 0.5, now["10"][t]
    worst = _worst_train_error()
    assert worst <= 1.5, worst
    # the cycle share alone: the 1 ms train reads > 2 points low at every rate
    old = sim.replay(LOWRATE, {"time_split_ns": 0})
    for rate in ("1000", "100", "10"):
        assert old[rate]["burst_1_5"]["err_pts"] < -2.0, (rate, old[rate]["burst_1_5"])
        assert abs(now[rate]["burst_1_5"]["err_pts"]) < abs(old[rate]["burst_1_5"]["err_pts"]) - 0.5
    # the time split alone: the r5l 0.2 ms train reads ≈ 2 points high
    assert _worst_train_error({"time_split_weight": 1.0}) > worst + 0.5
    # the blend where READ-only intervals among the kernels just measured the gaps' clock:
    # the 1 kHz 1 ms trains read up to 0.5 points lower
    fresh, stale = sim.replay(LOWRATE), sim.replay(LOWRATE, {"gap_clock_fresh_ns": 0})
    assert fresh["1000"]["burst_1_5"]["err_pts"] > stale["1000"]["burst_1_5"]["err_pts"] + 0.3, (fresh, stale)
    for rate in ("100", "10"):  # no READ-only interval inside a train at these rates
        assert fresh[rate]["burst_1_5"]["err_pts"] == stale[rate]["burst_1_5"]["err_pts"]


@pytest.mark.parametrize("override, load, rate", [
    ({"cpc_full_frac": 0.97}, "gemm", "8000"),         # r4b's threshold: a GEMM stream read 3 points low
    ({"quiet_active_frac": 0.005}, "burst_1_5", "8000"),  # learned only on the cheapest READs: trains read high
])
def test_a_rejected_threshold_breaks_the_replay(override, load, rate):
    r = sim.replay(DUMP, override)[rate][load]
    assert abs(r["err_pts"]) > 1.0, (override, r)


def test_replay_is_the_samplers_code(N):
    """The replay tool has no model of its own: it calls the bound C++ class, whose
    parameters are the sampler's."""
    p = N.sampler_estimator_params()
    assert p.cpc_full_frac == pytest.approx(0.90) and p.quiet_active_frac == pytest.approx(0.02)
    assert p.read_overlap_ns == 400000 and p.clock_split_ns == 400000 and p.time_split_ns == 400000
    assert p.read_only_bills_zero is True
    assert p.time_split_weight == pytest.approx(0.75) and p.gap_clock_fresh_ns == 10_000_000
    assert p.cp_only_min == pytest.approx(0.3) and p.num_simds == 1024
    src = open(os.path.join(REPO, "tools", "util_estimator_sim.py")).read()
    assert "DispatchEstimator" in src and "0.95 *" not in src  # no re-implemented EWMA


def test_estimator_learns_the_read_cost_and_goes_quiet(N):
    """Synthetic drains: 2.4 GHz, a 15 µs READ every 125 µs on an idle GPU, then a
    kernel.  The READ-only intervals teach the READ cost and, after the 5 ms hold, the
    quiet state; a busy interval counts whole and ends quiet."""
    p = N.sampler_estimator_params()
    e = N.DispatchEstimator()
    e.restart(0)
    clk_per_ns, t, cnt, spi, cpc = 2.4, 0, 0, 0, 0
    for i in range(80):  # 10 ms idle
        t += 125_000
        cnt += int(125_000 * clk_per_ns)
        cpc += int(15_000 * clk_per_ns)
        spi += 100
        s = e.feed(p, t, cnt, spi, cpc, mfma=0)
        assert s.dispatch_s < 1e-6
    assert e.cpc_read_us == pytest.approx(15.0, rel=0.01) and s.quiet
    t += 125_000
    cnt += int(125_000 * clk_per_ns)
    cpc += int(125_000 * clk_per_ns)
    spi += int(120_000 * clk_per_ns)
    s = e.feed(p, t, cnt, spi, cpc, mfma=10**9)
    assert s.dispatch_s == pytest.approx(125e-6) and not s.quiet
    assert e.clk_busy_hz == pytest.approx(2.4e9, rel=1e-3)


# ---- UtilBiller -------------------------------------------------------------------

def _simulate(N, hz, busy_of_t, secs=20.0, fw_period=0.020, drain_jitter=0.3, seed=1, fw_scale=1.0,
              max_carry=None, extrapolate=True):
    """The PMFW thread at min(hz, 100) reading a table quantised to fw_period; counter
    drains at hz with jittered host times, the counter integral exact at each drain.
    Returns (billed total, biller, [(firmware t, cumulative billed)])."""
    rnd = random.Random(seed)
    pmfw_rate = min(hz, 100.0)
    drain_t, t = [], 0.0
    while t < secs + 1:
        drain_t.append(t + rnd.uniform(0, drain_jitter / hz))
        t += 1.0 / hz
    b = N.UtilBiller()
    fresh = 3.0 / min(hz, 100.0) + 0.05
    billed, trace, last_fw, k = 0.0, [], None, 0
    t = last_t = 0.0
    while t < secs:
        t += 1.0 / pmfw_rate
        while k + 1 < len(drain_t) and drain_t[k + 1] <= t:
            k += 1
        fw = math.floor(t * fw_scale / fw_period) * fw_period
        dt = fw - last_fw if last_fw is not None else 0.0
        if last_fw is not None and dt <= 0:
            continue  # same table: not a distinct sample
        last_fw = fw
        share = 0.0
        if extrapolate and k > 0:
            share = (busy_of_t(drain_t[k]) - busy_of_t(drain_t[k - 1])) / (drain_t[k] - drain_t[k - 1])
        dgfx = min(dt, busy_of_t(t) - busy_of_t(last_t))  # the PMFW's busy of the interval
        last_t = t
        got, from_c = b.bill(dt, dgfx, True, 1, busy_of_t(drain_t[k]), max_carry or fresh, True, share,
                             t - drain_t[k], k)
        if dt > 0:
            assert from_c and got <= dt + 1e-12
            billed += got
        trace.append((fw, billed))
    return billed, b, trace


def _worst_window(trace, busy_of_fw, win=5.0):
    """Largest |billed − truth| share over every window of `win` firmware seconds."""
    worst = 0.0
    for i, (f0, b0) in enumerate(trace):
        for f1, b1 in trace[i + 1:]:
            if f1 - f0 >= win:
                worst = max(worst, abs((b1 - b0) - (busy_of_fw(f1) - busy_of_fw(f0))) / (f1 - f0))
                break
    return worst


def SQ(t: float) -> float:
    """∫ busy of a 50 % square wave of period 0.37 s (floor and remainder from one division)."""
    n = math.floor(t / 0.37)
    return n * 0.185 + min(max(t - n * 0.37, 0.0), 0.185)


@pytest.mark.parametrize("hz", [10, 25, 50, 100, 1000, 8000])
def test_biller_is_lossless_when_drains_alias_with_pmfw_intervals(N, hz):
    billed, b, trace = _simulate(N, hz, lambda t: t)  # saturated: busy integral = host time
    assert billed >= 0.99 * 20.0, billed
    assert _worst_window(trace, lambda f: f) < 0.01  # any 5 s window: ≥ 99 %
    assert b.dropped_s == 0.0
    billed, b, trace = _simulate(N, hz, SQ)
    assert billed == pytest.approx(SQ(20.0), abs=0.1), billed
    # A 5 s window's edges each sit within one drain period of the integral's last known
    # point: a load that flips every 185 ms is billed within that, and 50 ± 1 from 50 Hz.
    assert _worst_window(trace, SQ) < 2 / (5 * hz) + 0.005


@pytest.mark.parametrize("hz", [10, 100])
def test_run_on_guess_stops_with_the_load(N, hz):
    """A saturated 3 s load, then idle: the guess that runs the last drain on to each
    PMFW sample is bounded by that interval's PMFW busy, so nothing is billed past the
    load's end (r5j, 10 Hz: the unbounded guess billed 3 s of load as 3.04 s, for good —
    a counter cannot take it back)."""
    busy = lambda t: min(max(t - 1.0, 0.0), 3.0)  # noqa: E731
    billed, b, trace = _simulate(N, hz, busy, secs=8.0, drain_jitter=0.0)
    assert billed == pytest.approx(3.0, abs=0.005), billed
    assert b.carry_s == pytest.approx(0.0, abs=1e-6)
    # and the guess still keeps the billed integral current while the load runs
    mid = [bl for fw, bl in trace if 2.0 <= fw <= 3.5]
    fws = [fw for fw, bl in trace if 2.0 <= fw <= 3.5]
    assert max(abs(bl - busy(fw)) for fw, bl in zip(fws, mid)) < 1.5 / hz + 0.02


def test_clipping_each_interval_loses_busy_time(N):
    """The round-4 rule — an interval takes at most dt of counter busy, the excess is
    dropped — is the cap 0 here: at 10-100 Hz it loses 3-6 % of a saturated GPU."""
    for hz in (10, 25, 50):
        billed, b, _ = _simulate(N, hz, lambda t: t, max_carry=1e-12, extrapolate=False)
        assert billed < 0.97 * 20.0 and b.dropped_s > 0.5, (hz, billed)


def test_biller_caps_the_carry_when_the_firmware_clock_runs_slow(N):
    """A firmware clock 2 % slower than the host's hands a saturated GPU's counter
    integral more busy than firmware time: bill 100 %, bank no backlog beyond the cap."""
    billed, b, _ = _simulate(N, 100, lambda t: t, fw_scale=0.98, max_carry=0.08)
    assert b.carry_s <= 0.08 + 1e-9 and b.dropped_s > 0.2
    assert billed == pytest.approx(0.98 * 20.0, abs=0.05)


def test_biller_falls_back_to_pmfw_and_drops_the_carry_on_an_epoch_change(N):
    b = N.UtilBiller()
    assert b.bill(0.02, 0.02, True, 1, 0.0, 1.0) == (0.02, False)      # no previous view: PMFW
    assert b.bill(0.02, 0.02, True, 1, 0.05, 1.0) == (0.02, True)      # 0.05 in, 0.02 billed
    assert b.carry_s == pytest.approx(0.03)
    got, from_c = b.bill(0.02, 0.015, True, 2, 0.06, 1.0)              # counters restarted
    assert (got, from_c) == (0.015, False) and b.carry_s == 0
    got, from_c = b.bill(0.02, 0.02, False, 2, 0.07, 1.0)              # counter tier not fresh
    assert (got, from_c) == (0.02, False)
    assert b.bill(0.02, 0.0, True, 2, 0.08, 1.0) == (0.0, False)       # first interval after: PMFW again
    assert b.bill(0.02, 0.0, True, 2, 0.09, 1.0)[1] is True


def test_committed_replay_summary_matches(shipped):
    """profiles/r6/estimator_replay*.json are this replay's output, committed: the numbers
    README / BASELINE cite are the current code's (r6: READ-cost learning gated at 2 × the
    learned cost moved one row, r4f 1 kHz 1 ms / 5 ms, from −0.23 to +0.08; the time-split
    weight 0.6 → 0.7 → 0.75 moved the long-interval rows by ≤ 0.4, then ≤ 0.21)."""
    for path, res in ((os.path.join(REPO, "profiles", "r6", "estimator_replay.json"), shipped),
                      (os.path.join(REPO, "profiles", "r6", "estimator_replay_lowrate.json"), sim.replay(LOWRATE)),
                      (os.path.join(REPO, "profiles", "r6", "estimator_replay_r5l.json"), sim.replay(LOWRATE_R5L))):
        rec = json.load(open(path))
        for rate, rows in rec.items():
            for load, r in rows.items():
                if isinstance(r, dict):
                    assert res[rate][load]["err_pts"] == pytest.approx(r["err_pts"], abs=0.02), (path, rate, load)


def test_time_split_never_bills_a_deep_idle_stretch_as_busy(N):
    """A 10 ms interval (the 100 Hz tier) with one 50 µs kernel, its idle rest at 1.5 GHz
    — a GPU left quiet long enough to drop below the 2.4 GHz idle clock it learned
    between kernels.  The time split alone would call 37 % of the interval busy (its
    idle cycles at 2.4 GHz fill only 63 % of it); bounded to busy clocks ≥ 0.67 × the
    idle clock it stays within 1 point of the kernel's 0.5 %."""
    p = N.sampler_estimator_params()
    e = N.DispatchEstimator()
    e.restart(0)
    t, cnt, cpc, spi = 0, 0, 0, 0
    for _ in range(20):  # READ-only intervals between kernels teach the 2.4 GHz idle clock
        t += 10_000_000
        cnt += int(10_000_000 * 2.4)
        cpc += int(16_000 * 2.4)
        spi += 2000
        e.feed(p, t, cnt, spi, cpc, mfma=0)
    assert e.clk_idle_hz == pytest.approx(2.4e9, rel=0.01)
    busy_cyc = int(50_000 * 2.1)
    t += 10_000_000
    cnt += busy_cyc + int((10_000_000 - 50_000) * 1.5)
    cpc += busy_cyc + int(16_000 * 1.5)
    spi += busy_cyc
    s = e.feed(p, t, cnt, spi, cpc, mfma=10**6)
    assert s.dispatch_s / 0.010 < 0.015, s.dispatch_s


# ---- UtilBiller properties (hypothesis) ------------------------------------------

from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=60, deadline=None)
@given(hz=st.sampled_from([10.0, 25.0, 50.0, 100.0, 1000.0]),
       jitter=st.floats(min_value=0.0, max_value=0.9),
       duty=st.floats(min_value=0.0, max_value=1.0),
       period=st.floats(min_value=0.01, max_value=0.5),
       fw_period=st.sampled_from([0.01, 0.02]),
       seed=st.integers(0, 10_000))
def test_biller_properties(N, hz, jitter, duty, period, fw_period, seed):
    """For any drain rate and jitter, square-wave load and firmware cadence: every PMFW
    interval bills within [0, dt]; the carry stays within ± the cap; and over the run the
    billed total equals the counter integral at the last drain, give or take the carry
    and the run-on guess (never more than one freshness window)."""
    busy = lambda t: math.floor(t / period) * period * duty + min(max(t - math.floor(t / period) * period, 0.0),  # noqa: E731
                                                                   period * duty)
    rnd = random.Random(seed)
    secs = 6.0
    drain_t, t = [], 0.0
    while t < secs + 1:
        drain_t.append(t + rnd.uniform(0, jitter / hz))
        t += 1.0 / hz
    b = N.UtilBiller()
    cap = 3.0 / min(hz, 100.0) + 0.05
    pmfw_rate = min(hz, 100.0)
    billed, last_fw, last_t, k, t = 0.0, None, 0.0, 0, 0.0
    while t < secs:
        t += 1.0 / pmfw_rate
        while k + 1 < len(drain_t) and drain_t[k + 1] <= t:
            k += 1
        fw = math.floor(t / fw_period) * fw_period
        dt = fw - last_fw if last_fw is not None else 0.0
        if last_fw is not None and dt <= 0:
            continue
        last_fw = fw
        share = (busy(drain_t[k]) - busy(drain_t[k - 1])) / (drain_t[k] - drain_t[k - 1]) if k > 0 else 0.0
        dgfx = min(dt, busy(t) - busy(last_t))
        last_t = t
        got, _ = b.bill(dt, dgfx, True, 1, busy(drain_t[k]), cap, True, share, t - drain_t[k], k)
        assert -1e-12 <= got <= dt + 1e-12
        assert abs(b.carry_s) <= cap + 1e-9
        billed += got
    truth = busy(drain_t[k])
    assert b.dropped_s == pytest.approx(0.0, abs=1e-9)
    assert abs(billed - truth) <= cap + 1e-9, (billed, truth, b.carry_s)


def _synthetic_rows(busy_at, secs, hz, read_s=20e-6, f=2.1e9, t0=10.0, dither=0.25, seed=7):
    """Drains of a GPU at one clock: the CP and SPI busy while busy_at(t), plus each READ's
    own CP time (busy_at is a square wave).  The drains sit on the sampler's dithered tick
    grid (SamplerConfig::tick_dither: an offset random-walking ± dither of a period per
    tick, reflected into ± half a period), so a load whose period is a multiple of the tick
    does not phase-lock with it.  At 8 kHz every READ adds its CP time (r6a); at ≥ 400 µs
    intervals a READ that lands during a kernel adds none (r4f's 1 kHz raw READs, sampler.h
    kReadOverlapNs) — the READ lands at the drain."""
    rnd = random.Random(seed)
    rows, cnt, spi, cpc, t, off, k = [], 0.0, 0.0, 0.0, 0.0, 0.0, 0
    dt, step = 1.0 / hz, 5e-6
    while t < secs:
        rows.append([t0 + t, int(cnt), int(spi), int(cpc), -1, 1])
        k += 1
        off += rnd.uniform(-1.0, 1.0) * dither * dt
        if abs(off) > 0.5 * dt:  # reflected at ± half a period
            off = math.copysign(dt, off) - off
        nxt = k * dt + off
        s = t
        while s < nxt - 1e-12:
            b = busy_at(s)
            cnt += f * step
            if b:
                spi += f * step
                cpc += f * step
            s += step
        if not (nxt - t >= 400e-6 and busy_at(nxt)):
            cpc += read_s * f
        t = nxt
    return rows


@settings(max_examples=12, deadline=None)
@given(hz=st.sampled_from([8000.0, 1000.0]),
       period=st.floats(min_value=0.002, max_value=0.02),
       duty=st.floats(min_value=0.1, max_value=0.9))
def test_dispatch_estimator_reads_a_square_wave_at_one_clock(N, hz, period, duty):
    """At one shader clock (no power cap) the dispatch integral of any square-wave load is
    its duty within 1.5 points, at 8 kHz and 1 kHz, once the READ cost is learned on idle
    READs (sampler parameters, dithered ticks).  On a fixed tick grid a 2.5 ms period
    phase-locks with 1 ms intervals, and the kernel edges keep landing in intervals ≥ 90 %
    busy that count whole (cpc_full_frac): +1.74 points — the lock that tick_dither
    exists to break (tools/phase_probe.py); with it the worst of 200 draws is +0.98."""
    p = N.sampler_estimator_params()
    e = N.DispatchEstimator()
    e.replay(p, _synthetic_rows(lambda t: False, 0.1, hz, t0=1.0))
    rows = _synthetic_rows(lambda t: (t % period) < duty * period, 0.3, hz)
    e.invalidate(int(rows[0][0] * 1e9))
    r = e.replay(p, rows)
    truth = sum(min(max(rows[-1][0] - 10.0 - k * period, 0.0), duty * period)
                for k in range(int((rows[-1][0] - 10.0) / period) + 2)) / (rows[-1][0] - 10.0)
    assert 100 * r["dispatch_s"] / r["span_s"] == pytest.approx(100 * truth, abs=1.5), (r, truth)


@settings(max_examples=25, deadline=None)
@given(hz=st.sampled_from([8000.0, 1000.0, 100.0]),
       lo=st.floats(min_value=0.86, max_value=0.90),
       hi=st.floats(min_value=0.90, max_value=0.95),
       seed=st.integers(0, 10_000))
def test_a_saturated_stream_never_leaves_the_full_read_rate(N, hz, lo, hi, seed):
    """back-to-back MFMA kernels keep the CP busy every interval while
    their SPI share wanders 89.6-94.8 % from box to box (r3h, r3j, r4d, r5, GPUTEST_r05).
    Round 5's SPI-keyed gap rate put 28 % of such a stream on a slower READ rate at a 0.9
    threshold; the only rate machines left key on "no wave at all" (quiet) and on CP busy
    without waves (dispatch-bound, cp_only_min 0.3), so wherever the per-interval SPI share
    wanders in [0.86, 0.95] the stream keeps every tick and bills whole."""
    p = N.sampler_estimator_params()
    e = N.DispatchEstimator()
    e.restart(0)
    rnd = random.Random(seed)
    f, t, cnt, spi, cpc, mfma = 2.1, 0, 0, 0, 0, 0
    period = int(1e9 / hz)
    busy = span = 0.0
    for _ in range(int(min(hz, 1000) * 2)):  # 2 s at ≤ 1 kHz, 0.25 s at 8 kHz
        t += period
        clk = int(period * f)
        cnt += clk
        cpc += int(clk * rnd.uniform(0.97, 1.0))
        spi += int(clk * rnd.uniform(lo, hi))
        mfma += int(clk * 1024 * 0.8)
        s = e.feed(p, t, cnt, spi, cpc, mfma=mfma)
        assert not (s.quiet or s.dbound or s.quiet_interval or s.dbound_interval), (lo, hi, s.cp_only_share)
        busy += s.dispatch_s
        span += s.span_s
    assert busy / span == pytest.approx(1.0, abs=0.02)
    assert not hasattr(s, "gap") and not hasattr(p, "busy_min")


def test_a_microsecond_kernel_stream_is_dispatch_bound_after_the_hold(N):
    """The rate machine that replaced it: CP busy ≈100 % with waves ≈41 % of the clocks (a
    HIP graph of 1.7 µs copies on MI355X, profiles/r4/ r4b) turns dispatch-bound once the
    10 ms hold has passed, and a long kernel ends it on its first interval."""
    p = N.sampler_estimator_params()
    e = N.DispatchEstimator()
    e.restart(0)
    t = cnt = spi = cpc = 0
    period, f = 125_000, 2.4
    states = []
    for i in range(160):  # 20 ms at 8 kHz
        t += period
        clk = int(period * f)
        cnt += clk
        cpc += clk
        spi += int(0.41 * clk)
        states.append(e.feed(p, t, cnt, spi, cpc, mfma=0).dbound)
    assert not any(states[:79]) and all(states[81:]), states.index(True)
    t += period
    cnt += int(period * f)
    cpc += int(period * f)
    spi += int(0.95 * period * f)
    assert not e.feed(p, t, cnt, spi, cpc, mfma=10**9).dbound


def test_carry_is_dropped_when_the_gpu_changes_hands(N):
    """container_gpu_busy_seconds_total counts per allocation, so busy still
    carried when a pod's allocation ends belongs to that pod, not the next one.  The
    exporter drops it when the owner set changes (Exporter::set_device_owners →
    Sampler::drop_util_carry), and the carry is capped at MAX_UTIL_CARRY_S whatever the
    freshness window (pmc_idle_hz 0.01 makes that window 300 s)."""
    b = N.UtilBiller()
    b.bill(0.02, 0.02, True, 1, 0.0, 1.0)
    b.bill(0.02, 0.02, True, 1, 0.05, 1.0)            # two drains' worth in one interval: 0.03 carried
    assert b.carry_s == pytest.approx(0.03)
    b.drop_carry()
    assert b.carry_s == 0 and b.dropped_s == pytest.approx(0.03)
    got, from_c = b.bill(0.02, 0.0, True, 1, 0.05, 1.0)  # the new owner's idle interval bills nothing
    assert from_c and got == 0.0
    assert N.MAX_UTIL_CARRY_S == pytest.approx(1.0)


def test_reallocation_starts_the_new_pods_counter_at_zero(mock_exporter):
    """A saturated mock GPU handed from pod a to pod b: b's container_gpu_busy_seconds_total
    starts at 0 and never bills more than the time since its allocation (the old owner's
    carry is dropped, not billed to b)."""
    from kube_gpu_stats_amd.utils.scrape import parse_text

    ex = mock_exporter(n_gpus=1, hz=10, pmc_source="mock", proc_every=0, link_every=0,
                       mock={"util_base": 100, "util_amp": 0})
    ex.set_device_owners(0, [{"pod": "a", "namespace": "ns", "container": "c"}])
    import time as _t

    _t.sleep(1.2)
    d0 = ex.integrals(0)["util_dropped_seconds"]
    ex.set_device_owners(0, [{"pod": "a", "namespace": "ns", "container": "c"}])  # same owner: nothing dropped
    _t.sleep(0.3)
    t0 = _t.monotonic()
    ex.set_device_owners(0, [{"pod": "b", "namespace": "ns", "container": "c"}])
    _t.sleep(1.0)
    m = parse_text(ex.render())
    el = _t.monotonic() - t0
    busy = {lb["pod_name"]: v for lb, v in m["container_gpu_busy_seconds_total"]}
    assert set(busy) == {"b"} and 0.5 < busy["b"] <= el + 0.02, (busy, el)
    assert ex.integrals(0)["util_dropped_seconds"] >= d0


HELDOUT = os.path.join(REPO, "profiles", "r6", "r6c", "cp_dump_irregular.json.gz")


def test_held_out_irregular_loads_replay_within_one_and_a_half_points():
    """out of sample.  Every constant of the estimator was fitted on the
    r4f / r5b / r5l dumps of strictly periodic single-stream trains.  The r6c dump
    (recorded on MI355X in the exporter's READ mode at 8 kHz, 1 kHz, 100 Hz and 10 Hz)
    holds loads none of them saw — seeded random 5 µs - 20 ms MFMA kernels with random
    gaps on one and on two streams, and a bf16 decoder training step (duty: the union of
    its kernels' intervals, PyTorch profiler) — and replays within ±1.5 points of the
    duty at every rate with the shipped parameters, which test_replay_is_the_samplers_code
    pins, so nothing here was retuned to fit it."""
    res = sim.replay(HELDOUT)
    assert set(res) == {"8000", "1000", "100", "10"}
    for rate, rows in res.items():
        assert abs(rows["idle"]["err_pts"]) <= 0.05, (rate, rows["idle"])
        for load in ("random_kernels", "two_stream_random", "train_step"):
            r = rows[load]
            assert 20 < r["duty_gpu_pct"] < 90, (rate, load, r)
            assert abs(r["err_pts"]) <= 1.5, (rate, load, r)
    rec = json.load(open(os.path.join(REPO, "profiles", "r6", "estimator_replay_irregular_heldout.json")))
    for rate, rows in rec.items():
        for load, r in rows.items():
            if isinstance(r, dict):
                assert res[rate][load]["err_pts"] == pytest.approx(r["err_pts"], abs=0.02), (rate, load)


LIVE_10HZ = os.path.join(REPO, "profiles", "r6", "r6e", "gpu_tests", "irregular_raw_10hz.json")


def test_live_ten_hertz_drains_of_random_kernels_replay_within_one_point():
    """The tuning capture of round 6's time-split weight: the exporter's own drains at the
    DaemonSet's 10 Hz under seeded random MFMA kernels (one and two streams), recorded by
    tests/test_gpu.py::test_irregular_loads_bill_their_duty on MI355X (r6e), the kernels'
    event-timed intervals on the same clock.  At the old weight 0.6 the one-stream load read
    −1.53 (live −1.46); at 0.7 −0.99, at 0.75 (six more boxes' phase U) −0.72 — and the
    held-out r6c dump, not used for the choice, stays within 1.5 (test_held_out_irregular_loads_*)."""
    now = sim.replay_exporter_raw(LIVE_10HZ)
    for name, r in now.items():
        assert r["intervals"] >= 40 and abs(r["err_pts"]) <= 1.0, (name, r)
    old = sim.replay_exporter_raw(LIVE_10HZ, {"time_split_weight": 0.6})
    assert old["10/random_kernels"]["err_pts"] < -1.4, old["10/random_kernels"]
