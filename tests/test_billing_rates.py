"""container_gpu_busy_seconds_total bills the counter tier's busy integral without loss
at every counter rate the exporter ships with.

The reference bills each pod the mean of container_gpu_sm_util over the day
(/root/reference/gpu_util_stats/gpu_util_stats.py:159 → :62-94); the fixed report bills
100·rate(container_gpu_busy_seconds_total).  Round 4 clipped each PMFW interval's
counter increment to the interval, so at the DaemonSet's --hz=10 (two drains in one
20 ms-quantised interval, none in the next) a saturated mock GPU billed 75-78 %.  Here
the whole sampler runs on the mock (default fw_period_s 0.020, mock counters) at
10 / 25 / 50 / 100 / 1000 / 8000 Hz, all rates side by side.
"""
from __future__ import annotations

import time

import pytest

from kube_gpu_stats_amd.utils.scrape import parse_text

RATES = (10, 25, 50, 100, 1000, 8000)
WINDOW_S = 6.0


def _sweep(N, mock: dict) -> dict:
    exs = {}
    for hz in RATES:
        ex = N.Exporter({"backend": "mock", "mock": {"n_gpus": 1, **mock}, "hz": hz, "port": 0, "node_name": "n",
                         "pin_numa": False, "pmc_source": "mock"})
        ex.set_device_owners(0, [{"pod": "p", "namespace": "ns", "container": "c"}])
        ex.start()
        exs[hz] = ex
    try:
        time.sleep(1.0)
        one = lambda m, f: m[f][0][1]  # noqa: E731
        m0 = {hz: parse_text(ex.render()) for hz, ex in exs.items()}
        i0 = {hz: ex.integrals(0) for hz, ex in exs.items()}
        time.sleep(WINDOW_S)
        m1 = {hz: parse_text(ex.render()) for hz, ex in exs.items()}
        i1 = {hz: ex.integrals(0) for hz, ex in exs.items()}
        out = {}
        for hz in RATES:
            fw = i1[hz]["sampled_seconds"] - i0[hz]["sampled_seconds"]
            d = lambda f: one(m1[hz], f) - one(m0[hz], f)  # noqa: E731,B023
            out[hz] = {"billed": (i1[hz]["util_seconds"] - i0[hz]["util_seconds"]) / fw,
                       "metric": d("container_gpu_busy_seconds_total") / d("kgs_sampled_seconds_total"),
                       # the dispatch integral over the span between the drains it last took
                       "dispatch": (i1[hz]["dispatch_seconds"] - i0[hz]["dispatch_seconds"])
                       / ((i1[hz]["pmc_last_ns"] - i0[hz]["pmc_last_ns"]) * 1e-9),
                       "from_counters": (i1[hz]["util_counter_seconds"] - i0[hz]["util_counter_seconds"]) / fw,
                       "dropped": i1[hz]["util_dropped_seconds"]}
        return out
    finally:
        for ex in exs.values():
            ex.stop()


@pytest.mark.slow
def test_saturated_gpu_bills_at_least_99_percent_at_every_rate(N):
    r = _sweep(N, {"util_base": 100, "util_amp": 0})
    for hz, x in r.items():
        assert x["billed"] >= 0.99 and x["metric"] >= 0.99, (hz, x)
        # the counter integral, all of it
        assert x["billed"] == pytest.approx(x["dispatch"], abs=0.01), (hz, x)
        assert x["from_counters"] > 0.99 and x["dropped"] < 0.05, (hz, x)


@pytest.mark.slow
def test_half_duty_square_bills_fifty_at_every_rate(N):
    # a period incommensurate with every drain / PMFW rate: no aliasing luck either way
    r = _sweep(N, {"square_duty": 0.5, "util_base": 50, "util_amp": 50, "util_period_s": 0.13})
    for hz, x in r.items():
        assert 100 * x["billed"] == pytest.approx(50, abs=1), (hz, x)
        assert 100 * x["metric"] == pytest.approx(50, abs=1), (hz, x)
        assert x["billed"] == pytest.approx(x["dispatch"], abs=0.01), (hz, x)
