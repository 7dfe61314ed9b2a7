"""Phase K — samples/s delivered while each load component runs alone."""
from __future__ import annotations

import time

from kube_gpu_stats_amd.parallel import dist as D

from .common import scrape_at
from .exporter import Rates


def component_rates(ctx, load, exp, a) -> dict:
    """Phase K (untimed) — samples/s the exporter delivers at the primary rate while
    each load component runs alone for --component-s: the long MFMA kernel, the HBM
    triads, the dispatch-bound tiny-kernel graph (the headline's blend, split)."""
    if a.component_s <= 0:
        return {}
    names = getattr(load, "component_names", lambda: [])()
    if not names:
        return {}
    out: dict = {}
    for name in names:
        D.barrier(ctx)
        load.sync()
        before, w0 = scrape_at(exp.sc) if exp is not None else ({}, 0.0)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < a.component_s:
            load.run_component(name)
            k += 1
            if k % 4 == 0:
                load.sync()
        load.sync()
        D.barrier(ctx)
        if exp is None:
            continue
        after, w1 = scrape_at(exp.sc)
        r = Rates()
        r.add(before, after, w1 - w0)
        pg, src = r.per_gpu(exp.ready.get("pmc", "none") != "none")
        out[name] = {"samples_per_sec_per_gpu": {g: round(v, 1) for g, v in pg.items()}, "sample_source": src,
                     "launches": k, "seconds": round(w1 - w0, 3)}
    return out
