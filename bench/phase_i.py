"""Phase I — interleaved rounds of paused / released / sampling blocks: the paired GPU-time overhead."""
from __future__ import annotations

import math

from kube_gpu_stats_amd.parallel import dist as D
from kube_gpu_stats_amd.utils.scrape import Scraper

from .common import RELEASED, cond_label, mean_ci95, progress, scrape_at, t975, timed_block
from .exporter import PmfwProbe, Rates


def order_design(conds: list[float], rounds: int) -> list[tuple]:
    """Every permutation of the conditions in turn (3 conditions: all 6 orders), so
    each condition sits in each block position equally often and a block-position
    effect cannot pose as a sampling cost."""
    import itertools

    perms = list(itertools.permutations(conds))
    return [perms[r % len(perms)] for r in range(rounds)]


def position_adjusted(rows: list[dict], conds: list[float], orders: list[tuple]) -> dict:
    """Least squares on log(block seconds) = round + condition + position effects;
    the condition effects are the position-adjusted overheads (exp(b) − 1, with a
    95 % interval from the residual variance)."""
    import numpy as np

    R, C = len(rows), len(conds)
    P = C
    y, X = [], []
    for r, (row, order) in enumerate(zip(rows, orders)):
        for pos, c in enumerate(order):
            x = np.zeros(R + (C - 1) + (P - 1))
            x[r] = 1.0
            ci = conds.index(c)
            if ci > 0:
                x[R + ci - 1] = 1.0
            if pos > 0:
                x[R + C - 1 + pos - 1] = 1.0
            X.append(x)
            y.append(math.log(row[c]))
    X, y = np.array(X), np.array(y)
    beta, *_ = np.linalg.lstsq(X, y, rcond=None)
    resid = y - X @ beta
    dof = len(y) - np.linalg.matrix_rank(X)
    out: dict = {"model": "log t = round + condition + position", "dof": int(dof)}
    if dof <= 0:
        return out
    s2 = float(resid @ resid) / dof
    cov = s2 * np.linalg.pinv(X.T @ X)
    for ci in range(1, C):
        k = R + ci - 1
        b, se = float(beta[k]), math.sqrt(max(0.0, float(cov[k, k])))
        out[cond_label(conds[ci])] = {"overhead_pct": 100 * (math.exp(b) - 1),
                                 "overhead_ci95_pct": 100 * math.exp(b) * t975(dof) * se}
    out["position_effect_pct"] = {str(p): 100 * (math.exp(float(beta[R + C - 1 + p - 1])) - 1) for p in range(1, P)}
    return out


def interleaved(ctx, load, exp, a, hzs: list[float]) -> dict:
    """Rounds of blocks: exporter paused (0), released (--released: also the counter
    session STOPped and the reader's READ queue destroyed, re-acquired after the
    block) and sampling at each rate in ``hzs``, the block order cycling through every
    permutation of the conditions (order_design).  Paused means the sampler threads
    are stopped — no PMFW read, no counter READ, no scrape — while the process and its
    counter session stay up, so the paired difference is the cost of sampling +
    scraping; released vs paused is the cost of a programmed perfmon session and a
    mapped READ queue alone, with CIs like every tier.

    Per block and rank: its own GPU-work time, the all-rank (MAX) time, the GPU time
    of each load component (HIP events: MFMA kernel, triads, tiny-kernel graph,
    all-reduce) and the block's power from the rank's own PMFW table.  The headline
    overhead is the paired MAX-time ratio; per rank and per component the same pairing
    on that rank's / component's own times."""
    if a.rounds <= 0:
        return {}
    conds = [0.0] + ([RELEASED] if a.released else []) + list(hzs)  # the same on every rank
    orders = order_design(conds, a.rounds)
    released_now = False
    probe = None if a.mock else PmfwProbe(load.pci_bdf(ctx.local_rank))
    rates = {h: Rates() for h in hzs}
    lat: dict[float, list[float]] = {h: [] for h in hzs}
    paused_reads = 0.0
    local: list[dict] = []  # per round: {cond: {"own", "all", "comp", "power"}}
    for ri, order in enumerate(orders):
        blk: dict = {}
        if ri % 8 == 0:
            progress(ctx, f"phase I round {ri + 1}/{len(orders)}")
        for c in order:
            sc = None
            before: dict = {}
            w0 = 0.0
            if exp is not None:
                if released_now and c != RELEASED:  # leave "released": threads up, counters re-acquired
                    exp.resume()
                    exp.acquire()
                    released_now = False
                if c == 0:
                    exp.pause()
                elif c == RELEASED:
                    exp.resume()
                    if not released_now:
                        exp.release(drop_queue=True)
                        released_now = True
                    exp.pause()
                else:
                    exp.set_rate(c)
                    exp.resume()
                if c > 0:
                    sc = Scraper("127.0.0.1", exp.port).start(a.scrape_hz)
                before, w0 = scrape_at(exp.sc)
            p0 = probe.read() if probe is not None else None
            load.components_start()
            own, dt = timed_block(ctx, load, a.block_steps)
            comp = load.components_end()
            pw = PmfwProbe.delta(p0, probe.read() if probe is not None else None)
            if exp is not None:
                if sc is not None:
                    sc.stop()
                after, w1 = scrape_at(exp.sc)
                win = w1 - w0
                if c > 0:
                    rates[c].add(before, after, win)
                    lat[c].extend(sc.latencies_s)
                elif c == 0:  # paused really means no reads
                    rb = {lb["gpu"]: v for lb, v in before.get("kgs_reads_total", [])}
                    paused_reads += sum(v - rb.get(g, 0.0) for g, v in
                                        ((lb["gpu"], v) for lb, v in after.get("kgs_reads_total", [])))
            blk[c] = {"own": own, "all": dt, "comp": comp, "power": pw}
        local.append(blk)
    if exp is not None:
        exp.resume()
        if released_now:
            exp.acquire()
        exp.set_rate(a.hz)
    ranks = D.all_gather_object(ctx, local)  # [rank][round][cond]
    rows = [{c: max(rk[r][c]["all"] for rk in ranks) for c in conds} for r in range(a.rounds)]
    out: dict = {"rounds": a.rounds, "block_steps": a.block_steps,
                 "order_design": {"kind": "all permutations in turn", "orders": [[cond_label(c) for c in o]
                                                                                for o in dict.fromkeys(orders)],
                                  "balanced": a.rounds % len(dict.fromkeys(orders)) == 0},
                 "paused_reads": paused_reads, "tiers": {}}
    for h in hzs:
        diffs = [100.0 * (row[h] / row[0.0] - 1.0) for row in rows]
        m, ci, sd = mean_ci95(diffs)
        srt = sorted(diffs)
        med = (srt[(len(srt) - 1) // 2] + srt[len(srt) // 2]) / 2 if srt else float("nan")
        tier = {"overhead_pct": m, "overhead_ci95_pct": ci, "overhead_sd_pct": sd,
                # robustness next to the mean: a few disturbed rounds (another tenant of the
                # box, a clock event) move the mean and its CI, not the median
                "overhead_median_pct": med,
                "overhead_per_round_pct": [round(d, 4) for d in diffs],
                "_rates": rates[h], "_lat": lat[h]}
        # per component (rank 0's GPU, and the mean of every rank's own estimate)
        names = sorted({n for rk in ranks for rd in rk for n in rd[h]["comp"]})
        by_comp: dict = {}
        for n in names:
            per_rank = []
            for rk in ranks:
                d = [100.0 * (rd[h]["comp"][n] / rd[0.0]["comp"][n] - 1.0) for rd in rk
                     if rd[0.0]["comp"].get(n, 0) > 0 and n in rd[h]["comp"]]
                per_rank.append(mean_ci95(d))
            m0, c0, _ = per_rank[0]
            share = sum(rd[0.0]["comp"].get(n, 0.0) for rd in ranks[0]) / max(
                1e-12, sum(rd[0.0]["own"] for rd in ranks[0]))
            by_comp[n] = {"overhead_pct": m0, "overhead_ci95_pct": c0, "share_of_block_time": round(share, 4)}
            if len(ranks) > 1:
                by_comp[n]["per_rank_overhead_pct"] = [round(x[0], 4) for x in per_rank]
        tier["overhead_by_component"] = by_comp
        if RELEASED in conds:
            # The same pairing against "released" (counter session STOPped, READ queue
            # destroyed, threads stopped): paused keeps a programmed session and its
            # queue, which shifts a dispatch-bound stream's power state (BENCH_r04:
            # µs-kernel graph −1.23 % at 100 Hz vs paused), so this is the neutral base
            # for the cost of sampling.
            vs_rel: dict = {}
            for n in names:
                d = [100.0 * (rd[h]["comp"][n] / rd[RELEASED]["comp"][n] - 1.0) for rd in ranks[0]
                     if rd[RELEASED]["comp"].get(n, 0) > 0 and n in rd[h]["comp"]]
                m_r, c_r, _ = mean_ci95(d)
                vs_rel[n] = {"overhead_pct": m_r, "overhead_ci95_pct": c_r}
            tier["overhead_by_component_vs_released"] = vs_rel
        # per rank: that rank's own work time, paired by round
        per_rank = []
        for k, rk in enumerate(ranks):
            m_k, c_k, _ = mean_ci95([100.0 * (rd[h]["own"] / rd[0.0]["own"] - 1.0) for rd in rk])
            per_rank.append({"rank": k, "overhead_pct": round(m_k, 4), "overhead_ci95_pct": round(c_k, 4)})
        tier["overhead_by_rank"] = per_rank
        out["tiers"][f"{h:g}"] = tier
    if RELEASED in conds:
        # Released vs paused: the cost of a STARTed perfmon session + a mapped READ
        # queue with nothing sampling; each rate vs released: everything the
        # counter tier costs, session and queue included.
        rel: dict = {}
        m, ci, _ = mean_ci95([100.0 * (row[0.0] / row[RELEASED] - 1.0) for row in rows])
        rel["paused_vs_released_pct"], rel["paused_vs_released_ci95_pct"] = m, ci
        for h in hzs:
            m, ci, _ = mean_ci95([100.0 * (row[h] / row[RELEASED] - 1.0) for row in rows])
            rel[f"{h:g}_vs_released_pct"], rel[f"{h:g}_vs_released_ci95_pct"] = m, ci
        out["released"] = rel
    out["block_seconds"] = [[cond_label(c), round(rows[r][c], 6)] for r, o in enumerate(orders) for c in o]
    # Block-position means (every condition pooled, and per condition): with the
    # permutation design each condition's mean covers every position equally.
    pos_all: dict[int, list[float]] = {}
    pos_c: dict[str, dict[int, list[float]]] = {}
    for r, o in enumerate(orders):
        for p, c in enumerate(o):
            pos_all.setdefault(p, []).append(rows[r][c])
            pos_c.setdefault(cond_label(c), {}).setdefault(p, []).append(rows[r][c])
    out["position_means"] = {"all": {str(p): round(sum(v) / len(v), 6) for p, v in sorted(pos_all.items())},
                             "by_condition": {c: {str(p): round(sum(v) / len(v), 6) for p, v in sorted(d.items())}
                                              for c, d in pos_c.items()}}
    try:
        out["position_adjusted"] = position_adjusted(rows, conds, orders)
    except Exception as e:  # noqa: BLE001 - report, never fail the bench on the side estimate
        out["position_adjusted"] = {"error": repr(e)}
    # Power state per condition of every rank's GPU (PMFW energy / PPT accumulators).
    power_by_rank = []
    for k, rk in enumerate(ranks):
        power: dict = {}
        for c in conds:
            pw = [rd[c]["power"] for rd in rk if rd[c]["power"]]
            if not pw:
                continue
            ws = [d["power_w"] for d in pw]
            ps = [d["ppt_pct"] for d in pw if "ppt_pct" in d]
            power[cond_label(c)] = {"blocks": len(ws), "power_w_mean": round(sum(ws) / len(ws), 2),
                                    "ppt_pct_mean": round(sum(ps) / len(ps), 3) if ps else None}
            paired = [(rd[c]["power"], rd[0.0]["power"]) for rd in rk if rd[c]["power"] and rd[0.0]["power"]]
            if c != 0 and paired:
                m, ci, _ = mean_ci95([x["power_w"] - y["power_w"] for x, y in paired])
                power[cond_label(c)]["power_w_vs_paused"] = round(m, 2)
                power[cond_label(c)]["power_w_vs_paused_ci95"] = round(ci, 2)
        power_by_rank.append(power)
    if any(power_by_rank):
        out["power"] = {"by_condition": power_by_rank[0], "by_rank": power_by_rank,
                        "note": "PMFW energy / PPT-residency accumulators read by each rank at its own GPU's block "
                                "edges ('0' = exporter paused)"}
    return out
