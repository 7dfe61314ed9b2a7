"""In-process fake Prometheus HTTP API (tests only).

Two kinds of answers:

* canned — exact query string → vector/matrix result (how SURVEY.md §4.2's
  golden harness drove the reference's five queries);
* evaluated — a tiny TSDB fed from exporter scrapes (``ingest``) that evaluates
  the query shapes the report layer issues for the utilisation series:
  ``avg|sum|max(<metric>) by (l1, l2, ...)``, over a bare metric, ``avg_over_time``,
  ``rate`` or ``increase`` of it,
  instant or ranged, with Prometheus' 5-minute staleness lookback.
"""
from __future__ import annotations

import json
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

LOOKBACK_S = 300.0
_AVG_BY = re.compile(r"^\s*(?:([0-9.]+)\s*\*\s*)?(avg|sum|max)\((.+)\)\s*by\s*\(([^)]*)\)\s*$")
_AGG = {"avg": lambda vs: sum(vs) / len(vs), "sum": sum, "max": max}
_AOT = re.compile(r"^\s*avg_over_time\(\s*([a-zA-Z_:][a-zA-Z0-9_:]*)\s*\[(\d+)([smh])\]\s*\)\s*$")
_RATE = re.compile(r"^\s*(rate|increase)\(\s*([a-zA-Z_:][a-zA-Z0-9_:]*)\s*\[(\d+)([smh])\]\s*\)\s*$")
_UNIT = {"s": 1, "m": 60, "h": 3600}


def extrapolated(pts: list[tuple[float, float]], start: float, end: float, is_rate: bool) -> float | None:
    """Prometheus' extrapolatedRate (promql/functions.go) for a counter over (start, end]."""
    if len(pts) < 2:
        return None
    result, prev = 0.0, pts[0][1]
    for _, v in pts[1:]:
        result += v - prev if v >= prev else v  # counter reset: count from 0
        prev = v
    t0, t1 = pts[0][0], pts[-1][0]
    sampled = t1 - t0
    if sampled <= 0:
        return None
    avg_gap = sampled / (len(pts) - 1)
    to_start, to_end = t0 - start, end - t1
    if result > 0 and pts[0][1] >= 0:  # a counter does not extrapolate below zero
        to_start = min(to_start, sampled * (pts[0][1] / result))
    thr = avg_gap * 1.1
    interval = sampled + (to_start if to_start < thr else avg_gap / 2) + (to_end if to_end < thr else avg_gap / 2)
    result *= interval / sampled
    return result / (end - start) if is_rate else result
_NAME = re.compile(r"^\s*([a-zA-Z_:][a-zA-Z0-9_:]*)\s*$")


class FakeProm:
    def __init__(self):
        self.canned_instant: dict[str, list] = {}
        self.canned_range: dict[str, list] = {}
        self.series: dict[str, dict[tuple, list[tuple[float, float]]]] = {}
        self.calls: list[tuple[str, dict]] = []
        self.via_proxy: list[bool] = []
        self._srv: ThreadingHTTPServer | None = None
        self._th: threading.Thread | None = None
        self.lock = threading.Lock()

    # ------------------------------------------------------------------ data
    def add_instant(self, query: str, result: list) -> None:
        self.canned_instant[query] = result

    def add_range(self, query: str, result: list) -> None:
        self.canned_range[query] = result

    def ingest(self, samples: dict[str, list[tuple[dict, float]]], ts: float, extra: dict | None = None) -> None:
        """Store a parsed scrape (utils.scrape.parse_text output) at time ``ts``."""
        with self.lock:
            for name, rows in samples.items():
                m = self.series.setdefault(name, {})
                for labels, v in rows:
                    lb = dict(labels)
                    if extra:
                        lb.update(extra)
                    m.setdefault(tuple(sorted(lb.items())), []).append((ts, v))

    # ------------------------------------------------------------------ evaluation
    def _inner(self, expr: str, t: float) -> list[tuple[dict, float]]:
        m = _RATE.match(expr)
        if m:
            fn, name, n, unit = m.group(1), m.group(2), int(m.group(3)), m.group(4)
            rng = n * _UNIT[unit]
            out = []
            for key, pts in self.series.get(name, {}).items():
                v = extrapolated([(ts, x) for ts, x in pts if t - rng < ts <= t], t - rng, t, fn == "rate")
                if v is not None:
                    out.append((dict(key), v))
            return out
        m = _AOT.match(expr)
        if m:
            name, n, unit = m.group(1), int(m.group(2)), m.group(3)
            rng = n * {"s": 1, "m": 60, "h": 3600}[unit]
            out = []
            for key, pts in self.series.get(name, {}).items():
                vs = [v for ts, v in pts if t - rng < ts <= t]
                if vs:
                    out.append((dict(key), sum(vs) / len(vs)))
            return out
        m = _NAME.match(expr)
        if m:
            out = []
            for key, pts in self.series.get(m.group(1), {}).items():
                best = None
                for ts, v in pts:
                    if t - LOOKBACK_S < ts <= t:
                        best = v
                if best is not None:
                    out.append((dict(key), best))
            return out
        raise ValueError(f"fake prometheus cannot evaluate {expr!r}")

    def eval_instant(self, q: str, t: float) -> list[dict]:
        m = _AVG_BY.match(q)
        if not m:
            raise ValueError(f"unsupported query {q!r}")
        k = float(m.group(1)) if m.group(1) else 1.0
        agg = _AGG[m.group(2)]
        by = [x.strip() for x in m.group(4).split(",") if x.strip()]
        groups: dict[tuple, list[float]] = {}
        for labels, v in self._inner(m.group(3), t):
            groups.setdefault(tuple(labels.get(b, "") for b in by), []).append(v)
        return [{"metric": {b: g[i] for i, b in enumerate(by) if g[i] != ""},
                 "value": [t, repr(k * agg(vs))]} for g, vs in sorted(groups.items())]

    def eval_range(self, q: str, start: float, end: float, step: float) -> list[dict]:
        out: dict[tuple, dict] = {}
        t = start
        while t <= end + 1e-9:
            for r in self.eval_instant(q, t):
                key = tuple(sorted(r["metric"].items()))
                out.setdefault(key, {"metric": r["metric"], "values": []})["values"].append([t, r["value"][1]])
            t += step
        return list(out.values())

    # ------------------------------------------------------------------ HTTP
    def handle(self, path: str, params: dict) -> tuple[int, dict]:
        q = params.get("query", "")
        self.calls.append((path, params))
        try:
            if path.endswith("/query_range"):
                if q in self.canned_range:
                    res = self.canned_range[q]
                else:
                    res = self.eval_range(q, float(params["start"]), float(params["end"]), float(params["step"]))
                return 200, {"status": "success", "data": {"resultType": "matrix", "result": res}}
            if path.endswith("/query"):
                if q in self.canned_instant:
                    res = self.canned_instant[q]
                else:
                    res = self.eval_instant(q, float(params.get("time", 0) or 0) or max(
                        (p[-1][0] for m in self.series.values() for p in m.values() if p), default=0.0))
                return 200, {"status": "success", "data": {"resultType": "vector", "result": res}}
        except ValueError as e:
            return 400, {"status": "error", "errorType": "bad_data", "error": str(e)}
        return 404, {"status": "error", "errorType": "not_found", "error": path}

    def start(self, host: str = "127.0.0.1", port: int = 0) -> str:
        outer = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                u = urlparse(self.path)
                # a request sent through an HTTP proxy (this server doubling as one)
                # carries the absolute URL in its request line
                outer.via_proxy.append(self.path.startswith("http"))
                params = {k: v[-1] for k, v in parse_qs(u.query).items()}
                code, body = outer.handle(u.path, params)
                data = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def log_message(self, *a):
                pass

        self._srv = ThreadingHTTPServer((host, port), H)
        self._th = threading.Thread(target=self._srv.serve_forever, daemon=True)
        self._th.start()
        return f"http://{host}:{self._srv.server_address[1]}/api/v1"

    def stop(self) -> None:
        if self._srv:
            self._srv.shutdown()
            self._srv.server_close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()
