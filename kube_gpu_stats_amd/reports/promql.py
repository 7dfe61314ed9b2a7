"""Prometheus HTTP API client (reference transport layer L1).

Reference: ``query_prom`` (gpu_util_stats.py:14-27, ``/query_range``) and
``query_prom_instant`` (:29-34, ``/query``), plus the two inline instant GETs of
``get_gpu_servers`` (:103-108, :115-120).  Differences, all deliberate:

* the proxy applies to every call by default; ``--compat`` reproduces the
  reference's inconsistency — its live-pod instant query (M4, ``query_prom_instant``
  :29-34) goes out without the proxy, :32 vs :24 (Q9; call order/proxy pattern
  T,T,T,F,T pinned by tests/test_reports.py);
* HTTP and Prometheus-level errors raise ``PromError`` (the reference KeyErrors
  on ``['data']`` — Q10);
* optional retries with backoff; the 5 s timeout stays the default (:24).
"""
from __future__ import annotations

import time
from datetime import datetime
from time import mktime

from ..utils.config import REF_TIMEOUT_S


class PromError(RuntimeError):
    pass


def to_unix(t) -> int:
    """datetime → int seconds the way the reference does it (local-time mktime, :16-17)."""
    if isinstance(t, datetime):
        return int(mktime(t.timetuple()))
    return int(t)


class PromClient:
    def __init__(self, base_url: str, proxy: str = "", timeout_s: float = REF_TIMEOUT_S, retries: int = 0,
                 session=None):
        import requests

        self.base_url = base_url.rstrip("/")
        self.timeout_s = timeout_s
        self.retries = retries
        self.s = session or requests.Session()
        self.proxy = proxy
        if proxy:
            self.s.proxies = {"http": proxy, "https": proxy}
        self._direct = None  # lazily: a session without the configured proxy
        self.calls: list[tuple[str, dict]] = []
        self.proxied: list[bool] = []  # per call, parallel to ``calls``

    def _session(self, proxied: bool):
        if proxied or not self.proxy:
            return self.s
        if self._direct is None:
            import requests

            self._direct = requests.Session()
        return self._direct

    def _get(self, path: str, params: dict, proxied: bool = True) -> dict:
        import requests

        url = self.base_url + path
        last = None
        sess = self._session(proxied)
        for attempt in range(self.retries + 1):
            try:
                self.calls.append((path, dict(params)))
                self.proxied.append(bool(self.proxy) and proxied)
                r = sess.get(url, params=params, timeout=self.timeout_s)
                try:
                    body = r.json()
                except ValueError as e:
                    raise PromError(f"{url}: HTTP {r.status_code}, non-JSON body") from e
                if r.status_code != 200 or body.get("status") != "success":
                    raise PromError(f"{url}: HTTP {r.status_code} {body.get('errorType', '')}: {body.get('error', '')}")
                if "data" not in body:
                    raise PromError(f"{url}: response without data")
                return body
            except (requests.RequestException, PromError) as e:
                last = e
                if attempt < self.retries:
                    time.sleep(min(2.0, 0.2 * (2 ** attempt)))
        raise last if isinstance(last, PromError) else PromError(str(last))

    def query(self, q: str, at=None, proxied: bool = True) -> dict:
        p = {"query": q}
        if at is not None:
            p["time"] = to_unix(at)
        return self._get("/query", p, proxied)

    MAX_POINTS = 11000  # Prometheus rejects range queries above 11 000 points per series

    def query_range(self, q: str, start, end, step_s: int, max_points: int | None = None) -> dict:
        """``/query_range``; windows longer than ``max_points`` steps are split into
        chunks and the per-series values concatenated."""
        s, e = to_unix(start), to_unix(end)
        cap = max_points or self.MAX_POINTS
        if (e - s) // step_s + 1 <= cap:
            return self._get("/query_range", {"query": q, "start": s, "end": e, "step": step_s})
        merged: dict[tuple, dict] = {}
        body = None
        t = s
        while t <= e:
            t_end = min(e, t + (cap - 1) * step_s)
            body = self._get("/query_range", {"query": q, "start": t, "end": t_end, "step": step_s})
            for r in body["data"]["result"]:
                key = tuple(sorted(r["metric"].items()))
                slot = merged.setdefault(key, {"metric": r["metric"], "values": []})
                slot["values"].extend(r.get("values", []))
            t = t_end + step_s
        body = dict(body)
        body["data"] = {"resultType": "matrix", "result": list(merged.values())}
        return body


def result(body: dict) -> list[dict]:
    return body["data"]["result"]
