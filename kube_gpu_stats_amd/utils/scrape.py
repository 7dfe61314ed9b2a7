"""Keep-alive /metrics scraper with latency accounting (bench + tests)."""
from __future__ import annotations

import http.client
import threading
import time


def parse_text(body: str) -> dict[str, list[tuple[dict, float]]]:
    """Tiny Prometheus text parser: name -> [(labels, value)].  Good enough for our own output."""
    out: dict[str, list[tuple[dict, float]]] = {}
    for line in body.splitlines():
        if not line or line[0] == "#":
            continue
        if "{" in line:
            name, rest = line.split("{", 1)
            lbl_s, val_s = rest.rsplit("} ", 1)
            labels = {}
            i = 0
            while i < len(lbl_s):
                eq = lbl_s.index("=", i)
                k = lbl_s[i:eq]
                j = eq + 2
                v = []
                while lbl_s[j] != '"':
                    if lbl_s[j] == "\\":
                        nxt = lbl_s[j + 1]
                        v.append({"n": "\n", "\\": "\\", '"': '"'}.get(nxt, nxt))
                        j += 2
                    else:
                        v.append(lbl_s[j])
                        j += 1
                labels[k] = "".join(v)
                i = j + 2 if j + 1 < len(lbl_s) and lbl_s[j + 1] == "," else j + 1
        else:
            name, val_s = line.split(" ", 1)
            labels = {}
        out.setdefault(name, []).append((labels, float(val_s.split()[0])))
    return out


class Scraper:
    def __init__(self, host: str, port: int, path: str = "/metrics", timeout: float = 5.0):
        self.host, self.port, self.path, self.timeout = host, port, path, timeout
        self._conn: http.client.HTTPConnection | None = None
        self.latencies_s: list[float] = []
        self.bytes = 0
        self.errors = 0
        self._stop = threading.Event()
        self._th: threading.Thread | None = None

    def get(self, path: str | None = None) -> str:
        for attempt in range(2):
            try:
                if self._conn is None:
                    self._conn = http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)
                self._conn.request("GET", path or self.path)
                r = self._conn.getresponse()
                body = r.read()
                if r.status != 200:
                    raise RuntimeError(f"HTTP {r.status}")
                return body.decode()
            except (OSError, http.client.HTTPException):
                self._conn = None
                if attempt:
                    raise
        raise RuntimeError("unreachable")

    def scrape_once(self) -> str:
        t0 = time.perf_counter()
        body = self.get()
        self.latencies_s.append(time.perf_counter() - t0)
        self.bytes += len(body)
        return body

    def _loop(self, hz: float) -> None:
        period = 1.0 / hz
        nxt = time.perf_counter()
        while not self._stop.is_set():
            try:
                self.scrape_once()
            except Exception:  # noqa: BLE001
                self.errors += 1
            nxt += period
            d = nxt - time.perf_counter()
            if d > 0:
                self._stop.wait(d)
            else:
                nxt = time.perf_counter()

    def start(self, hz: float) -> "Scraper":
        self._th = threading.Thread(target=self._loop, args=(hz,), name="kgs-scraper", daemon=True)
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._th:
            self._th.join(timeout=10)

    def percentile(self, q: float) -> float:
        if not self.latencies_s:
            return float("nan")
        s = sorted(self.latencies_s)
        return s[min(len(s) - 1, int(q * (len(s) - 1) + 0.5))]
