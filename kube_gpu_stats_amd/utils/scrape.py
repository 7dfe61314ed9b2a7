"""Keep-alive /metrics scraper with latency accounting (bench + tests).

``scrape_once`` times a scrape the way a Prometheus server sees the exporter:
from sending the request to receiving the last body byte, on a persistent
connection, with a lean raw-socket HTTP/1.1 client (``http.client`` adds
≈70 µs of Python per request, more than the 1-GPU render itself).  Decoding
the body happens after the clock stops.
"""
from __future__ import annotations

import http.client
import socket
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

    # ---- lean client: request → last byte ------------------------------
    _sock: socket.socket | None = None

    def _raw_get(self, path: str) -> tuple[bytes, float]:
        if self._sock is None:
            self._sock = socket.create_connection((self.host, self.port), timeout=self.timeout)
            self._sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._buf = bytearray(1 << 20)
        req = f"GET {path} HTTP/1.1\r\nHost: {self.host}\r\n\r\n".encode()
        sock, buf = self._sock, self._buf
        t0 = time.perf_counter()
        sock.sendall(req)
        view = memoryview(buf)
        got = 0
        while True:
            n = sock.recv_into(view[got:])
            if n == 0:
                raise ConnectionError("connection closed")
            got += n
            he = buf.find(b"\r\n\r\n", 0, got)
            if he >= 0:
                break
        head = bytes(buf[:he]).decode("latin-1")
        status = int(head.split(" ", 2)[1])
        clen = 0
        for line in head.split("\r\n")[1:]:
            k, _, v = line.partition(":")
            if k.strip().lower() == "content-length":
                clen = int(v)
        total = he + 4 + clen
        if total > len(buf):
            self._buf = buf = buf + bytearray(total - len(buf) + (1 << 16))
            view = memoryview(buf)
        while got < total:
            n = sock.recv_into(view[got:total])
            if n == 0:
                raise ConnectionError("connection closed")
            got += n
        dt = time.perf_counter() - t0
        if status != 200:
            raise RuntimeError(f"HTTP {status}")
        return bytes(buf[he + 4:total]), dt

    def scrape_once(self) -> str:
        for attempt in range(2):
            try:
                body, dt = self._raw_get(self.path)
                break
            except (OSError, ValueError):
                if self._sock is not None:
                    self._sock.close()
                self._sock = None
                if attempt:
                    raise
        self.latencies_s.append(dt)
        self.bytes += len(body)
        return body.decode()

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
