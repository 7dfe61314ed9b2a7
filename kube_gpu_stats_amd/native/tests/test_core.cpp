// Host-only concurrency tests of the data plane, built with -fsanitize=thread
// (SURVEY.md §5.2).  Run by tests/test_native_tsan.py.
//
//  1. Seqlock: one writer publishing self-consistent payloads (every word equal
//     to the sequence), many readers; a torn read would show mixed words.
//  2. SampleRing: readers walking back from head never see a slot out of order
//     by more than the ring can explain, and never a torn slot; a reader lapped
//     by the writer gets "absent", never a newer entry (generation check).
//  3. Sampler over the mock backend with fault injection, readers calling
//     window_busy / window_pmc / integ concurrently, then stop().
//  4. Recovery: a device that resets mid-run is re-opened and re-baselined.
//  6. Exporter: concurrent /metrics renders and /counters streams while the
//     samplers run at 2 kHz, the slow tier republishes link tables, the node
//     name changes (render caches under the exporter mutex), the counters are
//     handed over and taken back, and a square load flips the devices between
//     quiet (idle READ rate, changed at run time) and busy.
//  7. HTTP server: keep-alive, pipelined requests split at random bytes, HEAD,
//     gzip, bad methods / targets, oversized requests, and silent clients
//     (evicted past the connection cap, closed when idle).
//  5. PMFW table parser fuzz (ASAN build): random, truncated and mutated
//     v1.8-shaped buffers, each in an exactly-sized heap block so any read past
//     `len` is caught; the parser must reject or parse, never overrun.
//  8. AQL queue-slot reservation (aql_ring.h) against a fake queue whose read
//     index never advances: a bounded error, never a spin; abort cuts it short.
//  9. Counter-tier fault boundary: one GPU whose counter reads take 1 s, one whose
//     reads stop returning at all; the same GPUs keep their PMFW tier, the others
//     their counter rate, a per-GPU release does not wait for the hung one, and
//     stop() abandons the stuck thread within its deadline.
// 10. Circuit breaker: reads that time out open it (kgs_pmc_failed), a reset +
//     re-acquire after the backoff closes it, and the totals stay monotonic.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cmath>
#include <cerrno>
#include <chrono>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include <cstring>
#include <random>

#include "kgs/aql_batch.h"
#include "kgs/aql_ib.h"
#include "kgs/aql_ring.h"
#include "kgs/backend.h"
#include "kgs/exporter.h"
#include "kgs/gpu_metrics.h"
#include "kgs/kfd_procs.h"
#include "kgs/pmc.h"
#include "kgs/sampler.h"
#include "kgs/seqlock.h"
#include "kgs/unpark.h"
#include "kgs/util_estimator.h"

using namespace kgs;

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                  \
    }                                                                \
  } while (0)

struct Payload {
  uint64_t w[24];
};

static void test_seqlock() {
  Seqlock<Payload> sl;
  std::atomic<bool> done{false};
  std::thread wr([&] {
    Payload p;
    for (uint64_t s = 1; s <= 200000; ++s) {
      for (auto& x : p.w) x = s;
      sl.store(p);
    }
    done = true;
  });
  std::vector<std::thread> rd;
  std::atomic<uint64_t> reads{0};
  for (int t = 0; t < 3; ++t)
    rd.emplace_back([&] {
      Payload p;
      uint64_t last = 0;
      while (!done) {
        if (sl.load(p)) {
          for (auto x : p.w) CHECK(x == p.w[0]);
          CHECK(p.w[0] >= last);
          last = p.w[0];
          reads++;
        }
      }
    });
  wr.join();
  for (auto& t : rd) t.join();
  CHECK(reads > 0);
  std::printf("seqlock ok (%llu reads)\n", static_cast<unsigned long long>(reads.load()));
}

static void test_ring() {
  SampleRing<Payload, 64> ring;
  std::atomic<bool> done{false};
  std::thread wr([&] {
    Payload p;
    for (uint64_t s = 1; s <= 100000; ++s) {
      for (auto& x : p.w) x = s;
      ring.push(p);
    }
    done = true;
  });
  std::thread rd([&] {
    std::vector<Payload> buf(64);
    while (!done) {
      const size_t n = ring.recent(buf.data(), 64);
      for (size_t i = 0; i < n; ++i) {
        for (auto x : buf[i].w) CHECK(x == buf[i].w[0]);
      }
    }
  });
  wr.join();
  rd.join();
  std::vector<Payload> buf(64);
  const size_t n = ring.recent(buf.data(), 64);
  CHECK(n == 63);
  for (size_t i = 0; i < n; ++i) CHECK(buf[i].w[0] == 100000 - i);
  std::printf("ring ok\n");
}

// Generation check: a reader that holds an old head while
// the writer laps the ring must get "absent", never a newer entry under the old
// index — window searches rely on entries being time-ordered.
static void test_ring_lap() {
  SampleRing<Payload, 64> ring;
  Payload p;
  for (uint64_t s = 1; s <= 100; ++s) {
    for (auto& x : p.w) x = s;
    ring.push(p);
  }
  const uint64_t h = ring.head();  // entry e = h - 1 - i carries value e + 1
  Payload out;
  CHECK(ring.at_from(h, 5, out) && out.w[0] == h - 5);
  for (uint64_t s = 101; s <= 100 + 64; ++s) {  // one full lap
    for (auto& x : p.w) x = s;
    ring.push(p);
  }
  for (uint64_t i = 0; i < 63; ++i) CHECK(!ring.at_from(h, i, out));  // every old slot now holds a newer lap
  CHECK(ring.at(0, out) && out.w[0] == 164);
  // Concurrent: a slow reader's lookups are either exact or absent.
  std::atomic<bool> done{false};
  std::atomic<uint64_t> exact{0}, lapped{0};
  std::thread wr([&] {
    Payload q;
    for (uint64_t s = 165; s <= 200000; ++s) {
      for (auto& x : q.w) x = s;
      ring.push(q);
    }
    done = true;
  });
  std::thread rd([&] {
    Payload o;
    while (!done) {
      const uint64_t hh = ring.head();
      std::this_thread::yield();  // let the writer run ahead
      for (uint64_t i = 0; i < 63; i += 7) {
        if (ring.at_from(hh, i, o)) {
          for (auto x : o.w) CHECK(x == o.w[0]);
          CHECK(o.w[0] == hh - i);
          ++exact;
        } else {
          ++lapped;
        }
      }
    }
  });
  wr.join();
  rd.join();
  CHECK(exact > 0);
  std::printf("ring lap ok (%llu exact, %llu lapped)\n", static_cast<unsigned long long>(exact.load()),
              static_cast<unsigned long long>(lapped.load()));
}

static void test_sampler() {
  MockConfig mc;
  mc.n_gpus = 4;
  mc.fw_period_s = 0.002;
  mc.fail_rate = 0.1;
  mc.vanish_dev = 3;
  mc.vanish_after_s = 0.2;
  auto be = make_mock_backend(mc);
  auto pmc = make_mock_counter_source(*be, mc, MockPmcConfig{});
  SamplerConfig sc;
  sc.hz = 1000;
  sc.pmfw_hz = 0;  // read the (mock) table every tick
  sc.proc_every = 5;
  sc.link_every = 7;
  sc.pin_numa = false;
  sc.pmc = true;
  sc.max_backoff_ms = 20;
  Sampler s(be.get(), pmc.get(), sc);
  s.start();
  std::atomic<bool> done{false};
  std::vector<std::thread> rd;
  for (int t = 0; t < 2; ++t)
    rd.emplace_back([&] {
      while (!done) {
        for (int d = 0; d < 4; ++d) {
          double g, u;
          int n;
          PmcRates r;
          s.window_busy(d, 0.05, g, u, n);
          s.window_pmc(d, 0.05, r);
          Integrals I;
          I = s.state(d).integrals();
          auto p = s.state(d).get_procs();
          auto l = s.state(d).get_links();
          (void)p;
          (void)l;
        }
      }
    });
  std::this_thread::sleep_for(std::chrono::milliseconds(600));
  done = true;
  for (auto& t : rd) t.join();
  s.stop();
  Integrals I0, I3;
  I0 = s.state(0).integrals();
  I3 = s.state(3).integrals();
  CHECK(I0.distinct_samples > 50);
  CHECK(I0.read_errors > 0);             // 10 % injected failures
  CHECK(s.state(0).up.load() == 1);
  CHECK(s.state(3).up.load() == 0);      // vanished device marked down
  CHECK(I3.read_errors > 3);
  CHECK(I0.pmc_samples > 50);
  std::printf("sampler ok (dev0 %llu samples, %llu errors)\n", static_cast<unsigned long long>(I0.distinct_samples),
              static_cast<unsigned long long>(I0.read_errors));
}

// Reset + recover() on one device while readers hammer every device.
static void test_recovery() {
  MockConfig mc;
  mc.n_gpus = 2;
  mc.fw_period_s = 0.002;
  mc.vanish_dev = 1;
  mc.vanish_after_s = 0.1;
  mc.vanish_for_s = 0.1;
  auto be = make_mock_backend(mc);
  SamplerConfig sc;
  sc.hz = 500;
  sc.pmfw_hz = 0;
  sc.proc_every = 3;
  sc.link_every = 5;
  sc.pin_numa = false;
  sc.pmc = false;
  sc.max_backoff_ms = 10;
  Sampler s(be.get(), nullptr, sc);
  s.start();
  std::atomic<bool> done{false};
  std::thread rd([&] {
    while (!done)
      for (int d = 0; d < 2; ++d) {
        double g, u;
        int n;
        s.window_busy(d, 0.05, g, u, n);
        Integrals I;
        I = s.state(d).integrals();
      }
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(500));
  done = true;
  rd.join();
  s.stop();
  Integrals I1;
  I1 = s.state(1).integrals();
  CHECK(I1.recoveries == 1);
  CHECK(s.state(1).up.load() == 1);
  CHECK(I1.energy_joules > 0);
  std::printf("recovery ok (%llu attempts)\n", static_cast<unsigned long long>(I1.recover_attempts));
}

static void test_parser_fuzz() {
  std::mt19937_64 rng(12345);
  // a syntactically valid v1.8 header: structure_size 3872, format 1, content 8
  auto make = [&](size_t len) {
    std::vector<uint8_t> b(len);
    for (auto& x : b) x = static_cast<uint8_t>(rng());
    if (len >= 4) {
      b[0] = 3872 & 0xFF;
      b[1] = 3872 >> 8;
      b[2] = 1;
      b[3] = 8;
    }
    return b;
  };
  int parsed = 0, rejected = 0;
  for (int it = 0; it < 20000; ++it) {
    size_t len;
    switch (it % 4) {
      case 0: len = rng() % 64; break;                  // tiny
      case 1: len = 3872; break;                        // full size, random body
      case 2: len = rng() % 3872; break;                // truncated
      default: len = 3872 + rng() % 256; break;         // longer than the table
    }
    std::vector<uint8_t> b = make(len);
    if (it % 8 == 5 && len > 400) b[338] = static_cast<uint8_t>(rng());  // num_partition field
    // exact-size heap copy: ASAN flags any byte read past len
    uint8_t* heap = len ? static_cast<uint8_t*>(std::malloc(len)) : nullptr;
    if (len) std::memcpy(heap, b.data(), len);
    GpuSample s;
    const int rc = parse_gpu_metrics_v1_8(heap, len, s);
    (void)gpu_metrics_revision(heap, len);
    if (rc == 0) {
      ++parsed;
      CHECK(s.num_xcc <= static_cast<uint32_t>(kMaxXcc));
    } else {
      ++rejected;
    }
    std::free(heap);
  }
  CHECK(parsed > 0 && rejected > 0);
  std::printf("parser fuzz ok (%d parsed, %d rejected)\n", parsed, rejected);
}

static void test_exporter_concurrent() {
  ExporterConfig c;
  c.backend = "mock";
  c.mock.n_gpus = 4;
  c.sampler.hz = 2000;
  c.sampler.pin_numa = false;
  c.sampler.proc_every = 20;
  c.sampler.link_every = 50;  // new link table every 25 ms: the link-block cache churns
  c.pmc_source = "mock";
  c.port = -1;
  c.node_name = "node-a";
  c.mock.square_duty = 0.5;  // 25 ms busy / 25 ms idle: quiet ↔ busy transitions
  c.mock.util_period_s = 0.05;
  c.mock.util_base = 50;
  c.mock.util_amp = 50;
  c.sampler.pmc_idle_hz = 200;
  Exporter ex(c);
  CHECK(ex.init());
  ex.start();
  std::atomic<bool> stop{false};
  std::atomic<int> renders{0}, streams{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t)
    th.emplace_back([&] {
      std::string out;
      while (!stop.load()) {
        ex.render(out);
        CHECK(out.find("amdgpu_topology_link{") != std::string::npos);
        CHECK(out.find("amdgpu_xgmi_link_info{") != std::string::npos || renders.load() < 50);
        CHECK(out.back() == '\n');
        ++renders;
      }
    });
  th.emplace_back([&] {
    uint64_t since = 0;
    while (!stop.load()) {
      const std::string j = ex.counters_json(streams.load() % 4, 64, since);
      CHECK(j.find("\"samples\":[") != std::string::npos);
      ++streams;
    }
  });
  for (int i = 0; i < 40; ++i) {
    ex.set_node_name(i % 2 ? "node-b" : "node-a");
    if (i % 4 == 0) ex.set_pmc_enabled(i % 8 != 0);  // counter hand-over while the samplers run
    ex.sampler()->set_pmc_idle_hz(i % 3 == 0 ? 0 : 200);  // profiling mode on / off at run time
    std::this_thread::sleep_for(std::chrono::milliseconds(25));
  }
  stop = true;
  for (auto& t : th) t.join();
  ex.stop();
  std::string out;
  ex.render(out);
  CHECK(out.find("kubernetes_io_hostname=\"node-a\"") == std::string::npos);  // last rename: node-b
  CHECK(renders.load() > 10 && streams.load() > 10);
  CHECK(out.find("kgs_pmc_enabled{gpu=\"0\"") != std::string::npos);
  CHECK(ex.sampler()->state(0).pmc_releases.load() == 5);  // released at i = 0, 8, 16, 24, 32
  CHECK(ex.sampler()->state(0).pmc_quiet_skips.load() > 0);  // the idle halves were READ at the idle rate
  std::printf("exporter concurrent ok (%d renders, %d streams)\n", renders.load(), streams.load());
}

// ---- 7. HTTP server ---------------------------------------------------------
static int http_connect(int port) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  CHECK(fd >= 0);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(port));
  sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  CHECK(connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) == 0);
  timeval tv{5, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  return fd;
}

static void http_send(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t n = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n <= 0) return;  // the server may close first (oversized request)
    off += static_cast<size_t>(n);
  }
}

// Read `n` complete responses (status line + headers + Content-Length body; HEAD
// responses carry no body).  Returns the status codes; fewer on EOF / timeout.
static std::vector<int> http_read(int fd, int n, bool head, std::string* last_headers = nullptr) {
  std::vector<int> codes;
  std::string buf;
  char tmp[8192];
  while (static_cast<int>(codes.size()) < n) {
    const size_t he = buf.find("\r\n\r\n");
    if (he != std::string::npos) {
      const std::string hdr = buf.substr(0, he);
      size_t len = 0;
      const size_t cl = hdr.find("Content-Length: ");
      if (cl != std::string::npos) len = std::strtoul(hdr.c_str() + cl + 16, nullptr, 10);
      if (head) len = 0;
      if (buf.size() >= he + 4 + len) {
        codes.push_back(std::atoi(hdr.c_str() + 9));
        if (last_headers) *last_headers = hdr;
        buf.erase(0, he + 4 + len);
        continue;
      }
    }
    const ssize_t r = recv(fd, tmp, sizeof tmp, 0);
    if (r <= 0) break;
    buf.append(tmp, static_cast<size_t>(r));
  }
  return codes;
}

// The server closed the connection (an oversized request may end in a reset:
// the client's unread bytes are still in flight when the server closes).
static bool http_eof(int fd) {
  char c;
  const ssize_t r = recv(fd, &c, 1, 0);
  return r == 0 || (r < 0 && errno == ECONNRESET);
}

// The epoll server under the sanitizer: keep-alive, pipelined requests split at
// arbitrary byte boundaries, HEAD, gzip, unknown methods and targets, oversized
// requests, and clients that connect and never send (evicted past
// http_max_conns, closed after http_idle_s) — while the samplers publish and the
// renders run on the server thread.
static void test_http_server() {
  ExporterConfig c;
  c.backend = "mock";
  c.mock.n_gpus = 2;
  c.sampler.hz = 1000;
  c.sampler.pin_numa = false;
  c.pmc_source = "mock";
  c.listen_addr = "127.0.0.1";
  c.port = 0;
  c.node_name = "node-h";
  c.gzip_level = 1;
  c.http_max_conns = 8;
  c.http_idle_s = 0.3;
  Exporter ex(c);
  CHECK(ex.init());
  ex.start();
  const int port = ex.port();
  CHECK(port > 0);
  {  // silent clients first (alone, so no active client is the least recently used):
     // past the cap the least recently active go, the rest once idle for 0.3 s
    std::vector<int> fds;
    for (int i = 0; i < 12; ++i) {
      fds.push_back(http_connect(port));
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    for (int fd : fds) {
      CHECK(http_eof(fd));
      close(fd);
    }
    CHECK(ex.http_closed_limit.load() == 4 && ex.http_closed_idle.load() == 8);
  }
  std::atomic<int> ok{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t)
    th.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      for (int i = 0; i < 25; ++i) {
        const int fd = http_connect(port);
        // two pipelined requests, split at a random byte
        const std::string two =
            "GET /metrics HTTP/1.1\r\nHost: x\r\n\r\nGET /healthz?x=1 HTTP/1.1\r\nHost: x\r\n\r\n";
        const size_t cut = rng() % two.size();
        http_send(fd, two.substr(0, cut));
        std::this_thread::sleep_for(std::chrono::microseconds(rng() % 500));
        http_send(fd, two.substr(cut));
        std::vector<int> codes = http_read(fd, 2, false);
        CHECK(codes.size() == 2 && codes[0] == 200 && codes[1] == 200);
        http_send(fd, "HEAD /metrics HTTP/1.1\r\n\r\n");
        codes = http_read(fd, 1, true);
        CHECK(codes.size() == 1 && codes[0] == 200);
        std::string hdr;
        http_send(fd, "GET /metrics HTTP/1.1\r\naccept-encoding: gzip, deflate\r\n\r\n");
        codes = http_read(fd, 1, false, &hdr);
        CHECK(codes.size() == 1 && codes[0] == 200 && hdr.find("Content-Encoding: gzip") != std::string::npos);
        http_send(fd, "POST /metrics HTTP/1.1\r\n\r\nGET /nope HTTP/1.1\r\n\r\nGET /counters?gpu=7&n=99999 HTTP/1.1\r\n\r\n");
        codes = http_read(fd, 3, false);
        CHECK(codes.size() == 3 && codes[0] == 405 && codes[1] == 404 && codes[2] == 200);
        http_send(fd, "GET /devices HTTP/1.1\r\nConnection: close\r\n\r\n");
        codes = http_read(fd, 1, false);
        CHECK(codes.size() == 1 && codes[0] == 200 && http_eof(fd));
        close(fd);
        ++ok;
      }
    });
  th.emplace_back([&] {  // oversized request without an end of headers: dropped
    for (int i = 0; i < 5; ++i) {
      const int fd = http_connect(port);
      http_send(fd, "GET /metrics HTTP/1.1\r\nX: " + std::string(70000, 'a'));
      CHECK(http_eof(fd));
      close(fd);
    }
  });
  for (auto& t : th) t.join();
  CHECK(ok.load() == 75);
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  CHECK(ex.http_conns_open.load() == 0);
  ex.stop();
  std::printf("http server ok (%llu requests, %llu evicted, %llu idle-closed)\n",
              static_cast<unsigned long long>(ex.http_requests.load()),
              static_cast<unsigned long long>(ex.http_closed_limit.load()),
              static_cast<unsigned long long>(ex.http_closed_idle.load()));
}

static int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static void test_reserve_slot() {
  // A 64-slot queue the CP stopped consuming: read index stuck at 10, 64 packets in flight.
  std::atomic<uint64_t> rd{10}, wr{74};
  auto read_idx = [&] { return rd.load(); };
  auto write_idx = [&] { return wr.load(); };
  auto commit = [&](uint64_t i) { wr.store(i + 1); };
  auto pause = [] { std::this_thread::yield(); };
  uint64_t idx = 0;
  int64_t t0 = now_ns();
  SlotResult r = reserve_slot(64, t0 + 50000000, nullptr, read_idx, write_idx, commit, now_ns, pause, idx);
  int64_t el = now_ns() - t0;
  CHECK(r == SlotResult::kTimeout);
  CHECK(el >= 50000000 && el < 500000000);  // at the deadline, not forever
  CHECK(wr.load() == 74);                   // nothing reserved: no hole for the CP to stall on
  std::atomic<int> abort{0};
  std::thread aborter([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    abort.store(1);
  });
  t0 = now_ns();
  r = reserve_slot(64, t0 + 5000000000LL, &abort, read_idx, write_idx, commit, now_ns, pause, idx);
  el = now_ns() - t0;
  aborter.join();
  CHECK(r == SlotResult::kAborted && el < 1000000000);
  CHECK(wr.load() == 74);
  // The CP drains one packet: the next reservation gets slot 74 at once.
  rd.store(11);
  r = reserve_slot(64, now_ns() + 1000000, nullptr, read_idx, write_idx, commit, now_ns, pause, idx);
  CHECK(r == SlotResult::kOk && idx == 74 && wr.load() == 75);
  std::printf("reserve_slot ok (timeout %.1f ms)\n", 50.0);
}

static void test_pmc_fault_boundary() {
  ExporterConfig c;
  c.backend = "mock";
  c.mock.n_gpus = 8;
  c.mock.fw_period_s = 0.020;  // PMFW table cadence (≈50 distinct tables/s)
  c.sampler.hz = 1000;
  c.sampler.pmfw_hz = 100;
  c.sampler.pin_numa = false;
  c.sampler.proc_every = 0;
  c.sampler.link_every = 0;
  c.sampler.pmc_idle_hz = 0;
  c.sampler.stop_timeout_s = 1.0;
  c.pmc_source = "mock";
  c.mock_pmc.slow_dev = 2;  // every counter read on GPU 2 takes 1 s
  c.mock_pmc.slow_s = 1.0;
  c.mock_pmc.hang_dev = 5;  // GPU 5's reads stop returning after 200
  c.mock_pmc.hang_after = 200;
  c.mock_pmc.hang_timeout_s = -1;
  c.port = -1;
  // Never deleted: the abandoned thread may outlive the test.  A global keeps it
  // reachable, so the ASAN build's leak checker does not count it.
  static Exporter* ex = nullptr;
  ex = new Exporter(c);
  CHECK(ex->init());
  ex->start();
  std::this_thread::sleep_for(std::chrono::milliseconds(500));
  std::vector<Integrals> a(8), b(8);
  for (int d = 0; d < 8; ++d) a[d] = ex->sampler()->state(d).integrals();
  const int64_t t0 = now_ns();
  std::this_thread::sleep_for(std::chrono::milliseconds(1500));
  for (int d = 0; d < 8; ++d) b[d] = ex->sampler()->state(d).integrals();
  const double secs = (now_ns() - t0) * 1e-9;
  for (int d = 0; d < 8; ++d) {
    const double pmfw = (b[d].distinct_samples - a[d].distinct_samples) / secs;
    const double pmc = (b[d].pmc_samples - a[d].pmc_samples) / secs;
    CHECK(pmfw >= 45);  // PMFW tier untouched on every GPU, the slow and the hung one included
    if (d != 2 && d != 5) CHECK(pmc >= 0.85 * 1000);  // slack for TSAN scheduling on a shared 8-CPU host
  }
  // Per-GPU hand-over: releasing the hung GPU returns at once, and every other GPU
  // releases within a few of its own ticks.
  int64_t r0 = now_ns();
  ex->set_pmc_enabled(false, 5);
  ex->set_pmc_enabled(false, 3);
  CHECK(now_ns() - r0 < 10000000);
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  CHECK(ex->sampler()->state(3).pmc_on.load() == 0);
  CHECK(ex->sampler()->state(5).pmc_on.load() == 1);  // its thread is stuck: nothing happened, nobody waited
  ex->set_pmc_enabled(true, 3);
  r0 = now_ns();
  ex->stop();
  const double stop_s = (now_ns() - r0) * 1e-9;
  CHECK(stop_s < 2.0);
  CHECK(ex->sampler()->abandoned_threads() == 1);
  CHECK(ex->sampler()->state(5).thread_hung.load() == 1);
  std::string out;
  ex->render(out);
  CHECK(out.find("kgs_sampler_thread_hung{gpu=\"5\"") != std::string::npos);
  // Restart: every tier comes back except the stuck (GPU 5, counter) one.
  ex->start();
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  const Integrals c5 = ex->sampler()->state(5).integrals();
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  CHECK(ex->sampler()->state(5).integrals().distinct_samples > c5.distinct_samples);
  ex->stop();
  std::printf("pmc fault boundary ok (stop %.3f s)\n", stop_s);
}

static void test_pmc_breaker() {
  ExporterConfig c;
  c.backend = "mock";
  c.mock.n_gpus = 2;
  c.mock.fw_period_s = 0.005;
  c.sampler.hz = 1000;
  c.sampler.pin_numa = false;
  c.sampler.proc_every = 0;
  c.sampler.link_every = 0;
  c.sampler.pmc_idle_hz = 0;
  c.sampler.pmc_breaker_k = 3;
  c.sampler.pmc_retry_s = 0.1;
  c.pmc_source = "mock";
  c.mock_pmc.hang_dev = 1;      // after 100 reads, GPU 1's reads time out (50 ms each) ...
  c.mock_pmc.hang_after = 100;
  c.mock_pmc.hang_timeout_s = 0.05;
  c.mock_pmc.hang_heals_on_reset = true;  // ... until the breaker resets its queue
  c.port = -1;
  Exporter ex(c);
  CHECK(ex.init());
  ex.start();
  bool saw_failed = false;
  std::string out;
  for (int i = 0; i < 60 && !saw_failed; ++i) {
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
    if (ex.sampler()->state(1).pmc_failed.load()) {
      saw_failed = true;
      ex.render(out);
      CHECK(out.find("kgs_pmc_failed{gpu=\"1\",uuid=") != std::string::npos);
    }
  }
  CHECK(saw_failed);
  const Integrals f = ex.sampler()->state(1).integrals();
  std::this_thread::sleep_for(std::chrono::milliseconds(600));  // retry after 0.1 s: reset heals, READs resume
  const Integrals g = ex.sampler()->state(1).integrals();
  ex.stop();
  const DeviceState& st = ex.sampler()->state(1);
  CHECK(st.pmc_failed.load() == 0);
  CHECK(st.pmc_breaker_trips.load() == 1);
  CHECK(st.pmc_retries.load() >= 1);
  CHECK(ex.counters()->resets(1) >= 1);
  CHECK(g.pmc_samples > f.pmc_samples + 200);
  CHECK(f.pmc_errors >= 3);
  CHECK(ex.sampler()->state(0).pmc_breaker_trips.load() == 0);
  PmcSample p;
  CHECK(st.pmc_latest.load(p) && p.value[kPmcGrbmCount] > 0);
  std::printf("pmc breaker ok (%llu errors, %llu retries)\n", static_cast<unsigned long long>(g.pmc_errors),
              static_cast<unsigned long long>(st.pmc_retries.load()));
}

static void test_batch_plan() {
  // --pmc-batch 8, publish interval 1 ms (kgs/aql_batch.h).
  BatchPlan p;
  p.configure(8, 1000000);
  CHECK(p.nslots() == 16 && p.publisher(0) == 7 && p.publisher(1) == 15);
  int64_t t = 1000000000;
  auto submit = [&](int64_t dt) {
    t += dt;
    const int k = p.next_slot(t);
    p.submitted(k, t);
    return k;
  };
  int ks[32];
  // After a reset the tick interval is unknown: the first READ publishes at once.
  CHECK(submit(0) == 7 && p.closed(0) && p.current_half() == 1);
  CHECK(p.slots(0, ks) == 1 && ks[0] == 7);
  p.collected(0);
  // 8 kHz: half 1 fills in order and only its 8th READ (slot 15) publishes.
  for (int j = 0; j < 8; ++j) CHECK(submit(125000) == 8 + j);
  CHECK(p.closed(1) && !p.closed(0) && p.current_half() == 0 && p.last() == 15);
  CHECK(p.slots(1, ks) == 8 && ks[0] == 8 && ks[6] == 14 && ks[7] == 15);
  p.collected(1);
  // Three 8 kHz READs, then the GPU goes quiet (100 Hz): the next READ would wait
  // past 1 ms for a publisher, so it takes slot 7 and closes the half early.
  CHECK(submit(125000) == 0 && submit(125000) == 1 && submit(125000) == 2);
  CHECK(!p.closed(0));
  CHECK(submit(10000000) == 7 && p.closed(0));
  CHECK(p.slots(0, ks) == 4 && ks[0] == 0 && ks[1] == 1 && ks[2] == 2 && ks[3] == 7);
  p.collected(0);
  // At 100 Hz every READ publishes: halves of one READ, alternating.
  for (int i = 0; i < 4; ++i) {
    const int k = submit(10000000);
    CHECK(k == (i % 2 == 0 ? 15 : 7));
    CHECK(p.slots(k / 8, ks) == 1 && ks[0] == k);
    p.collected(k / 8);
  }
  // 4 kHz: a READ publishes once the next would be due more than 1 ms after the
  // half's first — 4 READs per writeback (the 1 kHz publication rate).
  CHECK(submit(250000) == 8 && submit(250000) == 9 && submit(250000) == 10 && submit(250000) == 15);
  p.collected(1);
  // 1 kHz: every READ publishes.
  CHECK(submit(1000000) == 7 && submit(1000000) == 15);
  p.collected(0);
  p.collected(1);
  // A late tick (a sampler overrun) only shortens a half.
  CHECK(submit(125000) == 0 && submit(900000) == 7);
  p.collected(0);
  // publish interval 0: only the B-th READ publishes, whatever the rate.
  p.configure(4, 0);
  for (int j = 0; j < 4; ++j) CHECK(submit(50000000) == j);
  CHECK(p.closed(0) && p.slots(0, ks) == 4);
  // Random tick intervals (10 µs .. 3 ms): every half holds its first slots in order
  // plus the publisher, never more than B READs, and no READ waits 1 ms or more for
  // the submission of its publisher unless it is the half's only READ.
  std::mt19937_64 rng(7);
  std::uniform_int_distribution<int64_t> dt(10000, 3000000);
  p.configure(8, 1000000);
  int64_t first = 0;
  int n_in_half = 0;
  for (int i = 0; i < 20000; ++i) {
    const int h = p.current_half();
    if (p.closed(h)) p.collected(h);
    const int64_t step = dt(rng);
    t += step;
    const int k = p.next_slot(t);
    CHECK(k / 8 == h);
    if (n_in_half == 0) first = t;
    p.submitted(k, t);
    ++n_in_half;
    if (p.is_publisher(k)) {
      CHECK(p.slots(h, ks) == n_in_half && n_in_half <= 8 && ks[n_in_half - 1] == k);
      for (int j = 0; j + 1 < n_in_half; ++j) CHECK(ks[j] == h * 8 + j);
      CHECK(n_in_half == 1 || t - first < 1000000 + 3000000);
      n_in_half = 0;
    } else {
      CHECK(t - first < 1000000);  // a non-publisher is only submitted while the half is young
    }
  }
  // Collection order: the CP delays half A's publisher past the time
  // half B closes, so both halves are closed when the sampler comes back.  The
  // half the next READ reuses (A) is the older one and must be folded first, even
  // when B's publisher is already done; folding B first would hand out samples
  // whose time and cumulative counts go backwards.
  p.configure(2, 0);
  int hv[2];
  bool wv[2];
  CHECK(p.collect_order(true, hv, wv) == 0);  // nothing closed: nothing to fold
  CHECK(submit(125000) == 0 && submit(125000) == 1 && p.closed(0) && p.current_half() == 1);
  CHECK(p.collect_order(false, hv, wv) == 0);  // A closed, its publisher not done: keep filling B
  CHECK(p.collect_order(true, hv, wv) == 1 && hv[0] == 0 && !wv[0]);  // the usual case: fold A, no wait
  CHECK(submit(125000) == 2 && submit(125000) == 3 && p.closed(1) && p.current_half() == 0);
  CHECK(p.collect_order(true, hv, wv) == 2 && hv[0] == 0 && wv[0] && hv[1] == 1 && !wv[1]);
  CHECK(p.collect_order(false, hv, wv) == 1 && hv[0] == 0 && wv[0]);  // B still running: A only
  p.collected(0);
  CHECK(p.collect_order(true, hv, wv) == 1 && hv[0] == 1 && !wv[0]);
  // A whole rotation driven through collect_order never folds a newer half first.
  p.configure(3, 0);
  int last_half_folded = -1, closes = 0;
  std::vector<int> close_order, fold_order;
  for (int i = 0; i < 600; ++i) {
    const int n = p.collect_order((i % 7) != 0, hv, wv);
    for (int j = 0; j < n; ++j) {
      fold_order.push_back(hv[j]);
      p.collected(hv[j]);
      last_half_folded = hv[j];
    }
    const int k = p.next_slot(t += 125000);
    p.submitted(k, t);
    if (p.is_publisher(k)) {
      close_order.push_back(k / 3);
      ++closes;
    }
  }
  CHECK(last_half_folded >= 0 && closes > 100);
  for (size_t j = 0; j < fold_order.size(); ++j) CHECK(fold_order[j] == close_order[j]);  // FIFO
  std::printf("batch plan ok\n");
}

// Lite READ IB (kgs/aql_ib.h): a synthetic READ shaped like aqlprofile's
// (profiles/r1/lean/read_packet_dump_base.txt): a latch, one PRED_EXEC region per
// XCC with three broadcast GRBM/CP counters and four per-SE SQ sections, lean NOPs,
// a trailing ACQUIRE_MEM.
namespace {
uint32_t t3(uint32_t op, uint32_t len) { return (3u << 30) | ((len - 2) << 16) | (op << 8); }
void put_index(std::vector<uint32_t>& ib, uint32_t v) {
  ib.push_back(t3(kPm4SetUconfigReg, 3));
  ib.push_back(kGrbmGfxIndexReg);
  ib.push_back(v);
}
void put_copy(std::vector<uint32_t>& ib, uint32_t reg, uint64_t dst) {
  ib.push_back(t3(kPm4CopyData, 6));
  ib.push_back(0x500);  // src_sel register, dst_sel memory (5)
  ib.push_back(reg);
  ib.push_back(0);
  ib.push_back(static_cast<uint32_t>(dst));
  ib.push_back(static_cast<uint32_t>(dst >> 32));
}
std::vector<uint32_t> synthetic_read(bool odd_se_section, uint64_t* n_global) {
  std::vector<uint32_t> ib;
  uint64_t dst = 0x7f0000001000ull;
  *n_global = 0;
  ib.push_back(t3(kPm4SetUconfigReg, 3));  // CP_PERFMON_CNTL latch
  ib.push_back(0x1808);
  ib.push_back(0x401);
  for (int x = 0; x < 8; ++x) {
    const size_t pred = ib.size();
    ib.push_back(t3(kPm4PredExec, 2));
    ib.push_back((1u << (24 + (x % 8))) | 0);  // count patched below
    const size_t body = ib.size();
    ib.push_back(t3(kPm4Nop, 2));  // CS_PARTIAL_FLUSH turned NOP by the lean rewrite
    ib.push_back(0);
    for (uint32_t c = 0; c < 3; ++c) {  // GRBM_COUNT, GRBM_SPI_BUSY, CPC busy: LO / HI
      put_index(ib, 0xe0000000u);
      put_copy(ib, 0xd040 + 3 * c, dst); dst += 4;
      put_copy(ib, 0xd041 + 3 * c, dst); dst += 4;
      *n_global += 2;
    }
    for (uint32_t se = 0; se < 4; ++se) {  // SQ MFMA busy per SE
      put_index(ib, 0x60000000u | (se << 16));
      put_copy(ib, 0xd1c0, dst); dst += 4;
      put_copy(ib, 0xd1c1, dst); dst += 4;
      if (odd_se_section && x == 3 && se == 2) {  // a non-copy packet inside a per-SE section: kept whole
        ib.push_back(t3(0x46, 2));
        ib.push_back(0x407);
      }
    }
    ib[pred + 1] |= static_cast<uint32_t>(ib.size() - body);
  }
  ib.push_back(t3(0x58, 7));  // ACQUIRE_MEM (L2 writeback)
  for (int k = 0; k < 6; ++k) ib.push_back(k == 0 ? (1u << 18) : 0);
  return ib;
}
}  // namespace

static void test_lite_ib() {
  uint64_t n_global = 0;
  std::vector<uint32_t> ib = synthetic_read(false, &n_global), out;
  std::vector<uint64_t> all;
  CHECK(ib_copy_dsts(ib.data(), static_cast<uint32_t>(ib.size()), &all));
  CHECK(all.size() == 8 * (6 + 8));
  IbCompact r = compact_se_sections(ib.data(), static_cast<uint32_t>(ib.size()), out);
  CHECK(r.ok);
  CHECK(r.dropped_copies == 8 * 4 * 2);
  CHECK(r.kept_copies + r.dropped_copies == all.size() && r.copy_bytes == 4);  // 32-bit LO / HI copies
  // the dropped results are the SQ ones: with 2 copies of 4 B per result in IB order,
  // ordinal = offset / 8 lands on the 4 SE results after each XCC's 3 global ones
  for (uint64_t d : r.dropped_dsts) CHECK((d - 0x7f0000001000ull) / 8 % 7 >= 3);
  std::vector<uint64_t> kept;
  std::string why;
  CHECK(ib_copy_dsts(out.data(), static_cast<uint32_t>(out.size()), &kept, &why));
  CHECK(kept.size() == n_global);
  // every kept packet sits under a broadcast GRBM_GFX_INDEX, and every region is closed
  bool se = false;
  uint32_t regions = 0;
  for (uint32_t i = 0; i < out.size();) {
    if (pm4_gfx_index(out.data() + i, &se)) CHECK(!se);
    if (pm4_op(out[i]) == kPm4PredExec) ++regions;
    CHECK(pm4_op(out[i]) != kPm4Nop);
    i += pm4_len(out[i]);
  }
  CHECK(regions == 8);
  CHECK(out.size() + r.dropped_dw == ib.size());
  // A per-SE section with anything but copies in it stays whole (its copies too).
  std::vector<uint32_t> ib2 = synthetic_read(true, &n_global), out2;
  IbCompact r2 = compact_se_sections(ib2.data(), static_cast<uint32_t>(ib2.size()), out2);
  CHECK(r2.ok && r2.dropped_copies == 8 * 4 * 2 - 2);
  // Malformed input: a PRED_EXEC whose region ends inside a packet.
  std::vector<uint32_t> bad = ib;
  bad[4] += 1;  // the first region's count
  std::vector<uint32_t> out3;
  CHECK(!compact_se_sections(bad.data(), static_cast<uint32_t>(bad.size()), out3).ok);
  // No per-SE section at all: nothing to gain, the caller keeps the full IB.
  std::vector<uint32_t> flat;
  put_index(flat, 0xe0000000u);
  put_copy(flat, 0xd040, 0x1000);
  CHECK(!compact_se_sections(flat.data(), static_cast<uint32_t>(flat.size()), out3).ok);
  // Fuzz: random READ shapes (XCC count, broadcast counters, SEs, stray packets, fillers).
  // Whenever compaction succeeds its output parses, writes the input's results less the
  // dropped ones in order, never copies under an SE-select index write, and shrinks.
  std::mt19937 rng(1234);
  int ok_n = 0;
  for (int it = 0; it < 500; ++it) {
    std::vector<uint32_t> f;
    uint64_t dst = 0x7f0000002000ull;
    const int nx = 1 + static_cast<int>(rng() % 8), ng = static_cast<int>(rng() % 4), ns = static_cast<int>(rng() % 5);
    for (int x = 0; x < nx; ++x) {
      const bool pred = rng() % 4 != 0;
      size_t at = 0, body = 0;
      if (pred) {
        at = f.size();
        f.push_back(t3(kPm4PredExec, 2));
        f.push_back(1u << 24);
        body = f.size();
      }
      if (rng() % 2) { f.push_back(t3(kPm4Nop, 2)); f.push_back(0); }
      for (int g = 0; g < ng; ++g) { put_index(f, 0xe0000000u); put_copy(f, 0xd040, dst); dst += 4; }
      for (int se = 0; se < ns; ++se) {
        put_index(f, 0x60000000u | (static_cast<uint32_t>(se) << 16));
        const int nc = static_cast<int>(rng() % 3);
        for (int c = 0; c < nc; ++c) { put_copy(f, 0xd1c0 + c, dst); dst += 4; }
        if (rng() % 10 == 0) { f.push_back(t3(0x46, 2)); f.push_back(0x407); }
        if (rng() % 10 == 0) f.push_back(0x80000000u);  // type-2 filler
      }
      if (pred) f[at + 1] |= static_cast<uint32_t>(f.size() - body);
    }
    std::vector<uint64_t> in;
    CHECK(ib_copy_dsts(f.data(), static_cast<uint32_t>(f.size()), &in));
    std::vector<uint32_t> o;
    IbCompact c = compact_se_sections(f.data(), static_cast<uint32_t>(f.size()), o);
    if (!c.ok) continue;
    ++ok_n;
    std::vector<uint64_t> got;
    CHECK(ib_copy_dsts(o.data(), static_cast<uint32_t>(o.size()), &got));
    CHECK(got.size() + c.dropped_dsts.size() == in.size());
    CHECK(o.size() < f.size());
    // copies made under an SE-select index write: only those of the sections kept whole remain
    auto se_copies = [](const std::vector<uint32_t>& v) {
      uint32_t n = 0;
      bool sel = false;
      for (uint32_t i = 0; i < v.size();) {
        if (pm4_type(v[i]) == 2) { ++i; continue; }
        bool se2 = false;
        if (pm4_gfx_index(v.data() + i, &se2)) sel = se2;
        if (sel && pm4_copy_to_mem(v.data() + i)) ++n;
        i += pm4_len(v[i]);
      }
      return n;
    };
    CHECK(se_copies(o) + c.dropped_copies == se_copies(f));
  }
  CHECK(ok_n > 100);
  std::printf("lite IB ok (%zu -> %zu dwords, %u per-SE copies dropped; fuzz %d/500 compacted)\n", ib.size(),
              out.size(), r.dropped_copies, ok_n);
}


// DispatchEstimator on a synthetic READ stream (2.4 GHz idle, 2.1 GHz under bursts,
// a 15 µs READ every 125 µs): the READ cost is learned on READ-only intervals, an
// idle GPU integrates ≈0, a 1 ms-every-5 ms train its 20 % duty, and the quiet state
// follows the hold.  Under the sanitizers: no UB in the fold, no out-of-range index.
static void test_dispatch_estimator() {
  const EstimatorParams p = estimator_params(SamplerConfig{}, 256);
  DispatchEstimator e;
  e.restart(0);
  int64_t t = 0;
  double cnt = 0, spi = 0, cpc = 0, mfma = 0, busy_s = 0, disp_s = 0;
  bool quiet_seen = false;
  auto read = [&](bool count) {
    Drain d;
    d.mono_ns = t;
    d.mask = kPmcSetBase;
    d.count = static_cast<uint64_t>(cnt);
    d.spi = static_cast<uint64_t>(spi);
    d.cpc = static_cast<uint64_t>(cpc);
    d.mfma = static_cast<uint64_t>(mfma);
    const DrainStep r = e.feed(d, p);
    if (count) disp_s += r.dispatch_s;
    quiet_seen |= r.quiet;
  };
  for (int i = 0; i < 400; ++i) {  // 50 ms idle: READs only
    t += 125000;
    cnt += 2.4e3 * 125;
    cpc += 2.4e3 * 15;
    spi += 2.4e3 * 0.9;
    read(false);
  }
  CHECK(quiet_seen);
  CHECK(std::abs(e.cpc_read_us() - 15.0) < 0.5);
  CHECK(std::abs(e.clk_idle_hz() - 2.4e9) < 0.02e9);
  for (int i = 0; i < 8000; ++i) {  // 1 s of a 1 ms / 5 ms train, READs every 125 µs
    const double ph = std::fmod(t * 1e-9, 0.005);
    const bool on = ph < 0.001;
    const double f = on ? 2.1e3 : 2.4e3;  // cycles per µs
    t += 125000;
    cnt += f * 125;
    cpc += f * 15 + (on ? f * 110 : 0.0);  // busy slice + the READ (hidden under the kernel when on)
    spi += on ? f * 120 : 2.4e3 * 0.9;
    mfma += on ? f * 120 * 512 : 0.0;
    busy_s += on ? 125e-6 : 0.0;
    read(true);
  }
  CHECK(std::abs(disp_s - busy_s) < 0.01 * 1.0);  // within 1 point of the 20 % duty
  CHECK(!e.quiet());
}

// an interval with no wave, no MFMA cycle and the CP busy ≈48 % of the clocks
// has the READ-learning rule's shape, but its CP time is four READs' worth: it bills that
// time (less one READ) and classifies as dispatch-bound — only intervals within
// 2 × the learned READ cost bill zero.
static void test_cp_only_work_is_not_read_only() {
  const EstimatorParams p = estimator_params(SamplerConfig{}, 256);
  DispatchEstimator e;
  e.restart(0);
  int64_t t = 0;
  double cnt = 0, spi = 0, cpc = 0;
  auto read = [&]() {
    Drain d;
    d.mono_ns = t;
    d.mask = kPmcSetBase;
    d.count = static_cast<uint64_t>(cnt);
    d.spi = static_cast<uint64_t>(spi);
    d.cpc = static_cast<uint64_t>(cpc);
    return e.feed(d, p);
  };
  for (int i = 0; i < 100; ++i) {  // idle READs teach the 15 µs READ cost
    t += 125000;
    cnt += 2.4e3 * 125;
    cpc += 2.4e3 * 15;
    spi += 2.4e3 * 0.9;
    read();
  }
  double disp = 0;
  bool dbound = false;
  for (int i = 0; i < 120; ++i) {  // 15 ms of CP-only work at 48 % of the clocks, SPI < 2 %
    t += 125000;
    cnt += 2.4e3 * 125;
    cpc += 2.4e3 * 60;
    spi += 2.4e3 * 0.9;
    const DrainStep r = read();
    disp += r.dispatch_s;
    CHECK(r.dispatch_s > 40e-6);  // 60 µs of CP time less the READ's 15
    dbound |= r.dbound_interval;
  }
  CHECK(std::abs(disp - 120 * 45e-6) < 120 * 3e-6);
  // each interval is CP-busy without waves for ≥ 0.3 of the clocks; the READ rate still
  // drops to the idle rate rather than the dispatch rate, since no wave ran (quiet wins)
  CHECK(dbound);
  CHECK(e.quiet() && !e.dbound());
  // a READ-only interval within the learned cost still bills nothing
  t += 125000;
  cnt += 2.4e3 * 125;
  cpc += 2.4e3 * 16;
  spi += 2.4e3 * 0.9;
  CHECK(read().dispatch_s == 0.0);
  std::printf("cp-only work billed ok (%.1f µs per interval, dispatch-bound %d)\n", disp / 120 * 1e6, dbound);
}

// UtilBiller: drains at 10 Hz land on host time, PMFW tables on a 20 ms firmware
// grid read at 10 Hz — an interval holds 0, 1 or 2 drains.  Carrying the excess
// bills a saturated GPU everything but the last drain's lag; the round-4 clip
// (cap 0) loses time; an epoch change falls back to PMFW and drops the carry.
static void test_util_biller() {
  auto run = [](double max_carry) {
    UtilBiller b;
    double billed = 0, last_fw = -1;
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> jit(0.0, 0.03);
    double drain_t = 0, next_drain = 0.1 + jit(rng);
    for (int k = 1; k <= 200; ++k) {
      const double t = 0.1 * k + 0.004;               // PMFW thread wake-up
      while (next_drain <= t) {
        drain_t = next_drain;
        next_drain += 0.1 + jit(rng) - 0.015;
      }
      const double fw = std::floor(t / 0.02) * 0.02;  // table time
      const double dt = last_fw < 0 ? 0.0 : fw - last_fw;
      last_fw = fw;
      CounterCover c;
      c.ok = true;
      c.epoch = 1;
      c.dispatch = true;
      c.busy_s = drain_t;  // saturated: busy integral == host time at the drain
      c.share = 1.0;
      c.since_s = t - drain_t;
      const UtilBiller::Bill r = b.bill(dt, 0.0, c, max_carry);
      CHECK(r.billed_s <= dt + 1e-12);
      billed += r.billed_s;
    }
    return billed;
  };
  const double fw_total = std::floor(20.004 / 0.02) * 0.02 - std::floor(0.104 / 0.02) * 0.02;
  CHECK(run(0.35) > 0.99 * fw_total);
  CHECK(run(1e-12) < 0.98 * fw_total);
  UtilBiller b;
  CounterCover c;
  c.ok = true;
  c.epoch = 1;
  c.dispatch = true;
  b.bill(0.02, 0.02, c, 1.0);
  c.busy_s = 0.05;
  CHECK(b.bill(0.02, 0.02, c, 1.0).from_counters && std::abs(b.carry_s() - 0.03) < 1e-9);
  c.epoch = 2;
  c.busy_s = 0.06;
  const UtilBiller::Bill r = b.bill(0.02, 0.015, c, 1.0);
  CHECK(!r.from_counters && std::abs(r.billed_s - 0.015) < 1e-12 && b.carry_s() == 0.0);
}

// TickDither: the offset stays within half a period, moves at most `dither` of a period
// per tick, spreads over the whole period (the READ phase cannot lock onto a periodic
// load) and averages out (the grid keeps the rate); dither 0 is the fixed grid.
static void test_tick_dither() {
  TickDither d(42);
  const int64_t period = 125000;
  double prev = 0, sum = 0;
  int bins[8] = {};
  const int n = 200000;
  for (int i = 0; i < n; ++i) {
    const double o = d.step(period, 0.25);
    CHECK(std::abs(o) <= 0.5 * period + 1e-6);
    CHECK(std::abs(o - prev) <= 0.25 * period + 1e-6);
    prev = o;
    sum += o;
    ++bins[std::min(7, static_cast<int>((o + 0.5 * period) / period * 8))];
  }
  CHECK(std::abs(sum / n) < 0.05 * period);
  for (int b : bins) CHECK(b > n / 8 / 2);  // every eighth of the period visited often
  CHECK(d.step(period, 0.0) == 0.0 && d.offset() == 0.0);
}

// read_kfd_procs from one slow thread per GPU at once (the fdinfo parse must not share
// tokenizer state: strtok_r), on a fake KFD + /proc tree under /tmp.
static void test_kfd_procs_concurrent() {
  char tmpl[] = "/tmp/kgs_kfd_XXXXXX";
  const char* root = mkdtemp(tmpl);
  CHECK(root != nullptr);
  const std::string r(root), kfd = r + "/kfd", proc = r + "/proc";
  auto mk = [](const std::string& d) { mkdir(d.c_str(), 0755); };
  auto put = [](const std::string& f, const std::string& v) {
    FILE* fp = std::fopen(f.c_str(), "w");
    std::fputs(v.c_str(), fp);
    std::fclose(fp);
  };
  mk(kfd);
  mk(proc);
  for (int pid = 100; pid < 108; ++pid) {
    const std::string kd = kfd + "/" + std::to_string(pid), pd = proc + "/" + std::to_string(pid);
    mk(kd);
    for (int g = 1; g <= 4; ++g) {
      put(kd + "/vram_" + std::to_string(g), std::to_string(g << 20) + "\n");
      mk(kd + "/stats_" + std::to_string(g));
      put(kd + "/stats_" + std::to_string(g) + "/cu_occupancy", std::to_string(pid % 7) + "\n");
    }
    mk(pd);
    mk(pd + "/fd");
    mk(pd + "/fdinfo");
    put(pd + "/comm", "proc" + std::to_string(pid) + "\n");
    for (int g = 1; g <= 4; ++g) {
      const std::string fd = std::to_string(10 + g);
      CHECK(symlink("/dev/dri/renderD128", (pd + "/fd/" + fd).c_str()) == 0);
      char bdf[32];
      std::snprintf(bdf, sizeof bdf, "0000:%02x:00.0", g);
      put(pd + "/fdinfo/" + fd, std::string("drm-client-id:\t") + fd + "\ndrm-pdev:\t" + bdf +
                                    "\ndrm-memory-gtt:\t4 KiB\ndrm-engine-gfx:\t100 ns\n");
    }
  }
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int g = 1; g <= 4; ++g)
    th.emplace_back([&, g] {
      char bdf[32];
      std::snprintf(bdf, sizeof bdf, "0000:%02x:00.0", g);
      DrmFdCache cache;  // one per thread, as one per GPU slow thread
      for (int it = 0; it < 50; ++it) {
        std::vector<ProcInfo> v;
        if (read_kfd_procs(kfd, proc, static_cast<uint64_t>(g), bdf, v, it % 2 ? &cache : nullptr, it * 1000000LL) != 0 ||
            v.size() != 8)
          ++bad;
        for (const ProcInfo& p : v)
          if (p.vram_bytes != (static_cast<uint64_t>(g) << 20) || p.gtt_bytes != 4096 || p.gfx_ns != 100 || !p.cu_valid)
            ++bad;
      }
    });
  for (auto& t : th) t.join();
  CHECK(bad.load() == 0);
  std::string cmd = "rm -rf " + r;
  CHECK(std::system(cmd.c_str()) == 0);
  std::printf("kfd procs concurrent ok\n");
}

// The parked tier's wake-up (kgs/unpark.h) on synthetic PMFW tables every 20 ms: a stray
// 0.2 ms blip (one table at 1 %) does not wake it, a table at ≥ 10 % does at once, a
// trickle of 2 % does within one 100 ms window, 0.5 % never, tables read during the
// 50 ms settle are skipped, and a PMFW that stops wakes it after `silent`.
static void test_unpark_detector() {
  const int64_t ms = 1000000;
  const int64_t silent = 1000 * ms;
  auto run = [&](auto pct_at, int64_t stop_at_ms, int64_t* woke_at_ms) {
    UnparkDetector u(kUnparkTablePct, kUnparkBusyPct, kUnparkWindowS);
    const int64_t park = 1000 * ms;
    u.parked(park);
    GpuSample g;
    double cum_gfx = 0, cum_dt = 10.0;
    bool have = false;
    for (int64_t t = park; t < park + 3000 * ms; t += 5 * ms) {
      const int64_t rel = (t - park) / ms;
      if (rel % 20 == 0 && rel < stop_at_ms) {  // a new table every 20 ms
        const double pct = pct_at(rel);
        cum_gfx += pct * 0.01 * 0.02;
        cum_dt += 0.02;
        g.mono_ns = t;
        g.gfx_busy_window_pct = static_cast<float>(pct);
        g.cum_gfx_s = cum_gfx;
        g.cum_dt_s = cum_dt;
        have = true;
      }
      int64_t busy = 0;
      if (u.poll(t, have ? &g : nullptr, silent, &busy)) {
        *woke_at_ms = rel;
        return busy;
      }
    }
    *woke_at_ms = -1;
    return int64_t{0};
  };
  int64_t at = 0;
  run([](int64_t r) { return r == 500 ? 1.0 : 0.0; }, 1 << 30, &at);
  CHECK(at == -1);                                       // one blip: stays parked
  const int64_t busy = run([](int64_t r) { return r >= 400 ? 60.0 : 0.0; }, 1 << 30, &at);
  CHECK(at == 400 && busy > 0);                          // a load: the first table wakes it
  run([](int64_t r) { return r >= 20 ? 2.0 : 0.0; }, 1 << 30, &at);
  CHECK(at > 0 && at <= 200);                            // a trickle: within a window or two
  run([](int64_t) { return 0.5; }, 1 << 30, &at);
  CHECK(at == -1);                                       // below 1 %: never
  run([](int64_t r) { return r < 50 ? 80.0 : 0.0; }, 1 << 30, &at);
  CHECK(at == -1);                                       // the park's own CP work: skipped
  run([](int64_t) { return 0.0; }, 500, &at);
  CHECK(at > 1480 && at <= 1490);                        // last table at 480 ms: silent 1 s later
}

int main() {
  test_unpark_detector();
  test_kfd_procs_concurrent();
  test_dispatch_estimator();
  test_cp_only_work_is_not_read_only();
  test_util_biller();
  test_tick_dither();
  test_lite_ib();
  test_batch_plan();
  test_reserve_slot();
  test_pmc_breaker();
  test_pmc_fault_boundary();
  test_http_server();
  test_exporter_concurrent();
  test_parser_fuzz();
  test_seqlock();
  test_ring();
  test_ring_lap();
  test_sampler();
  test_recovery();
  std::printf("ALL OK\n");
  return 0;
}
