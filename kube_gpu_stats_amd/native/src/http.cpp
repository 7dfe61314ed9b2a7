// epoll HTTP server.  See http.h.
#include "kgs/http.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>
#include <zlib.h>

#include <strings.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <unordered_map>

#include "kgs/exporter.h"

namespace kgs {

namespace {

struct Conn {
  std::string in;
  std::string out;
  size_t out_off = 0;
  bool close_after = false;
  bool loopback = false;  // peer is 127.0.0.0/8 or ::1: may use /control/*
  int64_t active_ns = 0;  // last byte received or sent (idle timeout, eviction order)
};

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

bool peer_is_loopback(const sockaddr_storage& a) {
  if (a.ss_family == AF_INET)
    return (ntohl(reinterpret_cast<const sockaddr_in&>(a).sin_addr.s_addr) >> 24) == 127;
  if (a.ss_family == AF_INET6) {
    const in6_addr& x = reinterpret_cast<const sockaddr_in6&>(a).sin6_addr;
    if (IN6_IS_ADDR_LOOPBACK(&x)) return true;
    return IN6_IS_ADDR_V4MAPPED(&x) && x.s6_addr[12] == 127;
  }
  return false;
}

double query_double(const std::string& q, const char* key, double dflt) {
  const std::string k = std::string(key) + "=";
  size_t p = 0;
  while ((p = q.find(k, p)) != std::string::npos) {
    if (p == 0 || q[p - 1] == '&') return std::strtod(q.c_str() + p + k.size(), nullptr);
    p += k.size();
  }
  return dflt;
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

int query_int(const std::string& q, const char* key, int dflt) {
  const std::string k = std::string(key) + "=";
  size_t p = 0;
  while ((p = q.find(k, p)) != std::string::npos) {
    if (p == 0 || q[p - 1] == '&' || q[p - 1] == '?') return std::atoi(q.c_str() + p + k.size());
    p += k.size();
  }
  return dflt;
}

uint64_t query_u64(const std::string& q, const char* key, uint64_t dflt) {
  const std::string k = std::string(key) + "=";
  size_t p = 0;
  while ((p = q.find(k, p)) != std::string::npos) {
    if (p == 0 || q[p - 1] == '&' || q[p - 1] == '?') return std::strtoull(q.c_str() + p + k.size(), nullptr, 10);
    p += k.size();
  }
  return dflt;
}

// Case-insensitive search for a header line `name:` whose value contains `token`.
bool header_has(const std::string& req, const char* name, const char* token) {
  const size_t nl = std::strlen(name);
  size_t p = req.find("\r\n");
  while (p != std::string::npos) {
    const size_t s = p + 2;
    const size_t e = req.find("\r\n", s);
    const size_t end = e == std::string::npos ? req.size() : e;
    if (end - s > nl && req[s + nl] == ':' && strncasecmp(req.c_str() + s, name, nl) == 0) {
      const std::string v = req.substr(s + nl + 1, end - s - nl - 1);
      if (v.find(token) != std::string::npos) return true;
    }
    p = e;
  }
  return false;
}

// One-shot gzip (RFC 1952) of `in` into `out`; reuses the deflate state across calls.
class Gzip {
 public:
  ~Gzip() {
    if (init_) deflateEnd(&z_);
  }
  bool compress(const std::string& in, std::string& out, int level) {
    if (!init_ || level != level_) {
      if (init_) deflateEnd(&z_);
      z_ = z_stream{};
      init_ = deflateInit2(&z_, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) == Z_OK;
      level_ = level;
      if (!init_) return false;
    } else if (deflateReset(&z_) != Z_OK) {
      return false;
    }
    out.resize(deflateBound(&z_, in.size()) + 64);
    z_.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
    z_.avail_in = static_cast<uInt>(in.size());
    z_.next_out = reinterpret_cast<Bytef*>(&out[0]);
    z_.avail_out = static_cast<uInt>(out.size());
    const int rc = deflate(&z_, Z_FINISH);
    out.resize(z_.total_out);
    return rc == Z_STREAM_END;
  }

 private:
  z_stream z_{};
  bool init_ = false;
  int level_ = -1;
};

void respond(Conn& c, int code, const char* reason, const char* ctype, const std::string& body,
             const char* encoding = nullptr) {
  c.out.clear();
  c.out_off = 0;
  c.out.reserve(body.size() + 256);
  c.out += "HTTP/1.1 ";
  c.out += std::to_string(code);
  c.out += ' ';
  c.out += reason;
  c.out += "\r\nContent-Type: ";
  c.out += ctype;
  if (encoding) {
    c.out += "\r\nContent-Encoding: ";
    c.out += encoding;
    c.out += "\r\nVary: Accept-Encoding";
  }
  c.out += "\r\nContent-Length: ";
  c.out += std::to_string(body.size());
  c.out += c.close_after ? "\r\nConnection: close\r\n\r\n" : "\r\nConnection: keep-alive\r\n\r\n";
  c.out += body;
}

}  // namespace

HttpServer::HttpServer(Exporter* ex, std::string addr, int port) : ex_(ex), addr_(std::move(addr)), port_(port) {}
HttpServer::~HttpServer() { stop(); }

bool HttpServer::start(std::string& err) {
  lfd_ = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) { err = "socket: " + std::string(strerror(errno)); return false; }
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(port_));
  if (inet_pton(AF_INET, addr_.c_str(), &sa.sin_addr) != 1) sa.sin_addr.s_addr = htonl(INADDR_ANY);
  if (bind(lfd_, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
    err = "bind " + addr_ + ":" + std::to_string(port_) + ": " + strerror(errno);
    close(lfd_);
    lfd_ = -1;
    return false;
  }
  socklen_t sl = sizeof sa;
  getsockname(lfd_, reinterpret_cast<sockaddr*>(&sa), &sl);
  port_ = ntohs(sa.sin_port);
  listen(lfd_, 128);
  set_nonblock(lfd_);
  efd_ = epoll_create1(EPOLL_CLOEXEC);
  wake_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd_;
  epoll_ctl(efd_, EPOLL_CTL_ADD, lfd_, &ev);
  ev.data.fd = wake_fd_;
  epoll_ctl(efd_, EPOLL_CTL_ADD, wake_fd_, &ev);
  stop_.store(false);
  th_ = std::thread([this] { loop(); });
  return true;
}

void HttpServer::stop() {
  if (!th_.joinable()) return;
  stop_.store(true);
  uint64_t one = 1;
  if (write(wake_fd_, &one, sizeof one) < 0) {}
  th_.join();
  if (lfd_ >= 0) close(lfd_);
  if (efd_ >= 0) close(efd_);
  if (wake_fd_ >= 0) close(wake_fd_);
  lfd_ = efd_ = wake_fd_ = -1;
}

void HttpServer::loop() {
  pthread_setname_np(pthread_self(), "kgs-http");
  std::unordered_map<int, Conn> conns;
  std::string body, zbody;
  Gzip gz;
  epoll_event evs[64];
  auto drop = [&](int fd) {
    epoll_ctl(efd_, EPOLL_CTL_DEL, fd, nullptr);
    close(fd);
    conns.erase(fd);
    ex_->http_conns_open.store(conns.size(), std::memory_order_relaxed);
  };
  const ExporterConfig& cfg = ex_->config();
  const int64_t idle_ns = cfg.http_idle_s > 0 ? static_cast<int64_t>(cfg.http_idle_s * 1e9) : 0;
  const size_t max_conns = cfg.http_max_conns > 0 ? static_cast<size_t>(cfg.http_max_conns) : 0;
  int64_t next_sweep = mono_ns();
  auto flush = [&](int fd, Conn& c) -> bool {  // false = connection gone
    while (c.out_off < c.out.size()) {
      const ssize_t n = send(fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (n > 0) { c.out_off += static_cast<size_t>(n); c.active_ns = mono_ns(); continue; }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLOUT;
        ev.data.fd = fd;
        epoll_ctl(efd_, EPOLL_CTL_MOD, fd, &ev);
        return true;
      }
      drop(fd);
      return false;
    }
    c.out.clear();
    c.out_off = 0;
    if (c.close_after) { drop(fd); return false; }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = fd;
    epoll_ctl(efd_, EPOLL_CTL_MOD, fd, &ev);
    return true;
  };

  while (!stop_.load()) {
    const int n = epoll_wait(efd_, evs, 64, 500);
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == wake_fd_) continue;
      if (fd == lfd_) {
        for (;;) {
          sockaddr_storage peer{};
          socklen_t plen = sizeof peer;
          const int c = accept4(lfd_, reinterpret_cast<sockaddr*>(&peer), &plen, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (c < 0) break;
          if (max_conns > 0 && conns.size() >= max_conns) {  // evict the least recently active
            auto lru = conns.begin();
            for (auto jt = conns.begin(); jt != conns.end(); ++jt)
              if (jt->second.active_ns < lru->second.active_ns) lru = jt;
            drop(lru->first);
            ex_->http_closed_limit.fetch_add(1, std::memory_order_relaxed);
          }
          int one = 1;
          setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.fd = c;
          epoll_ctl(efd_, EPOLL_CTL_ADD, c, &ev);
          Conn& nc = conns[c];
          nc.loopback = peer_is_loopback(peer);
          nc.active_ns = mono_ns();
          ex_->http_conns_open.store(conns.size(), std::memory_order_relaxed);
        }
        continue;
      }
      auto it = conns.find(fd);
      // Dropped earlier in this batch (evicted): its fd is closed and off the epoll
      // set already, and the number may belong to a newer connection or file.
      if (it == conns.end()) continue;
      Conn& c = it->second;
      if (evs[i].events & EPOLLOUT) {
        if (!flush(fd, c)) continue;
        if (!c.out.empty()) continue;
      }
      if (!(evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR))) continue;
      char buf[4096];
      bool gone = false;
      for (;;) {
        const ssize_t r = recv(fd, buf, sizeof buf, 0);
        if (r > 0) { c.active_ns = mono_ns(); c.in.append(buf, static_cast<size_t>(r)); if (c.in.size() > (1u << 16)) { gone = true; break; } continue; }
        if (r == 0) { gone = true; break; }
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        gone = true;
        break;
      }
      // Serve every complete request in the buffer (pipelining-safe).
      size_t hdr_end;
      while (!gone && c.out.empty() && (hdr_end = c.in.find("\r\n\r\n")) != std::string::npos) {
        const std::string req = c.in.substr(0, hdr_end);
        c.in.erase(0, hdr_end + 4);
        ex_->http_requests.fetch_add(1);
        const size_t sp1 = req.find(' ');
        const size_t sp2 = sp1 == std::string::npos ? std::string::npos : req.find(' ', sp1 + 1);
        const std::string method = req.substr(0, sp1);
        std::string target = sp1 == std::string::npos ? "/" : req.substr(sp1 + 1, sp2 - sp1 - 1);
        std::string query;
        const size_t q = target.find('?');
        if (q != std::string::npos) { query = target.substr(q + 1); target.resize(q); }
        const bool http10 = req.find("HTTP/1.0") != std::string::npos;
        const bool conn_close = header_has(req, "Connection", "close");
        c.close_after = conn_close || (http10 && req.find("eep-Alive") == std::string::npos);
        if (method != "GET" && method != "HEAD") {
          respond(c, 405, "Method Not Allowed", "text/plain", "only GET\n");
        } else if (target == "/metrics") {
          ex_->render(body);
          const int lvl = ex_->config().gzip_level;
          if (lvl > 0 && header_has(req, "Accept-Encoding", "gzip") && gz.compress(body, zbody, lvl))
            respond(c, 200, "OK", "text/plain; version=0.0.4; charset=utf-8", zbody, "gzip");
          else
            respond(c, 200, "OK", "text/plain; version=0.0.4; charset=utf-8", body);
        } else if (target.compare(0, 9, "/control/") == 0 && !c.loopback) {
          // Control is for processes on the exporter's own host / pod network
          // namespace (`kubectl exec <pod> -- kgs pmc release`), never for scrapers.
          respond(c, 403, "Forbidden", "text/plain", "control endpoints are loopback-only\n");
        } else if (target == "/control/pmc/release" || target == "/control/pmc/acquire") {
          // ?gpu=N: that device only (its own sampler thread acts; a hung GPU delays nobody).
          const int gpu = query_int(query, "gpu", -1);
          Sampler* s = ex_->sampler();
          if (gpu >= 0 && (!s || gpu >= s->device_count())) {
            respond(c, 400, "Bad Request", "text/plain", "gpu out of range\n");
          } else {
            const bool on = target == "/control/pmc/acquire";
            // drop_queue=1 (release): destroy the READ queue as well (benchmarks'
            // "released" condition: nothing of the counter tier left on the GPU).
            ex_->set_pmc_enabled(on, gpu, query_int(query, "drop_queue", 0) != 0);
            std::string j = gpu >= 0 ? "{\"gpu\":" + std::to_string(gpu) + ",\"pmc\":" + (on ? "true" : "false") + "}"
                                     : std::string(ex_->pmc_enabled() ? "{\"pmc\":true}" : "{\"pmc\":false}");
            respond(c, 200, "OK", "application/json", j);
          }
        } else if (target == "/control/pmc/idle") {
          // Quiet-GPU counter READ rate (--pmc-idle-hz); hz=0 = READ every tick (profiling
          // mode); hz < 0 (or none) only reads the setting.  Out of range → 400.
          Sampler* s = ex_->sampler();
          const double hz = query_double(query, "hz", -1.0);
          if (s && hz >= 0 && !s->set_pmc_idle_hz(hz)) {
            respond(c, 400, "Bad Request", "text/plain", "hz must be 0 or within [0.01, 100000]\n");
          } else {
            respond(c, 200, "OK", "application/json",
                    "{\"pmc_idle_hz\":" + std::to_string(s ? s->pmc_idle_hz() : 0.0) + "}");
          }
        } else if (target == "/control/pmc/dispatch") {
          // Dispatch-bound READ rate (--pmc-dispatch-hz); no hz only reads the setting.
          // Out of range → 400.
          Sampler* s = ex_->sampler();
          const double hz = query_double(query, "hz", -1.0);
          if (s && hz != -1.0 && !s->set_pmc_dispatch_hz(hz)) {
            respond(c, 400, "Bad Request", "text/plain", "hz must be within (0, 100000]\n");
          } else {
            respond(c, 200, "OK", "application/json",
                    "{\"pmc_dispatch_hz\":" + std::to_string(s ? s->pmc_dispatch_hz() : 0.0) + "}");
          }
        } else if (target == "/control/pmc/quiet_release") {
          // Quiet-release delay (--pmc-quiet-release-s); s=0 never parks; no s only reads it.
          Sampler* s = ex_->sampler();
          const double v = query_double(query, "s", -1.0);
          if (s && v != -1.0 && !s->set_pmc_quiet_release_s(v)) {
            respond(c, 400, "Bad Request", "text/plain", "s must be within [0, 86400]\n");
          } else {
            respond(c, 200, "OK", "application/json",
                    "{\"pmc_quiet_release_s\":" + std::to_string(s ? s->pmc_quiet_release_s() : 0.0) + "}");
          }
        } else if (ex_->config().control_http && (target == "/control/pause" || target == "/control/resume")) {
          if (target == "/control/pause") ex_->pause_sampling();
          else ex_->resume_sampling();
          respond(c, 200, "OK", "application/json", ex_->sampling() ? "{\"sampling\":true}" : "{\"sampling\":false}");
        } else if (ex_->config().control_http && target == "/control/rate") {
          // Benchmarks: switch the tick rate in place (one exporter serves every tier).
          const double hz = query_double(query, "hz", -1.0);
          if (hz != -1.0 && !ex_->set_sample_rate(hz))
            respond(c, 400, "Bad Request", "text/plain", "hz must be within (0, 100000]\n");
          else
            respond(c, 200, "OK", "application/json", "{\"hz\":" + std::to_string(ex_->sample_rate()) + "}");
        } else if (ex_->config().control_http && target == "/control/pmc/stall") {
          // Benchmarks / hardware tests only: wedge one GPU's counter READ queue (a
          // never-completing packet at its head) so the circuit breaker must trip and
          // recreate the queue (Sampler::inject_pmc_stall).
          const int gpu = query_int(query, "gpu", -1);
          Sampler* s = ex_->sampler();
          if (!s || gpu < 0 || gpu >= s->device_count() || !s->inject_pmc_stall(gpu))
            respond(c, 400, "Bad Request", "text/plain", "gpu out of range or no counter tier\n");
          else
            respond(c, 200, "OK", "application/json", "{\"gpu\":" + std::to_string(gpu) + ",\"stall\":true}");
        } else if (ex_->config().control_http && target == "/control/mock/xgmi") {
          // Benchmarks on the mock provider (bench.py --mock phase X): account a peer copy
          // on the xGMI link between two mock GPUs.  Other backends: 404.
          const int src = query_int(query, "src", -1), dst = query_int(query, "dst", -1);
          const uint64_t bytes = query_u64(query, "bytes", 0);
          if (ex_->backend()->inject_xgmi(src, dst, bytes) == 0)
            respond(c, 200, "OK", "application/json", "{\"injected\":" + std::to_string(bytes) + "}");
          else
            respond(c, 404, "Not Found", "text/plain", "xGMI injection needs the mock backend and two GPUs\n");
        } else if (target == "/healthz") {
          const bool ok = ex_->healthy();
          respond(c, ok ? 200 : 503, ok ? "OK" : "Service Unavailable", "text/plain", ok ? "ok\n" : "no device sampled\n");
        } else if (target == "/topology") {
          respond(c, 200, "OK", "application/json", ex_->topology_json());
        } else if (target == "/devices") {
          respond(c, 200, "OK", "application/json", ex_->devices_json());
        } else if (target == "/samples") {
          respond(c, 200, "OK", "application/json",
                  ex_->samples_json(query_int(query, "gpu", 0), query_int(query, "n", 100)));
        } else if (target == "/counters") {
          respond(c, 200, "OK", "application/json",
                  ex_->counters_json(query_int(query, "gpu", 0), query_int(query, "n", 100),
                                     query_u64(query, "since", 0)));
        } else if (target == "/") {
          respond(c, 200, "OK", "text/html",
                  "<html><body><h1>kube_gpu_stats_amd exporter</h1><a href=\"/metrics\">/metrics</a> "
                  "<a href=\"/topology\">/topology</a> <a href=\"/devices\">/devices</a> "
                  "<a href=\"/samples\">/samples</a> <a href=\"/counters\">/counters</a></body></html>\n");
        } else {
          respond(c, 404, "Not Found", "text/plain", "not found\n");
        }
        if (method == "HEAD") {
          const size_t he = c.out.find("\r\n\r\n");
          if (he != std::string::npos) c.out.resize(he + 4);
        }
        if (!flush(fd, c)) { gone = true; break; }
      }
      if (gone && conns.count(fd)) drop(fd);
    }
    // Idle sweep after the batch (at most twice a second, O(connections)), so no
    // event of this batch refers to a connection closed under it.
    const int64_t now = mono_ns();
    if (idle_ns > 0 && now >= next_sweep) {
      next_sweep = now + 500000000LL;
      std::vector<int> idle;
      for (const auto& kvp : conns)
        if (now - kvp.second.active_ns >= idle_ns) idle.push_back(kvp.first);
      for (int fd : idle) {
        drop(fd);
        ex_->http_closed_idle.fetch_add(1, std::memory_order_relaxed);
      }
    }
  }
  for (auto& kvp : conns) close(kvp.first);
  ex_->http_conns_open.store(0, std::memory_order_relaxed);
}

}  // namespace kgs
