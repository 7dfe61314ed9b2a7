// Minimal single-threaded epoll HTTP/1.1 server for /metrics (keep-alive,
// no allocation per request beyond the response buffer).  Endpoints:
//   GET /metrics            Prometheus text format 0.0.4
//   GET /healthz            200 if any GPU is being sampled, else 503
//   GET /topology           JSON: devices, pairwise edges, per-link peers
//   GET /devices            JSON device inventory
//   GET /samples?gpu=N&n=K  JSON: the K most recent distinct samples of GPU N
#pragma once

#include <atomic>
#include <string>
#include <thread>

namespace kgs {

class Exporter;

class HttpServer {
 public:
  HttpServer(Exporter* ex, std::string addr, int port);
  ~HttpServer();
  bool start(std::string& err);
  void stop();
  int port() const { return port_; }

 private:
  void loop();
  Exporter* ex_;
  std::string addr_;
  int port_;
  int lfd_ = -1, efd_ = -1, wake_fd_ = -1;
  std::thread th_;
  std::atomic<bool> stop_{false};
};

}  // namespace kgs
