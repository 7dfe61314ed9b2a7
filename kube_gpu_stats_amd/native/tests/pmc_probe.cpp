// Diagnostic: drive libkgs_pmc.so directly with an arbitrary counter list and
// print per-interval rates + read latency as JSON lines (GPU box only).
//   pmc_probe <libkgs_pmc.so> <kfd_gpu_id> <seconds> <period_ms> NAME[:max] ...
#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using init_fn = int (*)(char*, int);
using open_fn = int (*)(uint64_t, const char* const*, const int*, int, char*, int);
using sample_fn = int (*)(int, uint64_t*, int, uint32_t*);
using info_fn = int (*)(int, char*, int);

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s lib gpu_id seconds period_ms NAME[:max]...\n", argv[0]);
    return 2;
  }
  void* lib = dlopen(argv[1], RTLD_NOW);
  if (!lib) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 1;
  }
  auto init = reinterpret_cast<init_fn>(dlsym(lib, "kgs_pmc_init"));
  auto open = reinterpret_cast<open_fn>(dlsym(lib, "kgs_pmc_open"));
  auto sample = reinterpret_cast<sample_fn>(dlsym(lib, "kgs_pmc_sample"));
  auto info = reinterpret_cast<info_fn>(dlsym(lib, "kgs_pmc_info"));
  char err[1024] = {};
  if (init(err, sizeof err) != 0) {
    std::printf("{\"error\":\"init: %s\"}\n", err);
    return 1;
  }
  const uint64_t gpu = std::strtoull(argv[2], nullptr, 10);
  const double secs = std::atof(argv[3]);
  const int period_ms = std::atoi(argv[4]);
  std::vector<std::string> names;
  std::vector<int> is_max;
  for (int i = 5; i < argc; ++i) {
    std::string s = argv[i];
    const size_t c = s.find(':');
    is_max.push_back(c != std::string::npos && s.substr(c + 1) == "max");
    names.push_back(c == std::string::npos ? s : s.substr(0, c));
  }
  std::vector<const char*> cn;
  for (auto& n : names) cn.push_back(n.c_str());
  const int h = open(gpu, cn.data(), is_max.data(), static_cast<int>(names.size()), err, sizeof err);
  if (h < 0) {
    std::printf("{\"error\":\"open: %s\"}\n", err);
    return 1;
  }
  char ib[2048] = {};
  info(h, ib, sizeof ib);
  std::printf("{\"info\":\"%s\"}\n", ib);
  std::vector<uint64_t> prev(names.size()), cur(names.size());
  uint32_t rns = 0;
  sample(h, prev.data(), static_cast<int>(names.size()), &rns);
  auto t_prev = std::chrono::steady_clock::now();
  const auto t_end = t_prev + std::chrono::duration<double>(secs);
  double lat_sum = 0;
  uint32_t lat_max = 0;
  int n = 0;
  while (std::chrono::steady_clock::now() < t_end) {
    std::this_thread::sleep_for(std::chrono::milliseconds(period_ms));
    if (sample(h, cur.data(), static_cast<int>(names.size()), &rns) != 0) {
      std::printf("{\"error\":\"sample failed\"}\n");
      continue;
    }
    ++n;
    lat_sum += rns;
    if (rns > lat_max) lat_max = rns;
    const auto now = std::chrono::steady_clock::now();
    const double dt = std::chrono::duration<double>(now - t_prev).count();
    const double wall = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    std::printf("{\"t\":%.3f,\"dt\":%.4f,\"read_us\":%.1f", wall, dt, rns * 1e-3);
    for (size_t k = 0; k < names.size(); ++k)
      std::printf(",\"%s\":%.4g", names[k].c_str(), (static_cast<double>(cur[k]) - static_cast<double>(prev[k])) / dt);
    std::printf("}\n");
    std::fflush(stdout);
    prev = cur;
    t_prev = now;
  }
  std::printf("{\"reads\":%d,\"read_us_mean\":%.1f,\"read_us_max\":%.1f}\n", n, n ? lat_sum / n * 1e-3 : 0.0,
              lat_max * 1e-3);
  return 0;
}
