// Which thread of a PMC-enabled exporter burns CPU?  Drives libkgs_pmc.so
// through its lifecycle (init = force_configure + hsa_init, open = start
// context, idle, 1 kHz sampling) and after each phase prints, per thread:
// name, CPU seconds used during the phase, scheduler state, and a histogram of
// /proc/self/task/<tid>/syscall samples ("running" = spinning in user space).
//   g++ -O2 -std=c++17 tools/pmc_threads.cpp -o build/pmc_threads -ldl -pthread
//   pmc_threads <libkgs_pmc.so> <kfd_gpu_id>
#include <dirent.h>
#include <dlfcn.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

using init_fn = int (*)(char*, int);
using open_fn = int (*)(uint64_t, const char* const*, const int*, int, char*, int);
using sample_fn = int (*)(int, uint64_t*, int, uint32_t*);

struct T {
  std::string comm;
  char state = '?';
  double cpu = 0;
};

static std::map<int, T> threads() {
  std::map<int, T> out;
  DIR* d = opendir("/proc/self/task");
  if (!d) return out;
  const double tck = static_cast<double>(sysconf(_SC_CLK_TCK));
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    const int tid = std::atoi(e->d_name);
    std::ifstream f(std::string("/proc/self/task/") + e->d_name + "/stat");
    std::string raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const size_t a = raw.find('('), b = raw.rfind(')');
    if (a == std::string::npos || b == std::string::npos) continue;
    T t;
    t.comm = raw.substr(a + 1, b - a - 1);
    std::istringstream rest(raw.substr(b + 2));
    std::vector<std::string> fl;
    std::string x;
    while (rest >> x) fl.push_back(x);
    if (fl.size() > 12) {
      t.state = fl[0][0];
      t.cpu = (std::atof(fl[11].c_str()) + std::atof(fl[12].c_str())) / tck;
    }
    out[tid] = t;
  }
  closedir(d);
  return out;
}

static std::string syscall_of(int tid) {
  std::ifstream f("/proc/self/task/" + std::to_string(tid) + "/syscall");
  std::string first;
  f >> first;
  return first.empty() ? "?" : first;
}

static void report(const char* phase, const std::map<int, T>& before, double secs, bool sample_syscalls) {
  std::map<int, std::map<std::string, int>> hist;
  if (sample_syscalls) {
    const int n = 40;
    for (int i = 0; i < n; ++i) {
      for (auto& kv : threads()) hist[kv.first][syscall_of(kv.first)]++;
      std::this_thread::sleep_for(std::chrono::duration<double>(secs / n));
    }
  } else {
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
  }
  const auto after = threads();
  std::printf("{\"phase\":\"%s\",\"threads\":[", phase);
  bool first = true;
  for (auto& kv : after) {
    auto it = before.find(kv.first);
    const double used = kv.second.cpu - (it == before.end() ? 0.0 : it->second.cpu);
    std::printf("%s{\"tid\":%d,\"comm\":\"%s\",\"state\":\"%c\",\"cpu_cores\":%.3f,\"new\":%s,\"syscalls\":{",
                first ? "" : ",", kv.first, kv.second.comm.c_str(), kv.second.state, used / secs,
                it == before.end() ? "true" : "false");
    bool f2 = true;
    for (auto& h : hist[kv.first]) {
      std::printf("%s\"%s\":%d", f2 ? "" : ",", h.first.c_str(), h.second);
      f2 = false;
    }
    std::printf("}}");
    first = false;
  }
  std::printf("]}\n");
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s libkgs_pmc.so kfd_gpu_id\n", argv[0]);
    return 2;
  }
  auto t0 = threads();
  void* lib = dlopen(argv[1], RTLD_NOW);
  if (!lib) {
    std::printf("{\"error\":\"dlopen %s\"}\n", dlerror());
    return 1;
  }
  auto init = reinterpret_cast<init_fn>(dlsym(lib, "kgs_pmc_init"));
  auto open = reinterpret_cast<open_fn>(dlsym(lib, "kgs_pmc_open"));
  auto sample = reinterpret_cast<sample_fn>(dlsym(lib, "kgs_pmc_sample"));
  char err[1024] = {};
  if (init(err, sizeof err) != 0) {
    std::printf("{\"error\":\"init: %s\"}\n", err);
    return 1;
  }
  report("after_init_idle_1s", t0, 1.0, true);
  auto t1 = threads();
  const char* names[] = {"GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"};
  const int is_max[] = {1, 1, 0};
  const int h = open(std::strtoull(argv[2], nullptr, 10), names, is_max, 3, err, sizeof err);
  if (h < 0) {
    std::printf("{\"error\":\"open: %s\"}\n", err);
    return 1;
  }
  report("after_open_idle_1s", t1, 1.0, true);
  auto t2 = threads();
  std::thread s([&] {
    uint64_t v[3];
    uint32_t ns;
    const auto end = std::chrono::steady_clock::now() + std::chrono::seconds(1);
    auto next = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() < end) {
      sample(h, v, 3, &ns);
      next += std::chrono::milliseconds(1);
      std::this_thread::sleep_until(next);
    }
  });
  report("sampling_1khz_1s", t2, 1.0, true);
  s.join();
  return 0;
}
