// Which thread of a PMC-enabled exporter burns CPU?  Drives libkgs_pmc.so
// through its lifecycle (init = force_configure + hsa_init, open = start
// context, idle, 1 kHz sampling) and after each phase prints, per thread:
// name, CPU seconds used during the phase, scheduler state, and a histogram of
// /proc/self/task/<tid>/syscall samples ("running" = spinning in user space).
//   g++ -O2 -std=c++17 tools/pmc_threads.cpp -o build/pmc_threads -ldl -pthread
//   pmc_threads <libkgs_pmc.so> <kfd_gpu_id>
#include <dirent.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <sched.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
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

// SIGUSR2: dump the receiving thread's user-space stack (diagnostic only).
static void on_usr2(int) {
  void* fr[32];
  const int n = backtrace(fr, 32);
  const char hdr[] = "--- backtrace\n";
  if (write(2, hdr, sizeof hdr - 1) < 0) {
  }
  backtrace_symbols_fd(fr, n, 2);
}

static int hottest(const std::map<int, T>& a, const std::map<int, T>& b) {
  int best = -1;
  double bu = 0.2;
  for (auto& kv : b) {
    auto it = a.find(kv.first);
    const double u = kv.second.cpu - (it == a.end() ? 0.0 : it->second.cpu);
    if (u > bu && kv.first != static_cast<int>(getpid())) {
      bu = u;
      best = kv.first;
    }
  }
  return best;
}

static void on_segv(int sig) {
  void* fr[48];
  const int n = backtrace(fr, 48);
  const char hdr[] = "--- SIGSEGV backtrace\n";
  if (write(2, hdr, sizeof hdr - 1) < 0) {
  }
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int main(int argc, char** argv) {
  signal(SIGUSR2, on_usr2);
  signal(SIGSEGV, on_segv);
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
  // optional counter list after the gpu id: NAME[:max|:mean] ...  (default: the first three of the exporter's)
  std::vector<std::string> nm = {"GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"};
  std::vector<int> red = {1, 1, 0};
  if (argc > 3) {
    nm.clear();
    red.clear();
    for (int i = 3; i < argc; ++i) {
      std::string a = argv[i];
      const size_t c = a.find(':');
      const std::string r = c == std::string::npos ? "" : a.substr(c + 1);
      nm.push_back(c == std::string::npos ? a : a.substr(0, c));
      red.push_back(r == "max" ? 1 : r == "mean" ? 2 : 0);
    }
  }
  std::vector<const char*> names;
  for (auto& x : nm) names.push_back(x.c_str());
  const int nc = static_cast<int>(names.size());
  const int h = open(std::strtoull(argv[2], nullptr, 10), names.data(), red.data(), nc, err, sizeof err);
  if (h < 0) {
    std::printf("{\"error\":\"open: %s\"}\n", err);
    return 1;
  }
  report("after_open_idle_1s", t1, 1.0, true);
  auto t2 = threads();
  {  // locate the spinner, sample its stack, optionally demote it
    auto a = threads();
    std::this_thread::sleep_for(std::chrono::milliseconds(300));
    const int spin = hottest(a, threads());
    std::printf("{\"spinner_tid\":%d}\n", spin);
    std::fflush(stdout);
    if (spin > 0) {
      for (int i = 0; i < 4; ++i) {
        syscall(SYS_tgkill, getpid(), spin, SIGUSR2);
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
      }
      if (std::getenv("KGS_PROBE_SCHED_IDLE")) {
        sched_param sp{};
        const int rc = sched_setscheduler(spin, SCHED_IDLE, &sp);
        std::printf("{\"sched_idle_rc\":%d}\n", rc);
      }
    }
    t2 = threads();
  }
  std::vector<double> lat_us;
  uint64_t first[16] = {}, last[16] = {};
  int rc_bad = 0;
  std::thread s([&] {
    uint64_t v[16];
    uint32_t ns;
    if (sample(h, first, nc, &ns) != 0) ++rc_bad;
    const auto end = std::chrono::steady_clock::now() + std::chrono::seconds(1);
    auto next = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() < end) {
      if (sample(h, v, nc, &ns) != 0) ++rc_bad;
      else std::memcpy(last, v, sizeof v);
      lat_us.push_back(ns * 1e-3);
      next += std::chrono::milliseconds(1);
      std::this_thread::sleep_until(next);
    }
  });
  report("sampling_1khz_1s", t2, 1.0, true);
  s.join();
  std::sort(lat_us.begin(), lat_us.end());
  if (!lat_us.empty())
  {
    std::printf("{\"samples\":%zu,\"errors\":%d,\"read_us_p50\":%.1f,\"read_us_p99\":%.1f,\"delta\":{",
                lat_us.size(), rc_bad, lat_us[lat_us.size() / 2], lat_us[lat_us.size() * 99 / 100]);
    for (int k = 0; k < nc; ++k)
      std::printf("%s\"%s\":%llu", k ? "," : "", nm[static_cast<size_t>(k)].c_str(),
                  static_cast<unsigned long long>(last[k] - first[k]));
    std::printf("}}\n");
  }
  return 0;
}
