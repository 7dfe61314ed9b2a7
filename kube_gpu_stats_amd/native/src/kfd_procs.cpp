// Per-process GPU use from the KFD sysfs + DRM fdinfo (see include/kgs/kfd_procs.h).
#include "kgs/kfd_procs.h"

#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <set>

namespace kgs {

namespace {

// Whole small file into buf (NUL-terminated); false if it cannot be read.
bool slurp(const std::string& path, char* buf, size_t cap, size_t* len = nullptr) {
  const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  size_t n = 0;
  while (n + 1 < cap) {
    const ssize_t r = read(fd, buf + n, cap - 1 - n);
    if (r <= 0) break;
    n += static_cast<size_t>(r);
  }
  close(fd);
  buf[n] = 0;
  if (len) *len = n;
  return true;
}

bool read_u64(const std::string& path, uint64_t& v) {
  char buf[64];
  if (!slurp(path, buf, sizeof buf)) return false;
  char* end = nullptr;
  const unsigned long long x = std::strtoull(buf, &end, 10);
  if (end == buf) return false;
  v = x;
  return true;
}

bool all_digits(const char* s) {
  if (!*s) return false;
  for (; *s; ++s)
    if (*s < '0' || *s > '9') return false;
  return true;
}

// "1464 KiB" / "12 MiB" / "7 GiB" / "15483 ns" → the number scaled to bytes (ns as is).
uint64_t scaled(const char* v) {
  while (*v == ' ' || *v == '\t') ++v;
  char* end = nullptr;
  const unsigned long long x = std::strtoull(v, &end, 10);
  while (*end == ' ') ++end;
  if (!std::strncmp(end, "KiB", 3)) return x << 10;
  if (!std::strncmp(end, "MiB", 3)) return x << 20;
  if (!std::strncmp(end, "GiB", 3)) return x << 30;
  return x;
}

bool is_drm_fd(const std::string& fd_path) {
  char link[256];
  const ssize_t n = readlink(fd_path.c_str(), link, sizeof link - 1);
  if (n <= 0) return false;
  link[n] = 0;
  return std::strncmp(link, "/dev/dri/", 9) == 0;
}

// The DRM fds of `pid` (names under /proc/<pid>/fd): the cached list while it is fresh
// and every fd in it still a DRM link, else a full walk (kgs/kfd_procs.h DrmFdCache).
std::vector<std::string> drm_fds(const std::string& fd_dir, uint32_t pid, DrmFdCache* cache, int64_t now_ns) {
  if (cache) {
    auto it = cache->by_pid.find(pid);
    if (it != cache->by_pid.end() && now_ns - it->second.scan_ns < kDrmRescanNs) {
      bool ok = true;
      for (const std::string& fd : it->second.fds) ok = ok && is_drm_fd(fd_dir + "/" + fd);
      if (ok) return it->second.fds;
    }
  }
  std::vector<std::string> fds;
  DIR* d = opendir(fd_dir.c_str());
  if (!d) return fds;
  while (dirent* e = readdir(d))
    if (all_digits(e->d_name) && is_drm_fd(fd_dir + "/" + e->d_name)) fds.emplace_back(e->d_name);
  closedir(d);
  if (cache) {
    ++cache->walks;
    cache->by_pid[pid] = DrmFdCache::Ent{fds, now_ns};
  }
  return fds;
}

// The DRM clients of `pid` on the render node at `bdf`: Σ GTT / CPU bytes and gfx
// engine ns over distinct drm-client-ids (dup'd fds share one client).
void drm_fdinfo(const std::string& proc_root, uint32_t pid, const std::string& bdf, ProcInfo& p, DrmFdCache* cache,
                int64_t now_ns) {
  const std::string pid_dir = proc_root + "/" + std::to_string(pid);
  std::set<uint64_t> seen;
  char buf[4096];
  for (const std::string& fd : drm_fds(pid_dir + "/fd", pid, cache, now_ns)) {
    if (!slurp(pid_dir + "/fdinfo/" + fd, buf, sizeof buf)) continue;
    bool ours = false;
    uint64_t client = ~0ull, gtt = 0, cpu = 0, gfx = 0;
    char* save = nullptr;  // strtok_r: one slow thread per GPU runs this at once
    for (char* line = strtok_r(buf, "\n", &save); line; line = strtok_r(nullptr, "\n", &save)) {
      char* colon = std::strchr(line, ':');
      if (!colon) continue;
      *colon = 0;
      const char* key = line;
      const char* val = colon + 1;
      while (*val == ' ' || *val == '\t') ++val;
      if (!std::strcmp(key, "drm-pdev")) ours = bdf == val;
      else if (!std::strcmp(key, "drm-client-id")) client = std::strtoull(val, nullptr, 10);
      else if (!std::strcmp(key, "drm-memory-gtt") || !std::strcmp(key, "drm-total-gtt")) gtt = scaled(val);
      else if (!std::strcmp(key, "drm-memory-cpu") || !std::strcmp(key, "drm-total-cpu")) cpu = scaled(val);
      else if (!std::strcmp(key, "drm-engine-gfx")) gfx = scaled(val);
    }
    if (!ours || !seen.insert(client).second) continue;
    p.gtt_bytes += gtt;
    p.cpu_bytes += cpu;
    p.gfx_ns += gfx;
  }
}

}  // namespace

int read_kfd_procs(const std::string& kfd_root, const std::string& proc_root, uint64_t gpu_id,
                   const std::string& bdf, std::vector<ProcInfo>& out, DrmFdCache* cache, int64_t now_ns) {
  out.clear();
  DIR* d = opendir(kfd_root.c_str());
  if (!d) return -1;
  const std::string gid = std::to_string(gpu_id);
  std::vector<uint32_t> pids;
  while (dirent* e = readdir(d))
    if (all_digits(e->d_name)) pids.push_back(static_cast<uint32_t>(std::strtoul(e->d_name, nullptr, 10)));
  closedir(d);
  for (uint32_t pid : pids) {
    const std::string base = kfd_root + "/" + std::to_string(pid) + "/";
    ProcInfo p;
    // A process with a KFD context on this GPU has a vram_<gpu_id> file; one that exited
    // since the listing has none (skipped, as AMD SMI's list would not hold it either).
    if (!read_u64(base + "vram_" + gid, p.vram_bytes)) continue;
    p.pid = pid;
    uint64_t cu = 0, ev = 0;
    // The CU occupancy of a process whose stats directory is unreadable (tearing down,
    // a KFD without it) is unknown, not 0: the sampler neither integrates nor exports it.
    p.cu_valid = read_u64(base + "stats_" + gid + "/cu_occupancy", cu);
    p.cu_occupancy = p.cu_valid ? static_cast<uint32_t>(cu) : 0;
    if (read_u64(base + "stats_" + gid + "/evicted_ms", ev)) p.evicted_ms = static_cast<uint32_t>(ev);
    char comm[64];
    size_t n = 0;
    if (slurp(proc_root + "/" + std::to_string(pid) + "/comm", comm, sizeof comm, &n)) {
      while (n > 0 && (comm[n - 1] == '\n' || comm[n - 1] == 0)) --n;
      p.name.assign(comm, n);
    }
    drm_fdinfo(proc_root, pid, bdf, p, cache, now_ns);
    out.push_back(std::move(p));
  }
  if (cache)  // forget the processes that left this GPU
    for (auto it = cache->by_pid.begin(); it != cache->by_pid.end();) {
      bool here = false;
      for (const ProcInfo& q : out) here = here || q.pid == it->first;
      it = here ? std::next(it) : cache->by_pid.erase(it);
    }
  return 0;
}

}  // namespace kgs
