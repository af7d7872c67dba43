// Node memory monitor (reference behaviour: src/ray/common/memory_monitor.cc —
// periodically snapshot used/total memory of the node or of its cgroup and per-process
// usage, and report when usage crosses a threshold so the raylet can kill a worker).
//
// Design: a plain reader the raylet calls from its own tick (no extra thread): cgroup v2
// (memory.max / memory.current, minus inactive_file) or cgroup v1 when a limit is set,
// /proc/meminfo (MemTotal - MemAvailable) otherwise; per-process usage is the PRIVATE
// resident set (statm resident - shared), so the /dev/shm object-store segment every
// worker maps is not charged to each of them.
#include "memory_monitor.h"

#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <fstream>
#include <sstream>

namespace ray_amd {

static bool read_u64(const std::string& path, uint64_t* out) {
  std::ifstream f(path);
  if (!f) return false;
  std::string s;
  f >> s;
  if (s.empty() || s == "max") return false;
  try {
    *out = std::stoull(s);
  } catch (...) {
    return false;
  }
  return true;
}

static uint64_t stat_field(const std::string& path, const char* key) {
  std::ifstream f(path);
  std::string k;
  uint64_t v;
  while (f >> k >> v)
    if (k == key) return v;
  return 0;
}

MemorySnapshot MemoryMonitor::snapshot() const {
  MemorySnapshot s;
  uint64_t lim = 0, cur = 0;
  // cgroup v2
  if (read_u64(cgroup_root_ + "/memory.max", &lim) &&
      read_u64(cgroup_root_ + "/memory.current", &cur) && lim < (1ull << 60)) {
    const uint64_t inactive = stat_field(cgroup_root_ + "/memory.stat", "inactive_file");
    s.total = lim;
    s.used = cur > inactive ? cur - inactive : cur;
    s.source = "cgroup2";
    return s;
  }
  // cgroup v1
  if (read_u64(cgroup_root_ + "/memory/memory.limit_in_bytes", &lim) &&
      read_u64(cgroup_root_ + "/memory/memory.usage_in_bytes", &cur) && lim < (1ull << 60)) {
    const uint64_t inactive =
        stat_field(cgroup_root_ + "/memory/memory.stat", "total_inactive_file");
    s.total = lim;
    s.used = cur > inactive ? cur - inactive : cur;
    s.source = "cgroup1";
    return s;
  }
  std::ifstream f(proc_root_ + "/meminfo");
  std::string line;
  uint64_t total = 0, avail = 0;
  while (std::getline(f, line)) {
    unsigned long long v;
    if (sscanf(line.c_str(), "MemTotal: %llu kB", &v) == 1) total = v * 1024;
    if (sscanf(line.c_str(), "MemAvailable: %llu kB", &v) == 1) avail = v * 1024;
  }
  s.total = total;
  s.used = total > avail ? total - avail : 0;
  s.source = "meminfo";
  return s;
}

int64_t MemoryMonitor::process_private_bytes(int pid) const {
  std::ifstream f(proc_root_ + "/" + std::to_string(pid) + "/statm");
  uint64_t size, resident, shared;
  if (!(f >> size >> resident >> shared)) return -1;
  const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  return (int64_t)((resident > shared ? resident - shared : 0) * page);
}

bool MemoryMonitor::over_threshold(const MemorySnapshot& s) const {
  if (s.total == 0) return false;
  // usage threshold, optionally relaxed on big hosts by an absolute free-bytes floor:
  // the effective limit is max(threshold * total, total - min_free_bytes)
  double limit = threshold_ * (double)s.total;
  if (min_free_bytes_ >= 0) {
    const double alt = (double)s.total - (double)min_free_bytes_;
    if (alt > limit) limit = alt;
  }
  return (double)s.used > limit;
}

}  // namespace ray_amd
