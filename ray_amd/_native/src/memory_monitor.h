// Node memory monitor: see memory_monitor.cc.
#pragma once
#include <stdint.h>

#include <string>

namespace ray_amd {

struct MemorySnapshot {
  uint64_t used = 0, total = 0;
  std::string source;
};

class MemoryMonitor {
 public:
  MemoryMonitor(double threshold, int64_t min_free_bytes, std::string cgroup_root = "/sys/fs/cgroup",
                std::string proc_root = "/proc")
      : threshold_(threshold),
        min_free_bytes_(min_free_bytes),
        cgroup_root_(std::move(cgroup_root)),
        proc_root_(std::move(proc_root)) {}
  MemorySnapshot snapshot() const;
  int64_t process_private_bytes(int pid) const;
  bool over_threshold(const MemorySnapshot& s) const;
  double threshold() const { return threshold_; }

 private:
  double threshold_;
  int64_t min_free_bytes_;
  std::string cgroup_root_, proc_root_;
};

}  // namespace ray_amd
