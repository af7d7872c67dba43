// Cluster resource scheduler (raylet/GCS scheduling core) for ray_amd.
//
// Reference behaviour: src/ray/raylet/scheduling/{cluster_resource_scheduler.cc,
// policy/hybrid_scheduling_policy.cc, policy/spread_scheduling_policy.cc,
// policy/node_affinity_scheduling_policy.cc, policy/bundle_scheduling_policy.cc}
// and src/ray/common/scheduling/resource_instance_set.cc.
//
//  * resources are fixed-point (1e-4 granularity), so 0.5 GPU / 0.25 CPU are exact
//  * unit-instance resources ("GPU" and its placement-group variants) are tracked per
//    device so a lease gets concrete GPU indices (→ HIP_VISIBLE_DEVICES)
//  * policies: HYBRID (pack locally until `spread_threshold` utilisation, then
//    least-utilised node), SPREAD (round-robin least loaded), NODE_AFFINITY
//    (hard/soft), node-label constraints
//  * placement groups: PACK / SPREAD / STRICT_PACK / STRICT_SPREAD bundle placement,
//    reservation materialises `<res>_group_<pg>` and `<res>_group_<i>_<pg>` resources
//    exactly like the reference, so tasks inside a PG are plain resource requests.
#pragma once
#include <stdint.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace ray_amd {

using ResMap = std::map<std::string, double>;
using LabelMap = std::map<std::string, std::string>;

enum Strategy : int { kHybrid = 0, kSpread = 1, kAffinityHard = 2, kAffinitySoft = 3 };
enum PGStrategy : int { kPack = 0, kPGSpread = 1, kStrictPack = 2, kStrictSpread = 3 };

struct Allocation {
  std::string node;
  std::map<std::string, std::vector<std::pair<int, int64_t>>> instances;  // res -> [(idx, amt)]
};

struct NodeRes {
  std::map<std::string, int64_t> total, avail;
  std::map<std::string, std::vector<int64_t>> inst_total, inst_avail;  // unit-instance resources
  LabelMap labels;
  bool alive = true;
  bool draining = false;
};

class Scheduler {
 public:
  static constexpr int64_t kUnit = 10000;
  void add_node(const std::string& id, const ResMap& total, const LabelMap& labels);
  void remove_node(const std::string& id);
  void set_draining(const std::string& id, bool d);
  std::vector<std::string> nodes();
  ResMap total(const std::string& node);
  ResMap available(const std::string& node);
  ResMap cluster_total();
  ResMap cluster_available();
  LabelMap labels(const std::string& node);

  // "" = feasible but not now; "!" = infeasible on every node.
  std::string pick_node(const ResMap& req, int strategy, const std::string& target,
                        const std::string& local, const LabelMap& hard_labels,
                        const LabelMap& soft_labels);
  bool feasible_anywhere(const ResMap& req, const LabelMap& hard_labels);
  // Allocate on a node; on success fills `out` with instance assignment.
  bool allocate(const std::string& node, const ResMap& req, Allocation* out);
  void release(const Allocation& a, const ResMap& req);

  // Placement groups: returns node per bundle (empty vector if not placeable now).
  std::vector<std::string> place_bundles(const std::vector<ResMap>& bundles, int strategy,
                                         bool* infeasible);
  bool commit_bundles(const std::string& pg_id, const std::vector<ResMap>& bundles,
                      const std::vector<std::string>& nodes);
  void remove_bundles(const std::string& pg_id, const std::vector<ResMap>& bundles,
                      const std::vector<std::string>& nodes);
  // GPU instance indices reserved by each bundle of a committed placement group.
  std::vector<std::vector<int>> pg_gpu_instances(const std::string& pg_id);
  double spread_threshold = 0.5;

 private:
  bool fits(const NodeRes& n, const std::map<std::string, int64_t>& req, bool use_total) const;
  double utilization(const NodeRes& n) const;
  static bool is_instance_res(const std::string& name);
  static std::map<std::string, int64_t> to_fixed(const ResMap& m);
  bool labels_match(const NodeRes& n, const LabelMap& want) const;
  bool take_instances(NodeRes& n, const std::string& name, int64_t amt,
                      std::vector<std::pair<int, int64_t>>* got);
  std::mutex mu_;
  std::map<std::string, NodeRes> nodes_;
  std::map<std::string, std::vector<std::vector<std::pair<int, int64_t>>>> pg_gpu_;  // pg -> bundle -> instances
  uint64_t rr_ = 0;
};

}  // namespace ray_amd
