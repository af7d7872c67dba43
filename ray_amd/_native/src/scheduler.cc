#include "scheduler.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace ray_amd {

static const char* kGroupTag = "_group_";

bool Scheduler::is_instance_res(const std::string& name) {
  return name == "GPU" || name.rfind("GPU_group_", 0) == 0;
}

std::map<std::string, int64_t> Scheduler::to_fixed(const ResMap& m) {
  std::map<std::string, int64_t> o;
  for (auto& kv : m) {
    if (kv.second <= 0) continue;
    o[kv.first] = (int64_t)std::llround(kv.second * kUnit);
  }
  return o;
}

static ResMap to_double(const std::map<std::string, int64_t>& m) {
  ResMap o;
  for (auto& kv : m) o[kv.first] = (double)kv.second / Scheduler::kUnit;
  return o;
}

void Scheduler::add_node(const std::string& id, const ResMap& total, const LabelMap& labels) {
  std::lock_guard<std::mutex> g(mu_);
  NodeRes n;
  n.total = to_fixed(total);
  n.avail = n.total;
  n.labels = labels;
  auto it = n.total.find("GPU");
  if (it != n.total.end()) {
    int k = (int)(it->second / kUnit);
    n.inst_total["GPU"] = std::vector<int64_t>(k, kUnit);
    n.inst_avail["GPU"] = n.inst_total["GPU"];
  }
  nodes_[id] = n;
}

void Scheduler::remove_node(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  nodes_.erase(id);
}

void Scheduler::set_draining(const std::string& id, bool d) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = nodes_.find(id);
  if (it != nodes_.end()) it->second.draining = d;
}

std::vector<std::string> Scheduler::nodes() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> o;
  for (auto& kv : nodes_) o.push_back(kv.first);
  return o;
}

ResMap Scheduler::total(const std::string& node) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = nodes_.find(node);
  return it == nodes_.end() ? ResMap() : to_double(it->second.total);
}
ResMap Scheduler::available(const std::string& node) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = nodes_.find(node);
  return it == nodes_.end() ? ResMap() : to_double(it->second.avail);
}
ResMap Scheduler::cluster_total() {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, int64_t> s;
  for (auto& kv : nodes_)
    for (auto& r : kv.second.total) s[r.first] += r.second;
  return to_double(s);
}
ResMap Scheduler::cluster_available() {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, int64_t> s;
  for (auto& kv : nodes_)
    for (auto& r : kv.second.avail) s[r.first] += r.second;
  return to_double(s);
}
LabelMap Scheduler::labels(const std::string& node) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = nodes_.find(node);
  return it == nodes_.end() ? LabelMap() : it->second.labels;
}

// A wanted value is a comma-separated "in" list; a leading '!' negates it ("not in": a
// node without the label matches a negated constraint, as in the reference's
// label_selector "!value" / "!in(a,b)").
bool Scheduler::labels_match(const NodeRes& n, const LabelMap& want) const {
  for (auto& kv : want) {
    const std::string& raw = kv.second;
    const bool neg = !raw.empty() && raw[0] == '!';
    auto it = n.labels.find(kv.first);
    if (it == n.labels.end()) {
      if (neg) continue;
      return false;
    }
    const size_t s0 = neg ? 1 : 0;
    size_t s = s0;
    bool in = false;
    while (s <= raw.size()) {
      size_t e = raw.find(',', s);
      if (e == std::string::npos) e = raw.size();
      if (raw.compare(s, e - s, it->second) == 0) { in = true; break; }
      s = e + 1;
    }
    if (neg ? in : !in) return false;
  }
  return true;
}

bool Scheduler::fits(const NodeRes& n, const std::map<std::string, int64_t>& req,
                     bool use_total) const {
  const auto& pool = use_total ? n.total : n.avail;
  for (auto& kv : req) {
    auto it = pool.find(kv.first);
    if (it == pool.end() || it->second < kv.second) return false;
    if (is_instance_res(kv.first)) {
      const auto& inst = use_total ? n.inst_total : n.inst_avail;
      auto iv = inst.find(kv.first);
      if (iv == inst.end()) return false;
      if (kv.second >= kUnit) {
        int need = (int)((kv.second + kUnit - 1) / kUnit);
        int have = 0;
        for (int64_t a : iv->second) have += (a == kUnit);
        if (have < need) return false;
      } else {
        bool any = false;
        for (int64_t a : iv->second) any |= (a >= kv.second);
        if (!any) return false;
      }
    }
  }
  return true;
}

double Scheduler::utilization(const NodeRes& n) const {
  double u = 0;
  for (auto& kv : n.total) {
    if (kv.second <= 0 || kv.first.find(kGroupTag) != std::string::npos) continue;
    if (kv.first.rfind("node:", 0) == 0) continue;
    auto a = n.avail.find(kv.first);
    double used = (double)(kv.second - (a == n.avail.end() ? 0 : a->second)) / kv.second;
    u = std::max(u, used);
  }
  return u;
}

bool Scheduler::feasible_anywhere(const ResMap& req, const LabelMap& hard) {
  std::lock_guard<std::mutex> g(mu_);
  auto r = to_fixed(req);
  for (auto& kv : nodes_)
    if (kv.second.alive && labels_match(kv.second, hard) && fits(kv.second, r, true)) return true;
  return false;
}

std::string Scheduler::pick_node(const ResMap& req, int strategy, const std::string& target,
                                 const std::string& local, const LabelMap& hard,
                                 const LabelMap& soft) {
  std::lock_guard<std::mutex> g(mu_);
  auto r = to_fixed(req);
  if (strategy == kAffinityHard || strategy == kAffinitySoft) {
    auto it = nodes_.find(target);
    bool ok = it != nodes_.end() && it->second.alive;
    if (ok && fits(it->second, r, true)) {
      if (fits(it->second, r, false)) return target;
      if (strategy == kAffinityHard) return "";
    } else if (strategy == kAffinityHard) {
      return "!";
    }
  }
  std::vector<std::string> feasible, avail;
  for (auto& kv : nodes_) {
    const NodeRes& n = kv.second;
    if (!n.alive || !labels_match(n, hard)) continue;
    if (!fits(n, r, true)) continue;
    feasible.push_back(kv.first);
    if (!n.draining && fits(n, r, false)) avail.push_back(kv.first);
  }
  if (feasible.empty()) return "!";
  if (avail.empty()) return "";
  if (!soft.empty()) {
    std::vector<std::string> pref;
    for (auto& id : avail)
      if (labels_match(nodes_[id], soft)) pref.push_back(id);
    if (!pref.empty()) avail.swap(pref);
  }
  if (strategy == kSpread) {
    // least loaded, round-robin among ties
    double best = 1e9;
    std::vector<std::string> ties;
    for (auto& id : avail) {
      double u = utilization(nodes_[id]);
      if (u < best - 1e-9) { best = u; ties.clear(); }
      if (u <= best + 1e-9) ties.push_back(id);
    }
    return ties[(rr_++) % ties.size()];
  }
  // hybrid
  if (!local.empty() && std::find(avail.begin(), avail.end(), local) != avail.end() &&
      utilization(nodes_[local]) < spread_threshold)
    return local;
  std::string best_id;
  double best = 1e9;
  for (auto& id : avail) {
    double u = utilization(nodes_[id]);
    if (id == local) u -= 1e-6;  // tie-break toward local
    if (u < best) { best = u; best_id = id; }
  }
  return best_id;
}

bool Scheduler::take_instances(NodeRes& n, const std::string& name, int64_t amt,
                               std::vector<std::pair<int, int64_t>>* got) {
  auto& av = n.inst_avail[name];
  std::vector<int> prefer;
  for (auto& p : *got) prefer.push_back(p.first);
  got->clear();
  if (amt >= kUnit) {
    int need = (int)((amt + kUnit - 1) / kUnit);
    std::vector<int> pick;
    for (int i : prefer)
      if ((int)pick.size() < need && i < (int)av.size() && av[i] == kUnit) pick.push_back(i);
    for (int i = 0; i < (int)av.size() && (int)pick.size() < need; ++i)
      if (av[i] == kUnit && std::find(pick.begin(), pick.end(), i) == pick.end()) pick.push_back(i);
    if ((int)pick.size() < need) return false;
    for (int i : pick) {
      av[i] = 0;
      got->push_back({i, kUnit});
    }
    return true;
  }
  int best = -1;
  for (int i : prefer)
    if (i < (int)av.size() && av[i] >= amt) { best = i; break; }
  if (best < 0)
    for (int i = 0; i < (int)av.size(); ++i)
      if (av[i] >= amt && (best < 0 || av[i] < av[best])) best = i;
  if (best < 0) return false;
  av[best] -= amt;
  got->push_back({best, amt});
  return true;
}

bool Scheduler::allocate(const std::string& node, const ResMap& req, Allocation* out) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return false;
  NodeRes& n = it->second;
  auto r = to_fixed(req);
  if (!fits(n, r, false)) return false;
  out->node = node;
  // instance resources: longest names (indexed PG resources) first so the wildcard
  // PG resource reuses the same device indices
  std::vector<std::string> inst;
  for (auto& kv : r)
    if (is_instance_res(kv.first)) inst.push_back(kv.first);
  std::sort(inst.begin(), inst.end(),
            [](const std::string& a, const std::string& b) { return a.size() > b.size(); });
  std::vector<std::pair<int, int64_t>> last;
  for (auto& name : inst) {
    std::vector<std::pair<int, int64_t>> got = last;
    if (!take_instances(n, name, r[name], &got)) {
      // roll back
      for (auto& kv : out->instances)
        for (auto& p : kv.second) n.inst_avail[kv.first][p.first] += p.second;
      out->instances.clear();
      return false;
    }
    out->instances[name] = got;
    last = got;
  }
  for (auto& kv : r) n.avail[kv.first] -= kv.second;
  return true;
}

void Scheduler::release(const Allocation& a, const ResMap& req) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = nodes_.find(a.node);
  if (it == nodes_.end()) return;
  NodeRes& n = it->second;
  for (auto& kv : to_fixed(req)) {
    auto t = n.total.find(kv.first);
    if (t == n.total.end()) continue;  // resource vanished (PG removed)
    n.avail[kv.first] = std::min(t->second, n.avail[kv.first] + kv.second);
  }
  for (auto& kv : a.instances) {
    auto iv = n.inst_avail.find(kv.first);
    if (iv == n.inst_avail.end()) continue;
    for (auto& p : kv.second)
      if (p.first < (int)iv->second.size())
        iv->second[p.first] = std::min(n.inst_total[kv.first][p.first], iv->second[p.first] + p.second);
  }
}

std::vector<std::string> Scheduler::place_bundles(const std::vector<ResMap>& bundles, int strategy,
                                                  bool* infeasible) {
  std::lock_guard<std::mutex> g(mu_);
  *infeasible = false;
  std::vector<std::map<std::string, int64_t>> req;
  for (auto& b : bundles) req.push_back(to_fixed(b));
  std::vector<std::string> ids;
  for (auto& kv : nodes_)
    if (kv.second.alive && !kv.second.draining) ids.push_back(kv.first);
  // work on a scratch copy of availability
  std::map<std::string, NodeRes> scratch;
  for (auto& id : ids) scratch[id] = nodes_[id];
  auto deduct = [&](NodeRes& n, const std::map<std::string, int64_t>& r) {
    for (auto& kv : r) {
      n.avail[kv.first] -= kv.second;
      if (is_instance_res(kv.first)) {
        std::vector<std::pair<int, int64_t>> got;
        take_instances(n, kv.first, kv.second, &got);
      }
    }
  };
  std::vector<std::string> out(bundles.size());
  if (strategy == kStrictPack) {
    std::map<std::string, int64_t> sum;
    for (auto& r : req)
      for (auto& kv : r) sum[kv.first] += kv.second;
    bool any_total = false;
    for (auto& id : ids) {
      if (fits(nodes_[id], sum, true)) any_total = true;
      if (fits(scratch[id], sum, false)) {
        for (auto& o : out) o = id;
        return out;
      }
    }
    *infeasible = !any_total;
    return {};
  }
  if (strategy == kStrictSpread) {
    if (ids.size() < bundles.size()) {
      *infeasible = true;
      return {};
    }
    std::vector<bool> used(ids.size(), false);
    for (size_t b = 0; b < req.size(); ++b) {
      int pick = -1;
      double best = 1e9;
      for (size_t i = 0; i < ids.size(); ++i) {
        if (used[i] || !fits(scratch[ids[i]], req[b], false)) continue;
        double u = utilization(scratch[ids[i]]);
        if (u < best) { best = u; pick = (int)i; }
      }
      if (pick < 0) return {};
      used[pick] = true;
      deduct(scratch[ids[pick]], req[b]);
      out[b] = ids[pick];
    }
    return out;
  }
  for (size_t b = 0; b < req.size(); ++b) {
    bool any_total = false;
    for (auto& id : ids) any_total |= fits(nodes_[id], req[b], true);
    if (!any_total) {
      *infeasible = true;
      return {};
    }
    int pick = -1;
    double best = 1e9;
    for (size_t i = 0; i < ids.size(); ++i) {
      NodeRes& n = scratch[ids[i]];
      if (!fits(n, req[b], false)) continue;
      double u = utilization(n);
      if (strategy == kPack) {
        // prefer the node already used by previous bundles, then most utilised
        bool prev = b > 0 && std::find(out.begin(), out.begin() + b, ids[i]) != out.begin() + b;
        double score = prev ? -2.0 : -u;
        if (score < best) { best = score; pick = (int)i; }
      } else {  // SPREAD: prefer nodes not yet used, then least utilised
        bool prev = std::find(out.begin(), out.begin() + b, ids[i]) != out.begin() + b;
        double score = (prev ? 10.0 : 0.0) + u;
        if (score < best) { best = score; pick = (int)i; }
      }
    }
    if (pick < 0) return {};
    deduct(scratch[ids[pick]], req[b]);
    out[b] = ids[pick];
  }
  return out;
}

bool Scheduler::commit_bundles(const std::string& pg, const std::vector<ResMap>& bundles,
                               const std::vector<std::string>& nodes) {
  std::lock_guard<std::mutex> g(mu_);
  auto& gpu_inst = pg_gpu_[pg];
  gpu_inst.assign(bundles.size(), {});
  for (size_t b = 0; b < bundles.size(); ++b) {
    auto it = nodes_.find(nodes[b]);
    if (it == nodes_.end()) return false;
    NodeRes& n = it->second;
    auto r = to_fixed(bundles[b]);
    if (!fits(n, r, false)) return false;
    for (auto& kv : r) {
      n.avail[kv.first] -= kv.second;
      std::vector<std::pair<int, int64_t>> got;
      if (is_instance_res(kv.first)) {
        take_instances(n, kv.first, kv.second, &got);
        gpu_inst[b] = got;
      }
      const std::string wild = kv.first + "_group_" + pg;
      const std::string idx = kv.first + "_group_" + std::to_string(b) + "_" + pg;
      for (const std::string* nm : {&wild, &idx}) {
        n.total[*nm] += kv.second;
        n.avail[*nm] += kv.second;
        if (!got.empty()) {
          size_t ng = n.inst_total["GPU"].size();
          auto& tt = n.inst_total[*nm];
          auto& aa = n.inst_avail[*nm];
          if (tt.size() < ng) { tt.resize(ng, 0); aa.resize(ng, 0); }
          for (auto& p : got) { tt[p.first] += p.second; aa[p.first] += p.second; }
        }
      }
    }
    const int64_t bun = 1000 * kUnit;
    n.total["bundle_group_" + pg] += bun;
    n.avail["bundle_group_" + pg] += bun;
    n.total["bundle_group_" + std::to_string(b) + "_" + pg] += bun;
    n.avail["bundle_group_" + std::to_string(b) + "_" + pg] += bun;
  }
  return true;
}

void Scheduler::remove_bundles(const std::string& pg, const std::vector<ResMap>& bundles,
                               const std::vector<std::string>& nodes) {
  std::lock_guard<std::mutex> g(mu_);
  auto gi = pg_gpu_.find(pg);
  for (size_t b = 0; b < bundles.size() && b < nodes.size(); ++b) {
    auto it = nodes_.find(nodes[b]);
    if (it == nodes_.end()) continue;
    NodeRes& n = it->second;
    for (auto& kv : to_fixed(bundles[b])) {
      n.avail[kv.first] = std::min(n.total[kv.first], n.avail[kv.first] + kv.second);
      if (is_instance_res(kv.first) && gi != pg_gpu_.end() && b < gi->second.size()) {
        for (auto& p : gi->second[b]) n.inst_avail[kv.first][p.first] += p.second;
      }
    }
  }
  // drop every resource tagged with this pg
  const std::string suffix = "_" + pg;
  for (auto& kv : nodes_) {
    NodeRes& n = kv.second;
    for (auto* m : {&n.total, &n.avail}) {
      for (auto it = m->begin(); it != m->end();) {
        const std::string& k = it->first;
        if (k.find(kGroupTag) != std::string::npos && k.size() > suffix.size() &&
            k.compare(k.size() - suffix.size(), suffix.size(), suffix) == 0)
          it = m->erase(it);
        else
          ++it;
      }
    }
    for (auto* m : {&n.inst_total, &n.inst_avail}) {
      for (auto it = m->begin(); it != m->end();) {
        const std::string& k = it->first;
        if (k.find(kGroupTag) != std::string::npos && k.size() > suffix.size() &&
            k.compare(k.size() - suffix.size(), suffix.size(), suffix) == 0)
          it = m->erase(it);
        else
          ++it;
      }
    }
  }
  if (gi != pg_gpu_.end()) pg_gpu_.erase(gi);
}

std::vector<std::vector<int>> Scheduler::pg_gpu_instances(const std::string& pg) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::vector<int>> out;
  auto it = pg_gpu_.find(pg);
  if (it == pg_gpu_.end()) return out;
  for (auto& b : it->second) {
    std::vector<int> ids;
    for (auto& p : b) ids.push_back(p.first);
    out.push_back(ids);
  }
  return out;
}

}  // namespace ray_amd
