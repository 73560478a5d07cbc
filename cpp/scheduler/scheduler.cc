#include "scheduler.h"

#include "../api/types.h"

#include <algorithm>
#include <climits>

namespace tfk {

static long long parse_quantity_milli(const Json& q) {
  if (q.is_number()) return (long long)(q.as_double() * 1000);
  std::string s = q.str();
  if (s.empty()) return 0;
  if (ends_with(s, "m")) return atoll(s.c_str());
  return (long long)(atof(s.c_str()) * 1000);
}

int pod_gpu_request(const Json& pod) {
  int n = 0;
  for (auto& c : pod.path("spec.containers").items()) {
    const Json& lim = c.path("resources.limits").at("amd.com/gpu");
    const Json& req = c.path("resources.requests").at("amd.com/gpu");
    const Json& q = lim.is_null() ? req : lim;
    n += q.is_number() ? (int)q.as_int() : atoi(q.str("0").c_str());
  }
  return n;
}

long long pod_cpu_request_milli(const Json& pod) {
  long long n = 0;
  for (auto& c : pod.path("spec.containers").items()) n += parse_quantity_milli(c.path("resources.requests").at("cpu"));
  return n;
}

static bool terminal(const Json& pod) {
  std::string ph = pod.path("status.phase").str();
  return ph == "Succeeded" || ph == "Failed";
}

std::vector<int> parse_int_list(const std::string& s) {
  std::vector<int> v;
  for (auto& t : split(s, ','))
    if (!t.empty()) v.push_back(atoi(t.c_str()));
  return v;
}

std::vector<int> pick_gpus(const NodeInfo& n, int need, int prefer_dom, int fit_total) {
  std::map<int, std::vector<int>> free_by_dom;  // NUMA domain -> free GPU ids (ascending)
  for (int g = 0; g < n.gpus; ++g)
    if (!n.used_gpus.count(g)) free_by_dom[g < (int)n.gpu_numa.size() ? n.gpu_numa[g] : 0].push_back(g);
  std::vector<int> ids;
  if (need <= 0) return ids;
  // the gang already holds GPUs in prefer_dom on this node: stay there while it has room
  auto pd = free_by_dom.find(prefer_dom);
  if (prefer_dom >= 0 && pd != free_by_dom.end() && (int)pd->second.size() >= need)
    return std::vector<int>(pd->second.begin(), pd->second.begin() + need);
  // best fit: the domain with the fewest free GPUs that still holds the whole gang (fit_total),
  // else the whole request
  for (int want : {std::max(fit_total, need), need}) {
    const std::vector<int>* best = nullptr;
    for (auto& kv : free_by_dom)
      if ((int)kv.second.size() >= want && (!best || kv.second.size() < best->size())) best = &kv.second;
    if (best) return std::vector<int>(best->begin(), best->begin() + need);
  }
  // spans domains: fewest domains -> take the largest domains first
  std::vector<const std::vector<int>*> doms;
  for (auto& kv : free_by_dom) doms.push_back(&kv.second);
  std::stable_sort(doms.begin(), doms.end(), [](const std::vector<int>* a, const std::vector<int>* b) {
    return a->size() > b->size();
  });
  for (auto* d : doms)
    for (int g : *d)
      if ((int)ids.size() < need) ids.push_back(g);
  std::sort(ids.begin(), ids.end());
  return ids;
}

GangScheduler::GangScheduler(std::shared_ptr<Client> c, SchedulerOptions o) : client_(std::move(c)), opts_(std::move(o)) {
  pods_.reset(new SharedInformer(client_, "pods", "", 30000));
  nodes_.reset(new SharedInformer(client_, "nodes", "", 30000));
  prio_.reset(new SharedInformer(client_, "priorityclasses", "", 30000));
}

long long GangScheduler::pod_priority(const Json& pod) const {
  const Json& pr = pod.path("spec.priority");
  if (pr.is_number()) return pr.as_int();
  std::string cls = pod.path("spec.priorityClassName").str();
  if (cls.empty()) return 0;
  if (cls == "system-node-critical") return 2000001000LL;
  if (cls == "system-cluster-critical") return 2000000000LL;
  for (auto& pc : prio_->indexer().list())
    if (pc.path("metadata.name").str() == cls) return pc.at("value").as_int();
  return 0;
}

bool GangScheduler::mine(const Json& pod) const {
  std::string s = pod.path("spec.schedulerName").str();
  if (s == opts_.name) return true;
  return opts_.schedule_default && (s.empty() || s == "default-scheduler");
}

std::vector<NodeInfo> GangScheduler::node_state() const {
  std::map<std::string, NodeInfo> nodes;
  for (auto& n : nodes_->indexer().list()) {
    NodeInfo ni;
    ni.name = n.path("metadata.name").str();
    const Json& alloc = n.path("status.allocatable").is_object() ? n.path("status.allocatable") : n.path("status.capacity");
    const Json& g = alloc.at("amd.com/gpu");
    ni.gpus = g.is_number() ? (int)g.as_int() : atoi(g.str("0").c_str());
    ni.cpu_milli = parse_quantity_milli(alloc.at("cpu"));
    ni.gpu_numa = parse_int_list(n.path("metadata.annotations").at("tfk.io/gpu-numa").str());
    bool ready = true;
    for (auto& c : n.path("status.conditions").items())
      if (c.at("type").str() == "Ready" && c.at("status").str() != "True") ready = false;
    if (n.path("spec.unschedulable").as_bool(false)) ready = false;
    if (ready) nodes[ni.name] = ni;
  }
  for (auto& p : pods_->indexer().list()) {
    std::string node = p.path("spec.nodeName").str();
    if (node.empty() || terminal(p) || !nodes.count(node)) continue;
    for (auto& id : split(p.path("metadata.annotations").at("tfk.io/gpu-ids").str(), ','))
      if (!id.empty()) nodes[node].used_gpus.insert(atoi(id.c_str()));
    nodes[node].used_cpu_milli += pod_cpu_request_milli(p);
  }
  std::vector<NodeInfo> v;
  for (auto& kv : nodes) v.push_back(kv.second);
  return v;
}

std::map<std::string, std::pair<std::string, std::vector<int>>> GangScheduler::place_group(
    const std::vector<Json>& pods, std::vector<NodeInfo> nodes) {
  std::map<std::string, std::pair<std::string, std::vector<int>>> out;
  // first-fit decreasing by GPU request; every pod must land or nothing is bound
  std::vector<const Json*> order;
  for (auto& p : pods) order.push_back(&p);
  std::stable_sort(order.begin(), order.end(), [](const Json* a, const Json* b) {
    return pod_gpu_request(*a) > pod_gpu_request(*b);
  });
  int remaining = 0;
  for (auto* p : order) remaining += pod_gpu_request(*p);
  std::map<std::string, int> gang_dom;  // node -> NUMA domain this gang packs into
  for (auto* p : order) {
    int need = pod_gpu_request(*p);
    long long cpu = pod_cpu_request_milli(*p);
    bool placed = false;
    for (auto& n : nodes) {
      int free = n.gpus - (int)n.used_gpus.size();
      if (free < need) continue;
      if (n.cpu_milli > 0 && n.used_cpu_milli + cpu > n.cpu_milli) continue;
      auto gd = gang_dom.find(n.name);
      std::vector<int> ids = pick_gpus(n, need, gd == gang_dom.end() ? -1 : gd->second, remaining);
      std::set<int> doms;
      for (int g : ids) doms.insert(g < (int)n.gpu_numa.size() ? n.gpu_numa[g] : 0);
      if (doms.size() == 1 && gd == gang_dom.end()) gang_dom[n.name] = *doms.begin();
      remaining -= need;
      for (int g : ids) n.used_gpus.insert(g);
      n.used_cpu_milli += cpu;
      out[p->path("metadata.namespace").str() + "/" + p->path("metadata.name").str()] = {n.name, ids};
      placed = true;
      break;
    }
    if (!placed) return {};
  }
  return out;
}

int GangScheduler::schedule_once() {
  auto nodes = node_state();
  if (nodes.empty()) return 0;
  std::map<std::string, std::vector<Json>> groups;        // pending by group
  std::map<std::string, int> bound_in_group, min_avail;
  for (auto& p : pods_->indexer().list()) {
    if (p.path("metadata.deletionTimestamp").is_string() || terminal(p)) continue;
    const Json& an = p.path("metadata.annotations");
    std::string g = an.at("scheduling.tfk.io/group-name").str();
    std::string key = g.empty() ? "pod:" + p.path("metadata.namespace").str() + "/" + p.path("metadata.name").str()
                                : "grp:" + p.path("metadata.namespace").str() + "/" + g;
    if (!g.empty()) min_avail[key] = std::max(min_avail[key], atoi(an.at("scheduling.tfk.io/min-available").str("1").c_str()));
    if (!p.path("spec.nodeName").str().empty()) { bound_in_group[key]++; continue; }
    if (!mine(p)) continue;
    groups[key].push_back(p);
  }
  // placement order: priority (highest first), then the oldest member's creation time, then key
  struct Pending { long long prio; std::string created, key; };
  std::vector<Pending> order;
  for (auto& kv : groups) {
    Pending pd{LLONG_MIN, "", kv.first};
    for (auto& p : kv.second) {
      pd.prio = std::max(pd.prio, pod_priority(p));
      std::string c = p.path("metadata.creationTimestamp").str();
      if (pd.created.empty() || c < pd.created) pd.created = c;
    }
    order.push_back(pd);
  }
  std::stable_sort(order.begin(), order.end(), [](const Pending& a, const Pending& b) {
    if (a.prio != b.prio) return a.prio > b.prio;
    if (a.created != b.created) return a.created < b.created;
    return a.key < b.key;
  });
  int bound = 0;
  for (auto& od : order) {
    auto& kv = *groups.find(od.key);
    int need_total = min_avail.count(kv.first) ? min_avail[kv.first] : 1;
    if ((int)kv.second.size() + bound_in_group[kv.first] < need_total) continue;  // gang incomplete: wait
    auto plan = place_group(kv.second, nodes);
    if (plan.empty()) {
      int64_t now = mono_ms();
      if (now - last_warned_[kv.first] > 10000) {
        last_warned_[kv.first] = now;
        TFK_LOG(Warn, "FailedScheduling: insufficient amd.com/gpu for gang", Json(Json::object_t{{"group", Json(kv.first)}}));
      }
      continue;
    }
    // gang-visible opt-in: the union of this gang's GPUs per node (sorted), recorded on each member
    std::map<std::string, std::set<int>> gang_gpus;
    for (auto& p : kv.second) {
      auto& pl = plan[p.path("metadata.namespace").str() + "/" + p.path("metadata.name").str()];
      gang_gpus[pl.first].insert(pl.second.begin(), pl.second.end());
    }
    for (auto& p : kv.second) {
      std::string k = p.path("metadata.namespace").str() + "/" + p.path("metadata.name").str();
      auto& pl = plan[k];
      Json next = p.clone();
      next["spec"]["nodeName"] = pl.first;
      std::string ids;
      for (size_t i = 0; i < pl.second.size(); ++i) ids += (i ? "," : "") + std::to_string(pl.second[i]);
      next["metadata"]["annotations"]["tfk.io/gpu-ids"] = ids;
      const Json& gv = p.path("metadata.annotations").at(api::kGangVisibleGpus);
      if (gv.is_string() && !gv.str().empty() && gv.str() != "false") {
        std::string all;
        for (int g : gang_gpus[pl.first]) all += (all.empty() ? "" : ",") + std::to_string(g);
        next["metadata"]["annotations"][api::kGangGpuIds] = all;
      }
      Json out;
      ApiStatus st = client_->update("pods", p.path("metadata.namespace").str(), next, &out);
      if (st.ok()) {
        bound++;
        bound_++;
        pods_->indexer().upsert(k, out);  // reflect immediately so the next group sees the GPUs as used
        for (auto& n : nodes)
          if (n.name == pl.first)
            for (int g : pl.second) n.used_gpus.insert(g);
        TFK_LOG(Info, "bound pod", Json(Json::object_t{{"pod", Json(k)}, {"node", Json(pl.first)}, {"gpus", Json(ids)}}));
      }
    }
  }
  return bound;
}

void GangScheduler::run(StopToken& stop) {
  pods_->start(stop);
  nodes_->start(stop);
  prio_->start(stop);
  while (!stop.stopped() && !wait_for_cache_sync({pods_.get(), nodes_.get(), prio_.get()}, 1000)) {
  }
  while (!stop.stopped()) {
    try {
      schedule_once();
    } catch (const std::exception& e) {
      TFK_LOG(Error, std::string("schedule pass failed: ") + e.what());
    }
    stop.wait_for(opts_.period_ms);
  }
}

}  // namespace tfk
