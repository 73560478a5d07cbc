// Gang scheduler (north star: "gang-schedules chief/PS/worker pods onto one 8xMI355X node").
// All-or-nothing placement per pod group (annotation scheduling.tfk.io/group-name, min-available),
// amd.com/gpu accounting per node with concrete, disjoint GPU ids handed to the node agent through
// the tfk.io/gpu-ids annotation (-> HIP_VISIBLE_DEVICES). Pods without a group are scheduled alone.
//
// Topology: the node agent publishes each GPU's NUMA node (annotation tfk.io/gpu-numa, e.g.
// "0,0,0,0,1,1,1,1" on a two-socket 8x MI355X node). xGMI connects every GPU pair directly, so GPU
// choice does not change collective bandwidth, but host-side work (input pipeline, pinned
// staging, the rank's CPU threads) is NUMA-local only if a gang's GPUs share a socket: GPU ids are
// taken best-fit per NUMA domain (the fullest domain that still fits), so a 4-GPU gang lands on
// one socket and leaves the other whole for the next gang. The kubelet then pins the container's
// CPUs to those domains.
// Priority: pending gangs are placed in order of priority (pod spec.priority, else the value of
// the PriorityClass named by spec.priorityClassName -- scheduling.k8s.io/v1 objects, plus the two
// built-in system classes), then age, so a high-priority TFJob gets contended GPUs first.
#pragma once
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "../cache/informer.h"

namespace tfk {

struct SchedulerOptions {
  std::string name = "tfk-gang";
  bool schedule_default = true;  // also place pods asking for default-scheduler / no scheduler
  int64_t period_ms = 100;
};

struct NodeInfo {
  std::string name;
  int gpus = 0;
  std::set<int> used_gpus;
  long long cpu_milli = 0, used_cpu_milli = 0;
  std::vector<int> gpu_numa;  // NUMA node of GPU i (empty: unknown -> one domain)
};

// GPU ids for `need` GPUs on n: the gang's domain (prefer_dom) while it has room, else the best-fit
// NUMA domain for the gang's remaining total (fit_total), else for `need`, else the fewest domains.
std::vector<int> pick_gpus(const NodeInfo& n, int need, int prefer_dom = -1, int fit_total = 0);
std::vector<int> parse_int_list(const std::string& s);

int pod_gpu_request(const Json& pod);
long long pod_cpu_request_milli(const Json& pod);

class GangScheduler {
 public:
  GangScheduler(std::shared_ptr<Client> c, SchedulerOptions o);
  void run(StopToken& stop);
  // One scheduling pass over cached state; returns number of pods bound.
  int schedule_once();
  // Pure placement: returns podname -> (node, gpu ids) for the whole group, or empty if it does not fit.
  static std::map<std::string, std::pair<std::string, std::vector<int>>> place_group(
      const std::vector<Json>& pods, std::vector<NodeInfo> nodes);
  std::vector<NodeInfo> node_state() const;
  long long bound() const { return bound_; }

 private:
  bool mine(const Json& pod) const;
  long long pod_priority(const Json& pod) const;
  std::shared_ptr<Client> client_;
  SchedulerOptions opts_;
  std::unique_ptr<SharedInformer> pods_, nodes_, prio_;
  std::atomic<long long> bound_{0};
  std::map<std::string, int64_t> last_warned_;
};

}  // namespace tfk
