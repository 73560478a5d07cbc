// Gang scheduler (north star: "gang-schedules chief/PS/worker pods onto one 8xMI355X node").
// All-or-nothing placement per pod group (annotation scheduling.tfk.io/group-name, min-available),
// amd.com/gpu accounting per node with concrete, disjoint GPU ids handed to the node agent through
// the tfk.io/gpu-ids annotation (-> HIP_VISIBLE_DEVICES). Pods without a group are scheduled alone.
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
};

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
  std::shared_ptr<Client> client_;
  SchedulerOptions opts_;
  std::unique_ptr<SharedInformer> pods_, nodes_;
  std::atomic<long long> bound_{0};
  std::map<std::string, int64_t> last_warned_;
};

}  // namespace tfk
