// Trainer: per-TFJob reconcile (reference: pkg/trainer/{labels.go,replicas.go,training.go},
// images/tf3.PNG:L59-L61; "TFJob CRUD is hand-implemented" k8s-operator.md:228; Job/Pod restart
// semantics k8s-operator.md:44-52). Level-triggered: given the TFJob and the pods/services that
// currently exist (from informer caches), create what is missing, apply restart/cleanup policies,
// and write back status. Deterministic pod/service names make creation idempotent (409 = exists).
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../api/types.h"
#include "../client/client.h"

namespace tfk {

// labels.go: the label set that identifies one replica of one job.
struct ReplicaLabels {
  static Json for_replica(const api::TFJob& job, api::RType t, int index);
  static std::string job_selector(const api::TFJob& job);  // "tf-job-name=<name>"
};

class EventRecorder {
 public:
  explicit EventRecorder(std::shared_ptr<Client> c, std::string component = "tf-operator")
      : client_(std::move(c)), component_(std::move(component)) {}
  void event(const Json& obj, const std::string& type, const std::string& reason, const std::string& msg);
  long long count() const { return count_; }

 private:
  std::shared_ptr<Client> client_;
  std::string component_;
  std::atomic<long long> count_{0};
};

struct TrainerOptions {
  std::string cluster_domain;          // appended to "<svc>.<ns>.svc"
  bool gang_scheduling = true;         // pods -> schedulerName tfk-gang + PodGroup
  std::string gang_scheduler_name = "tfk-gang";
  bool local_ports = false;            // single-node emulation: unique per-service ports
  int local_port_base = 20000;
  std::string default_ps_command = "python3 -m tensorflow_k8s_amd.runtime.ps_server";
  api::ControllerConfig controller_config = api::ControllerConfig::defaults();
};

struct ReconcileResult {
  bool requeue = false;          // try again soon (e.g. 409 on status write)
  int64_t requeue_after_ms = 0;  // e.g. TTL / deadline timers
  std::string error;
  int pods_created = 0, pods_deleted = 0, services_created = 0, services_deleted = 0;
  bool status_changed = false;
  bool job_deleted = false;
};

struct TrainerMetrics {
  std::atomic<long long> jobs_created{0}, jobs_succeeded{0}, jobs_failed{0}, jobs_restarted{0}, pods_created{0},
      pods_deleted{0};
};

class Trainer {
 public:
  Trainer(std::shared_ptr<Client> c, std::shared_ptr<EventRecorder> rec, TrainerOptions opts,
          TrainerMetrics* metrics = nullptr)
      : client_(std::move(c)), rec_(std::move(rec)), opts_(std::move(opts)), metrics_(metrics) {}

  ReconcileResult reconcile(const Json& tfjob, const std::vector<Json>& pods, const std::vector<Json>& services);

  // Pure helpers (tested directly)
  Json make_pod(const api::TFJob& job, api::RType t, int index, int generation) const;
  Json make_service(const api::TFJob& job, api::RType t, int index) const;
  std::map<std::string, int> service_ports(const api::TFJob& job) const;
  // Per-pod state from its "tensorflow" container: Running|Succeeded|Failed|Pending + retryable?
  struct PodState {
    std::string state;  // Pending | Running | Succeeded | Failed
    int exit_code = 0;
    std::string reason;
    bool retryable = false;
    int restarts = 0;
  };
  static PodState pod_state(const Json& pod);

 private:
  ApiStatus write_status(api::TFJob& job, const Json& orig);
  ReconcileResult cleanup(api::TFJob& job, const std::vector<Json>& pods, const std::vector<Json>& services,
                          bool all_pods, bool remove_finalizer, const Json& orig);
  void ensure_podgroup(const api::TFJob& job);
  std::shared_ptr<Client> client_;
  std::shared_ptr<EventRecorder> rec_;
  TrainerOptions opts_;
  TrainerMetrics* metrics_;
};

}  // namespace tfk
