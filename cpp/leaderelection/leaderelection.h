// Lease-based leader election (reference: k8s-operator.md:59 "leaderelection provides high
// availability", :237; client-go leaderelection.RunOrDie). Lock = a coordination.k8s.io/v1 Lease in
// tfk-apiserver; optimistic concurrency (resourceVersion) makes acquire/renew atomic.
#pragma once
#include <functional>
#include <memory>
#include <string>
#include <thread>

#include "../client/client.h"
#include "../common/util.h"

namespace tfk {

struct LeaderElectionConfig {
  std::string lock_namespace = "default";
  std::string lock_name = "tf-operator";
  std::string identity;
  int64_t lease_duration_ms = 15000;
  int64_t renew_deadline_ms = 10000;
  int64_t retry_period_ms = 2000;
  std::function<void(StopToken&)> on_started_leading;  // runs in its own thread
  std::function<void()> on_stopped_leading;
  std::function<void(const std::string&)> on_new_leader;
};

class LeaderElector {
 public:
  LeaderElector(std::shared_ptr<Client> c, LeaderElectionConfig cfg) : client_(std::move(c)), cfg_(std::move(cfg)) {}
  // Blocks: acquire, lead (callback thread), renew until lost or stopped. Returns after leadership
  // is lost (caller typically exits, like RunOrDie) or stop is requested.
  void run(StopToken& stop);
  bool is_leader() const { return leader_; }
  std::string observed_leader() const;
  // one acquire-or-renew attempt (exposed for tests)
  bool try_acquire_or_renew();

 private:
  std::shared_ptr<Client> client_;
  LeaderElectionConfig cfg_;
  std::atomic<bool> leader_{false};
  mutable std::mutex mu_;
  std::string observed_;
};

}  // namespace tfk
