// TFJob controller (reference: pkg/controller/controller.go, images/tf3.PNG:L58; the informer ->
// workqueue -> workers pattern of the sample, k8s-operator.md:80-203, with its bugs fixed:
// Done on every path, errors retried via AddRateLimited/Forget, real update detection, nonzero
// resync, a stop channel that actually stops). Watches TFJobs AND the Pods/Services it owns.
#pragma once
#include <atomic>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../cache/informer.h"
#include "../util/workqueue.h"
#include "trainer.h"

namespace tfk {

struct ControllerOptions {
  int threadiness = 2;
  int64_t resync_ms = 30000;
  std::string ns;  // "" = all namespaces
  TrainerOptions trainer;
  int max_retries_logged = 15;
};

class TFJobController {
 public:
  TFJobController(std::shared_ptr<Client> c, ControllerOptions opts);
  ~TFJobController();
  // Blocks until stop: starts informers, waits for cache sync, runs `threadiness` workers.
  void run(StopToken& stop);
  // Synchronously reconcile one key (tests / sync loop). Returns (forget, error).
  bool sync_handler(const std::string& key, std::string* err);
  RateLimitingQueue& queue() { return queue_; }
  std::string metrics_text() const;
  SharedInformer& tfjob_informer() { return *jobs_; }
  SharedInformer& pod_informer() { return *pods_; }
  bool synced() const;
  std::atomic<long long> syncs{0};

 private:
  void enqueue(const Json& tfjob);
  void enqueue_owner(const Json& obj);
  void worker(StopToken& stop);
  bool process_next();
  std::shared_ptr<Client> client_;
  ControllerOptions opts_;
  std::unique_ptr<SharedInformer> jobs_, pods_, services_;
  RateLimitingQueue queue_;
  std::shared_ptr<EventRecorder> recorder_;
  TrainerMetrics metrics_;
  std::unique_ptr<Trainer> trainer_;
  mutable std::mutex hist_mu_;
  std::vector<double> reconcile_ms_;  // histogram samples
  std::atomic<long long> errors_{0};
};

}  // namespace tfk
