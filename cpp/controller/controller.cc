#include "controller.h"

#include <sstream>

namespace tfk {

TFJobController::TFJobController(std::shared_ptr<Client> c, ControllerOptions opts)
    : client_(std::move(c)), opts_(std::move(opts)), queue_("TFJobs") {
  jobs_.reset(new SharedInformer(client_, "tfjobs", opts_.ns, opts_.resync_ms));
  pods_.reset(new SharedInformer(client_, "pods", opts_.ns, opts_.resync_ms, "tf-job-name"));
  services_.reset(new SharedInformer(client_, "services", opts_.ns, opts_.resync_ms, "tf-job-name"));
  pods_->indexer().add_indexer("job", [](const Json& o) {
    return std::vector<std::string>{o.path("metadata.namespace").str() + "/" + o.path("metadata.labels").at("tf-job-name").str()};
  });
  services_->indexer().add_indexer("job", [](const Json& o) {
    return std::vector<std::string>{o.path("metadata.namespace").str() + "/" + o.path("metadata.labels").at("tf-job-name").str()};
  });
  recorder_ = std::make_shared<EventRecorder>(client_);
  trainer_.reset(new Trainer(client_, recorder_, opts_.trainer, &metrics_));
  jobs_->add_event_handler({
      [this](const Json& o) { enqueue(o); },
      [this](const Json& oldo, const Json& newo) {
        // resync delivers old == new: still enqueue (level-triggered repair); a real change
        // is detected by resourceVersion (the reference's updatePod compared old with old).
        (void)oldo;
        enqueue(newo);
      },
      [this](const Json& o) { enqueue(o); },
  });
  EventHandlers owned{[this](const Json& o) { enqueue_owner(o); },
                      [this](const Json& oldo, const Json& newo) {
                        if (oldo.path("metadata.resourceVersion") != newo.path("metadata.resourceVersion"))
                          enqueue_owner(newo);
                      },
                      [this](const Json& o) { enqueue_owner(o); }};
  pods_->add_event_handler(owned);
  services_->add_event_handler(owned);
}

TFJobController::~TFJobController() { queue_.shutdown(); }

void TFJobController::enqueue(const Json& tfjob) { queue_.add(meta_namespace_key(tfjob)); }

void TFJobController::enqueue_owner(const Json& obj) {
  for (auto& ref : obj.path("metadata.ownerReferences").items())
    if (ref.at("kind").str() == api::kKind && ref.at("controller").as_bool(false)) {
      queue_.add(obj.path("metadata.namespace").str() + "/" + ref.at("name").str());
      return;
    }
}

bool TFJobController::synced() const { return jobs_->has_synced() && pods_->has_synced() && services_->has_synced(); }

bool TFJobController::sync_handler(const std::string& key, std::string* err) {
  int64_t t0 = mono_ms();
  syncs++;
  std::string ns, name;
  if (!split_meta_namespace_key(key, &ns, &name)) { *err = "invalid key " + key; return true; }
  Json job;
  if (!Lister(jobs_->indexer()).get(ns, name, &job)) {
    // deleted: owned pods/services are garbage-collected by ownerReference
    return true;
  }
  std::vector<Json> pods = pods_->indexer().by_index("job", ns + "/" + name);
  std::vector<Json> svcs = services_->indexer().by_index("job", ns + "/" + name);
  std::string uid = job.path("metadata.uid").str();
  auto owned = [&](std::vector<Json>& v) {
    std::vector<Json> out;
    for (auto& o : v)
      for (auto& ref : o.path("metadata.ownerReferences").items())
        if (ref.at("uid").str() == uid) { out.push_back(o); break; }
    v.swap(out);
  };
  owned(pods);
  owned(svcs);
  ReconcileResult r = trainer_->reconcile(job, pods, svcs);
  double ms = (double)(mono_ms() - t0);
  {
    std::lock_guard<std::mutex> g(hist_mu_);
    reconcile_ms_.push_back(ms);
    if (reconcile_ms_.size() > 10000) reconcile_ms_.erase(reconcile_ms_.begin(), reconcile_ms_.begin() + 5000);
  }
  TFK_LOG(Debug, "Finished syncing job", Json(Json::object_t{{"key", Json(key)}, {"ms", Json(ms)}}));
  if (!r.error.empty()) { *err = r.error; return false; }
  if (r.requeue) queue_.add_after(key, 50);
  if (r.requeue_after_ms > 0) queue_.add_after(key, r.requeue_after_ms + 10);
  return true;
}

bool TFJobController::process_next() {
  std::string key;
  if (!queue_.get(&key)) return false;
  // Done immediately after Get semantics: guarantee Done on EVERY path
  struct DoneGuard {
    RateLimitingQueue& q;
    const std::string& k;
    ~DoneGuard() { q.done(k); }
  } guard{queue_, key};
  std::string err;
  bool forget = false;
  try {
    forget = sync_handler(key, &err);
  } catch (const std::exception& e) {
    err = e.what();
  }
  if (err.empty() && forget) {
    queue_.forget(key);
  } else {
    errors_++;
    if (queue_.num_requeues(key) < opts_.max_retries_logged)
      TFK_LOG(Warn, "error syncing tfjob, requeueing", Json(Json::object_t{{"key", Json(key)}, {"error", Json(err)}}));
    queue_.add_rate_limited(key);
  }
  return true;
}

void TFJobController::worker(StopToken& stop) {
  while (!stop.stopped() && process_next()) {
  }
}

void TFJobController::run(StopToken& stop) {
  jobs_->start(stop);
  pods_->start(stop);
  services_->start(stop);
  TFK_LOG(Info, "waiting for informer caches to sync");
  while (!stop.stopped() && !wait_for_cache_sync({jobs_.get(), pods_.get(), services_.get()}, 1000)) {
  }
  TFK_LOG(Info, "starting workers", Json(Json::object_t{{"threadiness", Json(opts_.threadiness)}}));
  std::vector<std::thread> ws;
  for (int i = 0; i < opts_.threadiness; ++i) ws.emplace_back([this, &stop] { worker(stop); });
  while (!stop.wait_for(500)) {
  }
  queue_.shutdown();
  for (auto& t : ws) t.join();
  TFK_LOG(Info, "controller stopped");
}

std::string TFJobController::metrics_text() const {
  std::ostringstream os;
  os << "# TYPE tfjob_created_total counter\ntfjob_created_total " << metrics_.jobs_created << "\n";
  os << "# TYPE tfjob_succeeded_total counter\ntfjob_succeeded_total " << metrics_.jobs_succeeded << "\n";
  os << "# TYPE tfjob_failed_total counter\ntfjob_failed_total " << metrics_.jobs_failed << "\n";
  os << "# TYPE tfjob_restarted_total counter\ntfjob_restarted_total " << metrics_.jobs_restarted << "\n";
  os << "# TYPE tfjob_pods_created_total counter\ntfjob_pods_created_total " << metrics_.pods_created << "\n";
  os << "# TYPE tfjob_pods_deleted_total counter\ntfjob_pods_deleted_total " << metrics_.pods_deleted << "\n";
  os << "# TYPE workqueue_depth gauge\nworkqueue_depth{name=\"TFJobs\"} " << const_cast<RateLimitingQueue&>(queue_).len() << "\n";
  os << "# TYPE workqueue_retries_total counter\nworkqueue_retries_total{name=\"TFJobs\"} " << queue_.retries() << "\n";
  os << "# TYPE tfjob_sync_errors_total counter\ntfjob_sync_errors_total " << errors_ << "\n";
  static const double buckets[] = {1, 5, 10, 25, 50, 100, 250, 1000, 5000};
  std::lock_guard<std::mutex> g(hist_mu_);
  os << "# TYPE reconcile_duration_seconds histogram\n";
  double sum = 0;
  for (double b : buckets) {
    long long c = 0;
    for (double v : reconcile_ms_) c += v <= b;
    os << "reconcile_duration_seconds_bucket{le=\"" << b / 1000.0 << "\"} " << c << "\n";
  }
  for (double v : reconcile_ms_) sum += v;
  os << "reconcile_duration_seconds_bucket{le=\"+Inf\"} " << reconcile_ms_.size() << "\n";
  os << "reconcile_duration_seconds_sum " << sum / 1000.0 << "\nreconcile_duration_seconds_count " << reconcile_ms_.size() << "\n";
  return os.str();
}

}  // namespace tfk
