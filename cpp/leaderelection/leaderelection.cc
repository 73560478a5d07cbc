#include "leaderelection.h"

namespace tfk {

std::string LeaderElector::observed_leader() const {
  std::lock_guard<std::mutex> g(mu_);
  return observed_;
}

bool LeaderElector::try_acquire_or_renew() {
  int64_t now = now_ms();
  Json lease;
  ApiStatus st = client_->get("leases", cfg_.lock_namespace, cfg_.lock_name, &lease);
  if (st.code == 404) {
    Json l = Json::object();
    l["apiVersion"] = "coordination.k8s.io/v1";
    l["kind"] = "Lease";
    l["metadata"]["name"] = cfg_.lock_name;
    l["metadata"]["namespace"] = cfg_.lock_namespace;
    l["spec"]["holderIdentity"] = cfg_.identity;
    l["spec"]["leaseDurationSeconds"] = (double)cfg_.lease_duration_ms / 1000.0;
    l["spec"]["acquireTime"] = rfc3339(now);
    l["spec"]["renewTime"] = rfc3339(now);
    l["spec"]["leaseTransitions"] = 0;
    Json out;
    bool ok = client_->create("leases", cfg_.lock_namespace, l, &out).ok();
    if (ok) {
      std::lock_guard<std::mutex> g(mu_);
      observed_ = cfg_.identity;
    }
    return ok;
  }
  if (!st.ok()) return false;
  const Json& spec = lease.at("spec");
  std::string holder = spec.at("holderIdentity").str();
  int64_t renew = parse_rfc3339(spec.at("renewTime").str());
  int64_t dur = (int64_t)(spec.at("leaseDurationSeconds").as_double(15) * 1000);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (observed_ != holder && cfg_.on_new_leader) cfg_.on_new_leader(holder);
    observed_ = holder;
  }
  if (!holder.empty() && holder != cfg_.identity && renew >= 0 && now < renew + dur) return false;  // held by other
  Json next = lease.clone();
  if (holder != cfg_.identity) {
    next["spec"]["acquireTime"] = rfc3339(now);
    next["spec"]["leaseTransitions"] = spec.at("leaseTransitions").as_int(0) + (holder.empty() ? 0 : 1);
  }
  next["spec"]["holderIdentity"] = cfg_.identity;
  next["spec"]["renewTime"] = rfc3339(now);
  next["spec"]["leaseDurationSeconds"] = (double)cfg_.lease_duration_ms / 1000.0;
  Json out;
  bool ok = client_->update("leases", cfg_.lock_namespace, next, &out).ok();  // 409 => someone else won
  if (ok) {
    std::lock_guard<std::mutex> g(mu_);
    observed_ = cfg_.identity;
  }
  return ok;
}

void LeaderElector::run(StopToken& stop) {
  // acquire
  while (!stop.stopped()) {
    if (try_acquire_or_renew()) break;
    stop.wait_for(cfg_.retry_period_ms);
  }
  if (stop.stopped()) return;
  leader_ = true;
  TFK_LOG(Info, "became leader", Json(Json::object_t{{"identity", Json(cfg_.identity)}, {"lock", Json(cfg_.lock_name)}}));
  StopToken lead_stop;
  std::thread lead;
  if (cfg_.on_started_leading) lead = std::thread([&] { cfg_.on_started_leading(lead_stop); });
  // renew
  int64_t last_ok = mono_ms();
  while (!stop.stopped()) {
    if (stop.wait_for(cfg_.retry_period_ms)) break;
    if (try_acquire_or_renew()) {
      last_ok = mono_ms();
    } else if (mono_ms() - last_ok > cfg_.renew_deadline_ms) {
      TFK_LOG(Error, "leader election lost", Json(Json::object_t{{"identity", Json(cfg_.identity)}}));
      break;
    }
  }
  leader_ = false;
  lead_stop.stop();
  if (lead.joinable()) lead.join();
  if (cfg_.on_stopped_leading) cfg_.on_stopped_leading();
}

}  // namespace tfk
