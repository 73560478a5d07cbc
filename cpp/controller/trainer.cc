#include "trainer.h"

#include "../client/tfjob_client.h"

#include <algorithm>
#include <set>

#include "../common/util.h"

namespace tfk {

using api::RType;

// ------------------------------------------------------------------------------ labels
Json ReplicaLabels::for_replica(const api::TFJob& job, RType t, int index) {
  Json l = Json::object();
  // kubeflow v1 label set
  l["group-name"] = api::kGroupV1;
  l["tf-job-name"] = job.name();
  l["tf-replica-type"] = api::rtype_lower(t);
  l["tf-replica-index"] = std::to_string(index);
  if (t == RType::Chief || t == RType::Master) l["tf-job-role"] = "master";
  // v1alpha1 (tensorflow/k8s) label set: kubeflow.org, tf_job_name, job_type, runtime_id, task_index
  if (job.is_v1alpha1()) {
    l["kubeflow.org"] = "";
    l["tf_job_name"] = job.name();
    l["job_type"] = api::rtype_upper(t);
    l["runtime_id"] = job.runtime_id;
    l["task_index"] = std::to_string(index);
  }
  return l;
}

std::string ReplicaLabels::job_selector(const api::TFJob& job) { return "tf-job-name=" + job.name(); }

void EventRecorder::event(const Json& obj, const std::string& type, const std::string& reason, const std::string& msg) {
  Json e = Json::object();
  e["apiVersion"] = "v1";
  e["kind"] = "Event";
  std::string name = obj.path("metadata.name").str();
  std::string ns = obj.path("metadata.namespace").str("default");
  e["metadata"]["name"] = name + "." + rand_string(10);
  e["metadata"]["namespace"] = ns;
  e["involvedObject"]["kind"] = obj.at("kind").str();
  e["involvedObject"]["name"] = name;
  e["involvedObject"]["namespace"] = ns;
  e["involvedObject"]["uid"] = obj.path("metadata.uid").str();
  e["involvedObject"]["apiVersion"] = obj.at("apiVersion").str();
  e["reason"] = reason;
  e["message"] = msg;
  e["type"] = type;
  e["source"]["component"] = component_;
  std::string now = rfc3339(now_ms());
  e["firstTimestamp"] = now;
  e["lastTimestamp"] = now;
  e["count"] = 1;
  Json out;
  client_->create("events", ns, e, &out);
  count_++;
  TFK_LOG(Info, "event", Json(Json::object_t{{"object", Json(ns + "/" + name)}, {"type", Json(type)},
                                             {"reason", Json(reason)}, {"message", Json(msg)}}));
}

// ------------------------------------------------------------------------------ pods / services
std::map<std::string, int> Trainer::service_ports(const api::TFJob& job) const {
  std::map<std::string, int> m;
  if (!opts_.local_ports) return m;
  for (auto& r : job.replicas)
    for (int i = 0; i < std::max(0, r.replicas); ++i) {
      std::string svc = api::gen_name(job, r.type, i);
      std::string key = job.ns() + "/" + svc + "/" + job.uid();
      uint32_t h = crc32c(key.data(), key.size());
      m[svc] = opts_.local_port_base + (int)(h % 20000u);
    }
  return m;
}

static int total_replicas(const api::TFJob& job) {
  int n = 0;
  for (auto& r : job.replicas) n += std::max(0, r.replicas);
  return n;
}

Json Trainer::make_service(const api::TFJob& job, RType t, int index) const {
  Json s = Json::object();
  s["apiVersion"] = "v1";
  s["kind"] = "Service";
  std::string name = api::gen_name(job, t, index);
  s["metadata"]["name"] = name;
  s["metadata"]["namespace"] = job.ns();
  s["metadata"]["labels"] = ReplicaLabels::for_replica(job, t, index);
  s["metadata"]["ownerReferences"] = Json(Json::array_t{api::as_owner(job)});
  s["spec"]["selector"] = ReplicaLabels::for_replica(job, t, index);
  s["spec"]["clusterIP"] = "None";  // headless: stable DNS for the task
  int port = api::kDefaultPort;
  if (const api::ReplicaSpec* r = job.replica(t)) {
    if (r->tf_port > 0) port = r->tf_port;
  }
  auto ports = service_ports(job);
  if (ports.count(name)) port = ports[name];
  Json p = Json::object();
  p["name"] = api::kPortName;
  p["port"] = port;
  p["targetPort"] = port;
  s["spec"]["ports"] = Json(Json::array_t{p});
  return s;
}

// The training world a pod's TF_CONFIG describes: replica counts of every cluster member type
// (the Evaluator is outside the cluster spec). Pods carry it as an annotation so a replica-count
// change (scale up or down) is detected against the pods that are running.
static std::string world_signature(const api::TFJob& job) {
  std::map<std::string, int> m;
  for (auto& r : job.replicas)
    if (r.type != RType::Evaluator) m[api::rtype_title(r.type)] = r.replicas;
  std::string s;
  for (auto& kv : m) s += (s.empty() ? "" : ",") + kv.first + "=" + std::to_string(kv.second);
  return s;
}

Json Trainer::make_pod(const api::TFJob& job, RType t, int index, int generation) const {
  const api::ReplicaSpec* rs = job.replica(t);
  Json tmpl = rs && rs->template_.is_object() ? rs->template_.clone() : Json::object();
  Json pod = Json::object();
  pod["apiVersion"] = "v1";
  pod["kind"] = "Pod";
  std::string name = api::gen_name(job, t, index);
  Json md = tmpl.at("metadata").is_object() ? tmpl.at("metadata").clone() : Json::object();
  md["name"] = name;
  md["namespace"] = job.ns();
  md.erase("generateName");
  const Json labels = ReplicaLabels::for_replica(job, t, index);
  for (auto& kv : labels.fields()) md["labels"][kv.first] = kv.second;
  int min_avail = job.run_policy.scheduling.min_available >= 0 ? job.run_policy.scheduling.min_available
                                                               : total_replicas(job);
  md["annotations"]["scheduling.tfk.io/group-name"] = job.name();
  md["annotations"]["scheduling.tfk.io/min-available"] = std::to_string(min_avail);
  md["annotations"]["tfk.io/restart-generation"] = std::to_string(generation);
  md["annotations"]["tfk.io/world"] = world_signature(job);
  // opt-in (TFJob annotation): every gang member sees all of the gang's GPUs, so RCCL between the
  // pods of one node rides xGMI peer-to-peer (IPC) instead of falling back to host shared memory
  const Json& gv = job.metadata.path("annotations").at(api::kGangVisibleGpus);
  if (gv.is_string() && !gv.str().empty()) md["annotations"][api::kGangVisibleGpus] = gv.str();
  md["ownerReferences"] = Json(Json::array_t{api::as_owner(job)});
  pod["metadata"] = md;
  Json spec = tmpl.at("spec").is_object() ? tmpl.at("spec").clone() : Json::object();
  if (rs && rs->is_default_ps && spec.at("containers").size() == 0) {
    Json c = Json::object();
    c["name"] = api::kContainerName;
    c["image"] = job.tf_image.empty() ? "tfk/runtime:latest" : job.tf_image;
    c["command"] = Json(Json::array_t{Json("/bin/sh"), Json("-c"), Json(opts_.default_ps_command)});
    spec["containers"] = Json(Json::array_t{c});
  }
  // restart policy: controller-managed ExitCode -> kubelet "Never"
  std::string rp = rs ? rs->restart_policy : "";
  if (job.is_v1alpha1()) rp = spec.at("restartPolicy").str("OnFailure");
  spec["restartPolicy"] = (rp == "ExitCode" || rp.empty()) ? "Never" : rp;
  if (!job.run_policy.scheduling.priority_class.empty() && !spec.at("priorityClassName").is_string())
    spec["priorityClassName"] = job.run_policy.scheduling.priority_class;
  if (!job.scheduler_name.empty()) spec["schedulerName"] = job.scheduler_name;
  else if (opts_.gang_scheduling) spec["schedulerName"] = opts_.gang_scheduler_name;
  auto ports = service_ports(job);
  std::string tfc = api::tf_config(job, t, index, opts_.cluster_domain, opts_.local_ports ? &ports : nullptr);
  for (auto& c : spec["containers"].items_mut()) {
    if (c.at("name").str() != api::kContainerName) continue;
    auto add_env = [&](const std::string& k, const std::string& v) {
      for (auto& e : c["env"].items_mut())
        if (e.at("name").str() == k) { e["value"] = v; return; }
      Json e = Json::object();
      e["name"] = k;
      e["value"] = v;
      c["env"].push_back(e);
    };
    add_env("TF_CONFIG", tfc);
    add_env("TFK_JOB_NAME", job.name());
    add_env("TFK_JOB_NAMESPACE", job.ns());
    add_env("TFK_REPLICA_TYPE", api::rtype_lower(t));
    add_env("TFK_REPLICA_INDEX", std::to_string(index));
    add_env("TFK_RESTART_GENERATION", std::to_string(generation));
    if (opts_.local_ports) add_env("TFK_LOCAL_DNS", "1");
  }
  pod["spec"] = spec;
  return pod;
}

Trainer::PodState Trainer::pod_state(const Json& pod) {
  PodState ps;
  std::string phase = pod.path("status.phase").str("Pending");
  const Json* cs = nullptr;
  for (auto& c : pod.path("status.containerStatuses").items())
    if (c.at("name").str() == api::kContainerName) cs = &c;
  if (!cs && pod.path("status.containerStatuses").size()) cs = &pod.path("status.containerStatuses")[0];
  if (cs) ps.restarts = (int)cs->at("restartCount").as_int(0);
  if (phase == "Succeeded") { ps.state = "Succeeded"; return ps; }
  if (phase == "Failed") {
    ps.state = "Failed";
    if (cs) {
      const Json& term = cs->path("state.terminated").is_object() ? cs->path("state.terminated")
                                                                   : cs->path("lastState.terminated");
      ps.exit_code = (int)term.at("exitCode").as_int(1);
      ps.reason = term.at("reason").str();
    } else {
      ps.exit_code = 1;
      ps.reason = pod.path("status.reason").str();
    }
    ps.retryable = api::is_retryable_exit(ps.exit_code, ps.reason);
    return ps;
  }
  ps.state = phase == "Running" ? "Running" : "Pending";
  return ps;
}

// ------------------------------------------------------------------------------ reconcile
ApiStatus Trainer::write_status(api::TFJob& job, const Json& orig) {
  // typed TFJob client (typed/tensorflow/<version>/tfjob.go UpdateStatus) in the job's own version
  job.metadata["resourceVersion"] = orig.path("metadata.resourceVersion");
  return TFJobInterface(client_, job.ns(), job.api_version).UpdateStatus(job);
}

void Trainer::ensure_podgroup(const api::TFJob& job) {
  if (!opts_.gang_scheduling) return;
  Json pg = Json::object();
  pg["apiVersion"] = "scheduling.tfk.io/v1";
  pg["kind"] = "PodGroup";
  pg["metadata"]["name"] = job.name();
  pg["metadata"]["namespace"] = job.ns();
  pg["metadata"]["ownerReferences"] = Json(Json::array_t{api::as_owner(job)});
  int min_avail = job.run_policy.scheduling.min_available >= 0 ? job.run_policy.scheduling.min_available
                                                               : total_replicas(job);
  pg["spec"]["minMember"] = min_avail;
  if (!job.run_policy.scheduling.queue.empty()) pg["spec"]["queue"] = job.run_policy.scheduling.queue;
  if (!job.run_policy.scheduling.priority_class.empty())
    pg["spec"]["priorityClassName"] = job.run_policy.scheduling.priority_class;
  Json out;
  client_->create("podgroups", job.ns(), pg, &out);
}

ReconcileResult Trainer::cleanup(api::TFJob& job, const std::vector<Json>& pods, const std::vector<Json>& services,
                                 bool all_pods, bool remove_finalizer, const Json& orig) {
  ReconcileResult r;
  for (auto& p : pods) {
    if (p.path("metadata.deletionTimestamp").is_string()) continue;
    std::string phase = p.path("status.phase").str("Pending");
    bool active = phase != "Succeeded" && phase != "Failed";
    if (all_pods || active) {
      if (client_->remove("pods", job.ns(), p.path("metadata.name").str(), "Background").ok()) {
        r.pods_deleted++;
        if (metrics_) metrics_->pods_deleted++;
      }
    }
  }
  for (auto& s : services)
    if (client_->remove("services", job.ns(), s.path("metadata.name").str(), "Background").ok()) r.services_deleted++;
  if (remove_finalizer) {
    Json obj = orig.clone();
    Json fins = Json::array();
    for (auto& f : obj.path("metadata.finalizers").items())
      if (f.str() != api::kFinalizer) fins.push_back(f);
    obj["metadata"]["finalizers"] = fins;
    Json out;
    ApiStatus st = client_->update(api::kPlural, job.ns(), obj, &out);
    if (!st.ok() && st.code != 404) { r.requeue = true; r.error = st.message; }
  }
  return r;
}

static std::string join(const std::vector<std::string>& v, const std::string& sep) {
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) s += (i ? sep : "") + v[i];
  return s;
}

ReconcileResult Trainer::reconcile(const Json& orig, const std::vector<Json>& pods_in,
                                   const std::vector<Json>& services) {
  ReconcileResult res;
  api::TFJob job;
  try {
    job = api::from_json(orig);
  } catch (const std::exception& e) {
    res.error = std::string("malformed TFJob: ") + e.what();
    return res;
  }
  std::string now = rfc3339(now_ms());
  int64_t now_i = now_ms();
  // ---------------------------------------------------------------- deletion (finalizer path)
  if (orig.path("metadata.deletionTimestamp").is_string()) {
    return cleanup(job, pods_in, services, true, true, orig);
  }
  // ---------------------------------------------------------------- setup
  bool fresh = job.is_v1alpha1() ? job.status.phase.empty() : job.status.conditions.empty();
  if (fresh) {
    api::set_defaults(job);
    auto errs = api::validate(job);
    if (!errs.empty()) {
      std::string msg = join(errs, "; ");
      job.status.phase = "Failed";
      job.status.state = "Failed";
      job.status.reason = msg;
      api::set_condition(job.status, "Failed", "InvalidTFJobSpec", msg, now);
      if (metrics_) metrics_->jobs_failed++;
      rec_->event(orig, "Warning", "InvalidTFJobSpec", msg);
      ApiStatus st = write_status(job, orig);
      if (!st.ok()) res.requeue = true;
      res.status_changed = true;
      return res;
    }
    bool need_update = false;
    Json obj = orig.clone();
    bool has_fin = false;
    for (auto& f : orig.path("metadata.finalizers").items()) has_fin |= (f.str() == api::kFinalizer);
    if (!has_fin) {
      obj["metadata"]["finalizers"].push_back(Json(api::kFinalizer));
      need_update = true;
    }
    if (job.is_v1alpha1() && job.runtime_id.empty()) {
      job.runtime_id = rand_string(4);
      obj["spec"]["runtimeId"] = job.runtime_id;
      need_update = true;
    }
    Json cur = orig;
    if (need_update) {
      Json out;
      ApiStatus st = client_->update(api::kPlural, job.ns(), obj, &out);
      if (!st.ok()) { res.requeue = true; res.error = st.message; return res; }
      cur = out;
    }
    if (job.is_v1alpha1()) {
      job.status.phase = "Creating";
      job.status.state = "Running";
    }
    api::set_condition(job.status, "Created", "TFJobCreated", "TFJob " + job.name() + " is created.", now);
    job.status.start_time = now;
    if (metrics_) metrics_->jobs_created++;
    rec_->event(orig, "Normal", "TFJobCreated", "TFJob " + job.name() + " is created.");
    ApiStatus st = write_status(job, cur);
    res.status_changed = true;
    res.requeue = true;  // next pass creates resources against the fresh object
    if (!st.ok()) res.error = st.message;
    return res;
  }
  api::set_defaults(job);
  api::configure_accelerators(job, opts_.controller_config);
  const std::string old_status = api::to_json(job).at("status").dump();

  // ---------------------------------------------------------------- finished: cleanup + TTL
  if (api::is_finished(job.status)) {
    std::string policy = job.is_v1alpha1() ? "Running" : job.run_policy.clean_pod_policy;
    if (policy != "None") {
      std::vector<Json> keep_svcs;  // services go with the job's pods
      ReconcileResult c = cleanup(job, pods_in, policy == "None" ? keep_svcs : services, policy == "All", false, orig);
      res.pods_deleted = c.pods_deleted;
      res.services_deleted = c.services_deleted;
    }
    if (job.run_policy.ttl_seconds_after_finished >= 0 && !job.status.completion_time.empty()) {
      int64_t done = parse_rfc3339(job.status.completion_time);
      int64_t expire = done + job.run_policy.ttl_seconds_after_finished * 1000;
      if (now_i >= expire) {
        client_->remove(api::kPlural, job.ns(), job.name(), "Background");
        res.job_deleted = true;
      } else {
        res.requeue_after_ms = expire - now_i;
      }
    }
    if (job.is_v1alpha1() && job.status.phase != "Done" && job.status.phase != "Failed") {
      job.status.phase = "Done";
      write_status(job, orig);
      res.status_changed = true;
    }
    return res;
  }

  auto fail_job = [&](const std::string& reason, const std::string& msg) {
    job.status.phase = job.is_v1alpha1() ? "Failed" : job.status.phase;
    job.status.state = "Failed";
    job.status.reason = msg;
    api::set_condition(job.status, "Failed", reason, msg, now);
    if (job.status.completion_time.empty()) job.status.completion_time = now;
    if (metrics_) metrics_->jobs_failed++;
    rec_->event(orig, "Warning", reason, msg);
  };

  // ---------------------------------------------------------------- active deadline
  if (job.run_policy.active_deadline_seconds >= 0 && !job.status.start_time.empty()) {
    int64_t start = parse_rfc3339(job.status.start_time);
    int64_t dl = start + job.run_policy.active_deadline_seconds * 1000;
    if (now_i >= dl) {
      fail_job("DeadlineExceeded", "TFJob " + job.name() + " has run past its activeDeadlineSeconds");
      cleanup(job, pods_in, {}, false, false, orig);
      ApiStatus st = write_status(job, orig);
      res.status_changed = true;
      if (!st.ok()) res.requeue = true;
      return res;
    }
    res.requeue_after_ms = dl - now_i;
  }

  ensure_podgroup(job);
  // ---------------------------------------------------------------- index existing pods
  std::map<std::pair<RType, int>, Json> slot;
  std::vector<Json> extra;
  // Pods of an older generation were already acted upon (a gang restart or a resize deleted
  // them); a stale cache or a late kubelet status must not restart the job a second time.
  const int cur_gen = job.status.restart_count + job.status.resize_count;
  for (auto& p : pods_in) {
    if (p.path("metadata.deletionTimestamp").is_string()) continue;
    const Json& ga = p.path("metadata.annotations").at("tfk.io/restart-generation");
    if (ga.is_string() && atoi(ga.str().c_str()) < cur_gen) {
      if (client_->remove("pods", job.ns(), p.path("metadata.name").str(), "Background").ok()) res.pods_deleted++;
      continue;
    }
    const Json& l = p.path("metadata.labels");
    RType t = api::rtype_from(l.at("tf-replica-type").str());
    int idx = atoi(l.at("tf-replica-index").str("-1").c_str());
    const api::ReplicaSpec* rs = job.replica(t);
    if (!rs || idx < 0 || idx >= rs->replicas) { extra.push_back(p); continue; }
    auto key = std::make_pair(t, idx);
    if (!slot.count(key) || slot[key].path("metadata.creationTimestamp").str() < p.path("metadata.creationTimestamp").str())
      slot[key] = p;
  }
  // ---------------------------------------------------------------- coordinated resize (扩容/缩容)
  // A replica-count change alters the cluster every rank's TF_CONFIG lists, and collective
  // training (RCCL rings, PS shard maps) cannot admit or drop a rank in place: every pod built for
  // the old world is replaced together under a new generation, and the new gang resumes from the
  // chief's latest checkpoint at the new world size. Not counted against backoffLimit.
  const std::string world = world_signature(job);
  std::vector<Json> stale;
  for (auto& kv : slot) {
    const Json& w = kv.second.path("metadata.annotations").at("tfk.io/world");
    if (w.is_string() && w.str() != world && kv.first.first != RType::Evaluator) stale.push_back(kv.second);
  }
  if (!stale.empty()) {
    for (auto& p : extra) stale.push_back(p);
    for (auto& kv : slot)
      if (kv.first.first != RType::Evaluator) stale.push_back(kv.second);
    std::set<std::string> gone;
    for (auto& p : stale) {
      const std::string n = p.path("metadata.name").str();
      if (!gone.insert(n).second) continue;
      if (client_->remove("pods", job.ns(), n, "Background").ok()) {
        res.pods_deleted++;
        if (metrics_) metrics_->pods_deleted++;
      }
    }
    job.status.resize_count++;
    const std::string msg = "TFJob " + job.name() + " is resizing to " + world + " (generation " +
                            std::to_string(job.status.restart_count + job.status.resize_count) + ")";
    api::set_condition(job.status, "Restarting", "TFJobResized", msg, now);
    if (job.is_v1alpha1()) job.status.phase = "Running";
    rec_->event(orig, "Normal", "TFJobResized", msg);
    ApiStatus st = write_status(job, orig);
    res.status_changed = true;
    res.requeue = true;
    if (!st.ok()) res.error = st.message;
    return res;
  }
  // replicas beyond the count of a pre-annotation pod set (no world recorded): remove them
  for (auto& p : extra)
    if (client_->remove("pods", job.ns(), p.path("metadata.name").str(), "Background").ok()) {
      res.pods_deleted++;
      if (metrics_) metrics_->pods_deleted++;
    }
  std::set<std::string> have_svc;
  for (auto& s : services) have_svc.insert(s.path("metadata.name").str());
  // pod generation: gang restarts + coordinated resizes (TFK_RESTART_GENERATION in the pod)
  int generation = job.status.restart_count + job.status.resize_count;

  // ---------------------------------------------------------------- services + pods
  std::vector<std::string> permanent_failures;
  bool retry_needed = false;
  std::string retry_msg;
  job.status.replica_statuses.clear();
  for (auto& r : job.replicas) {
    api::ReplicaStatus rst;
    for (int i = 0; i < r.replicas; ++i) {
      std::string name = api::gen_name(job, r.type, i);
      if (r.type != RType::Evaluator && !have_svc.count(name)) {
        Json out;
        ApiStatus st = client_->create("services", job.ns(), make_service(job, r.type, i), &out);
        if (st.ok()) {
          res.services_created++;
          rec_->event(orig, "Normal", "SuccessfulCreateService", "Created service: " + name);
        } else if (st.code != 409) {
          rec_->event(orig, "Warning", "FailedCreateService", "Error creating service " + name + ": " + st.message);
          res.requeue = true;
        }
      }
      auto it = slot.find({r.type, i});
      if (it == slot.end()) {
        Json out;
        ApiStatus st = client_->create("pods", job.ns(), make_pod(job, r.type, i, generation), &out);
        if (st.ok()) {
          res.pods_created++;
          if (metrics_) metrics_->pods_created++;
          rec_->event(orig, "Normal", "SuccessfulCreatePod", "Created pod: " + name);
        } else if (st.code != 409) {
          rec_->event(orig, "Warning", "FailedCreatePod", "Error creating pod " + name + ": " + st.message);
          res.requeue = true;
        }
        rst.active++;
        rst.states["Pending"]++;
        continue;
      }
      PodState ps = pod_state(it->second);
      rst.states[ps.state]++;
      if (ps.state == "Succeeded") rst.succeeded++;
      else if (ps.state == "Failed") {
        rst.failed++;
        bool can_retry = ps.retryable && (job.is_v1alpha1() ? it->second.path("spec.restartPolicy").str() != "Never"
                                                            : (r.restart_policy == "ExitCode" ||
                                                               r.restart_policy == "OnFailure" ||
                                                               r.restart_policy == "Always"));
        // v1: ExitCode retries signals (exit >= 128); OnFailure/Always retry any failure the kubelet gave up on
        if (!job.is_v1alpha1() && (r.restart_policy == "OnFailure" || r.restart_policy == "Always") && !ps.retryable &&
            ps.reason != "OOMKilled")
          can_retry = true;
        if (can_retry) {
          retry_needed = true;
          retry_msg = name + " exited with code " + std::to_string(ps.exit_code) + (ps.reason.empty() ? "" : " (" + ps.reason + ")");
        } else if (r.type != RType::Evaluator) {
          permanent_failures.push_back(name + " exited with code " + std::to_string(ps.exit_code) +
                                       (ps.reason.empty() ? "" : " (" + ps.reason + ")"));
        }
      } else {
        rst.active++;
      }
    }
    rst.state = rst.failed ? "Failed" : (rst.active ? "Running" : (rst.succeeded == r.replicas ? "Succeeded" : "Unknown"));
    job.status.replica_statuses[r.type] = rst;
  }

  // ---------------------------------------------------------------- failures / restarts
  if (!permanent_failures.empty()) {
    fail_job("TFJobFailed", "TFJob " + job.name() + " has failed because " + join(permanent_failures, ", "));
  } else if (retry_needed) {
    if (job.run_policy.backoff_limit >= 0 && job.status.restart_count >= job.run_policy.backoff_limit) {
      fail_job("BackoffLimitExceeded", "TFJob " + job.name() + " has failed because it has reached the specified backoff limit");
    } else {
      // Collective training (MWMS / PS over RCCL) cannot lose one rank: restart the whole job's
      // pods together with a bumped restart generation; they resume from the latest checkpoint.
      job.status.restart_count++;
      for (auto& kv : slot) {
        if (client_->remove("pods", job.ns(), kv.second.path("metadata.name").str(), "Background").ok()) {
          res.pods_deleted++;
          if (metrics_) metrics_->pods_deleted++;
        }
      }
      api::set_condition(job.status, "Restarting", "TFJobRestarting",
                         "TFJob " + job.name() + " is restarting because " + retry_msg, now);
      if (job.is_v1alpha1()) job.status.phase = "Running";
      if (metrics_) metrics_->jobs_restarted++;
      rec_->event(orig, "Warning", "TFJobRestarting", "restarting job pods (generation " +
                                                          std::to_string(job.status.restart_count) + "): " + retry_msg);
      res.requeue = true;
    }
  } else {
    // ---------------------------------------------------------------- success / running
    RType chief = RType::Unknown;
    int chief_index = 0;
    if (job.is_v1alpha1()) {
      chief = api::rtype_from(job.chief_name);
      chief_index = std::max(0, job.chief_index);
    } else if (job.replica(RType::Chief)) {
      chief = RType::Chief;
    } else if (job.replica(RType::Master)) {
      chief = RType::Master;
    }
    bool succeeded = false, running = false;
    if (chief != RType::Unknown) {
      auto it = slot.find({chief, chief_index});
      if (it != slot.end()) {
        PodState ps = pod_state(it->second);
        succeeded = ps.state == "Succeeded";
        running = ps.state == "Running";
      }
    } else if (job.replica(RType::Worker)) {
      const auto& ws = job.status.replica_statuses[RType::Worker];
      if (job.success_policy == "AllWorkers") succeeded = ws.succeeded == job.replica(RType::Worker)->replicas;
      else {
        auto it = slot.find({RType::Worker, 0});
        succeeded = it != slot.end() && pod_state(it->second).state == "Succeeded";
      }
      auto it = slot.find({RType::Worker, 0});
      running = it != slot.end() && pod_state(it->second).state == "Running";
    }
    if (succeeded) {
      job.status.state = "Succeeded";
      if (job.is_v1alpha1()) job.status.phase = "Done";
      api::set_condition(job.status, "Succeeded", "TFJobSucceeded", "TFJob " + job.name() + " successfully completed.", now);
      job.status.completion_time = now;
      if (metrics_) metrics_->jobs_succeeded++;
      rec_->event(orig, "Normal", "TFJobSucceeded", "TFJob " + job.name() + " successfully completed.");
      res.requeue = true;  // apply cleanPodPolicy / TTL
    } else if (running) {
      job.status.state = "Running";
      if (job.is_v1alpha1()) job.status.phase = "Running";
      if (!api::has_condition(job.status, "Running"))
        api::set_condition(job.status, "Running", "TFJobRunning", "TFJob " + job.name() + " is running.", now);
    }
  }
  job.status.last_reconcile_time = api::to_json(job).at("status").dump() != old_status ? now : job.status.last_reconcile_time;
  if (api::to_json(job).at("status").dump() != old_status) {
    ApiStatus st = write_status(job, orig);
    res.status_changed = true;
    if (!st.ok()) { res.requeue = true; res.error = st.message; }
  }
  return res;
}

}  // namespace tfk
