#include "types.h"

#include <algorithm>
#include <stdexcept>

#include "../common/util.h"

namespace tfk {
namespace api {

RType rtype_from(const std::string& s) {
  std::string u = to_lower(s);
  if (u == "master") return RType::Master;
  if (u == "chief") return RType::Chief;
  if (u == "ps") return RType::PS;
  if (u == "worker") return RType::Worker;
  if (u == "evaluator") return RType::Evaluator;
  return RType::Unknown;
}
std::string rtype_upper(RType t) {
  switch (t) {
    case RType::Master: return "MASTER";
    case RType::Chief: return "CHIEF";
    case RType::PS: return "PS";
    case RType::Worker: return "WORKER";
    case RType::Evaluator: return "EVALUATOR";
    default: return "UNKNOWN";
  }
}
std::string rtype_title(RType t) {
  switch (t) {
    case RType::Master: return "Master";
    case RType::Chief: return "Chief";
    case RType::PS: return "PS";
    case RType::Worker: return "Worker";
    case RType::Evaluator: return "Evaluator";
    default: return "Unknown";
  }
}
std::string rtype_lower(RType t) { return to_lower(rtype_upper(t)); }

bool TFJob::is_v1alpha1() const { return ends_with(api_version, "/v1alpha1"); }
const ReplicaSpec* TFJob::replica(RType t) const {
  for (auto& r : replicas)
    if (r.type == t) return &r;
  return nullptr;
}
ReplicaSpec* TFJob::replica(RType t) {
  for (auto& r : replicas)
    if (r.type == t) return &r;
  return nullptr;
}

// ------------------------------------------------------------------------------ codec
static int opt_int(const Json& j, const char* k, int d = -1) { return j.has(k) ? (int)j.at(k).as_int(d) : d; }

TFJob from_json(const Json& j) {
  if (!j.is_object()) throw std::runtime_error("TFJob must be a JSON object");
  TFJob job;
  job.api_version = j.at("apiVersion").str("kubeflow.org/v1");
  if (j.at("kind").str("TFJob") != kKind) throw std::runtime_error("kind must be TFJob");
  job.metadata = j.at("metadata").is_object() ? j.at("metadata").clone() : Json::object();
  const Json& spec = j.at("spec");
  if (!spec.is_object()) throw std::runtime_error("TFJob.spec missing");
  // v1alpha1-only spec fields ride in annotations while the object is stored in the v1 shape, so
  // a v1alpha1 -> v1 -> v1alpha1 round trip is lossless (runtimeId names every replica's pods)
  const Json& ann = job.metadata.at("annotations");
  if (job.is_v1alpha1()) {
    job.runtime_id = spec.at("runtimeId").str(ann.at(kAnnRuntimeId).str());
    job.tf_image = spec.at("tfImage").str(ann.at(kAnnTfImage).str());
    job.scheduler_name = spec.at("schedulerName").str();
    if (spec.at("terminationPolicy").is_object()) {
      job.has_termination_policy = true;
      const Json& c = spec.at("terminationPolicy").at("chief");
      job.chief_name = c.at("replicaName").str();
      job.chief_index = opt_int(c, "replicaIndex", 0);
    }
    for (auto& r : spec.at("replicaSpecs").items()) {
      ReplicaSpec rs;
      rs.type = r.has("tfReplicaType") ? rtype_from(r.at("tfReplicaType").str()) : RType::Master;
      if (r.has("tfReplicaType") && rs.type == RType::Unknown)
        throw std::runtime_error("unknown tfReplicaType " + r.at("tfReplicaType").str());
      rs.replicas = opt_int(r, "replicas");
      rs.tf_port = opt_int(r, "tfPort");
      rs.is_default_ps = r.at("isDefaultPS").as_bool(false);
      rs.template_ = r.at("template").clone();
      rs.restart_policy = rs.template_.path("spec.restartPolicy").str();
      job.replicas.push_back(rs);
    }
  } else {
    const Json& m = spec.at("tfReplicaSpecs");
    static const char* order[] = {"Chief", "Master", "PS", "Worker", "Evaluator"};
    for (auto& kv : m.fields()) {
      if (rtype_from(kv.first) == RType::Unknown) throw std::runtime_error("unknown replica type " + kv.first);
    }
    for (const char* name : order) {
      for (auto& kv : m.fields()) {
        if (rtype_from(kv.first) != rtype_from(name)) continue;
        ReplicaSpec rs;
        rs.type = rtype_from(kv.first);
        rs.replicas = opt_int(kv.second, "replicas");
        rs.restart_policy = kv.second.at("restartPolicy").str();
        rs.template_ = kv.second.at("template").clone();
        rs.tf_port = -1;
        job.replicas.push_back(rs);
      }
    }
    const Json& rp = spec.has("runPolicy") ? spec.at("runPolicy") : spec;  // older v1 inlined the fields
    job.run_policy.clean_pod_policy = rp.at("cleanPodPolicy").str();
    if (rp.has("ttlSecondsAfterFinished")) job.run_policy.ttl_seconds_after_finished = rp.at("ttlSecondsAfterFinished").as_int();
    if (rp.has("activeDeadlineSeconds")) job.run_policy.active_deadline_seconds = rp.at("activeDeadlineSeconds").as_int();
    if (rp.has("backoffLimit")) job.run_policy.backoff_limit = (int)rp.at("backoffLimit").as_int();
    const Json& sp = rp.at("schedulingPolicy");
    job.run_policy.scheduling.min_available = opt_int(sp, "minAvailable");
    job.run_policy.scheduling.queue = sp.at("queue").str();
    job.run_policy.scheduling.priority_class = sp.at("priorityClass").str();
    job.success_policy = spec.at("successPolicy").str();
    job.scheduler_name = rp.path("schedulingPolicy.schedulerName").str(spec.at("schedulerName").str());
    job.runtime_id = ann.at(kAnnRuntimeId).str();
    job.tf_image = ann.at(kAnnTfImage).str();
    if (ann.at(kAnnChief).is_string()) {
      auto parts = split(ann.at(kAnnChief).str(), ':');
      job.has_termination_policy = parts.size() == 2;
      if (job.has_termination_policy) { job.chief_name = parts[0]; job.chief_index = atoi(parts[1].c_str()); }
    }
  }
  // status (both shapes tolerated)
  const Json& st = j.at("status");
  if (st.is_object()) {
    job.status.phase = st.at("phase").str();
    job.status.state = st.at("state").str();
    job.status.reason = st.at("reason").str();
    job.status.start_time = st.at("startTime").str();
    job.status.completion_time = st.at("completionTime").str();
    job.status.last_reconcile_time = st.at("lastReconcileTime").str();
    job.status.restart_count = (int)st.at("restartCount").as_int(0);
    job.status.resize_count = (int)st.at("resizeCount").as_int(0);
    for (auto& c : st.at("conditions").items()) {
      JobCondition jc;
      jc.type = c.at("type").str(); jc.status = c.at("status").str(); jc.reason = c.at("reason").str();
      jc.message = c.at("message").str(); jc.last_update = c.at("lastUpdateTime").str();
      jc.last_transition = c.at("lastTransitionTime").str();
      job.status.conditions.push_back(jc);
    }
    const Json& rs = st.at("replicaStatuses");
    if (rs.is_array()) {
      for (auto& r : rs.items()) {
        ReplicaStatus s;
        s.state = r.at("state").str();
        for (auto& kv : r.at("replicas_states").fields()) s.states[kv.first] = (int)kv.second.as_int();
        job.status.replica_statuses[rtype_from(r.at("tf_replica_type").str())] = s;
      }
    } else {
      for (auto& kv : rs.fields()) {
        ReplicaStatus s;
        s.active = (int)kv.second.at("active").as_int(0);
        s.succeeded = (int)kv.second.at("succeeded").as_int(0);
        s.failed = (int)kv.second.at("failed").as_int(0);
        job.status.replica_statuses[rtype_from(kv.first)] = s;
      }
    }
  }
  return job;
}

Json to_json(const TFJob& job) {
  Json j = Json::object();
  j["apiVersion"] = job.api_version;
  j["kind"] = kKind;
  j["metadata"] = job.metadata.clone();
  Json spec = Json::object();
  Json st = Json::object();
  if (job.is_v1alpha1()) {
    if (j["metadata"].at("annotations").is_object()) {
      for (const char* k : {kAnnRuntimeId, kAnnTfImage, kAnnChief}) j["metadata"]["annotations"].erase(k);
      if (j["metadata"]["annotations"].size() == 0) j["metadata"].erase("annotations");
    }
    if (!job.runtime_id.empty()) spec["runtimeId"] = job.runtime_id;
    if (!job.tf_image.empty()) spec["tfImage"] = job.tf_image;
    if (!job.scheduler_name.empty()) spec["schedulerName"] = job.scheduler_name;
    if (job.has_termination_policy) {
      spec["terminationPolicy"]["chief"]["replicaName"] = job.chief_name;
      spec["terminationPolicy"]["chief"]["replicaIndex"] = job.chief_index;
    }
    Json arr = Json::array();
    for (auto& r : job.replicas) {
      Json o = Json::object();
      if (r.replicas >= 0) o["replicas"] = r.replicas;
      if (r.tf_port >= 0) o["tfPort"] = r.tf_port;
      o["tfReplicaType"] = rtype_upper(r.type);
      if (r.is_default_ps) o["isDefaultPS"] = true;
      if (!r.template_.is_null()) o["template"] = r.template_.clone();
      arr.push_back(o);
    }
    spec["replicaSpecs"] = arr;
    if (!job.status.phase.empty()) st["phase"] = job.status.phase;
    if (!job.status.state.empty()) st["state"] = job.status.state;
    if (!job.status.reason.empty()) st["reason"] = job.status.reason;
    Json rs = Json::array();
    for (auto& kv : job.status.replica_statuses) {
      Json o = Json::object();
      o["tf_replica_type"] = rtype_upper(kv.first);
      o["state"] = kv.second.state.empty() ? "Unknown" : kv.second.state;
      Json m = Json::object();
      for (auto& s : kv.second.states) m[s.first] = s.second;
      o["replicas_states"] = m;
      rs.push_back(o);
    }
    if (rs.size()) st["replicaStatuses"] = rs;
  } else {
    if (!job.runtime_id.empty()) j["metadata"]["annotations"][kAnnRuntimeId] = job.runtime_id;
    if (!job.tf_image.empty()) j["metadata"]["annotations"][kAnnTfImage] = job.tf_image;
    if (job.has_termination_policy)
      j["metadata"]["annotations"][kAnnChief] = job.chief_name + ":" + std::to_string(job.chief_index);
    Json m = Json::object();
    for (auto& r : job.replicas) {
      Json o = Json::object();
      if (r.replicas >= 0) o["replicas"] = r.replicas;
      if (!r.restart_policy.empty()) o["restartPolicy"] = r.restart_policy;
      if (!r.template_.is_null()) o["template"] = r.template_.clone();
      m[rtype_title(r.type)] = o;
    }
    spec["tfReplicaSpecs"] = m;
    Json rp = Json::object();
    if (!job.run_policy.clean_pod_policy.empty()) rp["cleanPodPolicy"] = job.run_policy.clean_pod_policy;
    if (job.run_policy.ttl_seconds_after_finished >= 0) rp["ttlSecondsAfterFinished"] = job.run_policy.ttl_seconds_after_finished;
    if (job.run_policy.active_deadline_seconds >= 0) rp["activeDeadlineSeconds"] = job.run_policy.active_deadline_seconds;
    if (job.run_policy.backoff_limit >= 0) rp["backoffLimit"] = job.run_policy.backoff_limit;
    const auto& sp = job.run_policy.scheduling;
    if (sp.min_available >= 0 || !sp.queue.empty() || !sp.priority_class.empty() || !job.scheduler_name.empty()) {
      Json s = Json::object();
      if (sp.min_available >= 0) s["minAvailable"] = sp.min_available;
      if (!sp.queue.empty()) s["queue"] = sp.queue;
      if (!sp.priority_class.empty()) s["priorityClass"] = sp.priority_class;
      if (!job.scheduler_name.empty()) s["schedulerName"] = job.scheduler_name;
      rp["schedulingPolicy"] = s;
    }
    if (rp.size()) spec["runPolicy"] = rp;
    if (!job.success_policy.empty()) spec["successPolicy"] = job.success_policy;
    Json conds = Json::array();
    for (auto& c : job.status.conditions) {
      Json o = Json::object();
      o["type"] = c.type; o["status"] = c.status;
      if (!c.reason.empty()) o["reason"] = c.reason;
      if (!c.message.empty()) o["message"] = c.message;
      if (!c.last_update.empty()) o["lastUpdateTime"] = c.last_update;
      if (!c.last_transition.empty()) o["lastTransitionTime"] = c.last_transition;
      conds.push_back(o);
    }
    if (conds.size()) st["conditions"] = conds;
    Json rs = Json::object();
    for (auto& kv : job.status.replica_statuses) {
      Json o = Json::object();
      o["active"] = kv.second.active; o["succeeded"] = kv.second.succeeded; o["failed"] = kv.second.failed;
      rs[rtype_title(kv.first)] = o;
    }
    if (rs.size()) st["replicaStatuses"] = rs;
  }
  if (!job.status.start_time.empty()) st["startTime"] = job.status.start_time;
  if (!job.status.completion_time.empty()) st["completionTime"] = job.status.completion_time;
  if (!job.status.last_reconcile_time.empty()) st["lastReconcileTime"] = job.status.last_reconcile_time;
  if (job.status.restart_count) st["restartCount"] = job.status.restart_count;
  if (job.status.resize_count) st["resizeCount"] = job.status.resize_count;
  j["spec"] = spec;
  if (st.size()) j["status"] = st;
  return j;
}

Json convert(const Json& obj, const std::string& target) {
  TFJob job = from_json(obj);
  bool to_alpha = ends_with(target, "/v1alpha1");
  if (to_alpha && !job.is_v1alpha1()) {
    for (auto& r : job.replicas)
      if (r.type == RType::Chief) r.type = RType::Master;
    for (auto& r : job.replicas)
      if (r.type == RType::Evaluator) throw std::runtime_error("v1alpha1 has no Evaluator replica type");
    // conditions -> phase/state
    if (has_condition(job.status, "Succeeded")) { job.status.phase = "Done"; job.status.state = "Succeeded"; }
    else if (has_condition(job.status, "Failed")) { job.status.phase = "Done"; job.status.state = "Failed"; }
    else if (has_condition(job.status, "Running")) { job.status.phase = "Running"; job.status.state = "Running"; }
    else if (has_condition(job.status, "Created")) { job.status.phase = "Creating"; job.status.state = "Unknown"; }
  } else if (!to_alpha && job.is_v1alpha1()) {
    for (auto& r : job.replicas) {
      if (r.tf_port >= 0 && r.tf_port != kDefaultPort && r.template_.is_object()) {
        for (auto& c : r.template_["spec"]["containers"].items_mut())
          if (c.at("name").str() == kContainerName) {
            Json p = Json::object();
            p["name"] = kPortName; p["containerPort"] = r.tf_port;
            c["ports"] = Json(Json::array_t{p});
          }
      }
      r.tf_port = -1;
    }
    std::string now = rfc3339(now_ms());
    if (job.status.phase == "Creating") set_condition(job.status, "Created", "TFJobCreated", "", now);
    if (job.status.state == "Running") set_condition(job.status, "Running", "TFJobRunning", "", now);
    if (job.status.state == "Succeeded") set_condition(job.status, "Succeeded", "TFJobSucceeded", "", now);
    if (job.status.state == "Failed") set_condition(job.status, "Failed", "TFJobFailed", job.status.reason, now);
  }
  job.api_version = target;
  return to_json(job);
}

// ------------------------------------------------------------------------------ defaults
void set_defaults(TFJob& job) {
  if (job.is_v1alpha1()) {
    if (!job.has_termination_policy) {
      job.has_termination_policy = true;
      job.chief_name = "MASTER";
      job.chief_index = 0;
    }
    for (auto& r : job.replicas) {
      if (r.replicas < 0) r.replicas = 1;
      if (r.tf_port < 0) r.tf_port = kDefaultPort;
    }
  } else {
    for (auto& r : job.replicas) {
      if (r.replicas < 0) r.replicas = 1;
      if (r.restart_policy.empty()) r.restart_policy = "Never";
      // default port on the tensorflow container
      if (r.template_.is_object()) {
        for (auto& c : r.template_["spec"]["containers"].items_mut()) {
          if (c.at("name").str() != kContainerName) continue;
          bool has = false;
          for (auto& p : c.at("ports").items())
            if (p.at("name").str() == kPortName) has = true;
          if (!has) {
            Json p = Json::object();
            p["name"] = kPortName; p["containerPort"] = kDefaultPort;
            c["ports"].push_back(p);
          }
        }
      }
    }
    if (job.run_policy.clean_pod_policy.empty()) job.run_policy.clean_pod_policy = "Running";
  }
  if (!job.metadata.has("namespace")) job.metadata["namespace"] = "default";
}

// ------------------------------------------------------------------------------ validation
std::vector<std::string> validate(const TFJob& job) {
  std::vector<std::string> errs;
  if (job.name().empty()) errs.push_back("metadata.name is required");
  if (job.name().size() > 63) errs.push_back("metadata.name must be at most 63 characters");
  for (char c : job.name())
    if (!(islower((unsigned char)c) || isdigit((unsigned char)c) || c == '-' || c == '.')) {
      errs.push_back("metadata.name must be a DNS-1123 subdomain");
      break;
    }
  if (job.replicas.empty()) errs.push_back("spec must declare at least one replica spec");
  std::map<RType, int> seen;
  for (auto& r : job.replicas) {
    std::string t = rtype_upper(r.type);
    if (r.type == RType::Unknown) errs.push_back("invalid replica type");
    if (++seen[r.type] > 1) errs.push_back("duplicate replica type " + t);
    if (r.replicas < 0) errs.push_back(t + ": replicas must be set (defaulting not applied)");
    if (job.is_v1alpha1() && r.tf_port <= 0) errs.push_back(t + ": tfPort must be set");
    if ((r.type == RType::Master || r.type == RType::Chief) && r.replicas != 1)
      errs.push_back(t + ": must have exactly 1 replica");
    if (r.type == RType::Evaluator && r.replicas > 1) errs.push_back("EVALUATOR: at most 1 replica");
    if (r.is_default_ps) continue;  // default PS gets its container from the operator
    bool has_container = false;
    for (auto& c : r.template_.path("spec.containers").items())
      if (c.at("name").str() == kContainerName) has_container = true;
    if (!has_container) errs.push_back(t + ": template must contain a container named \"tensorflow\"");
    if (!job.is_v1alpha1() && !r.restart_policy.empty() && r.restart_policy != "Always" &&
        r.restart_policy != "OnFailure" && r.restart_policy != "Never" && r.restart_policy != "ExitCode")
      errs.push_back(t + ": invalid restartPolicy " + r.restart_policy);
  }
  if (job.is_v1alpha1()) {
    if (!job.has_termination_policy) errs.push_back("terminationPolicy.chief is required");
    else {
      const ReplicaSpec* c = job.replica(rtype_from(job.chief_name));
      if (!c) errs.push_back("terminationPolicy chief replica " + job.chief_name + " is not a replica type");
      else if (job.chief_index < 0 || job.chief_index >= std::max(1, c->replicas))
        errs.push_back("terminationPolicy chief replicaIndex out of range");
    }
  } else {
    if (job.replica(RType::Chief) && job.replica(RType::Master)) errs.push_back("Chief and Master are exclusive");
    const auto& cp = job.run_policy.clean_pod_policy;
    if (!cp.empty() && cp != "All" && cp != "Running" && cp != "None") errs.push_back("invalid cleanPodPolicy " + cp);
    if (!job.success_policy.empty() && job.success_policy != "AllWorkers")
      errs.push_back("invalid successPolicy " + job.success_policy);
  }
  return errs;
}

// ------------------------------------------------------------------------------ helpers
std::string crd_name() { return std::string(kPlural) + "." + kGroupV1; }

Json crd_manifest() {
  Json j = Json::parse(R"({
    "apiVersion": "apiextensions.k8s.io/v1beta1", "kind": "CustomResourceDefinition",
    "metadata": {"name": "tfjobs.kubeflow.org"},
    "spec": {"group": "kubeflow.org", "version": "v1", "scope": "Namespaced",
             "versions": [{"name": "v1", "served": true, "storage": true},
                          {"name": "v1alpha1", "served": true, "storage": false}],
             "names": {"plural": "tfjobs", "singular": "tfjob", "kind": "TFJob", "shortNames": ["tfj"]},
             "subresources": {"status": {}}}})");
  return j;
}

Json as_owner(const TFJob& job) {
  Json o = Json::object();
  o["apiVersion"] = job.api_version;
  o["kind"] = kKind;
  o["name"] = job.name();
  o["uid"] = job.uid();
  o["controller"] = true;
  o["blockOwnerDeletion"] = true;
  return o;
}

ControllerConfig ControllerConfig::defaults() {
  ControllerConfig c;
  AcceleratorConfig a;
  a.volumes.push_back({"kfd", {"/dev/kfd", "/dev/kfd"}});
  a.volumes.push_back({"dri", {"/dev/dri", "/dev/dri"}});
  a.env.push_back({"HSA_ENABLE_IPC_MODE_LEGACY", "0"});
  c.accelerators[kGPUResource] = a;
  return c;
}

ControllerConfig ControllerConfig::from_json(const Json& j) {
  ControllerConfig c;
  for (auto& kv : j.at("accelerators").fields()) {
    AcceleratorConfig a;
    for (auto& v : kv.second.at("volumes").items())
      a.volumes.push_back({v.at("name").str(), {v.at("hostPath").str(), v.at("mountPath").str()}});
    for (auto& e : kv.second.at("envVars").items()) a.env.push_back({e.at("name").str(), e.at("value").str()});
    c.accelerators[kv.first] = a;
  }
  c.grpc_server_file_path = j.at("grpcServerFilePath").str();
  return c;
}

void configure_accelerators(TFJob& job, const ControllerConfig& cfg) {
  for (auto& r : job.replicas) {
    if (!r.template_.is_object()) continue;
    Json& spec = r.template_["spec"];
    for (auto& c : spec["containers"].items_mut()) {
      if (c.at("name").str() != kContainerName) continue;
      for (auto& acc : cfg.accelerators) {
        const Json& lim = c.path("resources.limits").at(acc.first);
        if (lim.is_null() || (lim.is_number() && lim.as_int() == 0) || (lim.is_string() && lim.str() == "0")) continue;
        for (auto& v : acc.second.volumes) {
          bool present = false;
          for (auto& ev : spec.at("volumes").items())
            if (ev.at("name").str() == v.first) present = true;
          if (!present) {
            Json vol = Json::object();
            vol["name"] = v.first; vol["hostPath"]["path"] = v.second.first;
            spec["volumes"].push_back(vol);
          }
          Json vm = Json::object();
          vm["name"] = v.first; vm["mountPath"] = v.second.second;
          c["volumeMounts"].push_back(vm);
        }
        for (auto& e : acc.second.env) {
          Json ev = Json::object();
          ev["name"] = e.first; ev["value"] = e.second;
          c["env"].push_back(ev);
        }
      }
    }
  }
}

static std::string dns_clean(std::string s) {
  s = to_lower(s);
  for (auto& c : s)
    if (!(isalnum((unsigned char)c) || c == '-' || c == '.')) c = '-';
  return s;
}

std::string gen_general_name(const std::string& job_name, const std::string& rt, int index) {
  return dns_clean(job_name + "-" + rt + "-" + std::to_string(index));
}

std::string gen_name(const TFJob& job, RType t, int index) {
  if (job.is_v1alpha1())
    return dns_clean(job.name().substr(0, 40) + "-" + rtype_lower(t) + "-" + job.runtime_id + "-" + std::to_string(index));
  return gen_general_name(job.name(), rtype_lower(t), index);
}

static int replica_port(const ReplicaSpec& r) {
  if (r.tf_port > 0) return r.tf_port;
  for (auto& c : r.template_.path("spec.containers").items())
    if (c.at("name").str() == kContainerName)
      for (auto& p : c.at("ports").items())
        if (p.at("name").str() == kPortName) return (int)p.at("containerPort").as_int(kDefaultPort);
  return kDefaultPort;
}

Json cluster_spec(const TFJob& job, const std::string& domain, const std::map<std::string, int>* ports) {
  Json c = Json::object();
  for (auto& r : job.replicas) {
    if (r.type == RType::Evaluator) continue;  // evaluator is not part of the training cluster
    Json hosts = Json::array();
    for (int i = 0; i < std::max(r.replicas, 0); ++i) {
      std::string svc = gen_name(job, r.type, i);
      int port = replica_port(r);
      if (ports) {
        auto it = ports->find(svc);
        if (it != ports->end()) port = it->second;
      }
      std::string host = svc + "." + job.ns() + ".svc" + (domain.empty() ? "" : "." + domain);
      hosts.push_back(host + ":" + std::to_string(port));
    }
    c[rtype_lower(r.type)] = hosts;
  }
  return c;
}

std::string tf_config(const TFJob& job, RType t, int index, const std::string& domain,
                      const std::map<std::string, int>* ports) {
  Json j = Json::object();
  j["cluster"] = cluster_spec(job, domain, ports);
  j["task"]["type"] = rtype_lower(t);
  j["task"]["index"] = index;
  j["environment"] = "cloud";
  return j.dump();
}

void set_condition(TFJobStatus& st, const std::string& type, const std::string& reason, const std::string& msg,
                   const std::string& now) {
  // Running/Restarting/Succeeded/Failed are mutually exclusive "True" states (kubeflow semantics).
  auto exclusive = [](const std::string& t) {
    return t == "Running" || t == "Restarting" || t == "Succeeded" || t == "Failed";
  };
  for (auto& c : st.conditions) {
    if (c.type == type) {
      if (c.status != "True" || c.reason != reason || c.message != msg) {
        if (c.status != "True") c.last_transition = now;
        c.status = "True"; c.reason = reason; c.message = msg; c.last_update = now;
      }
    } else if (exclusive(type) && exclusive(c.type) && c.status == "True") {
      c.status = "False";
      c.last_transition = now;
      c.last_update = now;
    }
  }
  for (auto& c : st.conditions)
    if (c.type == type) return;
  st.conditions.push_back({type, "True", reason, msg, now, now});
}

bool has_condition(const TFJobStatus& st, const std::string& type) {
  for (auto& c : st.conditions)
    if (c.type == type && c.status == "True") return true;
  return false;
}

bool is_finished(const TFJobStatus& st) {
  return has_condition(st, "Succeeded") || has_condition(st, "Failed") || st.phase == "Done" ||
         st.phase == "Failed";
}

bool is_retryable_exit(int exit_code, const std::string& reason) {
  if (reason == "OOMKilled") return false;
  if (exit_code == 0) return false;
  return exit_code >= 128;
}

}  // namespace api
}  // namespace tfk
