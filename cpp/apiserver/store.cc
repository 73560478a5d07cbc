#include "store.h"

#include <unistd.h>

#include <fcntl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "../common/util.h"

namespace tfk {

Json ApiStatus::to_json() const {
  Json j = Json::object();
  j["kind"] = "Status";
  j["apiVersion"] = "v1";
  j["status"] = ok() ? "Success" : "Failure";
  j["code"] = code;
  if (!reason.empty()) j["reason"] = reason;
  if (!message.empty()) j["message"] = message;
  return j;
}

// ------------------------------------------------------------------------------ selectors
LabelSelector LabelSelector::parse(const std::string& s, std::string* err) {
  LabelSelector sel;
  std::string cur;
  int depth = 0;
  std::vector<std::string> parts;
  for (char c : s) {
    if (c == '(') depth++;
    if (c == ')') depth--;
    if (c == ',' && depth == 0) { parts.push_back(cur); cur.clear(); }
    else cur += c;
  }
  if (!cur.empty()) parts.push_back(cur);
  for (auto p : parts) {
    p = trim(p);
    if (p.empty()) continue;
    Req r;
    size_t pos;
    if ((pos = p.find(" notin ")) != std::string::npos || (pos = p.find(" in ")) != std::string::npos) {
      bool notin = p.find(" notin ") != std::string::npos;
      r.key = trim(p.substr(0, pos));
      r.op = notin ? "notin" : "in";
      size_t a = p.find('('), b = p.rfind(')');
      if (a == std::string::npos || b == std::string::npos) { if (err) *err = "bad set selector " + p; continue; }
      for (auto v : split(p.substr(a + 1, b - a - 1), ',')) r.vals.insert(trim(v));
    } else if ((pos = p.find("!=")) != std::string::npos) {
      r.key = trim(p.substr(0, pos)); r.op = "!="; r.vals.insert(trim(p.substr(pos + 2)));
    } else if ((pos = p.find("==")) != std::string::npos) {
      r.key = trim(p.substr(0, pos)); r.op = "="; r.vals.insert(trim(p.substr(pos + 2)));
    } else if ((pos = p.find('=')) != std::string::npos) {
      r.key = trim(p.substr(0, pos)); r.op = "="; r.vals.insert(trim(p.substr(pos + 1)));
    } else if (p[0] == '!') {
      r.key = trim(p.substr(1)); r.op = "!exists";
    } else {
      r.key = p; r.op = "exists";
    }
    sel.reqs_.push_back(r);
  }
  return sel;
}

LabelSelector LabelSelector::from_map(const Json& m) {
  LabelSelector sel;
  for (auto& kv : m.fields()) sel.reqs_.push_back({kv.first, "=", {kv.second.str()}});
  return sel;
}

bool LabelSelector::matches(const Json& labels) const {
  for (auto& r : reqs_) {
    bool has = labels.has(r.key);
    std::string v = labels.at(r.key).str();
    if (r.op == "=" && (!has || !r.vals.count(v))) return false;
    if (r.op == "!=" && has && r.vals.count(v)) return false;
    if (r.op == "exists" && !has) return false;
    if (r.op == "!exists" && has) return false;
    if (r.op == "in" && (!has || !r.vals.count(v))) return false;
    if (r.op == "notin" && has && r.vals.count(v)) return false;
  }
  return true;
}

std::string LabelSelector::str() const {
  std::string s;
  for (auto& r : reqs_) {
    if (!s.empty()) s += ",";
    if (r.op == "=" || r.op == "!=") s += r.key + r.op + *r.vals.begin();
    else if (r.op == "exists") s += r.key;
    else if (r.op == "!exists") s += "!" + r.key;
    else {
      s += r.key + " " + r.op + " (";
      bool f = true;
      for (auto& v : r.vals) { s += (f ? "" : ",") + v; f = false; }
      s += ")";
    }
  }
  return s;
}

FieldSelector FieldSelector::parse(const std::string& s) {
  FieldSelector f;
  for (auto p : split(s, ',')) {
    p = trim(p);
    if (p.empty()) continue;
    size_t pos = p.find("!=");
    if (pos != std::string::npos) f.reqs_.push_back({trim(p.substr(0, pos)), trim(p.substr(pos + 2)), true});
    else if ((pos = p.find("==")) != std::string::npos) f.reqs_.push_back({trim(p.substr(0, pos)), trim(p.substr(pos + 2)), false});
    else if ((pos = p.find('=')) != std::string::npos) f.reqs_.push_back({trim(p.substr(0, pos)), trim(p.substr(pos + 1)), false});
  }
  return f;
}

bool FieldSelector::matches(const Json& obj) const {
  for (auto& r : reqs_) {
    const Json& v = obj.path(r.path);
    std::string s = v.is_string() ? v.str() : (v.is_null() ? "" : v.dump());
    if (r.neq ? (s == r.val) : (s != r.val)) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------ watcher
bool Watcher::next(WatchEvent* ev, int64_t timeout_ms) {
  std::unique_lock<std::mutex> l(mu_);
  cv_wait_ms(cv_, l, timeout_ms, [&] { return !q_.empty() || closed_; });
  if (q_.empty()) return false;
  *ev = q_.front();
  q_.pop_front();
  return true;
}

void Watcher::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
  }
  cv_.notify_all();
}

void Watcher::deliver(const WatchEvent& ev) {
  if (ev.type != "BOOKMARK" && ev.type != "ERROR") {
    const Json& md = ev.object.at("metadata");
    if (!ns_.empty() && md.at("namespace").str() != ns_) return;
    if (!ls_.matches(md.at("labels"))) return;
    if (!fs_.matches(ev.object)) return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) return;
    if (q_.size() >= max_queue_) {  // slow consumer: terminate (client relists)
      closed_ = true;
      q_.clear();
    } else {
      q_.push_back(ev);
    }
  }
  cv_.notify_all();
}

// ------------------------------------------------------------------------------ store
Store::Store(const std::string& wal_path, size_t history, WalOptions wal_opts)
    : history_cap_(history), wal_path_(wal_path), wal_opts_(std::move(wal_opts)) {
  auto core = [&](const char* plural, const char* singular, const char* kind, bool ns) {
    register_resource({"", "v1", plural, singular, kind, ns, {"v1"}, {}});
  };
  core("pods", "pod", "Pod", true);
  core("services", "service", "Service", true);
  core("events", "event", "Event", true);
  core("configmaps", "configmap", "ConfigMap", true);
  core("endpoints", "endpoints", "Endpoints", true);
  core("nodes", "node", "Node", false);
  core("namespaces", "namespace", "Namespace", false);
  register_resource({"coordination.k8s.io", "v1", "leases", "lease", "Lease", true, {"v1"}, {}});
  register_resource({"apiextensions.k8s.io", "v1beta1", "customresourcedefinitions", "customresourcedefinition",
                     "CustomResourceDefinition", false, {"v1beta1", "v1"}, {"crd"}});
  register_resource({"scheduling.tfk.io", "v1", "podgroups", "podgroup", "PodGroup", true, {"v1"}, {"pg"}});
  register_resource({"scheduling.k8s.io", "v1", "priorityclasses", "priorityclass", "PriorityClass", false, {"v1"},
                     {"pc"}});
  if (!wal_path_.empty()) {
    replay_wal();
    wal_ = fopen(wal_path_.c_str(), "a");
    if (wal_opts_.sync == "interval") syncer_ = std::thread([this] { syncer_loop(); });
  }
}

void Store::syncer_loop() {
  while (!syncer_stop_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(std::max<int64_t>(1, wal_opts_.sync_interval_ms)));
    if (!wal_dirty_.exchange(false)) continue;
    int fd = -1;
    {
      std::lock_guard<std::mutex> g(mu_);
      // records are already fflush'ed under the lock. dup() the descriptor while holding it: a
      // concurrent compact_wal_locked() may fclose/reopen wal_, and fdatasync on the bare fileno
      // could then hit a closed fd or a number reused by another file or socket. The dup keeps
      // the old file description alive (syncing a compacted-away file is harmless).
      if (wal_) fd = dup(fileno(wal_));
      if (fd >= 0) ops_["wal_fsync"]++;
    }
    if (fd >= 0) {
      fdatasync(fd);
      close(fd);
    }
  }
}

Store::~Store() {
  syncer_stop_ = true;
  if (syncer_.joinable()) syncer_.join();
  if (wal_) {
    fflush(wal_);
    if (wal_opts_.sync != "none") fdatasync(fileno(wal_));
    fclose(wal_);
  }
  std::lock_guard<std::mutex> g(mu_);
  for (auto& w : watchers_)
    if (auto s = w.lock()) s->close();
}

void Store::register_resource(const ResourceInfo& ri) {
  std::lock_guard<std::mutex> g(mu_);
  resources_[ri.plural] = ri;
}

bool Store::resource(const std::string& plural, ResourceInfo* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = resources_.find(plural);
  if (it == resources_.end()) {
    for (auto& kv : resources_)
      for (auto& s : kv.second.short_names)
        if (s == plural) { if (out) *out = kv.second; return true; }
    return false;
  }
  if (out) *out = it->second;
  return true;
}

bool Store::resource_by_kind(const std::string& kind, ResourceInfo* out) const {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : resources_)
    if (kv.second.kind == kind) { if (out) *out = kv.second; return true; }
  return false;
}

std::vector<ResourceInfo> Store::resources() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<ResourceInfo> v;
  for (auto& kv : resources_) v.push_back(kv.second);
  return v;
}

void Store::set_converter(const std::string& plural, Converter c) {
  std::lock_guard<std::mutex> g(mu_);
  converters_[plural] = std::move(c);
}

Json Store::convert_for(const std::string& plural, const Json& obj, const std::string& api_version) const {
  if (api_version.empty() || obj.at("apiVersion").str() == api_version) return obj;
  Converter c;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = converters_.find(plural);
    if (it == converters_.end()) return obj;
    c = it->second;
  }
  try {
    return c(obj, api_version);
  } catch (...) {
    return obj;
  }
}

int64_t Store::resource_version() const {
  std::lock_guard<std::mutex> g(mu_);
  return rv_;
}

size_t Store::count(const std::string& plural) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = data_.find(plural);
  return it == data_.end() ? 0 : it->second.size();
}

std::map<std::string, long long> Store::counters() const {
  std::lock_guard<std::mutex> g(mu_);
  return ops_;
}

void Store::emit_locked(const std::string& plural, const std::string& type, const Json& obj, int64_t rv) {
  WatchEvent ev{type, obj, rv};
  history_.push_back(ev);
  history_plural_[rv] = plural;
  while (history_.size() > history_cap_) {
    history_plural_.erase(history_.front().rv);
    history_.pop_front();
  }
  std::vector<std::weak_ptr<Watcher>> live;
  for (auto& w : watchers_) {
    auto s = w.lock();
    if (!s || s->closed()) continue;
    live.push_back(w);
    if (s->plural() != plural) continue;
    if (!s->requested_version().empty() && plural == "tfjobs") {
      WatchEvent cv = ev;
      auto it = converters_.find(plural);
      if (it != converters_.end() && obj.at("apiVersion").str() != s->requested_version()) {
        try { cv.object = it->second(obj, s->requested_version()); } catch (...) {}
      }
      s->deliver(cv);
    } else {
      s->deliver(ev);
    }
  }
  watchers_.swap(live);
}

void Store::wal_locked(const std::string& op, const std::string& plural, const Json& obj) {
  if (!wal_ || replaying_) return;
  Json rec = Json::object();
  rec["op"] = op;
  rec["plural"] = plural;
  rec["object"] = obj;
  std::string line = rec.dump() + "\n";
  fwrite(line.data(), 1, line.size(), wal_);
  fflush(wal_);
  ++wal_records_;
  if (wal_opts_.sync == "always") {
    fdatasync(fileno(wal_));
    ops_["wal_fsync"]++;
  } else {
    wal_dirty_ = true;
  }
  if (wal_opts_.compact_records > 0 && wal_records_ >= wal_opts_.compact_records) {
    size_t live = 0;
    for (auto& kv : data_) live += kv.second.size();
    if (wal_records_ > 2 * live) compact_wal_locked();
  }
}

void Store::compact_wal_locked() {
  const std::string tmp = wal_path_ + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) return;
  size_t n = 0;
  auto put = [&](const std::string& op, const std::string& plural, const Json& obj) {
    Json rec = Json::object();
    rec["op"] = op;
    rec["plural"] = plural;
    rec["object"] = obj;
    std::string line = rec.dump() + "\n";
    fwrite(line.data(), 1, line.size(), f);
    ++n;
  };
  // resource-version high-water mark first: deleted objects' versions must never be reissued
  Json mark = Json::object();
  mark["metadata"]["resourceVersion"] = std::to_string(rv_ - 1);
  put("rv", "", mark);
  for (auto& kv : data_)  // CRDs first so their resources are registered before their objects
    if (kv.first == "customresourcedefinitions")
      for (auto& o : kv.second) put("crd", kv.first, o.second.data);
  for (auto& kv : data_)
    if (kv.first != "customresourcedefinitions")
      for (auto& o : kv.second) put("put", kv.first, o.second.data);
  fflush(f);
  const bool ok = fdatasync(fileno(f)) == 0;
  fclose(f);
  if (!ok || rename(tmp.c_str(), wal_path_.c_str()) != 0) {
    unlink(tmp.c_str());
    return;
  }
  std::string dir = wal_path_.substr(0, wal_path_.find_last_of('/') == std::string::npos ? 0 : wal_path_.find_last_of('/'));
  int dfd = open(dir.empty() ? "." : dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (dfd >= 0) {
    fsync(dfd);  // the rename itself is durable
    ::close(dfd);
  }
  fclose(wal_);
  wal_ = fopen(wal_path_.c_str(), "a");
  wal_records_ = n;
  ops_["wal_compactions"]++;
}

void Store::replay_wal() {
  FILE* f = fopen(wal_path_.c_str(), "r");
  if (!f) return;
  replaying_ = true;
  std::string line;
  char buf[65536];
  int n = 0;
  while (fgets(buf, sizeof buf, f)) {
    line += buf;
    if (line.empty() || line.back() != '\n') continue;
    try {
      Json rec = Json::parse(line);
      std::string op = rec.at("op").str(), plural = rec.at("plural").str();
      const Json& obj = rec.at("object");
      std::string ns = obj.path("metadata.namespace").str(), name = obj.path("metadata.name").str();
      int64_t rv = std::stoll(obj.path("metadata.resourceVersion").str("0"));
      std::lock_guard<std::mutex> g(mu_);
      ++wal_records_;
      if (op == "rv") {}  // compaction's resource-version high-water mark (applied below)
      else if (op == "delete") data_[plural].erase(key(ns, name));
      else data_[plural][key(ns, name)] = Obj{obj, rv};
      if (op == "crd") {
        ResourceInfo ri;
        ri.group = obj.path("spec.group").str(); ri.version = obj.path("spec.version").str();
        ri.plural = obj.path("spec.names.plural").str(); ri.kind = obj.path("spec.names.kind").str();
        resources_[ri.plural] = ri;
      }
      rv_ = std::max(rv_, rv + 1);
      ++n;
    } catch (...) {
    }
    line.clear();
  }
  fclose(f);
  replaying_ = false;
  TFK_LOG(Info, "apiserver WAL replayed", Json(Json::object_t{{"records", Json(n)}, {"resourceVersion", Json((long long)rv_)}}));
}

ApiStatus Store::create(const std::string& plural, const std::string& ns_in, Json obj, Json* out) {
  std::lock_guard<std::mutex> g(mu_);
  auto ri = resources_.find(plural);
  if (ri == resources_.end()) return ApiStatus::Err(404, "NotFound", "unknown resource " + plural);
  if (!obj.is_object()) return ApiStatus::Err(400, "BadRequest", "body must be an object");
  Json& md = obj["metadata"];
  std::string ns = ri->second.namespaced ? (ns_in.empty() ? md.at("namespace").str("default") : ns_in) : "";
  if (ri->second.namespaced && md.has("namespace") && md.at("namespace").str() != ns)
    return ApiStatus::Err(400, "BadRequest", "namespace in body does not match path");
  std::string name = md.at("name").str();
  if (name.empty() && md.has("generateName")) name = md.at("generateName").str() + rand_string(5);
  if (name.empty()) return ApiStatus::Err(422, "Invalid", "metadata.name is required");
  auto& b = data_[plural];
  if (b.count(key(ns, name))) return ApiStatus::Err(409, "AlreadyExists", plural + " \"" + name + "\" already exists");
  int64_t rv = rv_++;
  md["name"] = name;
  if (ri->second.namespaced) md["namespace"] = ns;
  md["uid"] = rand_string(8) + "-" + rand_string(4) + "-" + rand_string(4) + "-" + rand_string(12);
  md["resourceVersion"] = std::to_string(rv);
  md["creationTimestamp"] = rfc3339(now_ms());
  md["generation"] = 1;
  md.erase("deletionTimestamp");
  if (!obj.has("kind")) obj["kind"] = ri->second.kind;
  if (!obj.has("apiVersion"))
    obj["apiVersion"] = ri->second.group.empty() ? ri->second.version : ri->second.group + "/" + ri->second.version;
  b[key(ns, name)] = Obj{obj, rv};
  ops_["create_" + plural]++;
  if (plural == "customresourcedefinitions") {
    ResourceInfo cr;
    cr.group = obj.path("spec.group").str();
    cr.version = obj.path("spec.version").str();
    for (auto& v : obj.path("spec.versions").items()) cr.versions.push_back(v.at("name").str());
    if (cr.version.empty() && !cr.versions.empty()) cr.version = cr.versions[0];
    if (cr.versions.empty()) cr.versions.push_back(cr.version);
    cr.plural = obj.path("spec.names.plural").str();
    cr.singular = obj.path("spec.names.singular").str();
    cr.kind = obj.path("spec.names.kind").str();
    cr.namespaced = obj.path("spec.scope").str("Namespaced") == "Namespaced";
    for (auto& s : obj.path("spec.names.shortNames").items()) cr.short_names.push_back(s.str());
    resources_[cr.plural] = cr;
    wal_locked("crd", plural, obj);
  } else {
    wal_locked("put", plural, obj);
  }
  emit_locked(plural, "ADDED", obj, rv);
  if (out) *out = obj;
  return ApiStatus::Ok(201);
}

ApiStatus Store::get(const std::string& plural, const std::string& ns, const std::string& name, Json* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto ri = resources_.find(plural);
  if (ri == resources_.end()) return ApiStatus::Err(404, "NotFound", "unknown resource " + plural);
  auto b = data_.find(plural);
  std::string k = key(ri->second.namespaced ? ns : "", name);
  if (b == data_.end() || !b->second.count(k)) return ApiStatus::Err(404, "NotFound", plural + " \"" + name + "\" not found");
  *out = b->second.at(k).data;
  return ApiStatus::Ok();
}

ApiStatus Store::list(const std::string& plural, const std::string& ns, const LabelSelector& ls,
                      const FieldSelector& fs, std::vector<Json>* items, int64_t* rv) const {
  std::lock_guard<std::mutex> g(mu_);
  if (!resources_.count(plural)) return ApiStatus::Err(404, "NotFound", "unknown resource " + plural);
  auto b = data_.find(plural);
  if (b != data_.end())
    for (auto& kv : b->second) {
      const Json& o = kv.second.data;
      if (!ns.empty() && o.path("metadata.namespace").str() != ns) continue;
      if (!ls.matches(o.path("metadata.labels"))) continue;
      if (!fs.matches(o)) continue;
      items->push_back(o);
    }
  if (rv) *rv = rv_ - 1;
  return ApiStatus::Ok();
}

ApiStatus Store::update(const std::string& plural, const std::string& ns_in, const std::string& name, Json obj,
                        bool status_only, Json* out) {
  std::lock_guard<std::mutex> g(mu_);
  auto ri = resources_.find(plural);
  if (ri == resources_.end()) return ApiStatus::Err(404, "NotFound", "unknown resource " + plural);
  std::string ns = ri->second.namespaced ? ns_in : "";
  auto& b = data_[plural];
  auto it = b.find(key(ns, name));
  if (it == b.end()) return ApiStatus::Err(404, "NotFound", plural + " \"" + name + "\" not found");
  Json cur = it->second.data;
  std::string want_rv = obj.path("metadata.resourceVersion").str();
  if (!want_rv.empty() && want_rv != cur.path("metadata.resourceVersion").str())
    return ApiStatus::Err(409, "Conflict",
                          "Operation cannot be fulfilled on " + plural + " \"" + name +
                              "\": the object has been modified; please apply your changes to the latest version");
  Json next;
  if (status_only) {
    next = cur.clone();
    next["status"] = obj.at("status").clone();
  } else {
    next = obj.clone();
    // immutable / server-managed metadata
    Json& md = next["metadata"];
    const Json& cmd = cur.at("metadata");
    for (const char* k : {"uid", "creationTimestamp", "namespace", "name"})
      if (cmd.has(k)) md[k] = cmd.at(k);
    if (cmd.has("deletionTimestamp")) md["deletionTimestamp"] = cmd.at("deletionTimestamp");
    if (cur.has("status") && plural != "pods" && plural != "services" && plural != "leases" && plural != "nodes" &&
        plural != "podgroups")
      next["status"] = cur.at("status");  // CRDs with the status subresource
    bool spec_changed = next.at("spec") != cur.at("spec");
    md["generation"] = cmd.at("generation").as_int(1) + (spec_changed ? 1 : 0);
  }
  int64_t rv = rv_++;
  next["metadata"]["resourceVersion"] = std::to_string(rv);
  ops_["update_" + plural]++;
  // finalizer removal on a terminating object completes the delete
  if (next.path("metadata.deletionTimestamp").is_string() && next.path("metadata.finalizers").size() == 0) {
    it->second = Obj{next, rv};
    if (out) *out = next;
    return finish_delete_locked(plural, ns, name, "Background", out);
  }
  it->second = Obj{next, rv};
  wal_locked("put", plural, next);
  emit_locked(plural, "MODIFIED", next, rv);
  if (out) *out = next;
  return ApiStatus::Ok();
}

Json merge_patch(const Json& target, const Json& patch) {
  if (!patch.is_object()) return patch.clone();
  Json t = target.is_object() ? target.clone() : Json::object();
  for (auto& kv : patch.fields()) {
    if (kv.second.is_null()) t.erase(kv.first);
    else t[kv.first] = merge_patch(t.at(kv.first), kv.second);
  }
  return t;
}

ApiStatus Store::patch(const std::string& plural, const std::string& ns, const std::string& name, const Json& p,
                       bool status_only, Json* out) {
  Json cur;
  for (int attempt = 0; attempt < 5; ++attempt) {
    ApiStatus s = get(plural, ns, name, &cur);
    if (!s.ok()) return s;
    Json next = merge_patch(cur, p);
    next["metadata"]["resourceVersion"] = cur.path("metadata.resourceVersion");
    s = update(plural, ns, name, next, status_only, out);
    if (s.code != 409) return s;
  }
  return ApiStatus::Err(409, "Conflict", "patch retries exhausted");
}

ApiStatus Store::remove(const std::string& plural, const std::string& ns_in, const std::string& name,
                        const std::string& propagation, Json* out) {
  std::lock_guard<std::mutex> g(mu_);
  auto ri = resources_.find(plural);
  if (ri == resources_.end()) return ApiStatus::Err(404, "NotFound", "unknown resource " + plural);
  std::string ns = ri->second.namespaced ? ns_in : "";
  auto& b = data_[plural];
  auto it = b.find(key(ns, name));
  if (it == b.end()) return ApiStatus::Err(404, "NotFound", plural + " \"" + name + "\" not found");
  Json& obj = it->second.data;
  if (obj.path("metadata.finalizers").size() > 0) {
    if (!obj.path("metadata.deletionTimestamp").is_string()) {
      Json next = obj.clone();
      next["metadata"]["deletionTimestamp"] = rfc3339(now_ms());
      int64_t rv = rv_++;
      next["metadata"]["resourceVersion"] = std::to_string(rv);
      it->second = Obj{next, rv};
      wal_locked("put", plural, next);
      emit_locked(plural, "MODIFIED", next, rv);
      if (out) *out = next;
    } else if (out) {
      *out = obj;
    }
    ops_["delete_pending_" + plural]++;
    return ApiStatus::Ok(202);
  }
  return finish_delete_locked(plural, ns, name, propagation, out);
}

ApiStatus Store::finish_delete_locked(const std::string& plural, const std::string& ns, const std::string& name,
                                      const std::string& propagation, Json* out) {
  auto& b = data_[plural];
  auto it = b.find(key(ns, name));
  if (it == b.end()) return ApiStatus::Err(404, "NotFound", name);
  Json obj = it->second.data;
  b.erase(it);
  int64_t rv = rv_++;
  obj["metadata"]["resourceVersion"] = std::to_string(rv);
  ops_["delete_" + plural]++;
  wal_locked("delete", plural, obj);
  emit_locked(plural, "DELETED", obj, rv);
  if (out) *out = obj;
  if (propagation != "Orphan") gc_dependents_locked(obj.path("metadata.uid").str(), ns);
  return ApiStatus::Ok();
}

void Store::gc_dependents_locked(const std::string& owner_uid, const std::string& ns) {
  if (owner_uid.empty()) return;
  std::vector<std::pair<std::string, std::string>> victims;
  for (auto& pb : data_)
    for (auto& kv : pb.second) {
      const Json& o = kv.second.data;
      if (o.path("metadata.namespace").str() != ns) continue;
      for (auto& ref : o.path("metadata.ownerReferences").items())
        if (ref.at("uid").str() == owner_uid) victims.push_back({pb.first, o.path("metadata.name").str()});
    }
  for (auto& v : victims) {
    auto& b = data_[v.first];
    auto it = b.find(key(ns, v.second));
    if (it == b.end()) continue;
    if (it->second.data.path("metadata.finalizers").size() > 0) {
      Json next = it->second.data.clone();
      next["metadata"]["deletionTimestamp"] = rfc3339(now_ms());
      int64_t rv = rv_++;
      next["metadata"]["resourceVersion"] = std::to_string(rv);
      it->second = Obj{next, rv};
      wal_locked("put", v.first, next);  // the terminating state must survive a WAL replay
      emit_locked(v.first, "MODIFIED", next, rv);
      continue;
    }
    finish_delete_locked(v.first, ns, v.second, "Background", nullptr);
  }
}

std::shared_ptr<Watcher> Store::watch(const std::string& plural, const std::string& ns, int64_t from_rv,
                                      const LabelSelector& ls, const FieldSelector& fs, ApiStatus* st,
                                      const std::string& requested_version) {
  std::lock_guard<std::mutex> g(mu_);
  if (!resources_.count(plural)) {
    *st = ApiStatus::Err(404, "NotFound", "unknown resource " + plural);
    return nullptr;
  }
  auto w = std::make_shared<Watcher>(plural, ns, ls, fs, requested_version);
  if (from_rv <= 0) {
    // no resourceVersion: start with synthetic ADDED events for the current state
    auto b = data_.find(plural);
    if (b != data_.end())
      for (auto& kv : b->second) w->deliver({"ADDED", kv.second.data, kv.second.rv});
  } else {
    int64_t oldest = history_.empty() ? rv_ : history_.front().rv;
    if (from_rv < oldest - 1 && from_rv < rv_ - 1) {
      *st = ApiStatus::Err(410, "Expired", "too old resource version: " + std::to_string(from_rv) + " (" +
                                               std::to_string(oldest) + ")");
      return nullptr;
    }
    for (auto& ev : history_)
      if (ev.rv > from_rv && history_plural_[ev.rv] == plural) w->deliver(ev);
  }
  watchers_.push_back(w);
  *st = ApiStatus::Ok();
  return w;
}

}  // namespace tfk
