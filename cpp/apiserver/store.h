// Single-node Kubernetes-semantics object store for the tfk control plane (the L0 substrate the
// reference operator talks to: REST layout k8s-operator.md:33-34, List/Watch images/informer1.png,
// finalizers + deletionTimestamp k8s-operator.md:35-43). Provides:
//   resourceVersion (global, monotonic) + optimistic concurrency (409 on stale update),
//   uid/creationTimestamp/generation, status subresource, label/field selectors,
//   watch with replay from a resourceVersion (410 Gone when it fell out of the history window),
//   finalizers (delete -> deletionTimestamp, removal when the list empties), ownerReference
//   cascading garbage collection, CRD registry + TFJob version conversion, optional JSON-lines WAL.
#pragma once
#include <atomic>
#include <thread>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../common/json.h"

namespace tfk {

struct ApiStatus {
  int code = 200;
  std::string reason, message;
  bool ok() const { return code >= 200 && code < 300; }
  static ApiStatus Ok(int c = 200) { return {c, "", ""}; }
  static ApiStatus Err(int c, const std::string& reason, const std::string& msg) { return {c, reason, msg}; }
  Json to_json() const;
};

struct ResourceInfo {
  std::string group;  // "" for core
  std::string version;
  std::string plural, singular, kind;
  bool namespaced = true;
  std::vector<std::string> versions;  // served versions
  std::vector<std::string> short_names;
};

// Label selector: "a=b,c!=d,e,!f,g in (x,y),h notin (z)"
class LabelSelector {
 public:
  static LabelSelector parse(const std::string& s, std::string* err = nullptr);
  static LabelSelector from_map(const Json& match_labels);
  bool matches(const Json& labels) const;
  bool empty() const { return reqs_.empty(); }
  std::string str() const;

 private:
  struct Req {
    std::string key, op;  // = != exists !exists in notin
    std::set<std::string> vals;
  };
  std::vector<Req> reqs_;
};

// Field selector: "metadata.name=x,status.phase!=Failed,spec.nodeName="
class FieldSelector {
 public:
  static FieldSelector parse(const std::string& s);
  bool matches(const Json& obj) const;
  bool empty() const { return reqs_.empty(); }

 private:
  struct Req {
    std::string path, val;
    bool neq;
  };
  std::vector<Req> reqs_;
};

struct WatchEvent {
  std::string type;  // ADDED | MODIFIED | DELETED | BOOKMARK | ERROR
  Json object;
  int64_t rv = 0;
};

class Watcher {
 public:
  // requested_version is fixed at construction: the watcher is published to the store's fan-out
  // list (read by other request threads under the store lock) the moment Store::watch returns.
  Watcher(std::string plural, std::string ns, LabelSelector ls, FieldSelector fs, std::string requested_version = "")
      : plural_(std::move(plural)), ns_(std::move(ns)), requested_version_(std::move(requested_version)),
        ls_(std::move(ls)), fs_(std::move(fs)) {}
  // Blocks up to timeout_ms; returns false on timeout or when closed with no events left.
  bool next(WatchEvent* ev, int64_t timeout_ms);
  void close();
  bool closed() const {
    std::lock_guard<std::mutex> g(mu_);
    return closed_;
  }
  void deliver(const WatchEvent& ev);  // applies ns/selector filters
  void max_queue_for_test(size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    max_queue_ = n;
  }
  const std::string& plural() const { return plural_; }
  const std::string& requested_version() const { return requested_version_; }  // TFJob conversion target

 private:
  friend class Store;
  const std::string plural_, ns_, requested_version_;
  LabelSelector ls_;
  FieldSelector fs_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<WatchEvent> q_;
  bool closed_ = false;
  size_t max_queue_ = 100000;
};

// Write-ahead-log durability (etcd's WAL discipline, scaled down): every mutation is appended and
// flushed to the page cache under the store lock; fdatasync is per record ("always"), batched by a
// background syncer every sync_interval_ms ("interval", group commit: a crash loses at most that
// window) or left to the kernel ("none"). The log is compacted into a snapshot of the live objects
// (plus the resource-version high-water mark) once it holds compact_records records and more than
// twice as many records as live objects: written to <wal>.tmp, fdatasync'ed, renamed over the WAL.
struct WalOptions {
  std::string sync = "interval";  // always | interval | none
  int64_t sync_interval_ms = 100;
  size_t compact_records = 20000;
};

class Store {
 public:
  explicit Store(const std::string& wal_path = "", size_t history = 10000, WalOptions wal_opts = WalOptions());
  ~Store();

  void register_resource(const ResourceInfo& ri);
  bool resource(const std::string& plural, ResourceInfo* out) const;
  bool resource_by_kind(const std::string& kind, ResourceInfo* out) const;
  std::vector<ResourceInfo> resources() const;

  ApiStatus create(const std::string& plural, const std::string& ns, Json obj, Json* out);
  ApiStatus get(const std::string& plural, const std::string& ns, const std::string& name, Json* out) const;
  ApiStatus list(const std::string& plural, const std::string& ns, const LabelSelector& ls, const FieldSelector& fs,
                 std::vector<Json>* items, int64_t* rv) const;
  // Full replace. status_only: only .status changes (status subresource); otherwise .status is kept.
  ApiStatus update(const std::string& plural, const std::string& ns, const std::string& name, Json obj,
                   bool status_only, Json* out);
  // RFC 7386 JSON merge patch.
  ApiStatus patch(const std::string& plural, const std::string& ns, const std::string& name, const Json& patch,
                  bool status_only, Json* out);
  // propagation: Background (default) | Foreground | Orphan
  ApiStatus remove(const std::string& plural, const std::string& ns, const std::string& name,
                   const std::string& propagation, Json* out);
  // requested_version: apiVersion the watcher's TFJob events are converted to ("" = stored version).
  std::shared_ptr<Watcher> watch(const std::string& plural, const std::string& ns, int64_t from_rv,
                                 const LabelSelector& ls, const FieldSelector& fs, ApiStatus* st,
                                 const std::string& requested_version = "");
  int64_t resource_version() const;
  size_t count(const std::string& plural) const;
  std::map<std::string, long long> counters() const;  // for /metrics

  // Version conversion hook for multi-version CRDs: (obj, target apiVersion) -> converted
  using Converter = std::function<Json(const Json&, const std::string&)>;
  void set_converter(const std::string& plural, Converter c);
  Json convert_for(const std::string& plural, const Json& obj, const std::string& api_version) const;

 private:
  struct Obj {
    Json data;
    int64_t rv;
  };
  using Bucket = std::map<std::string, Obj>;  // key "ns/name"
  static std::string key(const std::string& ns, const std::string& name) { return ns + "/" + name; }
  void emit_locked(const std::string& plural, const std::string& type, const Json& obj, int64_t rv);
  void wal_locked(const std::string& op, const std::string& plural, const Json& obj);
  void replay_wal();
  void compact_wal_locked();
  void syncer_loop();
  ApiStatus finish_delete_locked(const std::string& plural, const std::string& ns, const std::string& name,
                                 const std::string& propagation, Json* out);
  void gc_dependents_locked(const std::string& owner_uid, const std::string& ns);

  mutable std::mutex mu_;
  std::map<std::string, ResourceInfo> resources_;
  std::map<std::string, Bucket> data_;
  int64_t rv_ = 1;
  std::deque<WatchEvent> history_;  // all resources, rv ordered
  std::map<int64_t, std::string> history_plural_;
  size_t history_cap_;
  std::vector<std::weak_ptr<Watcher>> watchers_;
  std::map<std::string, Converter> converters_;
  std::string wal_path_;
  FILE* wal_ = nullptr;
  bool replaying_ = false;
  WalOptions wal_opts_;
  size_t wal_records_ = 0;
  std::atomic<bool> wal_dirty_{false}, syncer_stop_{false};
  std::thread syncer_;
  std::map<std::string, long long> ops_;
};

// RFC 7386
Json merge_patch(const Json& target, const Json& patch);

}  // namespace tfk
