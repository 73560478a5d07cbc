// Informer machinery (reference: images/informer1.png — Reflector -> DeltaFIFO -> Local Store +
// OnAdd/OnUpdate/OnDelete callbacks; pkg/client/{informers,listers}, images/tf3.PNG:L41-L56;
// sample cache.NewIndexerInformer k8s-operator.md:110-127).
//   Reflector  : List then Watch from the list's resourceVersion; relist on 410/ERROR/stream end.
//   DeltaFIFO  : per-key accumulated deltas, popped in FIFO key order (Sync deltas for resync).
//   Indexer    : thread-safe local store with a namespace index + custom indexers.
//   SharedInformer: owns the three, dispatches handlers, periodic resync (the sample's resync=0
//                 bug, §0.5 #8, is not reproduced: default 30 s).
//   Lister     : read-only view (List by selector, Get by namespace/name).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../client/client.h"
#include "../common/util.h"

namespace tfk {

std::string meta_namespace_key(const Json& obj);  // "ns/name" (or "name" for cluster-scoped)
bool split_meta_namespace_key(const std::string& key, std::string* ns, std::string* name);

class Indexer {
 public:
  using IndexFunc = std::function<std::vector<std::string>(const Json&)>;
  Indexer();
  void add_indexer(const std::string& name, IndexFunc f);
  void upsert(const std::string& key, const Json& obj);
  void remove(const std::string& key);
  bool get_by_key(const std::string& key, Json* out) const;
  std::vector<Json> list() const;
  std::vector<std::string> list_keys() const;
  std::vector<Json> by_index(const std::string& index, const std::string& value) const;
  void replace(const std::map<std::string, Json>& items);
  size_t size() const;

 private:
  void index_locked(const std::string& key, const Json& obj, bool add);
  mutable std::mutex mu_;
  std::map<std::string, Json> items_;
  std::map<std::string, IndexFunc> indexers_;
  std::map<std::string, std::map<std::string, std::set<std::string>>> indices_;
};

enum class DeltaType { Added, Updated, Deleted, Sync };
struct Delta {
  DeltaType type;
  Json object;
};

class DeltaFIFO {
 public:
  void add(DeltaType t, const std::string& key, const Json& obj);
  // Blocks up to timeout; returns false on timeout/close.
  bool pop(std::string* key, std::vector<Delta>* deltas, int64_t timeout_ms);
  void close();
  bool has_synced() const { return synced_; }
  void set_populated(size_t initial) {
    std::lock_guard<std::mutex> g(mu_);
    initial_pop_ = initial;
    if (initial == 0) synced_ = true;
  }
  size_t len() const {
    std::lock_guard<std::mutex> g(mu_);
    return queue_.size();
  }

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> queue_;
  std::map<std::string, std::vector<Delta>> items_;
  bool closed_ = false;
  std::atomic<bool> synced_{false};
  size_t initial_pop_ = 0;
};

struct EventHandlers {
  std::function<void(const Json&)> on_add;
  std::function<void(const Json& old_obj, const Json& new_obj)> on_update;
  std::function<void(const Json&)> on_delete;
};

class SharedInformer {
 public:
  SharedInformer(std::shared_ptr<Client> c, std::string plural, std::string ns = "", int64_t resync_ms = 30000,
                 std::string label_selector = "", std::string field_selector = "");
  ~SharedInformer();
  void add_event_handler(EventHandlers h);
  void run(StopToken& stop);  // blocking: reflector + processor threads
  void start(StopToken& stop);  // non-blocking
  bool has_synced() const { return synced_; }
  bool wait_for_sync(int64_t timeout_ms) const;
  Indexer& indexer() { return indexer_; }
  long long relists() const { return relists_; }
  const std::string& plural() const { return plural_; }

 private:
  void reflector_loop(StopToken& stop);
  void process_loop(StopToken& stop);
  void resync_loop(StopToken& stop);
  std::shared_ptr<Client> client_;
  std::string plural_, ns_, ls_, fs_;
  int64_t resync_ms_;
  Indexer indexer_;
  DeltaFIFO fifo_;
  std::mutex hmu_;
  std::vector<EventHandlers> handlers_;
  std::atomic<bool> synced_{false};
  std::atomic<long long> relists_{0};
  std::vector<std::thread> threads_;
};

class Lister {
 public:
  explicit Lister(Indexer& idx) : idx_(idx) {}
  std::vector<Json> list(const std::string& ns = "", const std::string& label_selector = "") const;
  bool get(const std::string& ns, const std::string& name, Json* out) const;

 private:
  Indexer& idx_;
};

// Wait until every informer has synced (cache.WaitForCacheSync)
bool wait_for_cache_sync(const std::vector<SharedInformer*>& infs, int64_t timeout_ms);

}  // namespace tfk
