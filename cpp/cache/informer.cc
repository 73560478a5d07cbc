#include "informer.h"

#include <algorithm>

namespace tfk {

std::string meta_namespace_key(const Json& obj) {
  std::string ns = obj.path("metadata.namespace").str();
  std::string name = obj.path("metadata.name").str();
  return ns.empty() ? name : ns + "/" + name;
}

bool split_meta_namespace_key(const std::string& key, std::string* ns, std::string* name) {
  auto parts = split(key, '/');
  if (parts.size() == 1) { ns->clear(); *name = parts[0]; return !name->empty(); }
  if (parts.size() == 2) { *ns = parts[0]; *name = parts[1]; return !name->empty(); }
  return false;
}

// ------------------------------------------------------------------------------ indexer
Indexer::Indexer() {
  add_indexer("namespace", [](const Json& o) { return std::vector<std::string>{o.path("metadata.namespace").str()}; });
}

void Indexer::add_indexer(const std::string& name, IndexFunc f) {
  std::lock_guard<std::mutex> g(mu_);
  indexers_[name] = std::move(f);
  auto& idx = indices_[name];
  idx.clear();
  for (auto& kv : items_)
    for (auto& v : indexers_[name](kv.second)) idx[v].insert(kv.first);
}

void Indexer::index_locked(const std::string& key, const Json& obj, bool add) {
  for (auto& ix : indexers_) {
    for (auto& v : ix.second(obj)) {
      auto& s = indices_[ix.first][v];
      if (add) s.insert(key);
      else {
        s.erase(key);
        if (s.empty()) indices_[ix.first].erase(v);
      }
    }
  }
}

void Indexer::upsert(const std::string& key, const Json& obj) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = items_.find(key);
  if (it != items_.end()) index_locked(key, it->second, false);
  items_[key] = obj;
  index_locked(key, obj, true);
}

void Indexer::remove(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = items_.find(key);
  if (it == items_.end()) return;
  index_locked(key, it->second, false);
  items_.erase(it);
}

bool Indexer::get_by_key(const std::string& key, Json* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = items_.find(key);
  if (it == items_.end()) return false;
  *out = it->second;
  return true;
}

std::vector<Json> Indexer::list() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Json> v;
  for (auto& kv : items_) v.push_back(kv.second);
  return v;
}

std::vector<std::string> Indexer::list_keys() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> v;
  for (auto& kv : items_) v.push_back(kv.first);
  return v;
}

std::vector<Json> Indexer::by_index(const std::string& index, const std::string& value) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Json> v;
  auto ix = indices_.find(index);
  if (ix == indices_.end()) return v;
  auto s = ix->second.find(value);
  if (s == ix->second.end()) return v;
  for (auto& k : s->second) v.push_back(items_.at(k));
  return v;
}

void Indexer::replace(const std::map<std::string, Json>& items) {
  std::lock_guard<std::mutex> g(mu_);
  items_ = items;
  for (auto& ix : indices_) ix.second.clear();
  for (auto& kv : items_) index_locked(kv.first, kv.second, true);
}

size_t Indexer::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return items_.size();
}

// ------------------------------------------------------------------------------ delta fifo
void DeltaFIFO::add(DeltaType t, const std::string& key, const Json& obj) {
  std::lock_guard<std::mutex> g(mu_);
  if (closed_) return;
  auto& d = items_[key];
  if (d.empty()) queue_.push_back(key);
  // dedupe consecutive deletes (client-go dedupDeltas)
  if (!d.empty() && t == DeltaType::Deleted && d.back().type == DeltaType::Deleted) d.back() = {t, obj};
  else d.push_back({t, obj});
  cv_.notify_one();
}

bool DeltaFIFO::pop(std::string* key, std::vector<Delta>* deltas, int64_t timeout_ms) {
  std::unique_lock<std::mutex> l(mu_);
  cv_wait_ms(cv_, l, timeout_ms, [&] { return !queue_.empty() || closed_; });
  if (queue_.empty()) return false;
  *key = queue_.front();
  queue_.pop_front();
  *deltas = std::move(items_[*key]);
  items_.erase(*key);
  if (initial_pop_ > 0) {
    if (--initial_pop_ == 0) synced_ = true;
  }
  return true;
}

void DeltaFIFO::close() {
  std::lock_guard<std::mutex> g(mu_);
  closed_ = true;
  cv_.notify_all();
}

// ------------------------------------------------------------------------------ informer
SharedInformer::SharedInformer(std::shared_ptr<Client> c, std::string plural, std::string ns, int64_t resync_ms,
                               std::string ls, std::string fs)
    : client_(std::move(c)), plural_(std::move(plural)), ns_(std::move(ns)), ls_(std::move(ls)), fs_(std::move(fs)),
      resync_ms_(resync_ms) {}

SharedInformer::~SharedInformer() {
  fifo_.close();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
}

void SharedInformer::add_event_handler(EventHandlers h) {
  std::lock_guard<std::mutex> g(hmu_);
  handlers_.push_back(std::move(h));
}

void SharedInformer::start(StopToken& stop) {
  threads_.emplace_back([this, &stop] { reflector_loop(stop); });
  threads_.emplace_back([this, &stop] { process_loop(stop); });
  if (resync_ms_ > 0) threads_.emplace_back([this, &stop] { resync_loop(stop); });
}

void SharedInformer::run(StopToken& stop) {
  start(stop);
  while (!stop.wait_for(1000)) {
  }
  fifo_.close();
}

bool SharedInformer::wait_for_sync(int64_t timeout_ms) const {
  int64_t dl = mono_ms() + timeout_ms;
  while (mono_ms() < dl) {
    if (synced_) return true;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  return synced_;
}

void SharedInformer::reflector_loop(StopToken& stop) {
  bool first = true;
  while (!stop.stopped()) {
    ListResult lr;
    ApiStatus st = client_->list(plural_, ns_, ls_, fs_, &lr);
    if (!st.ok()) {
      TFK_LOG(Warn, "reflector list failed", Json(Json::object_t{{"resource", Json(plural_)}, {"error", Json(st.message)}}));
      if (stop.wait_for(1000)) break;
      continue;
    }
    relists_++;
    std::set<std::string> seen;
    for (auto& o : lr.items) {
      std::string k = meta_namespace_key(o);
      seen.insert(k);
      Json old;
      bool had = indexer_.get_by_key(k, &old);
      if (!had) fifo_.add(DeltaType::Added, k, o);
      else if (old.path("metadata.resourceVersion") != o.path("metadata.resourceVersion"))
        fifo_.add(DeltaType::Updated, k, o);
    }
    for (auto& k : indexer_.list_keys())
      if (!seen.count(k)) {
        Json old;
        if (indexer_.get_by_key(k, &old)) fifo_.add(DeltaType::Deleted, k, old);
      }
    if (first) {
      first = false;
      fifo_.set_populated(lr.items.size());
      if (lr.items.empty()) synced_ = true;
    }
    int64_t rv = lr.resource_version;
    // watch until error; resume from the last seen rv on clean stream end
    bool relist = false;
    while (!stop.stopped() && !relist) {
      ApiStatus ws;
      auto w = client_->watch(plural_, ns_, rv, ls_, fs_, &ws);
      if (!w) { relist = true; break; }
      while (!stop.stopped()) {
        WatchEvent ev;
        if (!w->next(&ev, 500)) {
          if (w->closed()) break;
          continue;
        }
        if (ev.type == "ERROR") {
          TFK_LOG(Info, "watch error, relisting", Json(Json::object_t{{"resource", Json(plural_)},
                                                                      {"status", ev.object}}));
          relist = true;
          break;
        }
        std::string evrv = ev.object.path("metadata.resourceVersion").str();
        if (!evrv.empty()) rv = std::max(rv, (int64_t)std::stoll(evrv));
        if (ev.type == "BOOKMARK") continue;
        std::string k = meta_namespace_key(ev.object);
        if (ev.type == "ADDED") fifo_.add(DeltaType::Added, k, ev.object);
        else if (ev.type == "MODIFIED") fifo_.add(DeltaType::Updated, k, ev.object);
        else if (ev.type == "DELETED") fifo_.add(DeltaType::Deleted, k, ev.object);
      }
      w->close();
      if (!relist && stop.wait_for(50)) break;
    }
  }
}

void SharedInformer::process_loop(StopToken& stop) {
  while (!stop.stopped()) {
    std::string key;
    std::vector<Delta> deltas;
    if (!fifo_.pop(&key, &deltas, 200)) {
      if (fifo_.has_synced()) synced_ = true;
      continue;
    }
    std::vector<EventHandlers> hs;
    {
      std::lock_guard<std::mutex> g(hmu_);
      hs = handlers_;
    }
    for (auto& d : deltas) {
      Json old;
      bool had = indexer_.get_by_key(key, &old);
      if (d.type == DeltaType::Deleted) {
        indexer_.remove(key);
        for (auto& h : hs)
          if (h.on_delete) h.on_delete(d.object);
      } else {
        indexer_.upsert(key, d.object);
        for (auto& h : hs) {
          if (!had) { if (h.on_add) h.on_add(d.object); }
          else if (h.on_update) h.on_update(old, d.object);
        }
      }
    }
    if (fifo_.has_synced()) synced_ = true;
  }
}

void SharedInformer::resync_loop(StopToken& stop) {
  while (!stop.wait_for(resync_ms_)) {
    for (auto& o : indexer_.list()) fifo_.add(DeltaType::Sync, meta_namespace_key(o), o);
  }
}

std::vector<Json> Lister::list(const std::string& ns, const std::string& label_selector) const {
  LabelSelector sel = LabelSelector::parse(label_selector);
  std::vector<Json> src = ns.empty() ? idx_.list() : idx_.by_index("namespace", ns);
  std::vector<Json> out;
  for (auto& o : src)
    if (sel.matches(o.path("metadata.labels"))) out.push_back(o);
  return out;
}

bool Lister::get(const std::string& ns, const std::string& name, Json* out) const {
  return idx_.get_by_key(ns.empty() ? name : ns + "/" + name, out);
}

bool wait_for_cache_sync(const std::vector<SharedInformer*>& infs, int64_t timeout_ms) {
  int64_t dl = mono_ms() + timeout_ms;
  for (auto* i : infs)
    if (!i->wait_for_sync(std::max<int64_t>(1, dl - mono_ms()))) return false;
  return true;
}

}  // namespace tfk
