#include "client.h"

#include <fstream>
#include <sstream>
#include <thread>

#include "../api/types.h"

namespace tfk {

void TokenBucket::refill() {
  int64_t now = mono_ms();
  tokens_ = std::min<double>(burst_, tokens_ + (now - last_) * qps_ / 1000.0);
  last_ = now;
}

bool TokenBucket::try_accept() {
  std::lock_guard<std::mutex> g(mu_);
  refill();
  if (tokens_ >= 1.0) { tokens_ -= 1.0; return true; }
  return false;
}

void TokenBucket::accept() {
  while (true) {
    double wait_ms;
    {
      std::lock_guard<std::mutex> g(mu_);
      refill();
      if (tokens_ >= 1.0) { tokens_ -= 1.0; return; }
      wait_ms = (1.0 - tokens_) * 1000.0 / qps_;
    }
    std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(wait_ms * 1000) + 100));
  }
}

// ------------------------------------------------------------------------------ REST
static void group_version(const std::string& plural, const std::string& tfjob_version, std::string* group,
                          std::string* version) {
  if (plural == "tfjobs") { *group = api::kGroupV1; *version = tfjob_version; }
  else if (plural == "leases") { *group = "coordination.k8s.io"; *version = "v1"; }
  else if (plural == "customresourcedefinitions") { *group = "apiextensions.k8s.io"; *version = "v1beta1"; }
  else if (plural == "podgroups") { *group = "scheduling.tfk.io"; *version = "v1"; }
  else if (plural == "priorityclasses") { *group = "scheduling.k8s.io"; *version = "v1"; }
  else { *group = ""; *version = "v1"; }
}

RestClient::RestClient(const RestConfig& cfg) : cfg_(cfg) {
  Endpoint ep;
  if (!parse_endpoint(cfg.host, &ep)) throw std::runtime_error("bad apiserver url " + cfg.host);
  std::shared_ptr<TlsContext> tls;
  if (ep.https) {
    std::string err;
    TlsOptions o = cfg.tls;
    o.enabled = true;
    tls = TlsContext::client(o, &err);
    if (!tls) throw std::runtime_error("TLS config for " + cfg.host + ": " + err);
  }
  http_.reset(new HttpClient(ep, tls, cfg.timeout_ms));
  http_->set_keepalive(cfg.keepalive);
  // NewForConfig: install a token bucket only when QPS > 0 (images/tf4.PNG:L4-L5)
  if (cfg.qps > 0) limiter_ = std::make_shared<TokenBucket>(cfg.qps, std::max(1, cfg.burst));
  if (cfg_.user_agent.empty()) cfg_.user_agent = "tfk-client/v0.1 (linux/amd64)";  // DefaultKubernetesUserAgent
  token_ = cfg_.bearer_token;
}

std::map<std::string, std::string> RestClient::auth_headers() {
  std::map<std::string, std::string> h{{"User-Agent", cfg_.user_agent}, {"Accept", "application/json"}};
  std::string tok;
  {
    // projected service-account tokens rotate: re-read the file at most once a minute (client-go)
    std::lock_guard<std::mutex> g(tok_mu_);
    if (!cfg_.bearer_token_file.empty() && mono_ms() - token_read_ms_ > 60000) {
      std::ifstream f(cfg_.bearer_token_file);
      std::stringstream ss;
      if (f) {
        ss << f.rdbuf();
        std::string t = trim(ss.str());
        if (!t.empty()) token_ = t;
      }
      token_read_ms_ = mono_ms();
    }
    tok = token_;
  }
  if (!tok.empty()) h["Authorization"] = "Bearer " + tok;
  else if (!cfg_.username.empty()) h["Authorization"] = "Basic " + base64_encode(cfg_.username + ":" + cfg_.password);
  return h;
}

std::string RestClient::path(const std::string& plural, const std::string& ns, const std::string& name,
                             const std::string& sub) const {
  std::string g, v;
  group_version(plural, cfg_.tfjob_version, &g, &v);
  std::string p = g.empty() ? "/api/" + v : "/apis/" + g + "/" + v;
  bool cluster_scoped = plural == "nodes" || plural == "namespaces" || plural == "customresourcedefinitions";
  if (!ns.empty() && !cluster_scoped) p += "/namespaces/" + ns;
  p += "/" + plural;
  if (!name.empty()) p += "/" + name;
  if (!sub.empty()) p += "/" + sub;
  return p;
}

ApiStatus RestClient::call(const std::string& method, const std::string& path, const std::string& body, Json* out,
                           const char* content_type) {
  if (limiter_) limiter_->accept();
  requests++;
  auto hdrs = auth_headers();
  if (!body.empty()) hdrs["Content-Type"] = content_type ? content_type : "application/json";
  HttpResponse r = http_->request(method, path, body, hdrs);
  if (r.status == 0) return ApiStatus::Err(503, "ServiceUnavailable", r.error);
  Json j;
  try { j = r.body.empty() ? Json() : Json::parse(r.body); } catch (...) { j = Json(r.body); }
  if (r.status >= 200 && r.status < 300) {
    if (out) *out = j;
    return ApiStatus::Ok(r.status);
  }
  return ApiStatus::Err(r.status, j.at("reason").str(http_status_text(r.status)), j.at("message").str(r.body));
}

ApiStatus RestClient::create(const std::string& plural, const std::string& ns, const Json& obj, Json* out) {
  return call("POST", path(plural, ns), obj.dump(), out);
}
ApiStatus RestClient::get(const std::string& plural, const std::string& ns, const std::string& name, Json* out) {
  return call("GET", path(plural, ns, name), "", out);
}
ApiStatus RestClient::list(const std::string& plural, const std::string& ns, const std::string& ls,
                           const std::string& fs, ListResult* out) {
  std::string q;
  if (!ls.empty()) q += "labelSelector=" + url_encode(ls);
  if (!fs.empty()) q += std::string(q.empty() ? "" : "&") + "fieldSelector=" + url_encode(fs);
  Json j;
  ApiStatus st = call("GET", path(plural, ns) + (q.empty() ? "" : "?" + q), "", &j);
  if (!st.ok()) return st;
  out->items = j.at("items").items();
  out->resource_version = std::stoll(j.path("metadata.resourceVersion").str("0"));
  return st;
}
ApiStatus RestClient::update(const std::string& plural, const std::string& ns, const Json& obj, Json* out) {
  return call("PUT", path(plural, ns, obj.path("metadata.name").str()), obj.dump(), out);
}
ApiStatus RestClient::update_status(const std::string& plural, const std::string& ns, const Json& obj, Json* out) {
  return call("PUT", path(plural, ns, obj.path("metadata.name").str(), "status"), obj.dump(), out);
}
ApiStatus RestClient::patch(const std::string& plural, const std::string& ns, const std::string& name, const Json& p,
                            Json* out) {
  // JSON merge patch (RFC 7386): the content type a kube-apiserver requires for this body
  return call("PATCH", path(plural, ns, name), p.dump(), out, "application/merge-patch+json");
}
ApiStatus RestClient::remove(const std::string& plural, const std::string& ns, const std::string& name,
                             const std::string& propagation) {
  return call("DELETE", path(plural, ns, name) + "?propagationPolicy=" + propagation, "", nullptr);
}

namespace {
// Background thread reading the HTTP watch stream into a queue.
class RestWatch : public WatchStream {
 public:
  RestWatch(HttpClient http, std::string path, std::map<std::string, std::string> hdrs)
      : http_(std::move(http)), path_(std::move(path)), hdrs_(std::move(hdrs)) {
    thr_ = std::thread([this] { run(); });
  }
  ~RestWatch() override {
    close();
    if (thr_.joinable()) thr_.join();
  }
  bool next(WatchEvent* ev, int64_t timeout_ms) override {
    std::unique_lock<std::mutex> l(mu_);
    cv_wait_ms(cv_, l, timeout_ms, [&] { return !q_.empty() || done_; });
    if (q_.empty()) return false;
    *ev = q_.front();
    q_.pop_front();
    return true;
  }
  bool closed() const override {
    std::lock_guard<std::mutex> g(mu_);
    return done_ && q_.empty();
  }
  void close() override { stop_ = true; }

 private:
  void run() {
    std::string err;
    http_.stream_lines(path_, [this](const std::string& line) {
      WatchEvent ev;
      try {
        Json j = Json::parse(line);
        ev.type = j.at("type").str();
        ev.object = j.at("object");
        if (ev.type.empty()) { ev.type = "ERROR"; ev.object = j; }
      } catch (...) {
        return true;
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        q_.push_back(ev);
      }
      cv_.notify_all();
      return !stop_.load();
    }, &stop_, &err, hdrs_);
    {
      std::lock_guard<std::mutex> g(mu_);
      done_ = true;
    }
    cv_.notify_all();
  }
  HttpClient http_;
  std::string path_;
  std::map<std::string, std::string> hdrs_;
  std::thread thr_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<WatchEvent> q_;
  bool done_ = false;
  std::atomic<bool> stop_{false};
};

class StoreWatch : public WatchStream {
 public:
  explicit StoreWatch(std::shared_ptr<Watcher> w) : w_(std::move(w)) {}
  ~StoreWatch() override { w_->close(); }
  bool next(WatchEvent* ev, int64_t timeout_ms) override { return w_->next(ev, timeout_ms); }
  bool closed() const override { return w_->closed(); }
  void close() override { w_->close(); }

 private:
  std::shared_ptr<Watcher> w_;
};
}  // namespace

std::unique_ptr<WatchStream> RestClient::watch(const std::string& plural, const std::string& ns, int64_t rv,
                                               const std::string& ls, const std::string& fs, ApiStatus* st) {
  if (limiter_) limiter_->accept();
  requests++;
  std::string q = "watch=true&resourceVersion=" + std::to_string(rv) + "&allowWatchBookmarks=false";
  if (!ls.empty()) q += "&labelSelector=" + url_encode(ls);
  if (!fs.empty()) q += "&fieldSelector=" + url_encode(fs);
  *st = ApiStatus::Ok();
  // copies of the HttpClient share its TLS context; the stream dials its own connection
  return std::unique_ptr<WatchStream>(new RestWatch(*http_, path(plural, ns) + "?" + q, auth_headers()));
}

// ------------------------------------------------------------------------------ fake
void FakeClient::record(const std::string& a) {
  std::lock_guard<std::mutex> g(mu_);
  actions_.push_back(a);
  requests++;
}
std::vector<std::string> FakeClient::actions() {
  std::lock_guard<std::mutex> g(mu_);
  return actions_;
}
void FakeClient::clear_actions() {
  std::lock_guard<std::mutex> g(mu_);
  actions_.clear();
}
ApiStatus FakeClient::create(const std::string& plural, const std::string& ns, const Json& obj, Json* out) {
  record("create " + plural + "/" + obj.path("metadata.name").str());
  return store_->create(plural, ns, obj.clone(), out);
}
ApiStatus FakeClient::get(const std::string& plural, const std::string& ns, const std::string& name, Json* out) {
  record("get " + plural + "/" + name);
  return store_->get(plural, ns, name, out);
}
ApiStatus FakeClient::list(const std::string& plural, const std::string& ns, const std::string& ls,
                           const std::string& fs, ListResult* out) {
  record("list " + plural);
  return store_->list(plural, ns, LabelSelector::parse(ls), FieldSelector::parse(fs), &out->items,
                      &out->resource_version);
}
ApiStatus FakeClient::update(const std::string& plural, const std::string& ns, const Json& obj, Json* out) {
  record("update " + plural + "/" + obj.path("metadata.name").str());
  return store_->update(plural, ns, obj.path("metadata.name").str(), obj.clone(), false, out);
}
ApiStatus FakeClient::update_status(const std::string& plural, const std::string& ns, const Json& obj, Json* out) {
  record("update " + plural + "/" + obj.path("metadata.name").str() + "/status");
  return store_->update(plural, ns, obj.path("metadata.name").str(), obj.clone(), true, out);
}
ApiStatus FakeClient::patch(const std::string& plural, const std::string& ns, const std::string& name, const Json& p,
                            Json* out) {
  record("patch " + plural + "/" + name);
  return store_->patch(plural, ns, name, p, false, out);
}
ApiStatus FakeClient::remove(const std::string& plural, const std::string& ns, const std::string& name,
                             const std::string& propagation) {
  record("delete " + plural + "/" + name);
  return store_->remove(plural, ns, name, propagation, nullptr);
}
std::unique_ptr<WatchStream> FakeClient::watch(const std::string& plural, const std::string& ns, int64_t rv,
                                               const std::string& ls, const std::string& fs, ApiStatus* st) {
  record("watch " + plural);
  auto w = store_->watch(plural, ns, rv, LabelSelector::parse(ls), FieldSelector::parse(fs), st);
  if (!w) return nullptr;
  return std::unique_ptr<WatchStream>(new StoreWatch(w));
}

std::shared_ptr<Client> new_for_config(const RestConfig& cfg) { return std::make_shared<RestClient>(cfg); }

}  // namespace tfk
