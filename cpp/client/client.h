// Clientset for the tfk control plane (reference: pkg/client/clientset/versioned/*, images/tf3.PNG:L18-L40;
// NewForConfig + token-bucket RateLimiter images/tf4.PNG:L2-L20; setConfigDefaults images/tf6.PNG).
// One untyped resource interface (CRUD + List + Watch keyed by plural) with two backends:
//   RestClient - HTTP/1.1 (or HTTPS) to tfk-apiserver or a real kube-apiserver: QPS/Burst token
//                bucket, UserAgent, GroupVersion table, bearer-token / basic / client-cert auth,
//                keep-alive connection reuse (config.h builds the RestConfig).
//   FakeClient - in-process Store (the generated "fake clientset": no server, records Actions()).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../apiserver/store.h"
#include "../common/http.h"
#include "config.h"

namespace tfk {

// flowcontrol.NewTokenBucketRateLimiter(qps, burst)
class TokenBucket {
 public:
  TokenBucket(double qps, int burst) : qps_(qps), burst_(burst), tokens_(burst), last_(mono_ms()) {}
  void accept();         // blocks until a token is available
  bool try_accept();
  double qps() const { return qps_; }

 private:
  void refill();
  std::mutex mu_;
  double qps_;
  int burst_;
  double tokens_;
  int64_t last_;
};

class WatchStream {
 public:
  virtual ~WatchStream() = default;
  virtual bool next(WatchEvent* ev, int64_t timeout_ms) = 0;  // false on timeout / closed
  virtual bool closed() const = 0;
  virtual void close() = 0;
};

struct ListResult {
  std::vector<Json> items;
  int64_t resource_version = 0;
};

class Client {
 public:
  virtual ~Client() = default;
  virtual ApiStatus create(const std::string& plural, const std::string& ns, const Json& obj, Json* out) = 0;
  virtual ApiStatus get(const std::string& plural, const std::string& ns, const std::string& name, Json* out) = 0;
  virtual ApiStatus list(const std::string& plural, const std::string& ns, const std::string& label_selector,
                         const std::string& field_selector, ListResult* out) = 0;
  virtual ApiStatus update(const std::string& plural, const std::string& ns, const Json& obj, Json* out) = 0;
  virtual ApiStatus update_status(const std::string& plural, const std::string& ns, const Json& obj, Json* out) = 0;
  virtual ApiStatus patch(const std::string& plural, const std::string& ns, const std::string& name, const Json& patch,
                          Json* out) = 0;
  virtual ApiStatus remove(const std::string& plural, const std::string& ns, const std::string& name,
                           const std::string& propagation = "Background") = 0;
  virtual std::unique_ptr<WatchStream> watch(const std::string& plural, const std::string& ns, int64_t rv,
                                             const std::string& label_selector, const std::string& field_selector,
                                             ApiStatus* st) = 0;
  std::atomic<long long> requests{0};
};

class RestClient : public Client {
 public:
  explicit RestClient(const RestConfig& cfg);
  ApiStatus create(const std::string& plural, const std::string& ns, const Json& obj, Json* out) override;
  ApiStatus get(const std::string& plural, const std::string& ns, const std::string& name, Json* out) override;
  ApiStatus list(const std::string& plural, const std::string& ns, const std::string& ls, const std::string& fs,
                 ListResult* out) override;
  ApiStatus update(const std::string& plural, const std::string& ns, const Json& obj, Json* out) override;
  ApiStatus update_status(const std::string& plural, const std::string& ns, const Json& obj, Json* out) override;
  ApiStatus patch(const std::string& plural, const std::string& ns, const std::string& name, const Json& patch,
                  Json* out) override;
  ApiStatus remove(const std::string& plural, const std::string& ns, const std::string& name,
                   const std::string& propagation) override;
  std::unique_ptr<WatchStream> watch(const std::string& plural, const std::string& ns, int64_t rv,
                                     const std::string& ls, const std::string& fs, ApiStatus* st) override;
  std::string path(const std::string& plural, const std::string& ns, const std::string& name = "",
                   const std::string& sub = "") const;
  const RestConfig& config() const { return cfg_; }
  HttpClient& http() { return *http_; }

 private:
  ApiStatus call(const std::string& method, const std::string& path, const std::string& body, Json* out,
                 const char* content_type = nullptr);
  std::map<std::string, std::string> auth_headers();
  RestConfig cfg_;
  std::unique_ptr<HttpClient> http_;
  std::shared_ptr<TokenBucket> limiter_;
  std::mutex tok_mu_;
  std::string token_;
  int64_t token_read_ms_ = 0;
};

// Fake clientset: talks to an in-process Store; records (verb, plural, name) actions.
class FakeClient : public Client {
 public:
  explicit FakeClient(std::shared_ptr<Store> s) : store_(std::move(s)) {}
  ApiStatus create(const std::string& plural, const std::string& ns, const Json& obj, Json* out) override;
  ApiStatus get(const std::string& plural, const std::string& ns, const std::string& name, Json* out) override;
  ApiStatus list(const std::string& plural, const std::string& ns, const std::string& ls, const std::string& fs,
                 ListResult* out) override;
  ApiStatus update(const std::string& plural, const std::string& ns, const Json& obj, Json* out) override;
  ApiStatus update_status(const std::string& plural, const std::string& ns, const Json& obj, Json* out) override;
  ApiStatus patch(const std::string& plural, const std::string& ns, const std::string& name, const Json& patch,
                  Json* out) override;
  ApiStatus remove(const std::string& plural, const std::string& ns, const std::string& name,
                   const std::string& propagation) override;
  std::unique_ptr<WatchStream> watch(const std::string& plural, const std::string& ns, int64_t rv,
                                     const std::string& ls, const std::string& fs, ApiStatus* st) override;
  std::vector<std::string> actions();  // "create pods/name" ...
  void clear_actions();
  Store& store() { return *store_; }

 private:
  void record(const std::string& a);
  std::shared_ptr<Store> store_;
  std::mutex mu_;
  std::vector<std::string> actions_;
};

std::shared_ptr<Client> new_for_config(const RestConfig& cfg);  // versioned.NewForConfig

}  // namespace tfk
