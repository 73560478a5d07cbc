// HTTP front of the tfk single-node API server: Kubernetes REST layout over Store.
//   /api/v1/namespaces/{ns}/{plural}[/{name}[/status|/log]]   core kinds
//   /apis/{group}/{version}/namespaces/{ns}/{plural}[/{name}[/status]]
//   /api/v1/{plural}, /apis/{g}/{v}/{plural}                    cluster-wide list/watch
//   ?watch=1&resourceVersion=N&labelSelector=..&fieldSelector=..&timeoutSeconds=..
//   /healthz /version /metrics /apis (discovery)
// Optional HTTPS (--tls-cert-file/--tls-private-key-file) and bearer-token authentication
// (--token-auth-file), so the operator's kube-apiserver client path is exercised locally.
#pragma once
#include <map>
#include <memory>
#include <string>

#include "../common/http.h"
#include "store.h"

namespace tfk {

class ApiServer {
 public:
  explicit ApiServer(std::shared_ptr<Store> store) : store_(std::move(store)) {}
  bool start(const std::string& host, int port, std::string* err);
  // Serve HTTPS with this certificate/key (call before start()).
  bool enable_tls(const TlsOptions& o, std::string* err) { return http_.enable_tls(o, err); }
  // Require "Authorization: Bearer <token>" (kube-apiserver --token-auth-file: token,user,uid[,...]
  // CSV). Health endpoints stay open. Returns false if the file cannot be read or is empty.
  bool load_token_file(const std::string& path, std::string* err);
  void add_token(const std::string& token, const std::string& user) { tokens_[token] = user; }
  bool tls() const { return http_.tls(); }
  long long connections_accepted() const { return http_.connections_accepted(); }
  long long connections_rejected() const { return http_.connections_rejected(); }
  void set_max_connections(int n) { http_.set_max_connections(n); }
  void stop() { http_.stop(); }
  int port() const { return http_.port(); }
  Store& store() { return *store_; }
  void handle(const HttpRequest& req, ResponseWriter& w);
  void set_log_root(const std::string& d) { log_root_ = d; }

 private:
  void do_watch(const HttpRequest& req, ResponseWriter& w, const std::string& plural, const std::string& ns,
                const std::string& api_version);
  std::shared_ptr<Store> store_;
  HttpServer http_;
  std::string log_root_;
  std::map<std::string, std::string> tokens_;  // bearer token -> user
};

// Install the TFJob CRD (+ v1alpha1<->v1 converter) into a store.
void install_tfjob_crd(Store& store);

}  // namespace tfk
