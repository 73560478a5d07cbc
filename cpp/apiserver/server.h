// HTTP front of the tfk single-node API server: Kubernetes REST layout over Store.
//   /api/v1/namespaces/{ns}/{plural}[/{name}[/status|/log]]   core kinds
//   /apis/{group}/{version}/namespaces/{ns}/{plural}[/{name}[/status]]
//   /api/v1/{plural}, /apis/{g}/{v}/{plural}                    cluster-wide list/watch
//   ?watch=1&resourceVersion=N&labelSelector=..&fieldSelector=..&timeoutSeconds=..
//   /healthz /version /metrics /apis (discovery)
#pragma once
#include <memory>
#include <string>

#include "../common/http.h"
#include "store.h"

namespace tfk {

class ApiServer {
 public:
  explicit ApiServer(std::shared_ptr<Store> store) : store_(std::move(store)) {}
  bool start(const std::string& host, int port, std::string* err);
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
};

// Install the TFJob CRD (+ v1alpha1<->v1 converter) into a store.
void install_tfjob_crd(Store& store);

}  // namespace tfk
