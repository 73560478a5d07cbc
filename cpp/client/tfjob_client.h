// Typed TFJob clientset (reference: pkg/client/clientset/versioned/clientset.go and
// typed/tensorflow/v1alpha1/{tensorflow_client.go,tfjob.go}, images/tf3.PNG:L20-L40;
// TensorflowV1alpha1Client.NewForConfig -> setConfigDefaults -> RESTClientFor, images/tf5.PNG,
// images/tf6.PNG). Operations take and return api::TFJob (the hub model) and speak the wire shape
// of the group-version the typed client was created for (kubeflow.org/v1 or .../v1alpha1).
//
//   auto cs = Clientset::NewForConfig(cfg);
//   api::TFJob j; cs->TensorflowV1()->TFJobs("default").Get("mnist", &j);
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "../api/types.h"
#include "client.h"

namespace tfk {

struct TFJobEvent {
  std::string type;  // ADDED | MODIFIED | DELETED | ERROR
  api::TFJob job;
  Json raw;
};

class TFJobWatch {
 public:
  explicit TFJobWatch(std::unique_ptr<WatchStream> s) : s_(std::move(s)) {}
  // false on timeout / closed; malformed objects surface as type ERROR with raw set
  bool next(TFJobEvent* ev, int64_t timeout_ms);
  void close() { if (s_) s_->close(); }
  bool closed() const { return !s_ || s_->closed(); }

 private:
  std::unique_ptr<WatchStream> s_;
};

// typed/tensorflow/<version>/tfjob.go: TFJobInterface scoped to one namespace
class TFJobInterface {
 public:
  TFJobInterface(std::shared_ptr<Client> c, std::string ns, std::string api_version)
      : c_(std::move(c)), ns_(std::move(ns)), api_version_(std::move(api_version)) {}
  ApiStatus Create(const api::TFJob& job, api::TFJob* out = nullptr);
  ApiStatus Get(const std::string& name, api::TFJob* out);
  ApiStatus List(const std::string& label_selector, std::vector<api::TFJob>* out, int64_t* resource_version = nullptr);
  ApiStatus Update(const api::TFJob& job, api::TFJob* out = nullptr);        // spec + metadata
  ApiStatus UpdateStatus(const api::TFJob& job, api::TFJob* out = nullptr);  // /status subresource
  ApiStatus Patch(const std::string& name, const Json& merge_patch, api::TFJob* out = nullptr);
  ApiStatus Delete(const std::string& name, const std::string& propagation = "Background");
  ApiStatus DeleteCollection(const std::string& label_selector, int* deleted = nullptr);
  std::unique_ptr<TFJobWatch> Watch(int64_t resource_version, const std::string& label_selector, ApiStatus* st);
  const std::string& api_version() const { return api_version_; }

 private:
  Json wire(const api::TFJob& job) const;  // hub -> this client's group-version
  ApiStatus decode(const ApiStatus& st, const Json& obj, api::TFJob* out) const;
  std::shared_ptr<Client> c_;
  std::string ns_, api_version_;
};

// typed/tensorflow/<version>/tensorflow_client.go: the group client
class TensorflowClient {
 public:
  TensorflowClient(std::shared_ptr<Client> c, std::string api_version)
      : c_(std::move(c)), api_version_(std::move(api_version)) {}
  TFJobInterface TFJobs(const std::string& ns) const { return TFJobInterface(c_, ns, api_version_); }
  Client& RESTClient() const { return *c_; }

 private:
  std::shared_ptr<Client> c_;
  std::string api_version_;
};

// versioned/clientset.go
class Clientset {
 public:
  // REST backends per served TFJob version (token bucket applied per client, as NewForConfig does)
  static std::shared_ptr<Clientset> NewForConfig(const RestConfig& cfg);
  // Over an existing client (e.g. FakeClient): both versions share it.
  static std::shared_ptr<Clientset> ForClient(std::shared_ptr<Client> c);
  TensorflowClient* TensorflowV1() { return v1_.get(); }
  TensorflowClient* TensorflowV1alpha1() { return v1alpha1_.get(); }
  std::shared_ptr<Client> Core() { return core_; }  // pods, services, events, leases

 private:
  std::shared_ptr<Client> core_;
  std::unique_ptr<TensorflowClient> v1_, v1alpha1_;
};

}  // namespace tfk
