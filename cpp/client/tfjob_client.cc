#include "tfjob_client.h"

namespace tfk {

bool TFJobWatch::next(TFJobEvent* ev, int64_t timeout_ms) {
  if (!s_) return false;
  WatchEvent w;
  if (!s_->next(&w, timeout_ms)) return false;
  ev->type = w.type;
  ev->raw = w.object;
  if (w.type != "ERROR") {
    try {
      ev->job = api::from_json(w.object);
    } catch (const std::exception&) {
      ev->type = "ERROR";
    }
  }
  return true;
}

Json TFJobInterface::wire(const api::TFJob& job) const {
  Json j = api::to_json(job);
  if (j.at("apiVersion").str() != api_version_) j = api::convert(j, api_version_);
  if (!j.path("metadata.namespace").is_string() && !ns_.empty()) j["metadata"]["namespace"] = ns_;
  return j;
}

ApiStatus TFJobInterface::decode(const ApiStatus& st, const Json& obj, api::TFJob* out) const {
  if (!st.ok() || !out) return st;
  try {
    *out = api::from_json(obj);
  } catch (const std::exception& e) {
    return ApiStatus::Err(500, "InternalError", std::string("undecodable TFJob: ") + e.what());
  }
  return st;
}

ApiStatus TFJobInterface::Create(const api::TFJob& job, api::TFJob* out) {
  Json o;
  return decode(c_->create(api::kPlural, ns_, wire(job), &o), o, out);
}

ApiStatus TFJobInterface::Get(const std::string& name, api::TFJob* out) {
  Json o;
  return decode(c_->get(api::kPlural, ns_, name, &o), o, out);
}

ApiStatus TFJobInterface::List(const std::string& ls, std::vector<api::TFJob>* out, int64_t* rv) {
  ListResult lr;
  ApiStatus st = c_->list(api::kPlural, ns_, ls, "", &lr);
  if (!st.ok()) return st;
  out->clear();
  for (auto& it : lr.items) {
    try {
      out->push_back(api::from_json(it));
    } catch (const std::exception& e) {
      return ApiStatus::Err(500, "InternalError", std::string("undecodable TFJob in list: ") + e.what());
    }
  }
  if (rv) *rv = lr.resource_version;
  return st;
}

ApiStatus TFJobInterface::Update(const api::TFJob& job, api::TFJob* out) {
  Json o;
  return decode(c_->update(api::kPlural, ns_, wire(job), &o), o, out);
}

ApiStatus TFJobInterface::UpdateStatus(const api::TFJob& job, api::TFJob* out) {
  Json o;
  return decode(c_->update_status(api::kPlural, ns_, wire(job), &o), o, out);
}

ApiStatus TFJobInterface::Patch(const std::string& name, const Json& patch, api::TFJob* out) {
  Json o;
  return decode(c_->patch(api::kPlural, ns_, name, patch, &o), o, out);
}

ApiStatus TFJobInterface::Delete(const std::string& name, const std::string& propagation) {
  return c_->remove(api::kPlural, ns_, name, propagation);
}

ApiStatus TFJobInterface::DeleteCollection(const std::string& ls, int* deleted) {
  ListResult lr;
  ApiStatus st = c_->list(api::kPlural, ns_, ls, "", &lr);
  if (!st.ok()) return st;
  int n = 0;
  for (auto& it : lr.items) {
    ApiStatus d = c_->remove(api::kPlural, it.path("metadata.namespace").str(ns_), it.path("metadata.name").str(),
                             "Background");
    if (d.ok()) ++n;
    else if (d.code != 404) st = d;
  }
  if (deleted) *deleted = n;
  return st;
}

std::unique_ptr<TFJobWatch> TFJobInterface::Watch(int64_t rv, const std::string& ls, ApiStatus* st) {
  auto w = c_->watch(api::kPlural, ns_, rv, ls, "", st);
  if (!w) return nullptr;
  return std::unique_ptr<TFJobWatch>(new TFJobWatch(std::move(w)));
}

std::shared_ptr<Clientset> Clientset::NewForConfig(const RestConfig& cfg) {
  auto cs = std::make_shared<Clientset>();
  RestConfig v1 = cfg, v1a = cfg;
  v1.tfjob_version = "v1";
  v1a.tfjob_version = "v1alpha1";
  cs->core_ = std::make_shared<RestClient>(v1);
  cs->v1_.reset(new TensorflowClient(cs->core_, std::string(api::kGroupV1) + "/v1"));
  cs->v1alpha1_.reset(new TensorflowClient(std::make_shared<RestClient>(v1a), std::string(api::kGroupV1) + "/v1alpha1"));
  return cs;
}

std::shared_ptr<Clientset> Clientset::ForClient(std::shared_ptr<Client> c) {
  auto cs = std::make_shared<Clientset>();
  cs->core_ = c;
  cs->v1_.reset(new TensorflowClient(c, std::string(api::kGroupV1) + "/v1"));
  cs->v1alpha1_.reset(new TensorflowClient(c, std::string(api::kGroupV1) + "/v1alpha1"));
  return cs;
}

}  // namespace tfk
