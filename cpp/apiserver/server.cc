#include "server.h"

#include <fstream>
#include <sstream>

#include "../api/types.h"

namespace tfk {

void install_tfjob_crd(Store& store) {
  Json crd = api::crd_manifest();
  Json out;
  store.create("customresourcedefinitions", "", crd, &out);  // 409 if present: fine
  ResourceInfo ri;
  ri.group = api::kGroupV1;
  ri.version = "v1";
  ri.plural = api::kPlural;
  ri.singular = api::kSingular;
  ri.kind = api::kKind;
  ri.namespaced = true;
  ri.versions = {"v1", "v1alpha1"};
  ri.short_names = {api::kShortName};
  store.register_resource(ri);
  store.set_converter(api::kPlural, [](const Json& obj, const std::string& v) { return api::convert(obj, v); });
}

bool ApiServer::start(const std::string& host, int port, std::string* err) {
  if (!http_.listen(host, port, err)) return false;
  http_.serve([this](const HttpRequest& r, ResponseWriter& w) { handle(r, w); });
  return true;
}

bool ApiServer::load_token_file(const std::string& path, std::string* err) {
  std::ifstream f(path);
  if (!f) { *err = "cannot read token file " + path; return false; }
  std::string line;
  size_t n0 = tokens_.size();
  while (std::getline(f, line)) {
    line = trim(line);
    if (line.empty() || line[0] == '#') continue;
    auto cols = split(line, ',');
    if (cols.size() < 2) { *err = "token file " + path + ": want token,user,uid"; return false; }
    tokens_[trim(cols[0])] = trim(cols[1]);
  }
  if (tokens_.size() == n0) { *err = "token file " + path + " has no tokens"; return false; }
  return true;
}

static void reply(ResponseWriter& w, const ApiStatus& st, const Json& body) {
  w.respond(st.code, st.ok() ? body.dump() : st.to_json().dump());
}

void ApiServer::handle(const HttpRequest& req, ResponseWriter& w) {
  const std::string& p = req.path;
  if (p == "/healthz" || p == "/readyz" || p == "/livez") { w.respond(200, "ok", "text/plain"); return; }
  if (!tokens_.empty()) {
    auto it = req.headers.find("authorization");
    std::string tok = it == req.headers.end() ? "" : it->second;
    if (!starts_with(tok, "Bearer ") || !tokens_.count(trim(tok.substr(7)))) {
      w.respond(401, ApiStatus::Err(401, "Unauthorized", "Unauthorized").to_json().dump());
      return;
    }
  }
  if (p == "/version") {
    w.respond(200, R"({"major":"1","minor":"9","gitVersion":"v1.9.0-tfk","platform":"linux/amd64"})");
    return;
  }
  if (p == "/metrics") {
    std::ostringstream os;
    os << "# TYPE apiserver_resource_version gauge\napiserver_resource_version " << store_->resource_version() << "\n";
    os << "# TYPE apiserver_request_total counter\n";
    for (auto& kv : store_->counters()) os << "apiserver_request_total{op=\"" << kv.first << "\"} " << kv.second << "\n";
    os << "# TYPE apiserver_objects gauge\n";
    for (auto& ri : store_->resources()) os << "apiserver_objects{resource=\"" << ri.plural << "\"} " << store_->count(ri.plural) << "\n";
    w.respond(200, os.str(), "text/plain; version=0.0.4");
    return;
  }
  if (p == "/apis" || p == "/api") {
    Json j = Json::object();
    j["kind"] = "APIGroupList";
    for (auto& ri : store_->resources()) {
      Json g = Json::object();
      g["name"] = ri.group.empty() ? "core" : ri.group;
      g["resource"] = ri.plural;
      g["kind"] = ri.kind;
      Json vs = Json::array();
      for (auto& v : ri.versions) vs.push_back(v);
      g["versions"] = vs;
      j["groups"].push_back(g);
    }
    w.respond(200, j.dump());
    return;
  }
  auto seg = split(p, '/');
  std::vector<std::string> s;
  for (auto& x : seg)
    if (!x.empty()) s.push_back(x);
  // normalise to: group, version, ns, plural, name, sub
  std::string group, version, ns, plural, name, sub;
  size_t i = 0;
  if (s.size() >= 2 && s[0] == "api") { group = ""; version = s[1]; i = 2; }
  else if (s.size() >= 3 && s[0] == "apis") { group = s[1]; version = s[2]; i = 3; }
  else { w.respond(404, ApiStatus::Err(404, "NotFound", "no route " + p).to_json().dump()); return; }
  if (i < s.size() && s[i] == "namespaces") {
    if (s.size() == i + 1) { plural = "namespaces"; i = s.size(); }
    else if (s.size() == i + 2) { plural = "namespaces"; name = s[i + 1]; i = s.size(); }
    else { ns = s[i + 1]; i += 2; }
  }
  if (plural.empty()) {
    if (i >= s.size()) { w.respond(404, ApiStatus::Err(404, "NotFound", "no resource").to_json().dump()); return; }
    plural = s[i++];
    if (i < s.size()) name = s[i++];
    if (i < s.size()) sub = s[i++];
  }
  ResourceInfo ri;
  if (!store_->resource(plural, &ri)) {
    w.respond(404, ApiStatus::Err(404, "NotFound", "the server could not find the requested resource " + plural).to_json().dump());
    return;
  }
  plural = ri.plural;
  if (ri.group != group) {
    w.respond(404, ApiStatus::Err(404, "NotFound", "resource " + plural + " is not in group " + group).to_json().dump());
    return;
  }
  bool served = false;
  for (auto& v : ri.versions) served |= (v == version);
  if (!served && ri.version != version) {
    w.respond(404, ApiStatus::Err(404, "NotFound", "version " + version + " not served for " + plural).to_json().dump());
    return;
  }
  std::string api_version = group.empty() ? version : group + "/" + version;
  auto q = [&](const char* k) {
    auto it = req.query.find(k);
    return it == req.query.end() ? std::string() : it->second;
  };
  std::string err;
  LabelSelector ls = LabelSelector::parse(q("labelSelector"), &err);
  FieldSelector fs = FieldSelector::parse(q("fieldSelector"));
  const std::string& m = req.method;

  if (name.empty()) {
    if (m == "GET") {
      if (q("watch") == "1" || q("watch") == "true") { do_watch(req, w, plural, ns, api_version); return; }
      std::vector<Json> items;
      int64_t rv = 0;
      ApiStatus st = store_->list(plural, ns, ls, fs, &items, &rv);
      if (!st.ok()) { reply(w, st, Json()); return; }
      Json out = Json::object();
      out["kind"] = ri.kind + "List";
      out["apiVersion"] = api_version;
      out["metadata"]["resourceVersion"] = std::to_string(rv);
      Json arr = Json::array();
      for (auto& it : items) arr.push_back(store_->convert_for(plural, it, plural == api::kPlural ? api_version : ""));
      out["items"] = arr;
      w.respond(200, out.dump());
      return;
    }
    if (m == "POST") {
      Json body;
      try { body = Json::parse(req.body); } catch (const std::exception& e) {
        reply(w, ApiStatus::Err(400, "BadRequest", e.what()), Json()); return;
      }
      if (plural == api::kPlural) {
        // admission: validate TFJob shape before storing
        try { api::from_json(body); } catch (const std::exception& e) {
          reply(w, ApiStatus::Err(422, "Invalid", e.what()), Json()); return;
        }
      }
      Json out;
      ApiStatus st = store_->create(plural, ns, body, &out);
      reply(w, st, store_->convert_for(plural, out, plural == api::kPlural ? api_version : ""));
      return;
    }
    if (m == "DELETE") {  // deletecollection
      std::vector<Json> items;
      store_->list(plural, ns, ls, fs, &items, nullptr);
      for (auto& it : items)
        store_->remove(plural, it.path("metadata.namespace").str(), it.path("metadata.name").str(), "Background", nullptr);
      w.respond(200, ApiStatus::Ok().to_json().dump());
      return;
    }
    w.respond(405, ApiStatus::Err(405, "MethodNotAllowed", m).to_json().dump());
    return;
  }

  if (sub == "log" && plural == "pods" && m == "GET") {
    Json pod;
    ApiStatus st = store_->get(plural, ns, name, &pod);
    if (!st.ok()) { reply(w, st, Json()); return; }
    std::string path = pod.path("metadata.annotations").at("tfk.io/log-path").str();
    std::ifstream f(path);
    if (!f) { w.respond(404, ApiStatus::Err(404, "NotFound", "no log for pod " + name).to_json().dump()); return; }
    std::stringstream ss;
    ss << f.rdbuf();
    std::string data = ss.str();
    std::string tail = q("tailLines");
    if (!tail.empty()) {
      int n = atoi(tail.c_str());
      size_t pos = data.size();
      for (int k = 0; k <= n && pos != std::string::npos && pos > 0; ++k) pos = data.rfind('\n', pos - 1);
      if (pos != std::string::npos && pos < data.size()) data = data.substr(pos + 1);
    }
    w.respond(200, data, "text/plain");
    return;
  }
  bool status_only = (sub == "status");
  if (!sub.empty() && !status_only) { w.respond(404, ApiStatus::Err(404, "NotFound", "subresource " + sub).to_json().dump()); return; }
  Json out;
  if (m == "GET") {
    ApiStatus st = store_->get(plural, ns, name, &out);
    reply(w, st, store_->convert_for(plural, out, plural == api::kPlural ? api_version : ""));
    return;
  }
  if (m == "PUT" || m == "PATCH") {
    Json body;
    try { body = Json::parse(req.body); } catch (const std::exception& e) {
      reply(w, ApiStatus::Err(400, "BadRequest", e.what()), Json()); return;
    }
    if (plural == api::kPlural && body.has("apiVersion")) {
      // store in the stored object's version
      Json cur;
      if (store_->get(plural, ns, name, &cur).ok() && cur.at("apiVersion").str() != body.at("apiVersion").str() && m == "PUT") {
        std::string rvv = body.path("metadata.resourceVersion").str();
        try { body = api::convert(body, cur.at("apiVersion").str()); } catch (...) {}
        if (!rvv.empty()) body["metadata"]["resourceVersion"] = rvv;
      }
    }
    ApiStatus st = m == "PUT" ? store_->update(plural, ns, name, body, status_only, &out)
                              : store_->patch(plural, ns, name, body, status_only, &out);
    reply(w, st, store_->convert_for(plural, out, plural == api::kPlural ? api_version : ""));
    return;
  }
  if (m == "DELETE") {
    std::string prop = q("propagationPolicy");
    if (!req.body.empty()) {
      try {
        Json b = Json::parse(req.body);
        if (b.has("propagationPolicy")) prop = b.at("propagationPolicy").str();
      } catch (...) {
      }
    }
    ApiStatus st = store_->remove(plural, ns, name, prop.empty() ? "Background" : prop, &out);
    reply(w, st, out);
    return;
  }
  w.respond(405, ApiStatus::Err(405, "MethodNotAllowed", m).to_json().dump());
}

void ApiServer::do_watch(const HttpRequest& req, ResponseWriter& w, const std::string& plural, const std::string& ns,
                         const std::string& api_version) {
  auto q = [&](const char* k) {
    auto it = req.query.find(k);
    return it == req.query.end() ? std::string() : it->second;
  };
  int64_t rv = q("resourceVersion").empty() ? 0 : std::stoll(q("resourceVersion"));
  int64_t timeout_s = q("timeoutSeconds").empty() ? 1800 : std::stoll(q("timeoutSeconds"));
  ApiStatus st;
  auto watcher = store_->watch(plural, ns, rv, LabelSelector::parse(q("labelSelector")),
                               FieldSelector::parse(q("fieldSelector")), &st,
                               plural == api::kPlural ? api_version : "");
  if (!watcher) {
    // Kubernetes sends 410 as an ERROR event inside a 200 stream; do the same.
    if (!w.start_stream(200)) return;
    Json ev = Json::object();
    ev["type"] = "ERROR";
    ev["object"] = st.to_json();
    w.write_chunk(ev.dump() + "\n");
    w.end_stream();
    return;
  }
  if (!w.start_stream(200)) { watcher->close(); return; }
  int64_t deadline = mono_ms() + timeout_s * 1000;
  int64_t last_write = mono_ms();
  while (mono_ms() < deadline && w.alive()) {
    WatchEvent ev;
    if (watcher->next(&ev, 500)) {
      Json j = Json::object();
      j["type"] = ev.type;
      j["object"] = plural == api::kPlural ? store_->convert_for(plural, ev.object, api_version) : ev.object;
      if (!w.write_chunk(j.dump() + "\n")) break;
      last_write = mono_ms();
    } else if (watcher->closed()) {
      break;
    } else if (mono_ms() - last_write > 5000) {
      // heartbeat bookmark keeps dead peers detectable
      Json j = Json::object();
      j["type"] = "BOOKMARK";
      j["object"]["metadata"]["resourceVersion"] = std::to_string(store_->resource_version() - 1);
      if (!w.write_chunk(j.dump() + "\n")) break;
      last_write = mono_ms();
    }
  }
  watcher->close();
  w.end_stream();
}

}  // namespace tfk
