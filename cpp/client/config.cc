#include "config.h"

#include <cstdlib>
#include <fstream>
#include <sstream>

#include "../common/yaml.h"

namespace tfk {

static bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

static std::string dir_of(const std::string& path) {
  size_t s = path.rfind('/');
  return s == std::string::npos ? "." : path.substr(0, s);
}

static std::string resolve(const std::string& base, const std::string& p) {
  if (p.empty() || p[0] == '/' || base.empty()) return p;
  return base + "/" + p;
}

std::string base64_decode(const std::string& in) {
  static int T[256];
  static bool init = false;
  if (!init) {
    for (int& t : T) t = -1;
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) T[(unsigned char)a[i]] = i;
    T[(unsigned char)'-'] = 62;  // url-safe alphabet too
    T[(unsigned char)'_'] = 63;
    init = true;
  }
  std::string out;
  int val = 0, bits = -8;
  for (unsigned char c : in) {
    if (T[c] < 0) continue;  // skips '=', whitespace, newlines
    val = (val << 6) + T[c];
    bits += 6;
    if (bits >= 0) {
      out.push_back((char)((val >> bits) & 0xFF));
      bits -= 8;
    }
  }
  return out;
}

std::string base64_encode(const std::string& in) {
  const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  int val = 0, bits = -6;
  for (unsigned char c : in) {
    val = (val << 8) + c;
    bits += 8;
    while (bits >= 0) {
      out.push_back(a[(val >> bits) & 0x3F]);
      bits -= 6;
    }
  }
  if (bits > -6) out.push_back(a[((val << 8) >> (bits + 8)) & 0x3F]);
  while (out.size() % 4) out.push_back('=');
  return out;
}

static const Json* find_named(const Json& list, const std::string& name) {
  if (!list.is_array()) return nullptr;
  for (auto& e : list.items())
    if (e.at("name").str() == name) return &e;
  return nullptr;
}

bool load_kubeconfig_text(const std::string& text, const std::string& base_dir, const std::string& context,
                          RestConfig* rc, std::string* err) {
  Json k;
  try {
    size_t i = text.find_first_not_of(" \t\r\n");
    k = (i != std::string::npos && text[i] == '{') ? Json::parse(text) : yaml_parse(text);
  } catch (const std::exception& e) {
    *err = std::string("kubeconfig: ") + e.what();
    return false;
  }
  if (!k.is_object()) { *err = "kubeconfig: not a mapping"; return false; }
  if (!k.has("clusters") && k.has("server")) {
    // legacy tfk shorthand {"server": url, "qps": .., "burst": ..}
    rc->host = k.at("server").str();
    if (k.has("qps")) rc->qps = k.at("qps").as_double();
    if (k.has("burst")) rc->burst = (int)k.at("burst").as_int();
    return true;
  }
  std::string ctx_name = context.empty() ? k.at("current-context").str() : context;
  const Json* ctx = find_named(k.at("contexts"), ctx_name);
  if (!ctx) {
    // a kubeconfig with one cluster and no contexts is still usable
    if (k.at("clusters").size() == 1 && ctx_name.empty()) {
      static Json empty = Json::object();
      ctx = &empty;
    } else {
      *err = "kubeconfig: context \"" + ctx_name + "\" not found";
      return false;
    }
  }
  const Json& c = ctx->at("context");
  std::string cluster_name = c.at("cluster").str(), user_name = c.at("user").str();
  const Json* cl = cluster_name.empty() && k.at("clusters").size() == 1 ? &k.at("clusters")[0]
                                                                          : find_named(k.at("clusters"), cluster_name);
  if (!cl) { *err = "kubeconfig: cluster \"" + cluster_name + "\" not found"; return false; }
  const Json& cd = cl->at("cluster");
  rc->host = cd.at("server").str();
  if (rc->host.empty()) { *err = "kubeconfig: cluster has no server"; return false; }
  rc->tls.enabled = starts_with(rc->host, "https://");
  rc->tls.insecure_skip_verify = cd.at("insecure-skip-tls-verify").as_bool(false);
  rc->tls.server_name = cd.at("tls-server-name").str();
  if (cd.has("certificate-authority-data")) rc->tls.ca_data = base64_decode(cd.at("certificate-authority-data").str());
  else if (cd.has("certificate-authority")) rc->tls.ca_file = resolve(base_dir, cd.at("certificate-authority").str());
  rc->ns = c.at("namespace").str();
  if (!user_name.empty()) {
    const Json* u = find_named(k.at("users"), user_name);
    if (!u) { *err = "kubeconfig: user \"" + user_name + "\" not found"; return false; }
    const Json& ud = u->at("user");
    if (ud.has("exec") || ud.has("auth-provider")) {
      *err = "kubeconfig: user \"" + user_name + "\" uses an exec/auth-provider plugin (not supported; use a token)";
      return false;
    }
    rc->bearer_token = ud.at("token").str();
    if (ud.has("tokenFile")) rc->bearer_token_file = resolve(base_dir, ud.at("tokenFile").str());
    rc->username = ud.at("username").str();
    rc->password = ud.at("password").str();
    if (ud.has("client-certificate-data")) rc->tls.cert_data = base64_decode(ud.at("client-certificate-data").str());
    else if (ud.has("client-certificate")) rc->tls.cert_file = resolve(base_dir, ud.at("client-certificate").str());
    if (ud.has("client-key-data")) rc->tls.key_data = base64_decode(ud.at("client-key-data").str());
    else if (ud.has("client-key")) rc->tls.key_file = resolve(base_dir, ud.at("client-key").str());
  }
  return true;
}

bool load_kubeconfig(const std::string& path, const std::string& context, RestConfig* rc, std::string* err) {
  std::string text;
  if (!read_file(path, &text)) { *err = "kubeconfig: cannot read " + path; return false; }
  return load_kubeconfig_text(text, dir_of(path), context, rc, err);
}

bool in_cluster_config(RestConfig* rc, std::string* err, const std::string& sa_dir) {
  const char* h = getenv("KUBERNETES_SERVICE_HOST");
  const char* p = getenv("KUBERNETES_SERVICE_PORT");
  if (!h || !*h || !p || !*p) {
    *err = "unable to load in-cluster configuration, KUBERNETES_SERVICE_HOST and KUBERNETES_SERVICE_PORT must be defined";
    return false;
  }
  std::string host = h;
  if (host.find(':') != std::string::npos) host = "[" + host + "]";  // IPv6 service IP
  rc->host = "https://" + host + ":" + p;
  std::string tok;
  if (!read_file(sa_dir + "/token", &tok)) { *err = "in-cluster: cannot read " + sa_dir + "/token"; return false; }
  rc->bearer_token = trim(tok);
  rc->bearer_token_file = sa_dir + "/token";
  rc->tls.enabled = true;
  rc->tls.ca_file = sa_dir + "/ca.crt";
  std::string ns;
  if (read_file(sa_dir + "/namespace", &ns)) rc->ns = trim(ns);
  return true;
}

bool build_config_from_flags(const std::string& master, const std::string& kubeconfig, RestConfig* rc,
                             std::string* err) {
  if (!kubeconfig.empty()) {
    if (!load_kubeconfig(kubeconfig, "", rc, err)) return false;
    if (!master.empty()) {
      rc->host = master;
      rc->tls.enabled = starts_with(master, "https://");
    }
    return true;
  }
  if (!master.empty()) {
    rc->host = master;
    rc->tls.enabled = starts_with(master, "https://");
    return true;
  }
  return in_cluster_config(rc, err);
}

}  // namespace tfk
