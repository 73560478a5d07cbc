// Client-layer tests (reference: NewForConfig + token bucket images/tf4.PNG,
// TensorflowV1alpha1Client.NewForConfig images/tf5.PNG, BuildConfigFromFlags k8s-operator.md:92-101):
// YAML subset parser, kubeconfig / in-cluster config, HTTPS + bearer-token auth against a local
// tfk-apiserver with a throw-away self-signed certificate, keep-alive reuse, typed TFJob client.
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>
#include <openssl/x509v3.h>
#include <stdlib.h>
#include <unistd.h>

#include <cstdio>
#include <fstream>
#include <string>

#include "../api/types.h"
#include "../apiserver/server.h"
#include "../client/config.h"
#include "../client/tfjob_client.h"
#include "../common/yaml.h"
#include "testing.h"

using namespace tfk;

namespace {

Json J(const std::string& s) { return Json::parse(s); }

std::string tmpdir() {
  char tmpl[] = "/tmp/tfk-ct-XXXXXX";
  return mkdtemp(tmpl);
}

void write_file(const std::string& p, const std::string& s) {
  std::ofstream f(p, std::ios::binary);
  f << s;
}

// Self-signed CA-less server certificate for 127.0.0.1 / localhost, written as PEM files.
void make_cert(const std::string& dir, const std::string& cn = "tfk-apiserver") {
  EVP_PKEY* key = EVP_RSA_gen(2048);
  X509* x = X509_new();
  X509_set_version(x, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(x), 1);
  X509_gmtime_adj(X509_getm_notBefore(x), -60);
  X509_gmtime_adj(X509_getm_notAfter(x), 3600);
  X509_set_pubkey(x, key);
  X509_NAME* name = X509_get_subject_name(x);
  X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, (const unsigned char*)cn.c_str(), -1, -1, 0);
  X509_set_issuer_name(x, name);
  X509V3_CTX ctx;
  X509V3_set_ctx_nodb(&ctx);
  X509V3_set_ctx(&ctx, x, x, nullptr, nullptr, 0);
  X509_EXTENSION* ext = X509V3_EXT_conf_nid(nullptr, &ctx, NID_subject_alt_name, "IP:127.0.0.1,DNS:localhost");
  X509_add_ext(x, ext, -1);
  X509_EXTENSION_free(ext);
  ext = X509V3_EXT_conf_nid(nullptr, &ctx, NID_basic_constraints, "critical,CA:TRUE");
  X509_add_ext(x, ext, -1);
  X509_EXTENSION_free(ext);
  X509_sign(x, key, EVP_sha256());
  FILE* f = fopen((dir + "/tls.crt").c_str(), "w");
  PEM_write_X509(f, x);
  fclose(f);
  f = fopen((dir + "/tls.key").c_str(), "w");
  PEM_write_PrivateKey(f, key, nullptr, nullptr, 0, nullptr, nullptr);
  fclose(f);
  X509_free(x);
  EVP_PKEY_free(key);
}

std::string slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  return std::string(std::istreambuf_iterator<char>(f), {});
}

Json tiny_job(const std::string& name) {
  return J(R"({"apiVersion":"kubeflow.org/v1","kind":"TFJob","metadata":{"name":")" + name +
           R"(","namespace":"default","labels":{"team":"a"}},"spec":{"tfReplicaSpecs":{"Worker":{"replicas":1,
           "template":{"spec":{"containers":[{"name":"tensorflow","image":"x"}]}}}}}})");
}

struct TlsServer {
  std::string dir;
  std::shared_ptr<Store> store = std::make_shared<Store>();
  std::unique_ptr<ApiServer> srv;
  TlsServer(bool tls, const std::string& token) {
    dir = tmpdir();
    install_tfjob_crd(*store);
    srv.reset(new ApiServer(store));
    std::string err;
    if (tls) {
      make_cert(dir);
      TlsOptions o;
      o.enabled = true;
      o.cert_file = dir + "/tls.crt";
      o.key_file = dir + "/tls.key";
      CHECK(srv->enable_tls(o, &err));
    }
    if (!token.empty()) srv->add_token(token, "operator");
    CHECK(srv->start("127.0.0.1", 0, &err));
  }
  ~TlsServer() {
    srv->stop();
    std::string cmd = "rm -rf " + dir;
    if (system(cmd.c_str()) != 0) perror("rm");
  }
  std::string url() const { return std::string(srv->tls() ? "https" : "http") + "://127.0.0.1:" + std::to_string(srv->port()); }
};

}  // namespace

// ----------------------------------------------------------------------------------- YAML
TEST(yaml_block_mappings_sequences_scalars) {
  Json j = yaml_parse(R"(---
# comment
apiVersion: v1
kind: Config
n: 42
f: 0.5
flag: true
none: ~
quoted: "a: b # not a comment\n"
single: 'it''s'
list:
- a
- b: 1
  c: [x, "y z", 3]
- - nested
nested:
  deeper:
    k: v   # trailing
  flow: {a: 1, b: two}
empty: []
lit: |
  line1
    indented
  line3
folded: >-
  one
  two
)");
  CHECK_EQ(j.at("kind").str(), std::string("Config"));
  CHECK_EQ(j.at("n").as_int(), 42LL);
  CHECK(j.at("f").as_double() == 0.5);
  CHECK(j.at("flag").as_bool());
  CHECK(j.at("none").is_null());
  CHECK_EQ(j.at("quoted").str(), std::string("a: b # not a comment\n"));
  CHECK_EQ(j.at("single").str(), std::string("it's"));
  CHECK_EQ(j.at("list").size(), (size_t)3);
  CHECK_EQ(j.at("list")[0].str(), std::string("a"));
  CHECK_EQ(j.at("list")[1].at("b").as_int(), 1LL);
  CHECK_EQ(j.at("list")[1].at("c")[1].str(), std::string("y z"));
  CHECK_EQ(j.at("list")[2][0].str(), std::string("nested"));
  CHECK_EQ(j.path("nested.deeper.k").str(), std::string("v"));
  CHECK_EQ(j.path("nested.flow.b").str(), std::string("two"));
  CHECK(j.at("empty").is_array() && j.at("empty").size() == 0);
  CHECK_EQ(j.at("lit").str(), std::string("line1\n  indented\nline3\n"));
  CHECK_EQ(j.at("folded").str(), std::string("one two"));
}

TEST(yaml_rejects_anchors_and_reports_lines) {
  bool threw = false;
  try {
    yaml_parse("a: &x 1\nb: *x\n");
  } catch (const std::runtime_error& e) {
    threw = std::string(e.what()).find("line 1") != std::string::npos;
  }
  CHECK(threw);
  auto docs = yaml_parse_all("a: 1\n---\nb: 2\n---\n");
  CHECK_EQ(docs.size(), (size_t)2);
  CHECK_EQ(docs[1].at("b").as_int(), 2LL);
}

TEST(yaml_parses_deploy_manifests) {
  // every manifest shipped under deploy/ parses (multi-document files included)
  // repo root = two levels above build/bin/<this binary>
  char exe[4096] = {0};
  CHECK(readlink("/proc/self/exe", exe, sizeof exe - 1) > 0);
  std::string root = exe;
  for (int up = 0; up < 3; ++up) root = root.substr(0, root.rfind('/'));
  for (const char* f : {"crd-tfjob-v1.yaml", "operator.yaml", "crd-tfjob.yaml"}) {
    std::string text = slurp(root + "/deploy/" + f);
    CHECK(!text.empty());
    auto docs = yaml_parse_all(text);
    CHECK(!docs.empty());
    for (auto& d : docs) CHECK(d.has("apiVersion") && d.has("kind"));
  }
}

// ----------------------------------------------------------------------------- kubeconfig
TEST(kubeconfig_contexts_users_and_paths) {
  std::string ca = "-----BEGIN CERTIFICATE-----\nMIIB\n-----END CERTIFICATE-----\n";
  std::string text = R"(apiVersion: v1
kind: Config
current-context: prod
clusters:
- name: dev
  cluster:
    server: http://127.0.0.1:8080
- name: prod
  cluster:
    server: https://10.0.0.1:6443
    certificate-authority-data: )" + base64_encode(ca) + R"(
    tls-server-name: kubernetes
contexts:
- name: dev
  context: {cluster: dev, user: dev-user}
- name: prod
  context:
    cluster: prod
    user: sa
    namespace: kubeflow
users:
- name: dev-user
  user:
    client-certificate: certs/dev.crt
    client-key: /abs/dev.key
- name: sa
  user:
    tokenFile: sa.token
    token: abc.def
)";
  RestConfig rc;
  std::string err;
  CHECK(load_kubeconfig_text(text, "/etc/kube", "", &rc, &err));
  CHECK_EQ(rc.host, std::string("https://10.0.0.1:6443"));
  CHECK_EQ(rc.tls.ca_data, ca);
  CHECK_EQ(rc.tls.server_name, std::string("kubernetes"));
  CHECK_EQ(rc.bearer_token, std::string("abc.def"));
  CHECK_EQ(rc.bearer_token_file, std::string("/etc/kube/sa.token"));
  CHECK_EQ(rc.ns, std::string("kubeflow"));
  RestConfig dev;
  CHECK(load_kubeconfig_text(text, "/etc/kube", "dev", &dev, &err));
  CHECK_EQ(dev.host, std::string("http://127.0.0.1:8080"));
  CHECK_EQ(dev.tls.cert_file, std::string("/etc/kube/certs/dev.crt"));
  CHECK_EQ(dev.tls.key_file, std::string("/abs/dev.key"));
  RestConfig bad;
  CHECK(!load_kubeconfig_text(text, "/", "nope", &bad, &err));
  CHECK(err.find("nope") != std::string::npos);
  std::string exec = "current-context: c\nclusters:\n- name: k\n  cluster: {server: https://h:1}\ncontexts:\n- name: c\n"
                     "  context: {cluster: k, user: u}\nusers:\n- name: u\n  user:\n    exec:\n      command: aws\n";
  CHECK(!load_kubeconfig_text(exec, "/", "", &bad, &err));
  CHECK(err.find("exec") != std::string::npos);
  // legacy tfk JSON shorthand still loads
  RestConfig legacy;
  CHECK(load_kubeconfig_text(R"({"server":"http://127.0.0.1:9","qps":7,"burst":9})", "/", "", &legacy, &err));
  CHECK_EQ(legacy.host, std::string("http://127.0.0.1:9"));
  CHECK_EQ(legacy.burst, 9);
}

TEST(in_cluster_config_reads_service_account) {
  std::string d = tmpdir();
  write_file(d + "/token", "tok-123\n");
  write_file(d + "/ca.crt", "x");
  write_file(d + "/namespace", "kubeflow");
  std::string err;
  RestConfig rc;
  unsetenv("KUBERNETES_SERVICE_HOST");
  CHECK(!in_cluster_config(&rc, &err, d));
  setenv("KUBERNETES_SERVICE_HOST", "10.96.0.1", 1);
  setenv("KUBERNETES_SERVICE_PORT", "443", 1);
  CHECK(in_cluster_config(&rc, &err, d));
  CHECK_EQ(rc.host, std::string("https://10.96.0.1:443"));
  CHECK_EQ(rc.bearer_token, std::string("tok-123"));
  CHECK_EQ(rc.tls.ca_file, d + "/ca.crt");
  CHECK_EQ(rc.ns, std::string("kubeflow"));
  unsetenv("KUBERNETES_SERVICE_HOST");
  unsetenv("KUBERNETES_SERVICE_PORT");
  CHECK(system(("rm -rf " + d).c_str()) == 0);
}

TEST(base64_roundtrip) {
  for (const std::string& s : std::vector<std::string>{"", "a", "ab", "abc", "abcd", std::string("\0\xff\x10", 3)}) CHECK_EQ(base64_decode(base64_encode(s)), s);
  CHECK_EQ(base64_encode("hello"), std::string("aGVsbG8="));
}

// ----------------------------------------------------------------------------- HTTPS + auth
TEST(https_bearer_token_and_verification) {
  TlsServer s(true, "s3cret");
  RestConfig rc;
  rc.host = s.url();
  rc.tls.ca_file = s.dir + "/tls.crt";
  rc.bearer_token = "s3cret";
  rc.qps = 0;
  RestClient c(rc);
  Json out;
  CHECK(c.create("tfjobs", "default", tiny_job("a"), &out).ok());
  CHECK(c.get("tfjobs", "default", "a", &out).ok());
  CHECK_EQ(out.path("metadata.name").str(), std::string("a"));
  // wrong token -> 401 Unauthorized
  RestConfig bad = rc;
  bad.bearer_token = "nope";
  ApiStatus st = RestClient(bad).get("tfjobs", "default", "a", &out);
  CHECK_EQ(st.code, 401);
  // token from a file (service-account style)
  write_file(s.dir + "/tok", "s3cret\n");
  RestConfig tf = rc;
  tf.bearer_token.clear();
  tf.bearer_token_file = s.dir + "/tok";
  CHECK(RestClient(tf).get("tfjobs", "default", "a", &out).ok());
  // the self-signed cert is not in the system store: verification fails unless trusted or skipped
  RestConfig untrusted = rc;
  untrusted.tls.ca_file.clear();
  st = RestClient(untrusted).get("tfjobs", "default", "a", &out);
  CHECK_EQ(st.code, 503);
  CHECK(st.message.find("TLS handshake") != std::string::npos);
  RestConfig insecure = untrusted;
  insecure.tls.insecure_skip_verify = true;
  CHECK(RestClient(insecure).get("tfjobs", "default", "a", &out).ok());
  // CA given inline (certificate-authority-data) works like the file
  RestConfig inl = rc;
  inl.tls.ca_file.clear();
  inl.tls.ca_data = slurp(s.dir + "/tls.crt");
  CHECK(RestClient(inl).get("tfjobs", "default", "a", &out).ok());
  // health endpoints stay unauthenticated
  Endpoint ep;
  CHECK(parse_endpoint(s.url(), &ep));
  TlsOptions o;
  o.ca_file = s.dir + "/tls.crt";
  std::string err;
  HttpClient hc(ep, TlsContext::client(o, &err), 5000);
  CHECK_EQ(hc.request("GET", "/healthz").status, 200);
}

TEST(https_watch_stream_and_kubeconfig_roundtrip) {
  TlsServer s(true, "tok");
  std::string kc = "apiVersion: v1\nkind: Config\ncurrent-context: local\nclusters:\n- name: local\n  cluster:\n"
                   "    server: " + s.url() + "\n    certificate-authority: tls.crt\ncontexts:\n- name: local\n"
                   "  context:\n    cluster: local\n    user: op\nusers:\n- name: op\n  user:\n    token: tok\n";
  write_file(s.dir + "/kubeconfig", kc);
  RestConfig rc;
  std::string err;
  CHECK(build_config_from_flags("", s.dir + "/kubeconfig", &rc, &err));
  auto cs = Clientset::NewForConfig(rc);
  auto jobs = cs->TensorflowV1()->TFJobs("default");
  ApiStatus st;
  auto w = jobs.Watch(0, "", &st);
  CHECK(st.ok() && w);
  api::TFJob created;
  CHECK(jobs.Create(api::from_json(tiny_job("w1")), &created).ok());
  TFJobEvent ev;
  bool seen = false;
  for (int i = 0; i < 50 && !seen; ++i)
    if (w->next(&ev, 100)) seen = ev.type == "ADDED" && ev.job.name() == "w1";
  CHECK(seen);
  w->close();
}

TEST(keepalive_reuses_connections) {
  TlsServer s(false, "");
  RestConfig rc;
  rc.host = s.url();
  rc.qps = 0;
  RestClient c(rc);
  Json out;
  ListResult lr;
  for (int i = 0; i < 20; ++i) CHECK(c.list("pods", "default", "", "", &lr).ok());
  CHECK(c.http().reuses() >= 19);
  CHECK(c.http().connects() <= 2);
  CHECK(s.srv->connections_accepted() <= 2);
  // with keep-alive off every request dials
  RestConfig nk = rc;
  nk.keepalive = false;
  RestClient c2(nk);
  for (int i = 0; i < 5; ++i) CHECK(c2.list("pods", "default", "", "", &lr).ok());
  CHECK_EQ(c2.http().connects(), 5LL);
}

TEST(keepalive_recovers_from_server_restart) {
  // a pooled connection whose server went away is retried on a fresh dial
  auto store = std::make_shared<Store>();
  install_tfjob_crd(*store);
  std::unique_ptr<ApiServer> a(new ApiServer(store));
  std::string err;
  CHECK(a->start("127.0.0.1", 0, &err));
  int port = a->port();
  RestConfig rc;
  rc.host = "http://127.0.0.1:" + std::to_string(port);
  rc.qps = 0;
  RestClient c(rc);
  ListResult lr;
  CHECK(c.list("pods", "default", "", "", &lr).ok());
  a->stop();
  a.reset(new ApiServer(store));
  CHECK(a->start("127.0.0.1", port, &err));
  CHECK(c.list("pods", "default", "", "", &lr).ok());
  a->stop();
}

// ----------------------------------------------------------------------------- typed client
static void exercise_typed(Clientset& cs) {
  auto v1 = cs.TensorflowV1()->TFJobs("default");
  api::TFJob j = api::from_json(tiny_job("t1")), out;
  CHECK(v1.Create(j, &out).ok());
  CHECK_EQ(out.name(), std::string("t1"));
  CHECK_EQ(v1.Create(j, &out).code, 409);
  CHECK(v1.Create(api::from_json(tiny_job("t2"))).ok());
  std::vector<api::TFJob> all;
  CHECK(v1.List("team=a", &all).ok());
  CHECK_EQ(all.size(), (size_t)2);
  CHECK(v1.Get("t1", &out).ok());
  api::set_condition(out.status, "Running", "TFJobRunning", "running", "2026-01-01T00:00:00Z");
  api::TFJob st;
  CHECK(v1.UpdateStatus(out, &st).ok());
  CHECK(api::has_condition(st.status, "Running"));
  CHECK(v1.Patch("t1", J(R"({"metadata":{"labels":{"team":"b"}}})"), &out).ok());
  CHECK_EQ(out.metadata.path("labels.team").str(), std::string("b"));
  // the v1alpha1 typed client sees the same object in its own wire shape
  api::TFJob old;
  CHECK(cs.TensorflowV1alpha1()->TFJobs("default").Get("t2", &old).ok());
  CHECK_EQ(old.name(), std::string("t2"));
  int n = 0;
  CHECK(v1.DeleteCollection("team=a", &n).ok());
  CHECK_EQ(n, 1);
  CHECK(v1.Delete("t1").ok());
  CHECK_EQ(v1.Get("t1", &out).code, 404);
}

TEST(typed_tfjob_client_over_fake) {
  auto store = std::make_shared<Store>();
  install_tfjob_crd(*store);
  auto fake = std::make_shared<FakeClient>(store);
  auto cs = Clientset::ForClient(fake);
  exercise_typed(*cs);
  bool saw_status = false;
  for (auto& a : fake->actions()) saw_status |= a == "update tfjobs/t1/status";
  CHECK(saw_status);
}

TEST(typed_tfjob_client_over_https) {
  TlsServer s(true, "tok");
  RestConfig rc;
  rc.host = s.url();
  rc.tls.ca_file = s.dir + "/tls.crt";
  rc.bearer_token = "tok";
  rc.qps = 0;
  exercise_typed(*Clientset::NewForConfig(rc));
}
