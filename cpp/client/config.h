// REST client configuration (client-go rest.Config + clientcmd), reference: the operator builds
// its config with clientcmd.BuildConfigFromFlags("", kubeconfig) (k8s-operator.md:92-101) and
// hands it to NewForConfig (images/tf4.PNG:L2, images/tf5.PNG:L2-L11).
//
//   load_kubeconfig      kubeconfig YAML/JSON: clusters / users / contexts / current-context with
//                        server, certificate-authority(-data), insecure-skip-tls-verify,
//                        tls-server-name, token, tokenFile, client-certificate(-data),
//                        client-key(-data), username/password; namespace of the context.
//   in_cluster_config    KUBERNETES_SERVICE_HOST/PORT + the pod's service-account token and CA.
//   build_config_from_flags   master URL and/or kubeconfig path, else in-cluster.
#pragma once
#include <string>

#include "../common/http.h"

namespace tfk {

constexpr const char* kServiceAccountDir = "/var/run/secrets/kubernetes.io/serviceaccount";

struct RestConfig {
  std::string host = "http://127.0.0.1:8080";
  double qps = 5;    // client-go defaults
  int burst = 10;
  std::string user_agent;
  std::string tfjob_version = "v1";  // GroupVersion for TFJobs (v1 | v1alpha1)
  int timeout_ms = 30000;
  // authentication
  std::string bearer_token;       // static token
  std::string bearer_token_file;  // re-read periodically (projected service-account tokens rotate)
  std::string username, password; // basic auth
  std::string ns;                 // namespace of the kubeconfig context / the pod (informational)
  // transport
  TlsOptions tls;                 // used when host is https://
  bool keepalive = true;
};

// Parse a kubeconfig (YAML or JSON) and fill rc from `context` (empty = current-context).
// Relative file paths in the kubeconfig resolve against the kubeconfig's directory.
bool load_kubeconfig(const std::string& path, const std::string& context, RestConfig* rc, std::string* err);
bool load_kubeconfig_text(const std::string& text, const std::string& base_dir, const std::string& context,
                          RestConfig* rc, std::string* err);
// rest.InClusterConfig. sa_dir lets tests point at a fake service-account mount.
bool in_cluster_config(RestConfig* rc, std::string* err, const std::string& sa_dir = kServiceAccountDir);
// clientcmd.BuildConfigFromFlags: kubeconfig if given (master overrides its server), else the
// master URL alone, else in-cluster.
bool build_config_from_flags(const std::string& master, const std::string& kubeconfig, RestConfig* rc,
                             std::string* err);

std::string base64_decode(const std::string& in);
std::string base64_encode(const std::string& in);

}  // namespace tfk
