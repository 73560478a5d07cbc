// tf-operator options + server (reference: cmd/tf_operator/app/options/options.go and app/server.go,
// images/tf.PNG:L1-L6; startup sequence New Option -> Add flag -> Init flag and initlog -> Run
// server, images/tf2.png; HA via leader election, k8s-operator.md:59).
#pragma once
#include <string>

#include "../common/util.h"

namespace tfk {

struct ServerOption {
  std::string apiserver;                // "" = from kubeconfig / in-cluster / http://127.0.0.1:8080
  std::string kubeconfig;              // kubeconfig YAML/JSON (client/config.h)
  std::string controller_config_file;  // JSON ControllerConfig (accelerators, grpcServerFilePath)
  std::string ns;                      // watch namespace ("" = all)
  long long threadiness = 2;
  long long resync_period_s = 30;
  bool json_log_format = false;
  bool print_version = false;
  bool leader_elect = true;
  std::string lock_namespace = "default";
  std::string lock_name = "tf-operator";
  std::string identity;                // default: hostname + pid
  double lease_duration_s = 15, renew_deadline_s = 10, retry_period_s = 2;
  long long metrics_port = 0;          // 0 = disabled; serves /metrics and /healthz
  double qps = 50;
  long long burst = 100;
  bool gang_scheduling = true;
  bool local_ports = true;             // single-node emulation (unique per-service ports)
  std::string cluster_domain;
  double chaos_level = 0;              // probability per resync tick of killing a random job pod
  std::string log_level = "info";

  static ServerOption New() { return ServerOption(); }
  void AddFlags(FlagSet& fs);
};

// app.Run: build clients, (optionally) leader-elect, run the controller until stop.
int RunServer(const ServerOption& opt, StopToken& stop);

void InitLogging(const std::string& component, bool json, const std::string& level);
// Installs SIGINT/SIGTERM handlers that stop the token (signal-safe via a watcher thread).
void HandleSignals(StopToken& stop);

}  // namespace tfk
