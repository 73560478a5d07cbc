#include "options.h"

#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <thread>

#include "../client/config.h"
#include "../controller/controller.h"
#include "../leaderelection/leaderelection.h"

namespace tfk {

void ServerOption::AddFlags(FlagSet& fs) {
  fs.add_string("apiserver", &apiserver, "API server URL (http[s]://host:port); overrides the kubeconfig server");
  fs.add_string("master", &apiserver, "alias of --apiserver (client-go --master)");
  fs.add_string("kubeconfig", &kubeconfig, "kubeconfig (YAML/JSON); default: in-cluster service account, else tfk-apiserver on 127.0.0.1:8080");
  fs.add_string("controller-config-file", &controller_config_file, "JSON controller config (accelerators)");
  fs.add_string("namespace", &ns, "namespace to watch (default all)");
  fs.add_int("threadiness", &threadiness, "number of reconcile workers");
  fs.add_int("resync-period", &resync_period_s, "informer resync period (seconds)");
  fs.add_bool("json-log-format", &json_log_format, "log as JSON lines");
  fs.add_bool("version", &print_version, "print version and exit");
  fs.add_bool("leader-elect", &leader_elect, "run leader election (HA)");
  fs.add_string("lock-namespace", &lock_namespace, "namespace of the leader lease");
  fs.add_string("lock-name", &lock_name, "name of the leader lease");
  fs.add_string("identity", &identity, "leader election identity");
  fs.add_double("lease-duration", &lease_duration_s, "lease duration seconds");
  fs.add_double("renew-deadline", &renew_deadline_s, "renew deadline seconds");
  fs.add_double("retry-period", &retry_period_s, "retry period seconds");
  fs.add_int("metrics-port", &metrics_port, "serve /metrics and /healthz on this port (0=off)");
  fs.add_double("qps", &qps, "client QPS (token bucket)");
  fs.add_int("burst", &burst, "client burst");
  fs.add_bool("gang-scheduling", &gang_scheduling, "schedule TFJob pods as a gang (tfk-gang)");
  fs.add_bool("local-ports", &local_ports, "single-node emulation: unique per-service ports in TF_CONFIG");
  fs.add_string("cluster-domain", &cluster_domain, "DNS cluster domain suffix for TF_CONFIG hosts");
  fs.add_double("chaos-level", &chaos_level, "probability (0-1) per tick of killing a random TFJob pod");
  fs.add_string("log-level", &log_level, "debug|info|warning|error");
}

void InitLogging(const std::string& component, bool json, const std::string& level) {
  auto& l = Logger::get();
  l.set_component(component);
  l.set_json(json);
  l.set_level(level == "debug" ? LogLevel::Debug : level == "warning" ? LogLevel::Warn
                                                 : level == "error" ? LogLevel::Error : LogLevel::Info);
}

void HandleSignals(StopToken& stop) {
  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGINT);
  sigaddset(&set, SIGTERM);
  pthread_sigmask(SIG_BLOCK, &set, nullptr);
  std::thread([set, &stop]() mutable {
    int sig = 0;
    sigwait(&set, &sig);
    TFK_LOG(Info, "signal received, shutting down", Json(Json::object_t{{"signal", Json(sig)}}));
    stop.stop();
  }).detach();
}

static std::string default_identity() {
  const char* pod = getenv("MY_POD_NAME");  // set from the downward API in deploy/operator.yaml
  if (pod && *pod) return pod;
  char host[256] = {0};
  gethostname(host, sizeof host - 1);
  return std::string(host) + "_" + std::to_string(getpid());
}

int RunServer(const ServerOption& opt_in, StopToken& stop) {
  ServerOption opt = opt_in;
  // clientcmd.BuildConfigFromFlags(master, kubeconfig) (k8s-operator.md:92-101); with neither flag an
  // operator pod uses its service account (rest.InClusterConfig), a dev box the local tfk-apiserver
  RestConfig rc;
  std::string cerr;
  if (!opt.kubeconfig.empty() || !opt.apiserver.empty() || getenv("KUBERNETES_SERVICE_HOST")) {
    if (!build_config_from_flags(opt.apiserver, opt.kubeconfig, &rc, &cerr)) {
      TFK_LOG(Error, "client config: " + cerr);
      return 1;
    }
  } else {
    rc.host = "http://127.0.0.1:8080";
  }
  rc.qps = opt.qps;
  rc.burst = (int)opt.burst;
  rc.user_agent = "tf-operator/v0.1 (tfk)";
  TFK_LOG(Info, "api server", Json(Json::object_t{{"host", Json(rc.host)},
                                                 {"auth", Json(!rc.bearer_token.empty() ? "bearer-token"
                                                               : !rc.tls.cert_file.empty() || !rc.tls.cert_data.empty()
                                                                   ? "client-certificate" : "none")}}));
  auto client = new_for_config(rc);
  ControllerOptions co;
  co.threadiness = (int)opt.threadiness;
  co.resync_ms = opt.resync_period_s * 1000;
  co.ns = opt.ns;
  co.trainer.gang_scheduling = opt.gang_scheduling;
  co.trainer.local_ports = opt.local_ports;
  co.trainer.cluster_domain = opt.cluster_domain;
  if (!opt.controller_config_file.empty()) {
    std::ifstream f(opt.controller_config_file);
    std::stringstream ss;
    ss << f.rdbuf();
    co.trainer.controller_config = api::ControllerConfig::from_json(Json::parse(ss.str()));
  }
  TFJobController ctl(client, co);
  HttpServer metrics;
  if (opt.metrics_port > 0) {
    std::string err;
    if (!metrics.listen("0.0.0.0", (int)opt.metrics_port, &err)) {
      TFK_LOG(Error, "metrics server: " + err);
      return 1;
    }
    metrics.serve([&](const HttpRequest& r, ResponseWriter& w) {
      if (r.path == "/metrics") w.respond(200, ctl.metrics_text(), "text/plain; version=0.0.4");
      else if (r.path == "/healthz") w.respond(200, "ok", "text/plain");
      else w.respond(404, "not found", "text/plain");
    });
  }
  std::thread chaos;
  if (opt.chaos_level > 0) {
    chaos = std::thread([&] {
      std::mt19937 rng(42);
      std::uniform_real_distribution<double> u(0, 1);
      while (!stop.wait_for(5000)) {
        if (u(rng) >= opt.chaos_level) continue;
        auto pods = ctl.pod_informer().indexer().list();
        if (pods.empty()) continue;
        auto& p = pods[rng() % pods.size()];
        TFK_LOG(Warn, "chaos: deleting pod", Json(Json::object_t{{"pod", Json(p.path("metadata.name").str())}}));
        client->remove("pods", p.path("metadata.namespace").str(), p.path("metadata.name").str());
      }
    });
  }
  if (!opt.leader_elect) {
    ctl.run(stop);
  } else {
    LeaderElectionConfig lc;
    lc.lock_namespace = opt.lock_namespace;
    lc.lock_name = opt.lock_name;
    lc.identity = opt.identity.empty() ? default_identity() : opt.identity;
    lc.lease_duration_ms = (int64_t)(opt.lease_duration_s * 1000);
    lc.renew_deadline_ms = (int64_t)(opt.renew_deadline_s * 1000);
    lc.retry_period_ms = (int64_t)(opt.retry_period_s * 1000);
    lc.on_started_leading = [&](StopToken& lead_stop) { ctl.run(lead_stop); };
    lc.on_new_leader = [](const std::string& id) {
      TFK_LOG(Info, "observed leader", Json(Json::object_t{{"identity", Json(id)}}));
    };
    LeaderElector le(client, lc);
    le.run(stop);
    if (!stop.stopped()) {
      // leadership lost: exit non-zero so the supervisor restarts us as a standby (RunOrDie)
      TFK_LOG(Error, "leader election lost, exiting");
      stop.stop();
      if (chaos.joinable()) chaos.join();
      return 2;
    }
  }
  stop.stop();
  if (chaos.joinable()) chaos.join();
  metrics.stop();
  return 0;
}

}  // namespace tfk
