// tfk-cluster: all-in-one single-node control plane (apiserver + tf-operator + gang scheduler +
// kubelet) in one process, for local TFJob runs and the end-to-end tests.
#include <cstdio>
#include <thread>

#include "../apiserver/server.h"
#include "../kubelet/kubelet.h"
#include "../operator/options.h"
#include "../scheduler/scheduler.h"

int main(int argc, char** argv) {
  using namespace tfk;
  std::string host = "127.0.0.1", wal, port_file;
  long long port = 8080, gpus = -1, backoff = 500;
  ServerOption so;
  KubeletOptions ko;
  so.leader_elect = false;
  FlagSet fs("tfk-cluster");
  fs.add_string("host", &host, "apiserver bind address");
  fs.add_int("port", &port, "apiserver port (0 = ephemeral)");
  fs.add_string("wal", &wal, "apiserver WAL path");
  fs.add_string("port-file", &port_file, "write the apiserver port here");
  fs.add_int("gpus", &gpus, "node amd.com/gpu capacity (-1 = detect)");
  fs.add_string("gpu-numa", &ko.gpu_numa, "NUMA node per GPU, e.g. 0,0,0,0,1,1,1,1 (default: sysfs)");
  fs.add_string("numa-cpus", &ko.numa_cpus, "CPU list per NUMA node, ';'-separated (default: sysfs)");
  fs.add_string("volume-mode", &ko.volume_mode, "volume mounts: auto | namespace (bind mounts) | substitute (path rewrite)");
  fs.add_string("root-dir", &ko.root_dir, "kubelet state/log dir");
  fs.add_int("restart-backoff-ms", &backoff, "kubelet restart backoff");
  fs.add_int("threadiness", &so.threadiness, "operator workers");
  fs.add_int("resync-period", &so.resync_period_s, "operator resync (s)");
  fs.add_bool("gang-scheduling", &so.gang_scheduling, "gang scheduling");
  fs.add_bool("json-log-format", &so.json_log_format, "JSON logs");
  fs.add_string("log-level", &so.log_level, "log level");
  fs.add_int("metrics-port", &so.metrics_port, "operator metrics port");
  fs.add_bool("leader-elect", &so.leader_elect, "operator leader election");
  std::string err;
  if (!fs.parse(argc, argv, &err)) { fprintf(stderr, "%s\n%s", err.c_str(), fs.usage().c_str()); return 2; }
  if (fs.help_requested()) { printf("%s", fs.usage().c_str()); return 0; }
  InitLogging("tfk-cluster", so.json_log_format, so.log_level);
  StopToken stop;
  HandleSignals(stop);
  auto store = std::make_shared<Store>(wal);
  install_tfjob_crd(*store);
  ApiServer srv(store);
  if (!srv.start(host, (int)port, &err)) { TFK_LOG(Error, "apiserver: " + err); return 1; }
  std::string url = "http://" + host + ":" + std::to_string(srv.port());
  if (!port_file.empty()) {
    // write-then-rename: a reader polling for the file never sees it created but still empty
    const std::string tmp = port_file + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (f) {
      fprintf(f, "%d\n", srv.port());
      fclose(f);
      std::rename(tmp.c_str(), port_file.c_str());
    }
  }
  printf("listening on %s\n", url.c_str());
  fflush(stdout);
  so.apiserver = url;
  RestConfig rc;
  rc.host = url;
  rc.qps = 200;
  rc.burst = 400;
  std::thread op([&] { RunServer(so, stop); });
  std::thread sch([&] {
    GangScheduler s(new_for_config(rc), SchedulerOptions());
    s.run(stop);
  });
  ko.gpus = (int)gpus;
  ko.restart_backoff_ms = backoff;
  std::thread kub([&] {
    Kubelet k(new_for_config(rc), ko);
    k.run(stop);
  });
  while (!stop.wait_for(500)) {
  }
  op.join();
  sch.join();
  kub.join();
  srv.stop();
  return 0;
}
