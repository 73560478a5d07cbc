// tfk-kubelet: node agent running pod containers as processes with GPU pinning.
#include <cstdio>

#include "../kubelet/kubelet.h"
#include "../operator/options.h"

int main(int argc, char** argv) {
  using namespace tfk;
  std::string apiserver = "http://127.0.0.1:8080", level = "info";
  KubeletOptions ko;
  long long gpus = -1, backoff = 1000, grace = 5000;
  bool json = false;
  FlagSet fs("tfk-kubelet");
  fs.add_string("apiserver", &apiserver, "apiserver URL");
  fs.add_string("node-name", &ko.node_name, "node name");
  fs.add_int("gpus", &gpus, "amd.com/gpu capacity (-1 = detect)");
  fs.add_string("gpu-numa", &ko.gpu_numa, "NUMA node per GPU, e.g. 0,0,0,0,1,1,1,1 (default: sysfs)");
  fs.add_string("numa-cpus", &ko.numa_cpus, "CPU list per NUMA node, ';'-separated (default: sysfs)");
  fs.add_string("volume-mode", &ko.volume_mode, "volume mounts: auto | namespace (bind mounts) | substitute (path rewrite)");
  fs.add_string("root-dir", &ko.root_dir, "state/log directory");
  fs.add_int("restart-backoff-ms", &backoff, "base container restart backoff");
  fs.add_int("grace-ms", &grace, "termination grace period");
  fs.add_bool("json-log-format", &json, "JSON logs");
  fs.add_string("log-level", &level, "log level");
  std::string err;
  if (!fs.parse(argc, argv, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 2; }
  if (fs.help_requested()) { printf("%s", fs.usage().c_str()); return 0; }
  InitLogging("tfk-kubelet", json, level);
  ko.gpus = (int)gpus;
  ko.restart_backoff_ms = backoff;
  ko.grace_ms = grace;
  StopToken stop;
  HandleSignals(stop);
  RestConfig rc;
  rc.host = apiserver;
  rc.qps = 100;
  rc.burst = 200;
  Kubelet k(new_for_config(rc), ko);
  k.run(stop);
  return 0;
}
