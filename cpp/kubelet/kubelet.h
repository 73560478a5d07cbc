// tfk node agent ("kubelet"): runs the containers of pods bound to this node as process groups,
// pins GPUs (HIP_VISIBLE_DEVICES from the scheduler's tfk.io/gpu-ids), implements the pod
// restart policies (k8s-operator.md:46-52: OnFailure restarts in place, Never leaves the failed
// pod, completed pods are retained), reports containerStatuses (exitCode, reason incl.
// OOMKilled via the termination-message file, restartCount, lastState), keeps per-container log
// files (tfk.io/log-path), heartbeats its Node object, and injects faults on request
// (annotation tfk.io/fault-kill-after-ms / tfk.io/fault-signal / tfk.io/fault-generation).
// Health checking (k8s-operator.md:1): liveness / readiness / startup probes (probe.h) -- a failed
// liveness or startup probe kills the container (restart per policy), readiness drives
// containerStatuses[].ready and the pod's Ready condition. Memory: resources.limits.memory is
// enforced by polling the container session's resident set; a breach is SIGKILLed with reason
// OOMKilled (permanent, k8s-operator.md:5). Storage (:2): hostPath, emptyDir (lives as long as the
// pod) and persistentVolumeClaim (a per-namespace directory under the kubelet root) volumes at
// their volumeMounts' mountPath -- bind mounts in a private mount namespace when the kubelet may
// create one, else path substitution in args/env/workingDir plus TFK_VOLUME_MAP for the runtime.
#pragma once
#include <sys/types.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../cache/informer.h"
#include "probe.h"

namespace tfk {

struct KubeletOptions {
  std::string node_name = "node-0";
  int gpus = -1;  // -1 = detect from /sys/class/kfd
  long long cpu_milli = 0;
  std::string root_dir = "/tmp/tfk-kubelet";
  int64_t restart_backoff_ms = 1000;
  int64_t max_backoff_ms = 30000;
  int64_t grace_ms = 5000;
  int64_t heartbeat_ms = 10000;
  bool local_dns = true;
  // topology (two-socket 8x MI355X): GPU i's NUMA node, and each NUMA node's CPU list; detected
  // from sysfs (KFD topology -> PCI numa_node, /sys/devices/system/node) unless given
  std::string gpu_numa;   // e.g. "0,0,0,0,1,1,1,1"
  std::string numa_cpus;  // e.g. "0-47,96-143;48-95,144-191" (';' separates NUMA nodes)
  bool pin_cpus = true;   // sched_setaffinity of containers to their GPUs' NUMA CPUs
  std::string volume_mode = "auto";  // auto | namespace | substitute (see header comment)
  int64_t memory_poll_ms = 200;      // resources.limits.memory enforcement period
};

struct Topology {
  std::vector<int> gpu_numa;                 // per GPU index (HIP order)
  std::vector<std::vector<int>> numa_cpus;   // per NUMA node
};
Topology detect_topology(int gpus);
std::vector<int> parse_cpulist(const std::string& s);  // "0-3,8,10-11" -> ids

struct ContainerRun {
  std::string name;
  pid_t pid = -1;
  int restarts = 0;
  std::string state = "waiting";  // waiting | running | terminated
  std::string waiting_reason = "ContainerCreating";
  int exit_code = 0;
  std::string reason;
  std::string started_at, finished_at;
  int64_t next_start_ms = 0;
  int64_t started_mono = 0;
  Json last_terminated;
  std::string log_path, term_path;
  bool done = false;  // terminal, no more restarts
  // health checking
  ProbeState liveness, readiness, startup;
  bool started = false;  // startupProbe passed (or none)
  bool ready = false;
  std::vector<std::string> env;  // the container's environment (exec probes run in it)
  // kill requested by the kubelet itself: reason reported at exit (OOMKilled) / SIGKILL deadline
  std::string kill_reason;
  int64_t kill_deadline = 0;
  long long mem_limit = 0;  // bytes, 0 = unlimited
  long long mem_peak = 0;
};

struct PodRun {
  std::string uid, ns, name;
  Json pod;
  std::vector<ContainerRun> containers;
  std::string start_time;
  bool fault_done = false;
  bool killing = false;
  int64_t kill_deadline = 0;
  std::string last_status;  // last status JSON written
};

int detect_gpus();
// CPUs a pod with these GPU ids is pinned to (union of their NUMA nodes' CPUs; empty = no pinning)
std::vector<int> cpus_for_gpus(const Topology& t, const std::vector<int>& gpu_ids);

class Kubelet {
 public:
  Kubelet(std::shared_ptr<Client> c, KubeletOptions o);
  ~Kubelet();
  void run(StopToken& stop);
  void sync_once();  // exposed for tests
  size_t running_pods() const { return pods_.size(); }

 private:
  void register_node(bool heartbeat);
  void start_container(PodRun& pr, ContainerRun& c);
  void reap();
  void kill_pod(PodRun& pr, int sig);
  void update_status(PodRun& pr);
  Json build_status(PodRun& pr);
  void probe_container(PodRun& pr, ContainerRun& c);
  bool step_probe(ProbeState& ps, ContainerRun& c);  // true when the result changed this call
  void kill_container(PodRun& pr, ContainerRun& c, const std::string& reason, const std::string& msg, bool now);
  void check_memory(PodRun& pr);
  // volume name -> host directory for this pod ("" + *err on a bad volume)
  std::map<std::string, std::string> pod_volumes(PodRun& pr, std::string* err);
  bool mount_ns_supported();
  std::shared_ptr<Client> client_;
  KubeletOptions opts_;
  std::unique_ptr<SharedInformer> pods_inf_;
  std::map<std::string, PodRun> pods_;  // uid -> run
  std::map<pid_t, std::pair<std::string, size_t>> pid_owner_;
  int64_t last_heartbeat_ = 0, last_mem_poll_ = 0;
  Topology topo_;
  std::shared_ptr<class EventRecorder> rec_;
  int mount_ns_ = -1;  // -1 unknown, 0 no, 1 yes
};

}  // namespace tfk
