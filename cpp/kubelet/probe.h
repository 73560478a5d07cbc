// Container health checking, memory accounting and volume plumbing of tfk-kubelet: the
// "health checking (健康监测)" and storage lifecycle goals (k8s-operator.md:1-2) and the OOM failure
// mode (:5) at the node level.
//
// Probes (livenessProbe / readinessProbe / startupProbe of a container spec) run OFF the kubelet's
// sync loop: each execution is a detached thread that writes its verdict into a shared slot the
// loop polls, so a probe that hangs until its timeoutSeconds never stalls status updates, restarts
// or other pods. Handlers: exec (the command in the container's environment, exit 0 = success),
// tcpSocket (connect within the timeout), httpGet (HTTP/1.0 GET, 200-399 = success).
#pragma once
#include <sys/types.h>

#include <atomic>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../common/json.h"

namespace tfk {

struct ProbeSpec {
  std::string kind;  // "" (none) | exec | tcp | http
  std::vector<std::string> command;
  std::string host = "127.0.0.1", path = "/";
  int port = 0;
  int64_t initial_delay_ms = 0, period_ms = 10000, timeout_ms = 1000;
  int failure_threshold = 3, success_threshold = 1;
  // spec: the probe object (e.g. container.livenessProbe); container: for named ports
  static ProbeSpec parse(const Json& spec, const Json& container);
  bool enabled() const { return !kind.empty(); }
};

// One probe execution's verdict: 0 = running, 1 = success, 2 = failure (message set before the
// state is published).
struct ProbeSlot {
  std::atomic<int> state{0};
  std::string message;
};

// Starts one probe execution on a detached thread. exec probes: argv resolved against env's PATH,
// run as their own process group with env, killed at the timeout.
std::shared_ptr<ProbeSlot> launch_probe(const ProbeSpec& spec, const std::vector<std::string>& env);

// Per-probe bookkeeping of a container (k8s prober semantics: consecutive failures / successes
// against the thresholds, one execution in flight at a time).
struct ProbeState {
  ProbeSpec spec;
  std::shared_ptr<ProbeSlot> inflight;
  int64_t next_ms = 0;
  int fails = 0, succ = 0;
  bool ok = false;          // settled result: success_threshold successes seen since the last failure run
  std::string last_message;
  void reset() {
    inflight.reset();
    next_ms = 0;
    fails = succ = 0;
    ok = false;
    last_message.clear();
  }
};

// Kubernetes resource quantity -> bytes ("512Mi", "1Gi", "2G", "1500k", "1e9", "100"); -1 if invalid.
long long parse_bytes(const std::string& q);

// Resident set per session id over every process, in bytes, from one /proc/<pid>/stat scan (a
// container's process tree is its session: the kubelet starts each container with setsid).
std::map<pid_t, long long> session_rss_bytes();

}  // namespace tfk
