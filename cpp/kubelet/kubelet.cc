#include "kubelet.h"

#include "../api/types.h"
#include "../controller/trainer.h"

#include <dirent.h>
#include <fcntl.h>
#include <ftw.h>
#include <sched.h>
#include <signal.h>
#include <sys/mount.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>

extern char** environ;

namespace tfk {

int detect_gpus() {
  int n = 0;
  DIR* d = opendir("/sys/class/kfd/kfd/topology/nodes");
  if (!d) return 0;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::ifstream f(std::string("/sys/class/kfd/kfd/topology/nodes/") + e->d_name + "/gpu_id");
    int id = 0;
    if (f >> id && id != 0) n++;
  }
  closedir(d);
  return n;
}

std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  for (auto& part : split(s, ',')) {
    std::string t = trim(part);
    if (t.empty()) continue;
    size_t dash = t.find('-');
    int a = atoi(t.c_str()), b = dash == std::string::npos ? a : atoi(t.c_str() + dash + 1);
    for (int c = a; c <= b && c - a < 65536; ++c) out.push_back(c);
  }
  return out;
}

static std::string read_first_line(const std::string& path) {
  std::ifstream f(path);
  std::string line;
  std::getline(f, line);
  return trim(line);
}

// KFD topology: GPU nodes (gpu_id != 0) in node-index order = HIP device order; each node's
// properties carry the PCI location_id (bus << 8 | devfn) and domain -> the PCI device's numa_node.
Topology detect_topology(int gpus) {
  Topology t;
  std::vector<std::pair<int, int>> gpu_nodes;  // (kfd node index, numa)
  if (DIR* d = opendir("/sys/class/kfd/kfd/topology/nodes")) {
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      std::string base = std::string("/sys/class/kfd/kfd/topology/nodes/") + e->d_name;
      if (atoi(read_first_line(base + "/gpu_id").c_str()) == 0) continue;
      long long loc = -1, dom = 0;
      std::ifstream f(base + "/properties");
      std::string k;
      long long v;
      while (f >> k >> v) {
        if (k == "location_id") loc = v;
        else if (k == "domain") dom = v;
      }
      int numa = 0;
      if (loc >= 0) {
        char bdf[64];
        snprintf(bdf, sizeof bdf, "/sys/bus/pci/devices/%04llx:%02llx:%02llx.%llx/numa_node", dom, (loc >> 8) & 0xff,
                 (loc >> 3) & 0x1f, loc & 0x7);
        numa = std::max(0, atoi(read_first_line(bdf).c_str()));
      }
      gpu_nodes.push_back({atoi(e->d_name), numa});
    }
    closedir(d);
  }
  std::sort(gpu_nodes.begin(), gpu_nodes.end());
  for (auto& g : gpu_nodes) t.gpu_numa.push_back(g.second);
  if ((int)t.gpu_numa.size() != gpus) t.gpu_numa.assign(std::max(gpus, 0), 0);
  for (int n = 0;; ++n) {
    std::string cl = read_first_line("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist");
    if (cl.empty()) break;
    t.numa_cpus.push_back(parse_cpulist(cl));
  }
  return t;
}

std::vector<int> cpus_for_gpus(const Topology& t, const std::vector<int>& gpu_ids) {
  std::set<int> nodes, cpus;
  for (int g : gpu_ids)
    if (g >= 0 && g < (int)t.gpu_numa.size()) nodes.insert(t.gpu_numa[g]);
  for (int n : nodes)
    if (n >= 0 && n < (int)t.numa_cpus.size()) cpus.insert(t.numa_cpus[n].begin(), t.numa_cpus[n].end());
  return std::vector<int>(cpus.begin(), cpus.end());
}

static void mkdirs(const std::string& p) {
  std::string cur;
  for (auto& part : split(p, '/')) {
    if (part.empty()) { cur += "/"; continue; }
    cur += part + "/";
    mkdir(cur.c_str(), 0755);
  }
}

static int rm_entry(const char* path, const struct stat*, int, struct FTW*) { return remove(path); }
static void remove_tree(const std::string& p) { nftw(p.c_str(), rm_entry, 16, FTW_DEPTH | FTW_PHYS); }

// One volumeMount resolved to its host directory.
struct MountSpec {
  std::string src, dst;
  bool ro = false;
};

// Path substitution (no mount namespace): a token that IS a mount path or starts with "<mountPath>/"
// -- at the start of the string or after '=', ':' or ',' (--flag=/mnt/x, PATH-like lists) -- is
// rewritten onto the host directory. Longest mount path first.
static std::string subst_paths(const std::string& s, const std::vector<MountSpec>& mounts) {
  std::string out = s;
  for (auto& m : mounts) {
    if (m.dst.empty() || m.dst == m.src) continue;
    size_t pos = 0;
    while ((pos = out.find(m.dst, pos)) != std::string::npos) {
      const bool start_ok = pos == 0 || out[pos - 1] == '=' || out[pos - 1] == ':' || out[pos - 1] == ',';
      const size_t e = pos + m.dst.size();
      const bool end_ok = e == out.size() || out[e] == '/' || out[e] == ':' || out[e] == ',';
      if (start_ok && end_ok) {
        out.replace(pos, m.dst.size(), m.src);
        pos += m.src.size();
      } else {
        pos = e;
      }
    }
  }
  return out;
}

Kubelet::Kubelet(std::shared_ptr<Client> c, KubeletOptions o) : client_(std::move(c)), opts_(std::move(o)) {
  if (opts_.gpus < 0) opts_.gpus = detect_gpus();
  if (opts_.cpu_milli <= 0) opts_.cpu_milli = (long long)sysconf(_SC_NPROCESSORS_ONLN) * 1000;
  topo_ = detect_topology(opts_.gpus);
  if (!opts_.gpu_numa.empty()) {
    topo_.gpu_numa.clear();
    for (auto& x : split(opts_.gpu_numa, ',')) topo_.gpu_numa.push_back(atoi(x.c_str()));
  }
  if (!opts_.numa_cpus.empty()) {
    topo_.numa_cpus.clear();
    for (auto& x : split(opts_.numa_cpus, ';')) topo_.numa_cpus.push_back(parse_cpulist(x));
  }
  mkdirs(opts_.root_dir + "/logs");
  mkdirs(opts_.root_dir + "/term");
  pods_inf_.reset(new SharedInformer(client_, "pods", "", 10000, "", "spec.nodeName=" + opts_.node_name));
  rec_ = std::make_shared<EventRecorder>(client_, "kubelet");
}

// Whether this kubelet may give containers a private mount namespace with bind mounts (needs
// CAP_SYS_ADMIN): tried once in a throw-away child.
bool Kubelet::mount_ns_supported() {
  if (mount_ns_ >= 0) return mount_ns_ == 1;
  std::string base = opts_.root_dir + "/nsprobe", src = base + "/src", dst = base + "/dst";
  mkdirs(src);
  mkdirs(dst);
  pid_t pid = fork();
  if (pid == 0) {
    if (unshare(CLONE_NEWNS) != 0) _exit(1);
    if (mount(nullptr, "/", nullptr, MS_REC | MS_PRIVATE, nullptr) != 0) _exit(2);
    if (mount(src.c_str(), dst.c_str(), nullptr, MS_BIND, nullptr) != 0) _exit(3);
    _exit(0);
  }
  int status = 1;
  if (pid > 0) waitpid(pid, &status, 0);
  mount_ns_ = (pid > 0 && WIFEXITED(status) && WEXITSTATUS(status) == 0) ? 1 : 0;
  TFK_LOG(Info, "volume mounts", Json(Json::object_t{{"mode", Json(mount_ns_ ? "namespace" : "substitute")}}));
  return mount_ns_ == 1;
}

std::map<std::string, std::string> Kubelet::pod_volumes(PodRun& pr, std::string* err) {
  std::map<std::string, std::string> out;
  for (auto& v : pr.pod.path("spec.volumes").items()) {
    const std::string name = v.at("name").str();
    if (v.at("hostPath").is_object()) {
      const std::string path = v.path("hostPath.path").str(), type = v.path("hostPath.type").str();
      struct stat sb;
      const bool exists = stat(path.c_str(), &sb) == 0;
      if (type == "DirectoryOrCreate" && !exists) {
        mkdirs(path);
      } else if (type == "Directory" && !(exists && S_ISDIR(sb.st_mode))) {
        *err = "hostPath type check failed: " + path + " is not a directory";
        return {};
      }
      out[name] = path;
    } else if (v.at("persistentVolumeClaim").is_object()) {
      // PVC-like: one directory per (namespace, claim) under the kubelet root, outliving pods
      std::string d = opts_.root_dir + "/pvc/" + pr.ns + "/" + v.path("persistentVolumeClaim.claimName").str();
      mkdirs(d);
      out[name] = d;
    } else {
      // emptyDir (and kinds this node does not implement): a per-pod directory removed with the pod
      std::string d = opts_.root_dir + "/pods/" + pr.uid + "/volumes/" + name;
      mkdirs(d);
      out[name] = d;
    }
  }
  return out;
}

Kubelet::~Kubelet() {
  for (auto& kv : pods_) kill_pod(kv.second, SIGKILL);
}

void Kubelet::register_node(bool heartbeat) {
  Json n = Json::object();
  n["apiVersion"] = "v1";
  n["kind"] = "Node";
  n["metadata"]["name"] = opts_.node_name;
  n["metadata"]["labels"]["kubernetes.io/hostname"] = opts_.node_name;
  n["metadata"]["labels"]["amd.com/gpu.product"] = "MI355X";
  std::string numa;
  for (size_t i = 0; i < topo_.gpu_numa.size(); ++i) numa += (i ? "," : "") + std::to_string(topo_.gpu_numa[i]);
  n["metadata"]["annotations"]["tfk.io/gpu-numa"] = numa;
  n["metadata"]["annotations"]["tfk.io/numa-nodes"] = std::to_string(std::max<size_t>(1, topo_.numa_cpus.size()));
  Json cap = Json::object();
  cap["amd.com/gpu"] = opts_.gpus;
  cap["cpu"] = std::to_string(opts_.cpu_milli) + "m";
  cap["pods"] = 110;
  n["status"]["capacity"] = cap;
  n["status"]["allocatable"] = cap;
  Json cond = Json::object();
  cond["type"] = "Ready";
  cond["status"] = "True";
  cond["reason"] = "KubeletReady";
  cond["lastHeartbeatTime"] = rfc3339(now_ms());
  n["status"]["conditions"] = Json(Json::array_t{cond});
  Json addr = Json::object();
  addr["type"] = "InternalIP";
  addr["address"] = "127.0.0.1";
  n["status"]["addresses"] = Json(Json::array_t{addr});
  Json out;
  if (!heartbeat) {
    ApiStatus st = client_->create("nodes", "", n, &out);
    if (st.code != 409) return;
  }
  Json cur;
  if (client_->get("nodes", "", opts_.node_name, &cur).ok()) {
    n["metadata"]["resourceVersion"] = cur.path("metadata.resourceVersion");
    n["spec"] = cur.at("spec");
    client_->update("nodes", "", n, &out);
  }
}

void Kubelet::start_container(PodRun& pr, ContainerRun& c) {
  const Json* spec = nullptr;
  for (auto& cs : pr.pod.path("spec.containers").items())
    if (cs.at("name").str() == c.name) spec = &cs;
  if (!spec) return;
  c.log_path = opts_.root_dir + "/logs/" + pr.ns + "_" + pr.name + "_" + c.name + ".log";
  c.term_path = opts_.root_dir + "/term/" + pr.uid + "_" + c.name;
  unlink(c.term_path.c_str());
  std::vector<std::string> argv;
  for (auto& a : spec->at("command").items()) argv.push_back(a.str());
  for (auto& a : spec->at("args").items()) argv.push_back(a.str());
  if (argv.empty()) argv.push_back("/bin/true");
  // volumes -> mounts of this container
  std::string verr;
  auto vols = pod_volumes(pr, &verr);
  std::vector<MountSpec> mounts;
  for (auto& vm : spec->at("volumeMounts").items()) {
    if (!verr.empty()) break;  // a volume of the pod failed its checks
    auto it = vols.find(vm.at("name").str());
    if (it == vols.end()) {
      verr = "volumeMount " + vm.at("name").str() + " names no volume of the pod";
      break;
    }
    MountSpec m;
    m.src = it->second;
    const std::string sub = vm.at("subPath").str();
    if (!sub.empty()) {
      m.src += "/" + sub;
      mkdirs(m.src);
    }
    m.dst = vm.at("mountPath").str();
    m.ro = vm.at("readOnly").as_bool(false);
    while (m.dst.size() > 1 && m.dst.back() == '/') m.dst.pop_back();
    if (!m.dst.empty() && m.dst != m.src) mounts.push_back(m);
  }
  if (!verr.empty()) {
    c.state = "waiting";
    c.waiting_reason = "CreateContainerConfigError";
    c.next_start_ms = mono_ms() + opts_.restart_backoff_ms;
    rec_->event(pr.pod, "Warning", "FailedMount", verr);
    return;
  }
  std::sort(mounts.begin(), mounts.end(), [](const MountSpec& a, const MountSpec& b) { return a.dst.size() > b.dst.size(); });
  const bool use_ns = !mounts.empty() && (opts_.volume_mode == "namespace" ||
                                          (opts_.volume_mode == "auto" && mount_ns_supported()));
  std::map<std::string, std::string> env;
  for (char** e = environ; *e; ++e) {
    std::string kv = *e;
    size_t eq = kv.find('=');
    if (eq != std::string::npos) env[kv.substr(0, eq)] = kv.substr(eq + 1);
  }
  for (auto& e : spec->at("env").items()) {
    std::string v = e.at("value").str();
    const Json& fr = e.path("valueFrom.fieldRef.fieldPath");
    if (fr.is_string()) {
      if (fr.str() == "metadata.name") v = pr.name;
      else if (fr.str() == "metadata.namespace") v = pr.ns;
      else if (fr.str() == "status.podIP") v = "127.0.0.1";
      else if (fr.str() == "spec.nodeName") v = opts_.node_name;
    }
    env[e.at("name").str()] = v;
  }
  std::string gpu_ids = pr.pod.path("metadata.annotations").at("tfk.io/gpu-ids").str();
  std::string gang_ids = pr.pod.path("metadata.annotations").at(api::kGangGpuIds).str();
  if (!gang_ids.empty() && !gpu_ids.empty()) {
    // gang-visible: the pod sees every GPU of its gang on this node; its own device is
    // TFK_LOCAL_DEVICE (index of its first assigned GPU in the visible list)
    auto vis = split(gang_ids, ',');
    std::string own = split(gpu_ids, ',')[0];
    int local = 0;
    for (size_t i = 0; i < vis.size(); ++i)
      if (vis[i] == own) local = (int)i;
    env["HIP_VISIBLE_DEVICES"] = gang_ids;
    env["TFK_LOCAL_DEVICE"] = std::to_string(local);
  } else if (!gpu_ids.empty()) {
    env["HIP_VISIBLE_DEVICES"] = gpu_ids;
    env["TFK_LOCAL_DEVICE"] = "0";
  }
  // NUMA-local CPUs of the pod's GPUs (built here: the child only calls sched_setaffinity)
  std::vector<int> gids;
  for (auto& x : split(gpu_ids, ','))
    if (!x.empty()) gids.push_back(atoi(x.c_str()));
  std::vector<int> pin = opts_.pin_cpus ? cpus_for_gpus(topo_, gids) : std::vector<int>();
  cpu_set_t cpuset;
  CPU_ZERO(&cpuset);
  std::string pin_list;
  for (int cpu : pin)
    if (cpu >= 0 && cpu < CPU_SETSIZE) {
      CPU_SET(cpu, &cpuset);
      pin_list += (pin_list.empty() ? "" : ",") + std::to_string(cpu);
    }
  const bool do_pin = !pin_list.empty();
  if (do_pin) env["TFK_CPU_AFFINITY"] = pin_list;
  env["TFK_POD_NAME"] = pr.name;
  env["TFK_POD_NAMESPACE"] = pr.ns;
  env["TFK_NODE_NAME"] = opts_.node_name;
  env["TFK_TERMINATION_LOG"] = c.term_path;
  if (opts_.local_dns) env["TFK_LOCAL_DNS"] = "1";
  std::string wd = spec->at("workingDir").str();
  if (!mounts.empty() && !use_ns) {
    // no mount namespace: the container sees its volumes at the host directories -- rewrite the
    // paths it was given, and tell the runtime the map for paths it reads from elsewhere
    std::string vmap;
    for (auto& m : mounts) vmap += (vmap.empty() ? "" : ";") + m.dst + "=" + m.src;
    for (auto& a : argv) a = subst_paths(a, mounts);
    for (auto& kv : env) kv.second = subst_paths(kv.second, mounts);
    wd = subst_paths(wd, mounts);
    env["TFK_VOLUME_MAP"] = vmap;
  }
  for (auto& m : mounts)
    if (use_ns) mkdirs(m.dst);  // the mount points (the namespace shares the host's tree)
  std::vector<std::string> msrc, mdst;
  std::vector<char> mro;
  if (use_ns)
    for (auto& m : mounts) { msrc.push_back(m.src); mdst.push_back(m.dst); mro.push_back(m.ro); }
  static const char kMountFail[] = "tfk-kubelet: volume mount failed\n";
  // resources.limits.memory (enforced by the sync loop's RSS poll)
  c.mem_limit = 0;
  c.mem_peak = 0;
  const Json& ml = spec->path("resources.limits").at("memory");
  if (ml.is_string() || ml.is_number()) {
    long long b = ml.is_number() ? (long long)ml.as_double() : parse_bytes(ml.str());
    if (b > 0) c.mem_limit = b;
  }
  // probes (their exec commands see the volumes at the host paths)
  c.liveness.reset();
  c.readiness.reset();
  c.startup.reset();
  c.liveness.spec = ProbeSpec::parse(spec->at("livenessProbe"), *spec);
  c.readiness.spec = ProbeSpec::parse(spec->at("readinessProbe"), *spec);
  c.startup.spec = ProbeSpec::parse(spec->at("startupProbe"), *spec);
  for (ProbeState* ps : {&c.liveness, &c.readiness, &c.startup})
    for (auto& a : ps->spec.command) a = subst_paths(a, mounts);
  c.started = !c.startup.spec.enabled();
  c.ready = false;
  c.kill_reason.clear();
  c.kill_deadline = 0;
  // Everything the child needs is built BEFORE fork(): the kubelet is multithreaded (informer,
  // HTTP and watch threads), so between fork and exec the child may only make async-signal-safe
  // calls -- a malloc there can deadlock on a lock another thread held at fork time.
  std::vector<std::string> envs;
  for (auto& kv : env) envs.push_back(kv.first + "=" + kv.second);
  // exec probes run outside any mount namespace: their environment sees the volumes at host paths
  c.env.clear();
  for (auto& kv : env) c.env.push_back(kv.first + "=" + subst_paths(kv.second, mounts));
  std::vector<char*> ev, av;
  for (auto& s : envs) ev.push_back((char*)s.c_str());
  ev.push_back(nullptr);
  for (auto& s : argv) av.push_back((char*)s.c_str());
  av.push_back(nullptr);
  // execvp's PATH search is not async-signal-safe: resolve the program here, execve in the child
  std::string prog = av[0] ? av[0] : "";
  if (prog.find('/') == std::string::npos) {
    for (const std::string& dir : split(env.count("PATH") ? env["PATH"] : std::string(getenv("PATH") ? getenv("PATH") : "/usr/bin:/bin"), ':')) {
      std::string cand = (dir.empty() ? std::string(".") : dir) + "/" + prog;
      if (access(cand.c_str(), X_OK) == 0) { prog = cand; break; }
    }
  }
  const char* log_path = c.log_path.c_str();
  const char* wd_c = wd.empty() ? nullptr : wd.c_str();
  static const char kExecFail[] = "tfk-kubelet: exec failed\n";
  // The kubelet blocks SIGINT/SIGTERM for its sigwait thread (HandleSignals) and ignores SIGPIPE;
  // both survive exec, so the container would ignore the SIGTERM of a graceful stop and only die
  // at the SIGKILL deadline. The child restores an empty mask and default dispositions.
  sigset_t none;
  sigemptyset(&none);
  pid_t pid = fork();
  if (pid == 0) {
    sigprocmask(SIG_SETMASK, &none, nullptr);
    if (do_pin) sched_setaffinity(0, sizeof(cpuset), &cpuset);  // best effort (cgroup may forbid)
    signal(SIGPIPE, SIG_DFL);
    signal(SIGTERM, SIG_DFL);
    signal(SIGINT, SIG_DFL);
    setsid();
    int fd = open(log_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (!msrc.empty()) {
      // private mount namespace: bind each volume at its mountPath (read-only when asked)
      bool ok = unshare(CLONE_NEWNS) == 0 && mount(nullptr, "/", nullptr, MS_REC | MS_PRIVATE, nullptr) == 0;
      for (size_t i = 0; ok && i < msrc.size(); ++i) {
        ok = mount(msrc[i].c_str(), mdst[i].c_str(), nullptr, MS_BIND | MS_REC, nullptr) == 0;
        if (ok && mro[i])
          ok = mount(nullptr, mdst[i].c_str(), nullptr, MS_BIND | MS_REMOUNT | MS_RDONLY | MS_REC, nullptr) == 0;
      }
      if (!ok) {
        if (fd >= 0) {
          ssize_t wr = write(fd, kMountFail, sizeof(kMountFail) - 1);
          (void)wr;
        }
        _exit(127);
      }
    }
    if (fd >= 0) { dup2(fd, 1); dup2(fd, 2); close(fd); }
    int nul = open("/dev/null", O_RDONLY);
    if (nul >= 0) { dup2(nul, 0); close(nul); }
    if (wd_c && chdir(wd_c) != 0) _exit(127);
    execve(prog.c_str(), av.data(), ev.data());
    ssize_t wr = write(2, kExecFail, sizeof(kExecFail) - 1);
    (void)wr;
    _exit(127);
  }
  if (pid < 0) {
    c.state = "waiting";
    c.waiting_reason = "StartError";
    c.next_start_ms = mono_ms() + opts_.restart_backoff_ms;
    return;
  }
  c.pid = pid;
  c.state = "running";
  c.started_at = rfc3339(now_ms());
  c.started_mono = mono_ms();
  for (size_t i = 0; i < pr.containers.size(); ++i)
    if (&pr.containers[i] == &c) pid_owner_[pid] = {pr.uid, i};
  TFK_LOG(Info, "started container", Json(Json::object_t{{"pod", Json(pr.ns + "/" + pr.name)}, {"container", Json(c.name)},
                                                         {"pid", Json((long long)pid)}, {"gpus", Json(gpu_ids)},
                                                         {"cpus", Json(pin_list)}}));
}

void Kubelet::kill_pod(PodRun& pr, int sig) {
  for (auto& c : pr.containers)
    if (c.pid > 0) kill(-c.pid, sig);
}

void Kubelet::kill_container(PodRun& pr, ContainerRun& c, const std::string& reason, const std::string& msg, bool now) {
  if (c.pid <= 0 || !c.kill_reason.empty()) return;
  c.kill_reason = reason;
  rec_->event(pr.pod, "Warning", reason == "OOMKilled" ? "OOMKilling" : "Unhealthy", c.name + ": " + msg);
  TFK_LOG(Warn, "killing container", Json(Json::object_t{{"pod", Json(pr.ns + "/" + pr.name)}, {"container", Json(c.name)},
                                                       {"reason", Json(reason)}, {"message", Json(msg)}}));
  std::ofstream(c.term_path + ".kubelet") << msg;
  if (now) {
    kill(-c.pid, SIGKILL);
  } else {
    const Json& g = pr.pod.path("spec.terminationGracePeriodSeconds");
    kill(-c.pid, SIGTERM);
    c.kill_deadline = mono_ms() + (g.is_number() ? (int64_t)(g.as_double() * 1000) : opts_.grace_ms);
  }
}

// One probe: settle a finished execution (consecutive-success / failure counting), start the next
// one when it is due. Returns whether a result was settled.
bool Kubelet::step_probe(ProbeState& ps, ContainerRun& c) {
  bool settled = false;
  if (ps.inflight) {
    const int st = ps.inflight->state.load(std::memory_order_acquire);
    if (st == 0) return false;
    if (st == 1) {
      ps.fails = 0;
      if (++ps.succ >= ps.spec.success_threshold) ps.ok = true;
    } else {
      ps.succ = 0;
      ps.last_message = ps.inflight->message;
      if (++ps.fails >= ps.spec.failure_threshold) ps.ok = false;
    }
    ps.inflight.reset();
    settled = true;
  }
  const int64_t now = mono_ms();
  if (ps.next_ms == 0) ps.next_ms = std::max(now, c.started_mono + ps.spec.initial_delay_ms);
  if (!ps.inflight && now >= ps.next_ms) {
    ps.inflight = launch_probe(ps.spec, c.env);
    ps.next_ms = now + ps.spec.period_ms;
  }
  return settled;
}

void Kubelet::probe_container(PodRun& pr, ContainerRun& c) {
  if (c.state != "running" || c.pid <= 0 || !c.kill_reason.empty()) return;
  if (!c.started) {
    step_probe(c.startup, c);
    if (c.startup.ok) {
      c.started = true;
    } else if (c.startup.fails >= c.startup.spec.failure_threshold) {
      kill_container(pr, c, "Unhealthy", "Startup probe failed: " + c.startup.last_message, false);
      return;
    }
  }
  if (!c.started) {
    c.ready = false;
    return;
  }
  if (c.liveness.spec.enabled()) {
    step_probe(c.liveness, c);
    if (c.liveness.fails >= c.liveness.spec.failure_threshold) {
      kill_container(pr, c, "Unhealthy", "Liveness probe failed: " + c.liveness.last_message, false);
      return;
    }
  }
  if (c.readiness.spec.enabled()) {
    step_probe(c.readiness, c);
    c.ready = c.readiness.ok;
  } else {
    c.ready = true;
  }
}

void Kubelet::check_memory(PodRun& pr) {
  bool any = false;
  for (auto& c : pr.containers) any |= c.mem_limit > 0 && c.pid > 0;
  if (!any) return;
  auto rss = session_rss_bytes();
  for (auto& c : pr.containers) {
    if (c.mem_limit <= 0 || c.pid <= 0 || !c.kill_reason.empty()) continue;
    auto it = rss.find(c.pid);
    const long long used = it == rss.end() ? 0 : it->second;
    c.mem_peak = std::max(c.mem_peak, used);
    if (used > c.mem_limit)
      kill_container(pr, c, "OOMKilled", "memory limit exceeded: resident " + std::to_string(used >> 20) + " MiB > limit " +
                                             std::to_string(c.mem_limit >> 20) + " MiB", true);
  }
}

void Kubelet::reap() {
  // only the containers' own pids: probe threads wait for their exec children themselves
  std::vector<pid_t> pids;
  for (auto& kv : pid_owner_) pids.push_back(kv.first);
  for (pid_t want : pids) {
    int status = 0;
    pid_t pid = waitpid(want, &status, WNOHANG);
    if (pid <= 0) continue;
    auto it = pid_owner_.find(pid);
    if (it == pid_owner_.end()) continue;
    auto pit = pods_.find(it->second.first);
    size_t ci = it->second.second;
    pid_owner_.erase(it);
    if (pit == pods_.end()) continue;
    PodRun& pr = pit->second;
    ContainerRun& c = pr.containers[ci];
    c.pid = -1;
    c.exit_code = WIFEXITED(status) ? WEXITSTATUS(status) : (WIFSIGNALED(status) ? 128 + WTERMSIG(status) : 1);
    c.reason = c.exit_code == 0 ? "Completed" : "Error";
    std::ifstream tf(c.term_path);
    std::string msg((std::istreambuf_iterator<char>(tf)), std::istreambuf_iterator<char>());
    if (msg.find("OOMKilled") != std::string::npos) c.reason = "OOMKilled";
    if (!c.kill_reason.empty()) {
      // killed by this kubelet (memory limit, failed probe): its reason and message win
      std::ifstream kf(c.term_path + ".kubelet");
      std::string km((std::istreambuf_iterator<char>(kf)), std::istreambuf_iterator<char>());
      if (c.kill_reason == "OOMKilled") c.reason = "OOMKilled";
      if (!km.empty()) msg = km + (msg.empty() ? "" : "\n" + msg);
      unlink((c.term_path + ".kubelet").c_str());
      c.kill_reason.clear();
      c.kill_deadline = 0;
    }
    c.ready = false;
    for (ProbeState* ps : {&c.liveness, &c.readiness, &c.startup}) ps->inflight.reset();
    c.finished_at = rfc3339(now_ms());
    c.state = "terminated";
    Json term = Json::object();
    term["exitCode"] = c.exit_code;
    term["reason"] = c.reason;
    term["startedAt"] = c.started_at;
    term["finishedAt"] = c.finished_at;
    if (!msg.empty()) term["message"] = msg.substr(0, 4096);
    c.last_terminated = term;
    std::string policy = pr.pod.path("spec.restartPolicy").str("Always");
    bool restart = !pr.killing && (policy == "Always" || (policy == "OnFailure" && c.exit_code != 0));
    if (restart) {
      int64_t backoff = opts_.restart_backoff_ms << std::min(c.restarts, 10);
      c.next_start_ms = mono_ms() + std::min(backoff, opts_.max_backoff_ms);
      c.waiting_reason = "CrashLoopBackOff";
    } else {
      c.done = true;
    }
    TFK_LOG(Info, "container exited", Json(Json::object_t{{"pod", Json(pr.ns + "/" + pr.name)}, {"container", Json(c.name)},
                                                          {"exitCode", Json(c.exit_code)}, {"reason", Json(c.reason)},
                                                          {"restart", Json(restart)}}));
  }
}

Json Kubelet::build_status(PodRun& pr) {
  Json st = Json::object();
  bool all_done = true, any_failed = false, all_zero = true, any_running = false, all_ready = !pr.containers.empty();
  Json css = Json::array();
  for (auto& c : pr.containers) {
    Json cs = Json::object();
    cs["name"] = c.name;
    cs["restartCount"] = c.restarts;
    cs["ready"] = c.state == "running" && c.ready;
    cs["started"] = c.state == "running" && c.started;
    cs["image"] = "";
    if (c.state == "running") {
      cs["state"]["running"]["startedAt"] = c.started_at;
      any_running = true;
    } else if (c.state == "terminated" && c.done) {
      cs["state"]["terminated"] = c.last_terminated;
    } else {
      cs["state"]["waiting"]["reason"] = c.waiting_reason;
    }
    if (c.last_terminated.is_object() && !(c.state == "terminated" && c.done))
      cs["lastState"]["terminated"] = c.last_terminated;
    css.push_back(cs);
    all_ready = all_ready && c.state == "running" && c.ready;
    if (!c.done) all_done = false;
    if (c.done && c.exit_code != 0) { any_failed = true; all_zero = false; }
  }
  std::string phase = "Pending";
  if (all_done && !pr.containers.empty()) phase = (any_failed || !all_zero) ? "Failed" : "Succeeded";
  else if (any_running || pr.containers.size()) {
    bool started = false;
    for (auto& c : pr.containers) started |= !c.started_at.empty();
    phase = started ? "Running" : "Pending";
  }
  st["phase"] = phase;
  st["hostIP"] = "127.0.0.1";
  st["podIP"] = "127.0.0.1";
  if (!pr.start_time.empty()) st["startTime"] = pr.start_time;
  st["containerStatuses"] = css;
  Json rc = Json::object();
  rc["type"] = "Ready";
  rc["status"] = all_ready ? "True" : "False";
  Json cr = Json::object();
  cr["type"] = "ContainersReady";
  cr["status"] = all_ready ? "True" : "False";
  st["conditions"] = Json(Json::array_t{rc, cr});
  return st;
}

void Kubelet::update_status(PodRun& pr) {
  Json st = build_status(pr);
  std::string s = st.dump();
  if (s == pr.last_status) return;
  Json cur;
  if (!pods_inf_->indexer().get_by_key(pr.ns + "/" + pr.name, &cur)) return;
  if (cur.path("metadata.uid").str() != pr.uid) return;
  Json next = cur.clone();
  next["status"] = st;
  Json out;
  ApiStatus r = client_->update_status("pods", pr.ns, next, &out);
  if (r.ok()) {
    pr.last_status = s;
    pods_inf_->indexer().upsert(pr.ns + "/" + pr.name, out);
  }
}

void Kubelet::sync_once() {
  reap();
  const bool poll_mem = mono_ms() - last_mem_poll_ >= opts_.memory_poll_ms;
  if (poll_mem) last_mem_poll_ = mono_ms();
  std::set<std::string> live;
  for (auto& p : pods_inf_->indexer().list()) {
    if (p.path("spec.nodeName").str() != opts_.node_name) continue;
    std::string uid = p.path("metadata.uid").str();
    live.insert(uid);
    auto it = pods_.find(uid);
    if (it == pods_.end()) {
      std::string phase = p.path("status.phase").str();
      if (phase == "Succeeded" || phase == "Failed") continue;  // already terminal (kubelet restart)
      // A replacement pod with the name of one still terminating (gang restart / resize) waits
      // until the old containers have exited, as the API's graceful deletion guarantees on a real
      // cluster: two incarnations of one rank would fight over its port and checkpoint.
      bool predecessor = false;
      for (auto& kv : pods_)
        if (kv.first != uid && kv.second.name == p.path("metadata.name").str() &&
            kv.second.ns == p.path("metadata.namespace").str())
          for (auto& c : kv.second.containers) predecessor |= c.pid > 0;
      if (predecessor) continue;
      PodRun pr;
      pr.uid = uid;
      pr.ns = p.path("metadata.namespace").str();
      pr.name = p.path("metadata.name").str();
      pr.pod = p;
      pr.start_time = rfc3339(now_ms());
      for (auto& cs : p.path("spec.containers").items()) {
        ContainerRun c;
        c.name = cs.at("name").str();
        pr.containers.push_back(c);
      }
      auto& ref = pods_[uid] = pr;
      std::string logp;
      for (auto& c : ref.containers) {
        start_container(ref, c);
        if (logp.empty() || c.name == "tensorflow") logp = c.log_path;
      }
      Json patch = Json::object();
      patch["metadata"]["annotations"]["tfk.io/log-path"] = logp;
      Json out;
      client_->patch("pods", ref.ns, ref.name, patch, &out);
      update_status(ref);
      continue;
    }
    PodRun& pr = it->second;
    pr.pod = p;
    if (p.path("metadata.deletionTimestamp").is_string() && !pr.killing) {
      pr.killing = true;
      pr.kill_deadline = mono_ms() + opts_.grace_ms;
      kill_pod(pr, SIGTERM);
    }
    // fault injection (once per restart generation)
    const Json& an = p.path("metadata.annotations");
    if (!pr.fault_done && an.has("tfk.io/fault-kill-after-ms") &&
        an.at("tfk.io/fault-generation").str("0") == an.at("tfk.io/restart-generation").str("0")) {
      int64_t after = atoll(an.at("tfk.io/fault-kill-after-ms").str().c_str());
      int sig = atoi(an.at("tfk.io/fault-signal").str("9").c_str());
      for (auto& c : pr.containers)
        if (c.pid > 0 && mono_ms() - c.started_mono >= after) {
          TFK_LOG(Warn, "fault injection: killing container", Json(Json::object_t{{"pod", Json(pr.name)}, {"signal", Json(sig)}}));
          kill(-c.pid, sig);
          pr.fault_done = true;
        }
    }
    for (auto& c : pr.containers)
      if (c.state != "running" && !c.done && !pr.killing && c.next_start_ms > 0 && mono_ms() >= c.next_start_ms) {
        c.restarts++;
        c.next_start_ms = 0;
        start_container(pr, c);
      }
    if (!pr.killing) {
      for (auto& c : pr.containers) {
        probe_container(pr, c);
        if (c.pid > 0 && c.kill_deadline > 0 && mono_ms() > c.kill_deadline) {
          kill(-c.pid, SIGKILL);  // a probe-killed container that ignored SIGTERM
          c.kill_deadline = 0;
        }
      }
      if (poll_mem) check_memory(pr);
    }
    update_status(pr);
  }
  // pods removed from the API (or rebound elsewhere): stop their containers
  for (auto it = pods_.begin(); it != pods_.end();) {
    PodRun& pr = it->second;
    if (!live.count(it->first) && !pr.killing) {
      pr.killing = true;
      pr.kill_deadline = mono_ms() + opts_.grace_ms;
      kill_pod(pr, SIGTERM);
    }
    bool alive = false;
    for (auto& c : pr.containers) alive |= c.pid > 0;
    if (pr.killing && alive && mono_ms() > pr.kill_deadline) kill_pod(pr, SIGKILL);
    if (pr.killing && !alive && !live.count(it->first)) {
      remove_tree(opts_.root_dir + "/pods/" + it->first);  // the pod's emptyDir volumes
      it = pods_.erase(it);
    } else {
      ++it;
    }
  }
  if (mono_ms() - last_heartbeat_ > opts_.heartbeat_ms) {
    register_node(true);
    last_heartbeat_ = mono_ms();
  }
}

void Kubelet::run(StopToken& stop) {
  register_node(false);
  last_heartbeat_ = mono_ms();
  pods_inf_->start(stop);
  while (!stop.stopped() && !pods_inf_->wait_for_sync(1000)) {
  }
  TFK_LOG(Info, "kubelet ready", Json(Json::object_t{{"node", Json(opts_.node_name)}, {"gpus", Json(opts_.gpus)}}));
  while (!stop.stopped()) {
    sync_once();
    stop.wait_for(100);
  }
  for (auto& kv : pods_) kill_pod(kv.second, SIGTERM);
  int64_t dl = mono_ms() + opts_.grace_ms;
  while (mono_ms() < dl) {
    reap();
    bool alive = false;
    for (auto& kv : pods_)
      for (auto& c : kv.second.containers) alive |= c.pid > 0;
    if (!alive) break;
    usleep(50000);
  }
  for (auto& kv : pods_) kill_pod(kv.second, SIGKILL);
  reap();
}

}  // namespace tfk
