#include "probe.h"

#include <arpa/inet.h>
#include <dirent.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>

#include "../common/util.h"

namespace tfk {

static int64_t secs_ms(const Json& j, int64_t dflt_ms) {
  return j.is_number() ? (int64_t)(j.as_double() * 1000.0) : dflt_ms;
}

// A probe's port: a number, or the name of one of the container's ports.
static int resolve_port(const Json& port, const Json& container) {
  if (port.is_number()) return (int)port.as_int();
  if (port.is_string()) {
    for (auto& p : container.at("ports").items())
      if (p.at("name").str() == port.str()) return (int)p.at("containerPort").as_int();
    return atoi(port.str().c_str());
  }
  return 0;
}

ProbeSpec ProbeSpec::parse(const Json& s, const Json& container) {
  ProbeSpec p;
  if (!s.is_object()) return p;
  if (s.at("exec").is_object()) {
    p.kind = "exec";
    for (auto& a : s.path("exec.command").items()) p.command.push_back(a.str());
    if (p.command.empty()) p.kind.clear();
  } else if (s.at("tcpSocket").is_object()) {
    p.kind = "tcp";
    p.host = s.path("tcpSocket.host").str("127.0.0.1");
    p.port = resolve_port(s.path("tcpSocket.port"), container);
  } else if (s.at("httpGet").is_object()) {
    p.kind = "http";
    p.host = s.path("httpGet.host").str("127.0.0.1");
    p.port = resolve_port(s.path("httpGet.port"), container);
    p.path = s.path("httpGet.path").str("/");
    if (p.path.empty() || p.path[0] != '/') p.path = "/" + p.path;
  }
  // Kubernetes defaults: period 10 s, timeout 1 s, failureThreshold 3, successThreshold 1
  p.initial_delay_ms = secs_ms(s.at("initialDelaySeconds"), 0);
  p.period_ms = std::max<int64_t>(100, secs_ms(s.at("periodSeconds"), 10000));
  p.timeout_ms = std::max<int64_t>(50, secs_ms(s.at("timeoutSeconds"), 1000));
  p.failure_threshold = std::max<int>(1, (int)s.at("failureThreshold").as_int(3));
  p.success_threshold = std::max<int>(1, (int)s.at("successThreshold").as_int(1));
  return p;
}

// Connected socket to host:port within timeout_ms, or -1 (message in *err).
static int connect_timeout(const std::string& host, int port, int64_t timeout_ms, std::string* err) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  std::string svc = std::to_string(port);
  if (getaddrinfo(host.c_str(), svc.c_str(), &hints, &res) != 0 || !res) {
    *err = "cannot resolve " + host;
    return -1;
  }
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (fd < 0) {
    freeaddrinfo(res);
    *err = "socket: " + std::string(strerror(errno));
    return -1;
  }
  int rc = connect(fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc != 0 && errno != EINPROGRESS) {
    *err = "dial " + host + ":" + svc + ": " + strerror(errno);
    close(fd);
    return -1;
  }
  if (rc != 0) {
    pollfd pf{fd, POLLOUT, 0};
    if (poll(&pf, 1, (int)timeout_ms) != 1) {
      *err = "dial " + host + ":" + svc + ": timeout";
      close(fd);
      return -1;
    }
    int soerr = 0;
    socklen_t l = sizeof soerr;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &l);
    if (soerr != 0) {
      *err = "dial " + host + ":" + svc + ": " + strerror(soerr);
      close(fd);
      return -1;
    }
  }
  return fd;
}

static bool probe_tcp(const ProbeSpec& s, std::string* msg) {
  int fd = connect_timeout(s.host, s.port, s.timeout_ms, msg);
  if (fd < 0) return false;
  close(fd);
  return true;
}

static bool probe_http(const ProbeSpec& s, std::string* msg) {
  const int64_t deadline = mono_ms() + s.timeout_ms;
  int fd = connect_timeout(s.host, s.port, s.timeout_ms, msg);
  if (fd < 0) return false;
  std::string req = "GET " + s.path + " HTTP/1.0\r\nHost: " + s.host + ":" + std::to_string(s.port) +
                    "\r\nUser-Agent: tfk-kubelet-probe\r\nConnection: close\r\n\r\n";
  size_t off = 0;
  while (off < req.size()) {
    pollfd pf{fd, POLLOUT, 0};
    if (poll(&pf, 1, (int)std::max<int64_t>(0, deadline - mono_ms())) != 1) break;
    ssize_t n = send(fd, req.data() + off, req.size() - off, MSG_NOSIGNAL);
    if (n <= 0) break;
    off += (size_t)n;
  }
  std::string resp;
  char buf[512];
  while (resp.find("\r\n") == std::string::npos && resp.size() < 4096) {
    pollfd pf{fd, POLLIN, 0};
    if (poll(&pf, 1, (int)std::max<int64_t>(0, deadline - mono_ms())) != 1) break;
    ssize_t n = recv(fd, buf, sizeof buf, 0);
    if (n <= 0) break;
    resp.append(buf, (size_t)n);
  }
  close(fd);
  // "HTTP/1.x <code> ..."
  size_t sp = resp.find(' ');
  if (resp.compare(0, 5, "HTTP/") != 0 || sp == std::string::npos) {
    *msg = off < req.size() || resp.empty() ? "HTTP probe: no response within timeout" : "HTTP probe: bad status line";
    return false;
  }
  int code = atoi(resp.c_str() + sp + 1);
  if (code >= 200 && code < 400) return true;
  *msg = "HTTP probe failed with statuscode: " + std::to_string(code);
  return false;
}

static bool probe_exec(const ProbeSpec& s, const std::vector<std::string>& env, std::string* msg) {
  // everything the child touches is built before fork (the kubelet is multithreaded)
  std::vector<char*> av, ev;
  for (auto& a : s.command) av.push_back((char*)a.c_str());
  av.push_back(nullptr);
  for (auto& e : env) ev.push_back((char*)e.c_str());
  ev.push_back(nullptr);
  std::string prog = s.command[0];
  if (prog.find('/') == std::string::npos) {
    std::string path = "/usr/bin:/bin";
    for (auto& e : env)
      if (e.compare(0, 5, "PATH=") == 0) path = e.substr(5);
    for (const std::string& dir : split(path, ':')) {
      std::string cand = (dir.empty() ? std::string(".") : dir) + "/" + prog;
      if (access(cand.c_str(), X_OK) == 0) { prog = cand; break; }
    }
  }
  sigset_t none;
  sigemptyset(&none);
  pid_t pid = fork();
  if (pid == 0) {
    sigprocmask(SIG_SETMASK, &none, nullptr);
    signal(SIGPIPE, SIG_DFL);
    setpgid(0, 0);
    int nul = open("/dev/null", O_RDWR);
    if (nul >= 0) { dup2(nul, 0); dup2(nul, 1); dup2(nul, 2); close(nul); }
    execve(prog.c_str(), av.data(), ev.data());
    _exit(127);
  }
  if (pid < 0) {
    *msg = "exec probe: fork failed";
    return false;
  }
  const int64_t deadline = mono_ms() + s.timeout_ms;
  int status = 0;
  while (true) {
    pid_t r = waitpid(pid, &status, WNOHANG);
    if (r == pid) break;
    if (r < 0) { *msg = "exec probe: wait failed"; return false; }
    if (mono_ms() >= deadline) {
      kill(-pid, SIGKILL);
      waitpid(pid, &status, 0);
      *msg = "command timed out after " + std::to_string(s.timeout_ms) + " ms";
      return false;
    }
    usleep(5000);
  }
  if (WIFEXITED(status) && WEXITSTATUS(status) == 0) return true;
  *msg = "command exited with " +
         (WIFEXITED(status) ? std::to_string(WEXITSTATUS(status)) : "signal " + std::to_string(WTERMSIG(status)));
  return false;
}

std::shared_ptr<ProbeSlot> launch_probe(const ProbeSpec& spec, const std::vector<std::string>& env) {
  auto slot = std::make_shared<ProbeSlot>();
  std::thread([slot, spec, env] {
    std::string msg;
    bool ok = spec.kind == "exec" ? probe_exec(spec, env, &msg)
              : spec.kind == "tcp" ? probe_tcp(spec, &msg)
              : spec.kind == "http" ? probe_http(spec, &msg) : true;
    slot->message = msg;
    slot->state.store(ok ? 1 : 2, std::memory_order_release);
  }).detach();
  return slot;
}

long long parse_bytes(const std::string& q_in) {
  std::string q = trim(q_in);
  if (q.empty()) return -1;
  char* end = nullptr;
  double v = strtod(q.c_str(), &end);
  if (end == q.c_str() || !std::isfinite(v) || v < 0) return -1;
  std::string suf(end);
  static const struct { const char* s; double m; } units[] = {
      {"Ki", 1024.0}, {"Mi", 1048576.0}, {"Gi", 1073741824.0}, {"Ti", 1099511627776.0},
      {"k", 1e3}, {"K", 1e3}, {"M", 1e6}, {"G", 1e9}, {"T", 1e12}, {"", 1.0}};
  for (auto& u : units)
    if (suf == u.s) return (long long)(v * u.m);
  return -1;
}

std::map<pid_t, long long> session_rss_bytes() {
  static const long page = sysconf(_SC_PAGESIZE);
  std::map<pid_t, long long> total;
  DIR* d = opendir("/proc");
  if (!d) return total;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    std::ifstream f(std::string("/proc/") + e->d_name + "/stat");
    std::string line;
    if (!std::getline(f, line)) continue;
    // fields after "(comm)": 3 state, 4 ppid, 5 pgrp, 6 session, ..., 24 rss (pages)
    size_t rp = line.rfind(')');
    if (rp == std::string::npos) continue;
    std::istringstream rest(line.substr(rp + 2));
    std::string tok;
    long long session = -1, rss = 0;
    for (int field = 3; rest >> tok; ++field) {
      if (field == 6) session = atoll(tok.c_str());
      if (field == 24) { rss = atoll(tok.c_str()); break; }
    }
    if (session > 0) total[(pid_t)session] += rss * page;
  }
  closedir(d);
  return total;
}

}  // namespace tfk
