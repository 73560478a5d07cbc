#include "http.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

namespace tfk {

std::string http_status_text(int c) {
  switch (c) {
    case 200: return "OK";
    case 201: return "Created";
    case 202: return "Accepted";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

static void ignore_sigpipe() {
  static std::once_flag f;
  std::call_once(f, [] { signal(SIGPIPE, SIG_IGN); });
}

bool ResponseWriter::write_all(const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = ::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return false;
    off += (size_t)n;
  }
  return true;
}

void ResponseWriter::respond(int status, const std::string& body, const std::string& ct) {
  if (responded_) return;
  responded_ = true;
  std::string h = "HTTP/1.1 " + std::to_string(status) + " " + http_status_text(status) + "\r\n";
  h += "Content-Type: " + ct + "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n";
  write_all(h + body);
}

bool ResponseWriter::start_stream(int status, const std::string& ct) {
  responded_ = streaming_ = true;
  std::string h = "HTTP/1.1 " + std::to_string(status) + " " + http_status_text(status) + "\r\n";
  h += "Content-Type: " + ct + "\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n";
  return write_all(h);
}

bool ResponseWriter::write_chunk(const std::string& d) {
  if (d.empty()) return true;
  char hex[32];
  snprintf(hex, sizeof hex, "%zx\r\n", d.size());
  return write_all(std::string(hex) + d + "\r\n");
}

void ResponseWriter::end_stream() { write_all("0\r\n\r\n"); }

HttpServer::~HttpServer() { stop(); }

bool HttpServer::listen(const std::string& host, int port, std::string* err) {
  ignore_sigpipe();
  lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (lfd_ < 0) { *err = strerror(errno); return false; }
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(lfd_, (sockaddr*)&a, sizeof a) < 0) {
    *err = std::string("bind ") + host + ":" + std::to_string(port) + ": " + strerror(errno) +
           (errno == EADDRINUSE ? " (port already in use)" : "");
    ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  if (::listen(lfd_, 256) < 0) { *err = strerror(errno); return false; }
  socklen_t len = sizeof a;
  getsockname(lfd_, (sockaddr*)&a, &len);
  port_ = ntohs(a.sin_port);
  return true;
}

void HttpServer::serve(HttpHandler h) {
  handler_ = std::move(h);
  accept_thr_ = std::thread([this] { accept_loop(); });
}

void HttpServer::stop() {
  if (stopping_.exchange(true)) return;
  if (lfd_ >= 0) {
    ::shutdown(lfd_, SHUT_RDWR);
    ::close(lfd_);
  }
  if (accept_thr_.joinable()) accept_thr_.join();
  for (int i = 0; i < 200 && active_.load() > 0; ++i) usleep(10000);
}

void HttpServer::accept_loop() {
  while (!stopping_) {
    pollfd p{lfd_, POLLIN, 0};
    int r = poll(&p, 1, 200);
    if (r <= 0) continue;
    sockaddr_in a{};
    socklen_t len = sizeof a;
    int fd = ::accept(lfd_, (sockaddr*)&a, &len);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    char ip[64];
    inet_ntop(AF_INET, &a.sin_addr, ip, sizeof ip);
    std::string peer = std::string(ip) + ":" + std::to_string(ntohs(a.sin_port));
    active_++;
    std::thread([this, fd, peer] {
      handle_conn(fd, peer);
      active_--;
    }).detach();
  }
}

// Read until "\r\n\r\n"; returns false on EOF/error. Leftover bytes stay in buf.
static bool read_headers(int fd, std::string& buf, std::string& head, int timeout_ms, std::atomic<bool>* stop) {
  while (true) {
    size_t pos = buf.find("\r\n\r\n");
    if (pos != std::string::npos) {
      head = buf.substr(0, pos);
      buf.erase(0, pos + 4);
      return true;
    }
    pollfd p{fd, POLLIN, 0};
    int r = poll(&p, 1, 200);
    if (stop && stop->load()) return false;
    if (r == 0) {
      timeout_ms -= 200;
      if (timeout_ms <= 0) return false;
      continue;
    }
    if (r < 0) return false;
    char tmp[8192];
    ssize_t n = ::recv(fd, tmp, sizeof tmp, 0);
    if (n <= 0) return false;
    buf.append(tmp, (size_t)n);
    if (buf.size() > (1u << 20)) return false;
  }
}

static bool read_n(int fd, std::string& buf, size_t n, int timeout_ms) {
  while (buf.size() < n) {
    pollfd p{fd, POLLIN, 0};
    int r = poll(&p, 1, timeout_ms);
    if (r <= 0) return false;
    char tmp[65536];
    ssize_t k = ::recv(fd, tmp, sizeof tmp, 0);
    if (k <= 0) return false;
    buf.append(tmp, (size_t)k);
  }
  return true;
}

void HttpServer::handle_conn(int fd, std::string peer) {
  std::string buf;
  while (!stopping_) {
    std::string head;
    if (!read_headers(fd, buf, head, 120000, &stopping_)) break;
    HttpRequest req;
    req.peer = peer;
    auto lines = split(head, '\n');
    if (lines.empty()) break;
    auto first = split(trim(lines[0]), ' ');
    if (first.size() < 2) break;
    req.method = first[0];
    std::string target = first[1];
    size_t q = target.find('?');
    req.path = url_decode(target.substr(0, q));
    if (q != std::string::npos) {
      req.query_string = target.substr(q + 1);
      req.query = parse_query(req.query_string);
    }
    for (size_t i = 1; i < lines.size(); ++i) {
      std::string l = trim(lines[i]);
      size_t c = l.find(':');
      if (c == std::string::npos) continue;
      req.headers[to_lower(trim(l.substr(0, c)))] = trim(l.substr(c + 1));
    }
    size_t clen = 0;
    auto it = req.headers.find("content-length");
    if (it != req.headers.end()) clen = (size_t)atoll(it->second.c_str());
    if (clen > (256u << 20)) break;
    if (!read_n(fd, buf, clen, 30000)) break;
    req.body = buf.substr(0, clen);
    buf.erase(0, clen);
    ResponseWriter w(fd);
    try {
      handler_(req, w);
    } catch (const std::exception& e) {
      if (!w.responded()) w.respond(500, Json(Json::object_t{{"message", Json(std::string(e.what()))}}).dump());
    }
    if (!w.responded()) w.respond(500, "{\"message\":\"no response\"}");
    if (w.streaming()) break;
    auto c = req.headers.find("connection");
    if (c != req.headers.end() && to_lower(c->second) == "close") break;
  }
  ::shutdown(fd, SHUT_RDWR);
  ::close(fd);
}

// ----------------------------------------------------------------------------------- client
bool parse_url(const std::string& url, std::string* host, int* port) {
  std::string u = url;
  if (starts_with(u, "http://")) u = u.substr(7);
  while (!u.empty() && u.back() == '/') u.pop_back();
  size_t c = u.rfind(':');
  if (c == std::string::npos) { *host = u; *port = 80; return !u.empty(); }
  *host = u.substr(0, c);
  *port = atoi(u.substr(c + 1).c_str());
  return !host->empty() && *port > 0;
}

int HttpClient::connect_fd(std::string* err) {
  ignore_sigpipe();
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  std::string h = host_ == "localhost" ? "127.0.0.1" : host_;
  if (getaddrinfo(h.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res) {
    if (err) *err = "resolve failed: " + host_;
    return -1;
  }
  int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  if (fd < 0) { freeaddrinfo(res); if (err) *err = strerror(errno); return -1; }
  if (::connect(fd, res->ai_addr, res->ai_addrlen) < 0) {
    if (err) *err = std::string("connect ") + host_ + ":" + std::to_string(port_) + ": " + strerror(errno);
    ::close(fd);
    freeaddrinfo(res);
    return -1;
  }
  freeaddrinfo(res);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  return fd;
}

static bool send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return false;
    off += (size_t)n;
  }
  return true;
}

static int parse_status(const std::string& head, std::map<std::string, std::string>* hdrs) {
  auto lines = split(head, '\n');
  if (lines.empty()) return 0;
  auto parts = split(trim(lines[0]), ' ');
  int status = parts.size() >= 2 ? atoi(parts[1].c_str()) : 0;
  for (size_t i = 1; i < lines.size(); ++i) {
    std::string l = trim(lines[i]);
    size_t c = l.find(':');
    if (c != std::string::npos) (*hdrs)[to_lower(trim(l.substr(0, c)))] = trim(l.substr(c + 1));
  }
  return status;
}

HttpResponse HttpClient::request(const std::string& method, const std::string& path, const std::string& body,
                                 const std::map<std::string, std::string>& headers) {
  HttpResponse r;
  int fd = connect_fd(&r.error);
  if (fd < 0) return r;
  std::string req = method + " " + path + " HTTP/1.1\r\nHost: " + host_ + ":" + std::to_string(port_) +
                    "\r\nConnection: close\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
  bool has_ct = false;
  for (auto& kv : headers) {
    req += kv.first + ": " + kv.second + "\r\n";
    if (to_lower(kv.first) == "content-type") has_ct = true;
  }
  if (!has_ct && !body.empty()) req += "Content-Type: application/json\r\n";
  req += "\r\n" + body;
  if (!send_all(fd, req)) { r.error = "send failed"; ::close(fd); return r; }
  std::string buf, head;
  if (!read_headers(fd, buf, head, timeout_ms_, nullptr)) { r.error = "no response"; ::close(fd); return r; }
  r.status = parse_status(head, &r.headers);
  auto it = r.headers.find("content-length");
  if (it != r.headers.end()) {
    size_t n = (size_t)atoll(it->second.c_str());
    if (!read_n(fd, buf, n, timeout_ms_)) r.error = "short body";
    r.body = buf.substr(0, n);
  } else if (r.headers.count("transfer-encoding")) {
    // de-chunk fully
    std::string out;
    while (true) {
      size_t e;
      while ((e = buf.find("\r\n")) == std::string::npos)
        if (!read_n(fd, buf, buf.size() + 1, timeout_ms_)) break;
      if (e == std::string::npos) break;
      size_t n = strtoul(buf.substr(0, e).c_str(), nullptr, 16);
      buf.erase(0, e + 2);
      if (n == 0) break;
      if (!read_n(fd, buf, n + 2, timeout_ms_)) break;
      out += buf.substr(0, n);
      buf.erase(0, n + 2);
    }
    r.body = out;
  } else {
    while (read_n(fd, buf, buf.size() + 1, 2000)) {
    }
    r.body = buf;
  }
  ::close(fd);
  return r;
}

int HttpClient::stream_lines(const std::string& path, const std::function<bool(const std::string&)>& on_line,
                             std::atomic<bool>* stop, std::string* err) {
  int fd = connect_fd(err);
  if (fd < 0) return 0;
  std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + host_ + "\r\nConnection: close\r\n\r\n";
  if (!send_all(fd, req)) { ::close(fd); return 0; }
  std::string buf, head;
  if (!read_headers(fd, buf, head, timeout_ms_, stop)) { ::close(fd); return 0; }
  std::map<std::string, std::string> hdrs;
  int status = parse_status(head, &hdrs);
  bool chunked = hdrs.count("transfer-encoding") > 0;
  std::string pending;  // de-chunked bytes not yet split into lines
  auto feed = [&](const std::string& data) -> bool {
    pending += data;
    size_t nl;
    while ((nl = pending.find('\n')) != std::string::npos) {
      std::string line = pending.substr(0, nl);
      pending.erase(0, nl + 1);
      if (!trim(line).empty() && !on_line(line)) return false;
    }
    return true;
  };
  if (status != 200) {
    // deliver the error body as one line
    std::string body = buf;
    feed(body + "\n");
    ::close(fd);
    return status;
  }
  bool go = true;
  while (go && !(stop && stop->load())) {
    if (chunked) {
      size_t e = buf.find("\r\n");
      if (e == std::string::npos) {
        pollfd p{fd, POLLIN, 0};
        int r = poll(&p, 1, 200);
        if (r < 0) break;
        if (r == 0) continue;
        char tmp[65536];
        ssize_t k = ::recv(fd, tmp, sizeof tmp, 0);
        if (k <= 0) break;
        buf.append(tmp, (size_t)k);
        continue;
      }
      size_t n = strtoul(buf.substr(0, e).c_str(), nullptr, 16);
      if (n == 0) break;
      while (buf.size() < e + 2 + n + 2 && !(stop && stop->load())) {
        pollfd p{fd, POLLIN, 0};
        int r = poll(&p, 1, 200);
        if (r < 0) { go = false; break; }
        if (r == 0) continue;
        char tmp[65536];
        ssize_t k = ::recv(fd, tmp, sizeof tmp, 0);
        if (k <= 0) { go = false; break; }
        buf.append(tmp, (size_t)k);
      }
      if (!go || buf.size() < e + 2 + n + 2) break;
      go = feed(buf.substr(e + 2, n));
      buf.erase(0, e + 2 + n + 2);
    } else {
      if (!buf.empty()) { go = feed(buf); buf.clear(); }
      pollfd p{fd, POLLIN, 0};
      int r = poll(&p, 1, 200);
      if (r < 0) break;
      if (r == 0) continue;
      char tmp[65536];
      ssize_t k = ::recv(fd, tmp, sizeof tmp, 0);
      if (k <= 0) break;
      buf.append(tmp, (size_t)k);
    }
  }
  ::shutdown(fd, SHUT_RDWR);
  ::close(fd);
  return status;
}

}  // namespace tfk
