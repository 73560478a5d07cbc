#include "http.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
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
    case 415: return "Unsupported Media Type";
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

// ------------------------------------------------------------------------------------ TLS
static std::string ssl_errors() {
  std::string out;
  unsigned long e;
  char buf[256];
  while ((e = ERR_get_error()) != 0) {
    ERR_error_string_n(e, buf, sizeof buf);
    if (!out.empty()) out += "; ";
    out += buf;
  }
  return out.empty() ? "unknown TLS error" : out;
}

static bool load_pem_cert(SSL_CTX* ctx, const TlsOptions& o, std::string* err) {
  if (!o.cert_file.empty()) {
    if (SSL_CTX_use_certificate_chain_file(ctx, o.cert_file.c_str()) != 1) {
      *err = "certificate " + o.cert_file + ": " + ssl_errors();
      return false;
    }
  } else if (!o.cert_data.empty()) {
    BIO* b = BIO_new_mem_buf(o.cert_data.data(), (int)o.cert_data.size());
    X509* x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
    BIO_free(b);
    if (!x || SSL_CTX_use_certificate(ctx, x) != 1) {
      if (x) X509_free(x);
      *err = "certificate data: " + ssl_errors();
      return false;
    }
    X509_free(x);
  } else {
    return true;  // no certificate configured
  }
  if (!o.key_file.empty()) {
    if (SSL_CTX_use_PrivateKey_file(ctx, o.key_file.c_str(), SSL_FILETYPE_PEM) != 1) {
      *err = "private key " + o.key_file + ": " + ssl_errors();
      return false;
    }
  } else if (!o.key_data.empty()) {
    BIO* b = BIO_new_mem_buf(o.key_data.data(), (int)o.key_data.size());
    EVP_PKEY* k = PEM_read_bio_PrivateKey(b, nullptr, nullptr, nullptr);
    BIO_free(b);
    if (!k || SSL_CTX_use_PrivateKey(ctx, k) != 1) {
      if (k) EVP_PKEY_free(k);
      *err = "private key data: " + ssl_errors();
      return false;
    }
    EVP_PKEY_free(k);
  } else {
    *err = "certificate given without a private key";
    return false;
  }
  if (SSL_CTX_check_private_key(ctx) != 1) {
    *err = "certificate and private key do not match";
    return false;
  }
  return true;
}

std::shared_ptr<TlsContext> TlsContext::client(const TlsOptions& o, std::string* err) {
  auto t = std::shared_ptr<TlsContext>(new TlsContext());
  t->opt_ = o;
  t->ctx_ = SSL_CTX_new(TLS_client_method());
  if (!t->ctx_) { *err = ssl_errors(); return nullptr; }
  SSL_CTX_set_min_proto_version(t->ctx_, TLS1_2_VERSION);
  if (o.insecure_skip_verify) {
    SSL_CTX_set_verify(t->ctx_, SSL_VERIFY_NONE, nullptr);
  } else {
    SSL_CTX_set_verify(t->ctx_, SSL_VERIFY_PEER, nullptr);
    if (!o.ca_file.empty()) {
      if (SSL_CTX_load_verify_locations(t->ctx_, o.ca_file.c_str(), nullptr) != 1) {
        *err = "CA file " + o.ca_file + ": " + ssl_errors();
        return nullptr;
      }
    } else if (!o.ca_data.empty()) {
      BIO* b = BIO_new_mem_buf(o.ca_data.data(), (int)o.ca_data.size());
      X509_STORE* st = SSL_CTX_get_cert_store(t->ctx_);
      int n = 0;
      while (X509* x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr)) {
        X509_STORE_add_cert(st, x);
        X509_free(x);
        ++n;
      }
      ERR_clear_error();  // PEM_read end-of-data
      BIO_free(b);
      if (n == 0) { *err = "CA data holds no PEM certificate"; return nullptr; }
    } else {
      SSL_CTX_set_default_verify_paths(t->ctx_);
    }
  }
  if (!load_pem_cert(t->ctx_, o, err)) return nullptr;
  return t;
}

std::shared_ptr<TlsContext> TlsContext::server(const TlsOptions& o, std::string* err) {
  if (o.cert_file.empty() && o.cert_data.empty()) { *err = "TLS server needs a certificate"; return nullptr; }
  auto t = std::shared_ptr<TlsContext>(new TlsContext());
  t->opt_ = o;
  t->ctx_ = SSL_CTX_new(TLS_server_method());
  if (!t->ctx_) { *err = ssl_errors(); return nullptr; }
  SSL_CTX_set_min_proto_version(t->ctx_, TLS1_2_VERSION);
  if (!load_pem_cert(t->ctx_, o, err)) return nullptr;
  return t;
}

TlsContext::~TlsContext() {
  if (ctx_) SSL_CTX_free(ctx_);
}

// ----------------------------------------------------------------------------------- Conn
Conn::~Conn() {
  if (ssl_) {
    SSL_shutdown(ssl_);
    SSL_free(ssl_);
  }
  if (fd_ >= 0) ::close(fd_);
}

bool Conn::peer_closed() const {
  pollfd p{fd_, POLLIN | POLLRDHUP, 0};
  if (poll(&p, 1, 0) <= 0) return false;
  if (p.revents & (POLLRDHUP | POLLHUP | POLLERR)) return true;
  if (ssl_) return false;  // pending TLS records are not EOF
  char b;
  ssize_t n = ::recv(fd_, &b, 1, MSG_PEEK | MSG_DONTWAIT);
  return n == 0;
}

void Conn::shutdown() {
  if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
}

int Conn::read_some(char* buf, int cap, int poll_ms) {
  if (!(ssl_ && SSL_pending(ssl_) > 0)) {
    pollfd p{fd_, POLLIN, 0};
    int r = poll(&p, 1, poll_ms);
    if (r == 0) return 0;
    if (r < 0) return errno == EINTR ? 0 : -1;
  }
  if (ssl_) {
    int n = SSL_read(ssl_, buf, cap);
    if (n > 0) return n;
    int e = SSL_get_error(ssl_, n);
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return 0;  // partial record
    return -1;
  }
  ssize_t n = ::recv(fd_, buf, (size_t)cap, 0);
  if (n < 0 && (errno == EINTR || errno == EAGAIN)) return 0;
  return n > 0 ? (int)n : -1;
}

bool Conn::send_all(const std::string& s) {
  std::lock_guard<std::mutex> g(wmu_);
  size_t off = 0;
  while (off < s.size()) {
    if (ssl_) {
      int n = SSL_write(ssl_, s.data() + off, (int)std::min<size_t>(s.size() - off, 1 << 30));
      if (n <= 0) return false;
      off += (size_t)n;
    } else {
      ssize_t n = ::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) return false;
      off += (size_t)n;
    }
  }
  return true;
}

// Read until "\r\n\r\n"; returns false on EOF/error/timeout. Leftover bytes stay in buf.
// got_bytes (optional): set when any byte arrived (distinguishes a stale keep-alive socket).
static bool read_headers(Conn& c, std::string& buf, std::string& head, int timeout_ms, std::atomic<bool>* stop,
                         bool* got_bytes = nullptr) {
  while (true) {
    size_t pos = buf.find("\r\n\r\n");
    if (pos != std::string::npos) {
      head = buf.substr(0, pos);
      buf.erase(0, pos + 4);
      return true;
    }
    char tmp[8192];
    int n = c.read_some(tmp, sizeof tmp, 200);
    if (stop && stop->load()) return false;
    if (n == 0) {
      timeout_ms -= 200;
      if (timeout_ms <= 0) return false;
      continue;
    }
    if (n < 0) return false;
    if (got_bytes) *got_bytes = true;
    buf.append(tmp, (size_t)n);
    if (buf.size() > (1u << 20)) return false;
  }
}

static bool read_n(Conn& c, std::string& buf, size_t n, int timeout_ms) {
  int waited = 0;
  while (buf.size() < n) {
    char tmp[65536];
    int k = c.read_some(tmp, sizeof tmp, 200);
    if (k < 0) return false;
    if (k == 0) {
      waited += 200;
      if (waited >= timeout_ms) return false;
      continue;
    }
    waited = 0;
    buf.append(tmp, (size_t)k);
  }
  return true;
}

// ------------------------------------------------------------------------------ server side
void ResponseWriter::respond(int status, const std::string& body, const std::string& ct) {
  if (responded_) return;
  responded_ = true;
  std::string h = "HTTP/1.1 " + std::to_string(status) + " " + http_status_text(status) + "\r\n";
  h += "Content-Type: " + ct + "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n";
  c_->send_all(h + body);
}

bool ResponseWriter::start_stream(int status, const std::string& ct) {
  responded_ = streaming_ = true;
  std::string h = "HTTP/1.1 " + std::to_string(status) + " " + http_status_text(status) + "\r\n";
  h += "Content-Type: " + ct + "\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n";
  return c_->send_all(h);
}

bool ResponseWriter::write_chunk(const std::string& d) {
  if (d.empty()) return true;
  char hex[32];
  snprintf(hex, sizeof hex, "%zx\r\n", d.size());
  return c_->send_all(std::string(hex) + d + "\r\n");
}

void ResponseWriter::end_stream() { c_->send_all("0\r\n\r\n"); }

bool ResponseWriter::alive() const { return !(stopping_ && stopping_->load()) && !c_->peer_closed(); }

HttpServer::~HttpServer() { stop(); }

bool HttpServer::enable_tls(const TlsOptions& o, std::string* err) {
  tls_ = TlsContext::server(o, err);
  return tls_ != nullptr;
}

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
  // Connection threads are detached and touch this object until they exit. Shut their sockets down
  // so a thread blocked in send() to a watch client that stopped reading, or in SSL_read() on a
  // partial record, returns at once; idle keep-alive reads poll the stop flag every 200 ms and
  // handlers poll ResponseWriter::alive(). Accepted sockets also carry send/receive timeouts, so
  // every blocking call is bounded even without the shutdown.
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  while (active_.load() > 0) usleep(5000);
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
    if (active_.load() >= max_conns_) {
      // every connection owns a thread (watches are long-lived): shed load instead of exhausting
      // threads/fds; clients retry (informers relist with backoff)
      static const char k503[] = "HTTP/1.1 503 Service Unavailable\r\nContent-Length: 0\r\nConnection: close\r\n\r\n";
      if (!tls_) {
        ssize_t wr = ::send(fd, k503, sizeof(k503) - 1, MSG_NOSIGNAL);
        (void)wr;
      }
      ::close(fd);
      rejected_++;
      continue;
    }
    active_++;
    accepted_++;
    std::thread([this, fd, peer] {
      handle_conn(fd, peer);
      active_--;
    }).detach();
  }
}

// Per-socket I/O bounds: a peer that stops reading fails send() after kSendTimeoutS instead of
// blocking its thread forever; SSL_read on a partial TLS record returns WANT_READ after
// kRecvSliceMs (read_some() treats that as "no data yet" and the caller re-checks its stop flag).
static constexpr int kSendTimeoutS = 10;
static constexpr int kRecvSliceMs = 1000;

static void set_io_timeouts(int fd, int send_s, int recv_ms) {
  timeval sv{send_s, 0};
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &sv, sizeof sv);
  timeval rv{recv_ms / 1000, (recv_ms % 1000) * 1000};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &rv, sizeof rv);
}

void HttpServer::handle_conn(int fd, std::string peer) {
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    conn_fds_.insert(fd);
  }
  // drop the fd from conn_fds_ BEFORE it is closed, so stop() never shuts down a reused fd number
  auto untrack = [this, fd] {
    std::lock_guard<std::mutex> g(conns_mu_);
    conn_fds_.erase(fd);
  };
  if (stopping_) {  // raced with stop(): it may have swept conn_fds_ before the insert
    untrack();
    ::close(fd);
    return;
  }
  SSL* ssl = nullptr;
  if (tls_) {
    ssl = SSL_new(tls_->ctx());
    SSL_set_fd(ssl, fd);
    timeval tv{10, 0};  // bound the handshake on a silent peer
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    if (SSL_accept(ssl) != 1) {
      ERR_clear_error();
      SSL_free(ssl);
      untrack();
      ::close(fd);
      return;
    }
  }
  set_io_timeouts(fd, kSendTimeoutS, kRecvSliceMs);
  Conn conn(fd, ssl);
  std::string buf;
  while (!stopping_) {
    std::string head;
    if (!read_headers(conn, buf, head, 120000, &stopping_)) break;
    HttpRequest req;
    req.peer = peer;
    req.tls = ssl != nullptr;
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
    if (!read_n(conn, buf, clen, 30000)) break;
    req.body = buf.substr(0, clen);
    buf.erase(0, clen);
    ResponseWriter w(&conn, &stopping_);
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
  conn.shutdown();
  untrack();  // ~Conn closes the fd right after
}

// ----------------------------------------------------------------------------------- client
bool parse_endpoint(const std::string& url, Endpoint* ep) {
  std::string u = url;
  ep->https = false;
  ep->port = 80;
  if (starts_with(u, "https://")) { ep->https = true; ep->port = 443; u = u.substr(8); }
  else if (starts_with(u, "http://")) u = u.substr(7);
  size_t slash = u.find('/');
  if (slash != std::string::npos) u = u.substr(0, slash);
  if (!u.empty() && u[0] == '[') {  // [v6]:port
    size_t e = u.find(']');
    if (e == std::string::npos) return false;
    ep->host = u.substr(1, e - 1);
    if (e + 1 < u.size() && u[e + 1] == ':') ep->port = atoi(u.substr(e + 2).c_str());
    return !ep->host.empty() && ep->port > 0;
  }
  size_t c = u.rfind(':');
  if (c == std::string::npos) { ep->host = u; return !u.empty(); }
  ep->host = u.substr(0, c);
  ep->port = atoi(u.substr(c + 1).c_str());
  return !ep->host.empty() && ep->port > 0;
}

bool parse_url(const std::string& url, std::string* host, int* port) {
  Endpoint ep;
  if (!parse_endpoint(url, &ep)) return false;
  *host = ep.host;
  *port = ep.port;
  return true;
}

HttpClient::HttpClient(std::string host, int port, int timeout_ms)
    : host_(std::move(host)), port_(port), timeout_ms_(timeout_ms), pool_(std::make_shared<Pool>()) {}

HttpClient::HttpClient(const Endpoint& ep, std::shared_ptr<TlsContext> tls, int timeout_ms)
    : host_(ep.host), port_(ep.port), timeout_ms_(timeout_ms), tls_(ep.https ? std::move(tls) : nullptr),
      pool_(std::make_shared<Pool>()) {
  if (ep.https && !tls_) {
    std::string err;
    TlsOptions o;
    o.enabled = true;
    tls_ = TlsContext::client(o, &err);
    if (!tls_) throw std::runtime_error("TLS client: " + err);
  }
}

std::unique_ptr<Conn> HttpClient::dial(std::string* err) {
  ignore_sigpipe();
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  std::string h = host_ == "localhost" ? "127.0.0.1" : host_;
  if (getaddrinfo(h.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res) {
    if (err) *err = "resolve failed: " + host_;
    return nullptr;
  }
  int fd = -1;
  std::string last;
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype, a->ai_protocol);
    if (fd < 0) { last = strerror(errno); continue; }
    if (::connect(fd, a->ai_addr, a->ai_addrlen) == 0) break;
    last = strerror(errno);
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) {
    if (err) *err = "connect " + host_ + ":" + std::to_string(port_) + ": " + last;
    return nullptr;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  pool_->connects++;
  if (!tls_) return std::unique_ptr<Conn>(new Conn(fd, nullptr));
  SSL* ssl = SSL_new(tls_->ctx());
  SSL_set_fd(ssl, fd);
  const std::string& sni = tls_->options().server_name.empty() ? host_ : tls_->options().server_name;
  in6_addr tmp6;
  in_addr tmp4;
  bool is_ip = inet_pton(AF_INET, sni.c_str(), &tmp4) == 1 || inet_pton(AF_INET6, sni.c_str(), &tmp6) == 1;
  if (!is_ip) SSL_set_tlsext_host_name(ssl, sni.c_str());
  if (!tls_->options().insecure_skip_verify) {
    X509_VERIFY_PARAM* vp = SSL_get0_param(ssl);
    if (is_ip) X509_VERIFY_PARAM_set1_ip_asc(vp, sni.c_str());
    else X509_VERIFY_PARAM_set1_host(vp, sni.c_str(), 0);
  }
  timeval tv{timeout_ms_ / 1000, (timeout_ms_ % 1000) * 1000};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  if (SSL_connect(ssl) != 1) {
    long vr = SSL_get_verify_result(ssl);
    if (err) {
      *err = "TLS handshake with " + host_ + ":" + std::to_string(port_) + " failed: " +
             (vr != X509_V_OK ? std::string(X509_verify_cert_error_string(vr)) : ssl_errors());
    }
    ERR_clear_error();
    SSL_free(ssl);
    ::close(fd);
    return nullptr;
  }
  // Keep SSL_read bounded after the handshake: a server that stalls mid-record (or sends only
  // non-data records such as TLS 1.3 session tickets) yields WANT_READ, which read_some() reports
  // as "no data yet", so timeouts and RestWatch's stop flag keep working over HTTPS.
  SSL_clear_mode(ssl, SSL_MODE_AUTO_RETRY);
  set_io_timeouts(fd, std::max(1, timeout_ms_ / 1000), kRecvSliceMs);
  return std::unique_ptr<Conn>(new Conn(fd, ssl));
}

std::unique_ptr<Conn> HttpClient::take_idle() {
  std::lock_guard<std::mutex> g(pool_->mu);
  while (!pool_->idle.empty()) {
    std::unique_ptr<Conn> c = std::move(pool_->idle.back());
    pool_->idle.pop_back();
    // a peer that closed the idle socket makes it readable (EOF): drop it
    pollfd p{c->fd(), POLLIN, 0};
    if (poll(&p, 1, 0) == 0) return c;
  }
  return nullptr;
}

void HttpClient::put_idle(std::unique_ptr<Conn> c) {
  std::lock_guard<std::mutex> g(pool_->mu);
  if (pool_->idle.size() < 8) pool_->idle.push_back(std::move(c));
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

HttpResponse HttpClient::round_trip(Conn& c, const std::string& wire, bool* reusable, bool* nothing_read) {
  HttpResponse r;
  *reusable = false;
  *nothing_read = true;
  if (!c.send_all(wire)) { r.error = "send failed"; return r; }
  std::string buf, head;
  bool got = false;
  if (!read_headers(c, buf, head, timeout_ms_, nullptr, &got)) {
    *nothing_read = !got;
    r.error = "no response";
    return r;
  }
  *nothing_read = false;
  r.status = parse_status(head, &r.headers);
  bool framed = true;
  auto it = r.headers.find("content-length");
  if (it != r.headers.end()) {
    size_t n = (size_t)atoll(it->second.c_str());
    if (!read_n(c, buf, n, timeout_ms_)) { r.error = "short body"; framed = false; }
    r.body = buf.substr(0, std::min(n, buf.size()));
  } else if (r.headers.count("transfer-encoding")) {
    std::string out;
    framed = false;
    while (true) {
      size_t e;
      bool ok = true;
      while ((e = buf.find("\r\n")) == std::string::npos)
        if (!(ok = read_n(c, buf, buf.size() + 1, timeout_ms_))) break;
      if (!ok) break;
      size_t n = strtoul(buf.substr(0, e).c_str(), nullptr, 16);
      buf.erase(0, e + 2);
      if (n == 0) {
        framed = read_n(c, buf, 2, timeout_ms_);  // trailing CRLF
        break;
      }
      if (!read_n(c, buf, n + 2, timeout_ms_)) break;
      out += buf.substr(0, n);
      buf.erase(0, n + 2);
    }
    r.body = out;
  } else {
    framed = false;  // close-delimited
    while (read_n(c, buf, buf.size() + 1, 2000)) {
    }
    r.body = buf;
  }
  auto ch = r.headers.find("connection");
  bool close = ch != r.headers.end() && to_lower(ch->second) == "close";
  *reusable = framed && !close && r.error.empty();
  return r;
}

HttpResponse HttpClient::request(const std::string& method, const std::string& path, const std::string& body,
                                 const std::map<std::string, std::string>& headers) {
  std::string wire = method + " " + path + " HTTP/1.1\r\nHost: " + host_ + ":" + std::to_string(port_) + "\r\n" +
                     (keepalive_ ? "" : "Connection: close\r\n") + "Content-Length: " + std::to_string(body.size()) +
                     "\r\n";
  bool has_ct = false;
  for (auto& kv : headers) {
    wire += kv.first + ": " + kv.second + "\r\n";
    if (to_lower(kv.first) == "content-type") has_ct = true;
  }
  if (!has_ct && !body.empty()) wire += "Content-Type: application/json\r\n";
  wire += "\r\n" + body;
  // A pooled connection the server already closed fails before any response byte: retry once on
  // a fresh connection. Only idempotent methods are retried -- the server may have processed a
  // POST/PATCH and dropped the connection before replying, and a blind retry would run it twice
  // (callers of non-idempotent requests handle the failure, e.g. with an AlreadyExists check).
  const bool idempotent = method == "GET" || method == "HEAD" || method == "PUT" || method == "DELETE" ||
                          method == "OPTIONS";
  for (int attempt = 0; attempt < (idempotent ? 2 : 1); ++attempt) {
    std::unique_ptr<Conn> c = keepalive_ ? take_idle() : nullptr;
    bool reused = c != nullptr;
    HttpResponse r;
    if (!c) {
      c = dial(&r.error);
      if (!c) return r;
    } else {
      pool_->reuses++;
    }
    bool reusable = false, nothing = true;
    r = round_trip(*c, wire, &reusable, &nothing);
    if (r.status == 0 && reused && nothing) continue;
    if (reusable && keepalive_) put_idle(std::move(c));
    return r;
  }
  HttpResponse r;
  r.error = "connection reset";
  return r;
}

int HttpClient::stream_lines(const std::string& path, const std::function<bool(const std::string&)>& on_line,
                             std::atomic<bool>* stop, std::string* err,
                             const std::map<std::string, std::string>& headers) {
  std::unique_ptr<Conn> c = dial(err);
  if (!c) return 0;
  std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + host_ + "\r\nConnection: close\r\n";
  for (auto& kv : headers) req += kv.first + ": " + kv.second + "\r\n";
  req += "\r\n";
  if (!c->send_all(req)) return 0;
  std::string buf, head;
  if (!read_headers(*c, buf, head, timeout_ms_, stop)) return 0;
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
    auto it = hdrs.find("content-length");
    if (it != hdrs.end()) read_n(*c, buf, (size_t)atoll(it->second.c_str()), 2000);
    feed(buf + "\n");  // deliver the error body as one line
    return status;
  }
  bool go = true;
  auto fill = [&]() -> int {  // 1 data, 0 idle, -1 closed
    char tmp[65536];
    int k = c->read_some(tmp, sizeof tmp, 200);
    if (k > 0) buf.append(tmp, (size_t)k);
    return k > 0 ? 1 : k;
  };
  while (go && !(stop && stop->load())) {
    if (chunked) {
      size_t e = buf.find("\r\n");
      if (e == std::string::npos) {
        if (fill() < 0) break;
        continue;
      }
      size_t n = strtoul(buf.substr(0, e).c_str(), nullptr, 16);
      if (n == 0) break;
      while (buf.size() < e + 2 + n + 2 && !(stop && stop->load())) {
        if (fill() < 0) { go = false; break; }
      }
      if (!go || buf.size() < e + 2 + n + 2) break;
      go = feed(buf.substr(e + 2, n));
      buf.erase(0, e + 2 + n + 2);
    } else {
      if (!buf.empty()) { go = feed(buf); buf.clear(); }
      if (fill() < 0) break;
    }
  }
  c->shutdown();
  return status;
}

}  // namespace tfk
