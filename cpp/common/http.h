// HTTP/1.1 server + client over POSIX sockets for the tfk control plane (REST + chunked watch
// streams, like the Kubernetes API), with optional TLS (OpenSSL) on both ends:
//   * client: http:// and https:// URLs, CA bundle (file or PEM data), insecure-skip-verify,
//     client certificate auth, bearer tokens (set by the REST layer), keep-alive connection pool
//     shared by copies of one HttpClient (client-go's transport reuses connections the same way);
//   * server: plain or TLS listener, keep-alive, thread per connection.
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "util.h"

typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace tfk {

// TLS material. Empty ca = system default verify paths (unless insecure).
struct TlsOptions {
  bool enabled = false;
  std::string ca_file, ca_data;           // PEM (file path or inline data)
  std::string cert_file, cert_data;       // client cert (client) / serving cert (server)
  std::string key_file, key_data;
  std::string server_name;                // SNI + hostname check (client); default: URL host
  bool insecure_skip_verify = false;
};

// OpenSSL context (client or server role), shared by all connections of an endpoint.
class TlsContext {
 public:
  static std::shared_ptr<TlsContext> client(const TlsOptions& o, std::string* err);
  static std::shared_ptr<TlsContext> server(const TlsOptions& o, std::string* err);
  ~TlsContext();
  SSL_CTX* ctx() const { return ctx_; }
  const TlsOptions& options() const { return opt_; }

 private:
  SSL_CTX* ctx_ = nullptr;
  TlsOptions opt_;
};

// One stream connection: a socket, optionally wrapped in TLS. Owns (and closes) the fd.
class Conn {
 public:
  Conn(int fd, SSL* ssl) : fd_(fd), ssl_(ssl) {}
  ~Conn();
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;
  // Waits up to poll_ms for data; >0 bytes read, 0 = timeout (no data yet), -1 = EOF / error.
  int read_some(char* buf, int cap, int poll_ms);
  bool send_all(const std::string& s);
  void shutdown();
  int fd() const { return fd_; }
  bool tls() const { return ssl_ != nullptr; }
  bool peer_closed() const;  // orderly shutdown / reset seen on the socket (non-blocking probe)

 private:
  int fd_;
  SSL* ssl_;
  std::mutex wmu_;
};

struct HttpRequest {
  std::string method, path, query_string, body;
  std::map<std::string, std::string> query;    // decoded
  std::map<std::string, std::string> headers;  // lower-case keys
  std::string peer;
  bool tls = false;
};

struct HttpResponse {
  int status = 0;
  std::map<std::string, std::string> headers;
  std::string body;
  std::string error;  // transport error (status == 0)
  bool ok() const { return status >= 200 && status < 300; }
};

class ResponseWriter {
 public:
  explicit ResponseWriter(Conn* c, const std::atomic<bool>* server_stopping = nullptr)
      : c_(c), stopping_(server_stopping) {}
  // False once the server is stopping or the peer has closed its end: long-running handlers
  // (watch streams) poll this so HttpServer::stop() can join every connection thread.
  bool alive() const;
  void respond(int status, const std::string& body, const std::string& content_type = "application/json");
  bool start_stream(int status, const std::string& content_type = "application/json");
  bool write_chunk(const std::string& data);  // false once the peer is gone
  void end_stream();
  bool responded() const { return responded_; }
  bool streaming() const { return streaming_; }

 private:
  Conn* c_;
  const std::atomic<bool>* stopping_;
  bool responded_ = false, streaming_ = false;
};

using HttpHandler = std::function<void(const HttpRequest&, ResponseWriter&)>;

class HttpServer {
 public:
  HttpServer() = default;
  ~HttpServer();
  // Serve TLS on this listener (call before listen()). Returns false if the cert/key do not load.
  bool enable_tls(const TlsOptions& o, std::string* err);
  // host "127.0.0.1", port 0 = ephemeral. Returns false on bind failure (err filled: e.g. port in use).
  bool listen(const std::string& host, int port, std::string* err);
  int port() const { return port_; }
  bool tls() const { return tls_ != nullptr; }
  void serve(HttpHandler h);  // spawns the accept thread
  void stop();
  long long connections_accepted() const { return accepted_.load(); }
  long long connections_rejected() const { return rejected_.load(); }
  int connections_active() const { return active_.load(); }
  void set_max_connections(int n) { max_conns_ = n > 0 ? n : 1; }

 private:
  void accept_loop();
  void handle_conn(int fd, std::string peer);
  int lfd_ = -1;
  int port_ = 0;
  std::atomic<bool> stopping_{false};
  std::atomic<int> active_{0};
  std::atomic<long long> accepted_{0};
  std::atomic<long long> rejected_{0};
  int max_conns_ = 4096;
  HttpHandler handler_;
  std::thread accept_thr_;
  std::shared_ptr<TlsContext> tls_;
  std::mutex conns_mu_;
  std::set<int> conn_fds_;  // live connection sockets: stop() shuts them down so no thread stays blocked
};

std::string http_status_text(int code);

// Parsed endpoint URL: scheme://host[:port]
struct Endpoint {
  bool https = false;
  std::string host;
  int port = 80;
};
bool parse_endpoint(const std::string& url, Endpoint* ep);
// "http://host:port" -> (host, port) (scheme optional)
bool parse_url(const std::string& url, std::string* host, int* port);

class HttpClient {
 public:
  HttpClient(std::string host, int port, int timeout_ms = 30000);
  // Full endpoint (https:// uses tls options; `tls` may be null for plain http).
  HttpClient(const Endpoint& ep, std::shared_ptr<TlsContext> tls, int timeout_ms = 30000);
  HttpResponse request(const std::string& method, const std::string& path, const std::string& body = "",
                       const std::map<std::string, std::string>& headers = {});
  // Streams a chunked (or close-delimited) body line by line on a dedicated connection. Returns
  // the status code, or 0 on a transport error. on_line returns false to stop. `stop` (optional)
  // aborts from another thread.
  int stream_lines(const std::string& path, const std::function<bool(const std::string&)>& on_line,
                   std::atomic<bool>* stop = nullptr, std::string* err = nullptr,
                   const std::map<std::string, std::string>& headers = {});
  const std::string& host() const { return host_; }
  int port() const { return port_; }
  bool https() const { return tls_ != nullptr; }
  // Connection reuse statistics (shared by copies of this client).
  long long connects() const { return pool_->connects.load(); }
  long long reuses() const { return pool_->reuses.load(); }
  void set_keepalive(bool on) { keepalive_ = on; }

 private:
  struct Pool {
    std::mutex mu;
    std::vector<std::unique_ptr<Conn>> idle;
    std::atomic<long long> connects{0}, reuses{0};
  };
  std::unique_ptr<Conn> dial(std::string* err);
  std::unique_ptr<Conn> take_idle();
  void put_idle(std::unique_ptr<Conn> c);
  HttpResponse round_trip(Conn& c, const std::string& wire, bool* reusable, bool* nothing_read);
  std::string host_;
  int port_;
  int timeout_ms_;
  bool keepalive_ = true;
  std::shared_ptr<TlsContext> tls_;
  std::shared_ptr<Pool> pool_;
};

}  // namespace tfk
