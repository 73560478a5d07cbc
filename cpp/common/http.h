// Minimal HTTP/1.1 server + client over POSIX sockets for the tfk control plane
// (REST + chunked watch streams, like the Kubernetes API). No external dependencies.
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "util.h"

namespace tfk {

struct HttpRequest {
  std::string method, path, query_string, body;
  std::map<std::string, std::string> query;    // decoded
  std::map<std::string, std::string> headers;  // lower-case keys
  std::string peer;
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
  explicit ResponseWriter(int fd) : fd_(fd) {}
  void respond(int status, const std::string& body, const std::string& content_type = "application/json");
  bool start_stream(int status, const std::string& content_type = "application/json");
  bool write_chunk(const std::string& data);  // false once the peer is gone
  void end_stream();
  bool responded() const { return responded_; }
  bool streaming() const { return streaming_; }

 private:
  bool write_all(const std::string& s);
  int fd_;
  bool responded_ = false, streaming_ = false;
};

using HttpHandler = std::function<void(const HttpRequest&, ResponseWriter&)>;

class HttpServer {
 public:
  HttpServer() = default;
  ~HttpServer();
  // host "127.0.0.1", port 0 = ephemeral. Returns false on bind failure (err filled: e.g. port in use).
  bool listen(const std::string& host, int port, std::string* err);
  int port() const { return port_; }
  void serve(HttpHandler h);  // spawns the accept thread
  void stop();

 private:
  void accept_loop();
  void handle_conn(int fd, std::string peer);
  int lfd_ = -1;
  int port_ = 0;
  std::atomic<bool> stopping_{false};
  std::atomic<int> active_{0};
  HttpHandler handler_;
  std::thread accept_thr_;
};

std::string http_status_text(int code);

class HttpClient {
 public:
  HttpClient(std::string host, int port, int timeout_ms = 30000)
      : host_(std::move(host)), port_(port), timeout_ms_(timeout_ms) {}
  HttpResponse request(const std::string& method, const std::string& path, const std::string& body = "",
                       const std::map<std::string, std::string>& headers = {});
  // Streams a chunked (or close-delimited) body line by line. Returns the status code, or 0 on a
  // transport error. on_line returns false to stop. `stop` (optional) aborts from another thread.
  int stream_lines(const std::string& path, const std::function<bool(const std::string&)>& on_line,
                   std::atomic<bool>* stop = nullptr, std::string* err = nullptr);
  const std::string& host() const { return host_; }
  int port() const { return port_; }

 private:
  int connect_fd(std::string* err);
  std::string host_;
  int port_;
  int timeout_ms_;
};

// "http://host:port" -> (host, port)
bool parse_url(const std::string& url, std::string* host, int* port);

}  // namespace tfk
