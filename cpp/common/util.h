// Small shared utilities: logging (text/JSON, glog-style levels), flags, time, random names,
// string helpers, CRC32C (checkpoint format), a stop token.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "json.h"

namespace tfk {

// ------------------------------------------------------------------------------ logging
enum class LogLevel { Debug = 0, Info = 1, Warn = 2, Error = 3 };
struct Logger {
  static Logger& get();
  void set_json(bool j) { json_ = j; }
  void set_level(LogLevel l) { level_ = l; }
  void set_component(const std::string& c) { component_ = c; }
  void log(LogLevel lvl, const std::string& msg, const Json& fields = Json());
  LogLevel level() const { return level_; }

 private:
  std::mutex mu_;
  bool json_ = false;
  LogLevel level_ = LogLevel::Info;
  std::string component_ = "tfk";
};
#define TFK_LOG(lvl, msg, ...) ::tfk::Logger::get().log(::tfk::LogLevel::lvl, (msg), ##__VA_ARGS__)

// ------------------------------------------------------------------------------ flags
// --name=value / --name value / --flag (bool). Unknown flags are an error.
class FlagSet {
 public:
  explicit FlagSet(std::string prog) : prog_(std::move(prog)) {}
  void add_string(const std::string& name, std::string* dst, const std::string& help);
  void add_int(const std::string& name, long long* dst, const std::string& help);
  void add_double(const std::string& name, double* dst, const std::string& help);
  void add_bool(const std::string& name, bool* dst, const std::string& help);
  // Returns false (and fills err) on a bad flag; positional args go to rest().
  bool parse(int argc, char** argv, std::string* err);
  std::string usage() const;
  const std::vector<std::string>& rest() const { return rest_; }
  bool help_requested() const { return help_; }

 private:
  struct F {
    char kind;
    void* dst;
    std::string help;
  };
  std::string prog_;
  std::map<std::string, F> flags_;
  std::vector<std::string> rest_;
  bool help_ = false;
};

// ------------------------------------------------------------------------------ time
inline int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}
inline int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
std::string rfc3339(int64_t ms_since_epoch);
int64_t parse_rfc3339(const std::string& s);  // -1 on error

// ------------------------------------------------------------------------------ strings
std::string rand_string(int n);  // lowercase alnum
std::vector<std::string> split(const std::string& s, char sep);
std::string trim(const std::string& s);
std::string to_lower(std::string s);
bool starts_with(const std::string& s, const std::string& p);
bool ends_with(const std::string& s, const std::string& p);
std::string url_decode(const std::string& s);
std::string url_encode(const std::string& s);
std::map<std::string, std::string> parse_query(const std::string& q);

// ------------------------------------------------------------------------------ crc32c
uint32_t crc32c(const void* data, size_t n, uint32_t init = 0);
inline uint32_t crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
inline uint32_t crc32c_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

// ------------------------------------------------------------------------------ stop token
// Timed condition-variable wait on the system clock (pthread_cond_timedwait). libstdc++'s
// steady-clock wait_for goes through pthread_cond_clockwait, which GCC 11's ThreadSanitizer does
// not intercept: it then loses track of the mutex and reports false double locks and races. The
// wall clock is good enough for these sub-second timeouts.
template <class Pred>
inline bool cv_wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& l, int64_t ms, Pred pred) {
  return cv.wait_until(l, std::chrono::system_clock::now() + std::chrono::milliseconds(ms), pred);
}
inline void cv_wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& l, int64_t ms) {
  cv.wait_until(l, std::chrono::system_clock::now() + std::chrono::milliseconds(ms));
}

class StopToken {
 public:
  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stopped_ = true;
    }
    cv_.notify_all();
  }
  bool stopped() const { return stopped_.load(); }
  // Sleeps up to ms; returns true if stopped.
  bool wait_for(int64_t ms) {
    std::unique_lock<std::mutex> l(mu_);
    cv_wait_ms(cv_, l, ms, [&] { return stopped_.load(); });
    return stopped_.load();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<bool> stopped_{false};
};

// Run fn every period until stopped (wait.Until equivalent; a panicking fn is logged, not fatal).
void until(const std::function<void()>& fn, int64_t period_ms, StopToken& stop);

}  // namespace tfk
