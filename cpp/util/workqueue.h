// Rate-limited work queue (client-go workqueue semantics; reference usage k8s-operator.md:87,108,138,
// 155,172,202). Invariants (regression-tested against the reference sample's bugs):
//   * a key is in the queue at most once (dedupe via the dirty set);
//   * a key being processed is never handed to a second worker; an Add during processing is
//     parked in dirty and re-queued by Done (so Done MUST be called on every path);
//   * AddRateLimited = AddAfter(key, limiter.When(key)); Forget resets the per-item backoff;
//   * ShutDown wakes every Get; Get returns quit=true once the queue has drained.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../common/util.h"

namespace tfk {

class RateLimiter {
 public:
  virtual ~RateLimiter() = default;
  virtual int64_t when_ms(const std::string& item) = 0;
  virtual void forget(const std::string& item) = 0;
  virtual int num_requeues(const std::string& item) = 0;
};

// base * 2^failures, capped (client-go: 5ms .. 1000s)
class ItemExponentialFailureRateLimiter : public RateLimiter {
 public:
  ItemExponentialFailureRateLimiter(int64_t base_ms = 5, int64_t max_ms = 1000000) : base_(base_ms), max_(max_ms) {}
  int64_t when_ms(const std::string& item) override {
    std::lock_guard<std::mutex> g(mu_);
    int f = failures_[item]++;
    double d = (double)base_ * std::pow(2.0, f);
    return d > (double)max_ ? max_ : (int64_t)d;
  }
  void forget(const std::string& item) override {
    std::lock_guard<std::mutex> g(mu_);
    failures_.erase(item);
  }
  int num_requeues(const std::string& item) override {
    std::lock_guard<std::mutex> g(mu_);
    auto it = failures_.find(item);
    return it == failures_.end() ? 0 : it->second;
  }

 private:
  std::mutex mu_;
  std::map<std::string, int> failures_;
  int64_t base_, max_;
};

// overall token bucket (client-go: 10 qps, burst 100) -> delay until the next token
class BucketRateLimiter : public RateLimiter {
 public:
  BucketRateLimiter(double qps = 10, int burst = 100) : qps_(qps), tokens_(burst), burst_(burst), last_(mono_ms()) {}
  int64_t when_ms(const std::string&) override {
    std::lock_guard<std::mutex> g(mu_);
    int64_t now = mono_ms();
    tokens_ = std::min<double>(burst_, tokens_ + (now - last_) * qps_ / 1000.0);
    last_ = now;
    tokens_ -= 1.0;  // reserve (may go negative -> wait)
    return tokens_ >= 0 ? 0 : (int64_t)std::ceil(-tokens_ * 1000.0 / qps_);
  }
  void forget(const std::string&) override {}
  int num_requeues(const std::string&) override { return 0; }

 private:
  std::mutex mu_;
  double qps_, tokens_;
  int burst_;
  int64_t last_;
};

class MaxOfRateLimiter : public RateLimiter {
 public:
  explicit MaxOfRateLimiter(std::vector<std::shared_ptr<RateLimiter>> ls) : ls_(std::move(ls)) {}
  int64_t when_ms(const std::string& item) override {
    int64_t m = 0;
    for (auto& l : ls_) m = std::max(m, l->when_ms(item));
    return m;
  }
  void forget(const std::string& item) override {
    for (auto& l : ls_) l->forget(item);
  }
  int num_requeues(const std::string& item) override {
    int m = 0;
    for (auto& l : ls_) m = std::max(m, l->num_requeues(item));
    return m;
  }

 private:
  std::vector<std::shared_ptr<RateLimiter>> ls_;
};

inline std::shared_ptr<RateLimiter> default_controller_rate_limiter() {
  return std::make_shared<MaxOfRateLimiter>(std::vector<std::shared_ptr<RateLimiter>>{
      std::make_shared<ItemExponentialFailureRateLimiter>(5, 1000 * 1000),
      std::make_shared<BucketRateLimiter>(10, 100)});
}

class RateLimitingQueue {
 public:
  explicit RateLimitingQueue(std::string name, std::shared_ptr<RateLimiter> rl = default_controller_rate_limiter())
      : name_(std::move(name)), rl_(std::move(rl)) {
    delay_thr_ = std::thread([this] { delay_loop(); });
  }
  ~RateLimitingQueue() {
    shutdown();
    if (delay_thr_.joinable()) delay_thr_.join();
  }
  RateLimitingQueue(const RateLimitingQueue&) = delete;

  void add(const std::string& item) {
    std::lock_guard<std::mutex> g(mu_);
    add_locked(item);
  }
  size_t len() {
    std::lock_guard<std::mutex> g(mu_);
    return queue_.size();
  }
  // Blocks until an item is available or the queue is shut down and drained.
  bool get(std::string* item) {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return !queue_.empty() || shutting_down_; });
    if (queue_.empty()) return false;  // quit
    *item = queue_.front();
    queue_.pop_front();
    processing_.insert(*item);
    dirty_.erase(*item);
    gets_++;
    return true;
  }
  void done(const std::string& item) {
    std::lock_guard<std::mutex> g(mu_);
    processing_.erase(item);
    if (dirty_.count(item)) {
      queue_.push_back(item);
      cv_.notify_one();
    }
  }
  void add_after(const std::string& item, int64_t delay_ms) {
    if (delay_ms <= 0) { add(item); return; }
    std::lock_guard<std::mutex> g(mu_);
    if (shutting_down_) return;
    waiting_.push({mono_ms() + delay_ms, item});
    delay_cv_.notify_all();
  }
  void add_rate_limited(const std::string& item) {
    retries_++;
    add_after(item, rl_->when_ms(item));
  }
  void forget(const std::string& item) { rl_->forget(item); }
  int num_requeues(const std::string& item) { return rl_->num_requeues(item); }
  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu_);
      shutting_down_ = true;
    }
    cv_.notify_all();
    delay_cv_.notify_all();
  }
  bool shutting_down() {
    std::lock_guard<std::mutex> g(mu_);
    return shutting_down_;
  }
  bool is_processing(const std::string& item) {
    std::lock_guard<std::mutex> g(mu_);
    return processing_.count(item) > 0;
  }
  long long retries() const { return retries_; }
  long long gets() const { return gets_; }
  const std::string& name() const { return name_; }

 private:
  void add_locked(const std::string& item) {
    if (shutting_down_) return;
    if (dirty_.count(item)) return;
    dirty_.insert(item);
    if (processing_.count(item)) return;  // re-queued by done()
    queue_.push_back(item);
    cv_.notify_one();
  }
  void delay_loop() {
    std::unique_lock<std::mutex> l(mu_);
    while (!shutting_down_) {
      if (waiting_.empty()) {
        delay_cv_.wait(l);
        continue;
      }
      int64_t now = mono_ms();
      auto top = waiting_.top();
      if (top.first <= now) {
        waiting_.pop();
        add_locked(top.second);
        continue;
      }
      cv_wait_ms(delay_cv_, l, top.first - now);
    }
  }
  std::string name_;
  std::shared_ptr<RateLimiter> rl_;
  std::mutex mu_;
  std::condition_variable cv_, delay_cv_;
  std::deque<std::string> queue_;
  std::set<std::string> dirty_, processing_;
  using WaitItem = std::pair<int64_t, std::string>;
  std::priority_queue<WaitItem, std::vector<WaitItem>, std::greater<WaitItem>> waiting_;
  bool shutting_down_ = false;
  std::thread delay_thr_;
  std::atomic<long long> retries_{0}, gets_{0};
};

}  // namespace tfk
