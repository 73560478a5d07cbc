// Minimal test harness shared by the tfk-unit-tests translation units: TEST(name) registers a
// case, CHECK/CHECK_EQ throw a Failure; run_all(argc, argv) runs the cases whose name contains
// argv[1] and returns 0 only if all pass.
//
// Hang diagnosis: every case prints "[ RUN ] name" before it starts, and a
// deadline thread watches it; a case still running after TFK_TEST_DEADLINE_S seconds (default 120)
// prints "[HANG] name", dumps every thread's stack (gdb attached to this process, batch mode) and
// aborts, so a stalled multi-threaded case names itself and its lock holders instead of hitting the
// caller's outer timeout silently.
#pragma once
#include <dirent.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tfk_test {
struct TestCase {
  const char* name;
  std::function<void()> fn;
};
inline std::vector<TestCase>& registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
struct Failure {
  std::string msg;
};

// Print every thread's backtrace of this process: each thread is sent SIGUSR2 (tgkill over
// /proc/self/task) and writes its own frames with backtrace_symbols_fd -- no debugger needed (the
// binary links with -rdynamic so frames carry function names). gdb, when installed, is tried first.
inline void stack_signal_handler(int) {
  void* fr[64];
  char hdr[64];
  const int n = backtrace(fr, 64);
  const int len = snprintf(hdr, sizeof hdr, "--- thread %ld ---\n", (long)syscall(SYS_gettid));
  if (write(2, hdr, len) < 0) return;
  backtrace_symbols_fd(fr, n, 2);
}

inline void dump_all_stacks() {
  fflush(stdout);
  fflush(stderr);
  if (system("command -v gdb >/dev/null 2>&1") == 0) {
    char cmd[160];
    snprintf(cmd, sizeof cmd, "gdb -p %d -batch -nx -ex 'set pagination off' -ex 'thread apply all bt' 1>&2",
             (int)getpid());
    if (system(cmd) == 0) return;
  }
  struct sigaction sa {};
  sa.sa_handler = stack_signal_handler;
  sigaction(SIGUSR2, &sa, nullptr);
  const long self = syscall(SYS_gettid);
  if (DIR* d = opendir("/proc/self/task")) {
    while (dirent* e = readdir(d)) {
      const long tid = atol(e->d_name);
      if (tid <= 0 || tid == self) continue;
      syscall(SYS_tgkill, (long)getpid(), tid, SIGUSR2);
      usleep(50000);  // one thread's frames at a time
    }
    closedir(d);
  }
  usleep(200000);
}

// One deadline per running case; fires dump + abort when the case overruns.
class Deadline {
 public:
  explicit Deadline(double secs) : secs_(secs), th_([this] { loop(); }) {}
  ~Deadline() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void arm(const char* name) {
    std::lock_guard<std::mutex> g(mu_);
    name_ = name;
    due_ = std::chrono::system_clock::now() + std::chrono::milliseconds((long long)(secs_ * 1000));
    armed_ = true;
    cv_.notify_all();
  }
  void disarm() {
    std::lock_guard<std::mutex> g(mu_);
    armed_ = false;
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      if (!armed_) {
        cv_.wait(lk);
        continue;
      }
      if (cv_.wait_until(lk, due_) == std::cv_status::timeout && armed_ && !stop_ &&
          std::chrono::system_clock::now() >= due_) {
        fprintf(stderr, "[HANG] %s exceeded %.0f s; thread stacks follow\n", name_, secs_);
        printf("[HANG] %s\n", name_);
        lk.unlock();
        dump_all_stacks();
        abort();
      }
    }
  }
  double secs_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false, armed_ = false;
  const char* name_ = "";
  // system_clock: a steady-clock wait_until is pthread_cond_clockwait, which GCC 11's TSan does not
  // intercept (it then reports the waiter as still holding mu_; cpp/common/util.h)
  std::chrono::system_clock::time_point due_;
  std::thread th_;
};

inline int run_all(int argc, char** argv) {
  const char* filter = argc > 1 ? argv[1] : "";
  int pass = 0, fail = 0;
  const char* dl = getenv("TFK_TEST_DEADLINE_S");
  Deadline deadline(dl ? atof(dl) : 120.0);
  for (auto& t : registry()) {
    if (*filter && !strstr(t.name, filter)) continue;
    auto t0 = std::chrono::steady_clock::now();
    printf("[ RUN ] %s\n", t.name);
    fflush(stdout);
    deadline.arm(t.name);
    try {
      t.fn();
      pass++;
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      printf("[ OK ] %s (%.0f ms)\n", t.name, ms);
    } catch (const Failure& f) {
      fail++;
      printf("[FAIL] %s: %s\n", t.name, f.msg.c_str());
    } catch (const std::exception& e) {
      fail++;
      printf("[FAIL] %s: exception %s\n", t.name, e.what());
    }
    deadline.disarm();
    fflush(stdout);
  }
  printf("%d passed, %d failed\n", pass, fail);
  return fail ? 1 : 0;
}
}  // namespace tfk_test

#define TEST(name)                                        \
  static void test_##name();                              \
  static tfk_test::Reg reg_##name(#name, test_##name);    \
  static void test_##name()
#define CHECK(cond)                                                                                             \
  do {                                                                                                          \
    if (!(cond)) throw tfk_test::Failure{std::string(__FILE__) + ":" + std::to_string(__LINE__) + ": " #cond}; \
  } while (0)
#define CHECK_EQ(a, b)                                                                                       \
  do {                                                                                                       \
    auto _a = (a);                                                                                           \
    auto _b = (b);                                                                                           \
    if (!(_a == _b))                                                                                         \
      throw tfk_test::Failure{std::string(__FILE__) + ":" + std::to_string(__LINE__) + ": " #a " == " #b " failed"}; \
  } while (0)
