// Minimal test harness shared by the tfk-unit-tests translation units: TEST(name) registers a
// case, CHECK/CHECK_EQ throw a Failure; run_all(argc, argv) runs the cases whose name contains
// argv[1] and returns 0 only if all pass.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
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

inline int run_all(int argc, char** argv) {
  const char* filter = argc > 1 ? argv[1] : "";
  int pass = 0, fail = 0;
  for (auto& t : registry()) {
    if (*filter && !strstr(t.name, filter)) continue;
    auto t0 = std::chrono::steady_clock::now();
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
