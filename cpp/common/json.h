// Minimal, dependency-free JSON value for the tfk control plane (apiserver storage, REST bodies,
// TF_CONFIG). Objects keep keys sorted (std::map) so serialisation is deterministic.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace tfk {

class Json {
 public:
  enum Type { Null, Bool, Number, String, Array, Object };
  using array_t = std::vector<Json>;
  using object_t = std::map<std::string, Json>;

  Json() : t_(Null) {}
  Json(std::nullptr_t) : t_(Null) {}
  // Value semantics with DEEP copies: no storage is ever shared between two Json values, so a
  // copy handed to another thread (informer caches, watch fan-out, work queues) can never race
  // with its source (copy-on-write sharing is a data race under the C++ memory model: the
  // use_count() probe has no acquire ordering). Moves stay O(1).
  Json(const Json& o);
  Json(Json&& o) noexcept = default;
  Json& operator=(const Json& o);
  Json& operator=(Json&& o) noexcept = default;
  Json(bool b) : t_(Bool), b_(b) {}
  Json(int v) : t_(Number), n_(v) {}
  Json(long v) : t_(Number), n_((double)v) {}
  Json(long long v) : t_(Number), n_((double)v) {}
  Json(unsigned v) : t_(Number), n_(v) {}
  Json(unsigned long v) : t_(Number), n_((double)v) {}
  Json(double v) : t_(Number), n_(v) {}
  Json(const char* s) : t_(String), s_(s) {}
  Json(const std::string& s) : t_(String), s_(s) {}
  Json(std::string&& s) : t_(String), s_(std::move(s)) {}
  Json(const array_t& a) : t_(Array), a_(std::make_shared<array_t>(a)) {}
  Json(const object_t& o) : t_(Object), o_(std::make_shared<object_t>(o)) {}

  static Json array() { return Json(array_t{}); }
  static Json object() { return Json(object_t{}); }
  static Json parse(const std::string& text);  // throws std::runtime_error

  Type type() const { return t_; }
  bool is_null() const { return t_ == Null; }
  bool is_bool() const { return t_ == Bool; }
  bool is_number() const { return t_ == Number; }
  bool is_string() const { return t_ == String; }
  bool is_array() const { return t_ == Array; }
  bool is_object() const { return t_ == Object; }

  bool as_bool(bool d = false) const { return t_ == Bool ? b_ : d; }
  double as_double(double d = 0) const { return t_ == Number ? n_ : d; }
  long long as_int(long long d = 0) const { return t_ == Number ? (long long)n_ : d; }
  const std::string& as_string() const;
  std::string str(const std::string& d = "") const { return t_ == String ? s_ : d; }

  // arrays
  size_t size() const;
  Json& operator[](size_t i);
  const Json& operator[](size_t i) const;
  void push_back(const Json& v);
  const array_t& items() const;
  array_t& items_mut();

  // objects (operator[] on a Null converts it to an Object)
  Json& operator[](const std::string& k);
  Json& operator[](const char* k) { return (*this)[std::string(k)]; }
  const Json& at(const std::string& k) const;  // returns a static Null if missing
  bool has(const std::string& k) const;
  void erase(const std::string& k);
  const object_t& fields() const;
  object_t& fields_mut();

  // deep path helpers: get("metadata.name")
  const Json& path(const std::string& dotted) const;

  std::string dump(int indent = -1) const;
  Json clone() const { return *this; }  // copies are deep (kept for call-site clarity)

  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  void ensure_unique();
  void dump_to(std::string& out, int indent, int depth) const;
  Type t_;
  bool b_ = false;
  double n_ = 0;
  std::string s_;
  std::shared_ptr<array_t> a_;
  std::shared_ptr<object_t> o_;
};

std::string json_escape(const std::string& s);

}  // namespace tfk
