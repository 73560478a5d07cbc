#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace tfk {

static const Json kNull;

const std::string& Json::as_string() const {
  static const std::string empty;
  return t_ == String ? s_ : empty;
}

Json::Json(const Json& o) : t_(o.t_), b_(o.b_), n_(o.n_), s_(o.s_) {
  if (o.a_) a_ = std::make_shared<array_t>(*o.a_);
  if (o.o_) o_ = std::make_shared<object_t>(*o.o_);
}

Json& Json::operator=(const Json& o) {
  if (this != &o) {
    Json tmp(o);
    *this = std::move(tmp);
  }
  return *this;
}

void Json::ensure_unique() {
  if (t_ == Array && a_ && a_.use_count() > 1) a_ = std::make_shared<array_t>(*a_);
  if (t_ == Object && o_ && o_.use_count() > 1) o_ = std::make_shared<object_t>(*o_);
}

size_t Json::size() const {
  if (t_ == Array) return a_->size();
  if (t_ == Object) return o_->size();
  return 0;
}
Json& Json::operator[](size_t i) {
  ensure_unique();
  if (t_ != Array || i >= a_->size()) throw std::out_of_range("json index");
  return (*a_)[i];
}
const Json& Json::operator[](size_t i) const {
  if (t_ != Array || i >= a_->size()) return kNull;
  return (*a_)[i];
}
void Json::push_back(const Json& v) {
  if (t_ == Null) { t_ = Array; a_ = std::make_shared<array_t>(); }
  if (t_ != Array) throw std::runtime_error("push_back on non-array");
  ensure_unique();
  a_->push_back(v);
}
const Json::array_t& Json::items() const {
  static const array_t empty;
  return t_ == Array ? *a_ : empty;
}
Json::array_t& Json::items_mut() {
  if (t_ == Null) { t_ = Array; a_ = std::make_shared<array_t>(); }
  ensure_unique();
  return *a_;
}
Json& Json::operator[](const std::string& k) {
  if (t_ == Null) { t_ = Object; o_ = std::make_shared<object_t>(); }
  if (t_ != Object) throw std::runtime_error("json: key access on non-object");
  ensure_unique();
  return (*o_)[k];
}
const Json& Json::at(const std::string& k) const {
  if (t_ != Object) return kNull;
  auto it = o_->find(k);
  return it == o_->end() ? kNull : it->second;
}
bool Json::has(const std::string& k) const { return t_ == Object && o_->count(k); }
void Json::erase(const std::string& k) {
  if (t_ != Object) return;
  ensure_unique();
  o_->erase(k);
}
const Json::object_t& Json::fields() const {
  static const object_t empty;
  return t_ == Object ? *o_ : empty;
}
Json::object_t& Json::fields_mut() {
  if (t_ == Null) { t_ = Object; o_ = std::make_shared<object_t>(); }
  ensure_unique();
  return *o_;
}
const Json& Json::path(const std::string& dotted) const {
  const Json* cur = this;
  size_t start = 0;
  while (start <= dotted.size()) {
    size_t dot = dotted.find('.', start);
    std::string key = dotted.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    cur = &cur->at(key);
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return *cur;
}

bool Json::operator==(const Json& o) const {
  if (t_ != o.t_) return false;
  switch (t_) {
    case Null: return true;
    case Bool: return b_ == o.b_;
    case Number: return n_ == o.n_;
    case String: return s_ == o.s_;
    case Array: return *a_ == *o.a_;
    case Object: return *o_ == *o.o_;
  }
  return false;
}

std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  return out;
}

static void newline(std::string& out, int indent, int depth) {
  if (indent < 0) return;
  out += '\n';
  out.append((size_t)indent * depth, ' ');
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  switch (t_) {
    case Null: out += "null"; break;
    case Bool: out += b_ ? "true" : "false"; break;
    case Number: {
      if (std::isfinite(n_) && n_ == std::floor(n_) && std::fabs(n_) < 9.007199254740992e15) {
        char buf[32];
        snprintf(buf, sizeof buf, "%lld", (long long)n_);
        out += buf;
      } else if (std::isfinite(n_)) {
        char buf[40];
        snprintf(buf, sizeof buf, "%.17g", n_);
        out += buf;
      } else {
        out += "null";
      }
      break;
    }
    case String: out += '"'; out += json_escape(s_); out += '"'; break;
    case Array: {
      out += '[';
      bool first = true;
      for (auto& v : *a_) {
        if (!first) out += ',';
        first = false;
        newline(out, indent, depth + 1);
        v.dump_to(out, indent, depth + 1);
      }
      if (!a_->empty()) newline(out, indent, depth);
      out += ']';
      break;
    }
    case Object: {
      out += '{';
      bool first = true;
      for (auto& kv : *o_) {
        if (!first) out += ',';
        first = false;
        newline(out, indent, depth + 1);
        out += '"'; out += json_escape(kv.first); out += "\":";
        if (indent >= 0) out += ' ';
        kv.second.dump_to(out, indent, depth + 1);
      }
      if (!o_->empty()) newline(out, indent, depth);
      out += '}';
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

// ----------------------------------------------------------------------------------- parser
namespace {
struct Parser {
  const std::string& s;
  size_t i = 0;
  int depth = 0;
  explicit Parser(const std::string& str) : s(str) {}
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json parse error: ") + what + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if (s.compare(i, n, w) == 0) { i += n; return true; }
    return false;
  }
  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    }
  }
  unsigned hex4() {
    if (i + 4 > s.size()) fail("short \\u escape");
    unsigned v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (true) {
      if (i >= s.size()) fail("unterminated string");
      char c = s[i++];
      if (c == '"') break;
      if (c == '\\') {
        if (i >= s.size()) fail("bad escape");
        char e = s[i++];
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            unsigned cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              i += 2;
              unsigned lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            utf8(out, cp);
            break;
          }
          default: fail("bad escape");
        }
      } else {
        out += c;
      }
    }
    return out;
  }
  Json value() {
    if (++depth > 512) fail("nesting too deep");
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    Json r;
    if (c == '{') {
      ++i;
      r = Json::object();
      ws();
      if (i < s.size() && s[i] == '}') { ++i; --depth; return r; }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (i >= s.size() || s[i] != ':') fail("expected ':'");
        ++i;
        r[k] = value();
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; break; }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      ++i;
      r = Json::array();
      ws();
      if (i < s.size() && s[i] == ']') { ++i; --depth; return r; }
      while (true) {
        r.push_back(value());
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == ']') { ++i; break; }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      r = Json(str());
    } else if (lit("true")) {
      r = Json(true);
    } else if (lit("false")) {
      r = Json(false);
    } else if (lit("null")) {
      r = Json();
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      size_t st = i;
      if (s[i] == '-') ++i;
      while (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                              s[i] == '+' || s[i] == '-'))
        ++i;
      std::string num = s.substr(st, i - st);
      char* end = nullptr;
      double v = strtod(num.c_str(), &end);
      if (!end || *end) fail("bad number");
      r = Json(v);
    } else {
      fail("unexpected character");
    }
    --depth;
    return r;
  }
};
}  // namespace

Json Json::parse(const std::string& text) {
  Parser p(text);
  Json v = p.value();
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

}  // namespace tfk
