#include "util.h"

#include <cstdio>
#include <cstring>
#include <ctime>
#include <iostream>
#include <random>
#include <thread>

namespace tfk {

Logger& Logger::get() {
  static Logger l;
  return l;
}

void Logger::log(LogLevel lvl, const std::string& msg, const Json& fields) {
  if (lvl < level_) return;
  static const char* names[] = {"debug", "info", "warning", "error"};
  std::string line;
  int64_t t = now_ms();
  if (json_) {
    Json j = fields.is_object() ? fields.clone() : Json::object();
    j["level"] = names[(int)lvl];
    j["msg"] = msg;
    j["time"] = rfc3339(t);
    j["component"] = component_;
    line = j.dump();
  } else {
    line = std::string(1, "DIWE"[(int)lvl]) + rfc3339(t) + " " + component_ + "] " + msg;
    if (fields.is_object())
      for (auto& kv : fields.fields())
        line += " " + kv.first + "=" + (kv.second.is_string() ? kv.second.as_string() : kv.second.dump());
  }
  std::lock_guard<std::mutex> g(mu_);
  std::cerr << line << std::endl;
}

// ------------------------------------------------------------------------------ flags
void FlagSet::add_string(const std::string& n, std::string* d, const std::string& h) { flags_[n] = {'s', d, h}; }
void FlagSet::add_int(const std::string& n, long long* d, const std::string& h) { flags_[n] = {'i', d, h}; }
void FlagSet::add_double(const std::string& n, double* d, const std::string& h) { flags_[n] = {'d', d, h}; }
void FlagSet::add_bool(const std::string& n, bool* d, const std::string& h) { flags_[n] = {'b', d, h}; }

bool FlagSet::parse(int argc, char** argv, std::string* err) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "-h" || a == "--help") { help_ = true; continue; }
    if (!starts_with(a, "-")) { rest_.push_back(a); continue; }
    std::string body = a.substr(a[1] == '-' ? 2 : 1);
    std::string name = body, val;
    bool has_val = false;
    size_t eq = body.find('=');
    if (eq != std::string::npos) { name = body.substr(0, eq); val = body.substr(eq + 1); has_val = true; }
    auto it = flags_.find(name);
    if (it == flags_.end()) { *err = "unknown flag --" + name; return false; }
    F& f = it->second;
    if (f.kind == 'b') {
      bool v = true;
      if (has_val) v = (val == "true" || val == "1" || val == "yes");
      *(bool*)f.dst = v;
      continue;
    }
    if (!has_val) {
      if (i + 1 >= argc) { *err = "flag --" + name + " needs a value"; return false; }
      val = argv[++i];
    }
    try {
      if (f.kind == 's') *(std::string*)f.dst = val;
      else if (f.kind == 'i') *(long long*)f.dst = std::stoll(val);
      else if (f.kind == 'd') *(double*)f.dst = std::stod(val);
    } catch (...) {
      *err = "bad value for --" + name + ": " + val;
      return false;
    }
  }
  return true;
}

std::string FlagSet::usage() const {
  std::string u = "usage: " + prog_ + " [flags]\n";
  for (auto& kv : flags_) u += "  --" + kv.first + "  " + kv.second.help + "\n";
  return u;
}

// ------------------------------------------------------------------------------ time
std::string rfc3339(int64_t ms) {
  time_t s = ms / 1000;
  struct tm tmv;
  gmtime_r(&s, &tmv);
  char buf[64];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tmv);
  char out[80];
  snprintf(out, sizeof out, "%s.%03dZ", buf, (int)(ms % 1000));
  return out;
}

int64_t parse_rfc3339(const std::string& s) {
  struct tm tmv;
  memset(&tmv, 0, sizeof tmv);
  int ms = 0;
  if (sscanf(s.c_str(), "%d-%d-%dT%d:%d:%d", &tmv.tm_year, &tmv.tm_mon, &tmv.tm_mday, &tmv.tm_hour, &tmv.tm_min,
             &tmv.tm_sec) != 6)
    return -1;
  size_t dot = s.find('.');
  if (dot != std::string::npos) ms = atoi(s.substr(dot + 1, 3).c_str());
  tmv.tm_year -= 1900;
  tmv.tm_mon -= 1;
  return (int64_t)timegm(&tmv) * 1000 + ms;
}

// ------------------------------------------------------------------------------ strings
std::string rand_string(int n) {
  static thread_local std::mt19937_64 rng(std::random_device{}() ^ (uint64_t)now_ms());
  static const char* al = "bcdfghjklmnpqrstvwxz2456789";
  std::string s;
  for (int i = 0; i < n; ++i) s += al[rng() % strlen(al)];
  return s;
}
std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) { out.push_back(cur); cur.clear(); }
    else cur += c;
  }
  out.push_back(cur);
  return out;
}
std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}
std::string to_lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}
bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
bool ends_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}
std::string url_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      o += (char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16);
      i += 2;
    } else if (s[i] == '+') {
      o += ' ';
    } else {
      o += s[i];
    }
  }
  return o;
}
std::string url_encode(const std::string& s) {
  std::string o;
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') o += (char)c;
    else {
      char b[4];
      snprintf(b, sizeof b, "%%%02X", c);
      o += b;
    }
  }
  return o;
}
std::map<std::string, std::string> parse_query(const std::string& q) {
  std::map<std::string, std::string> m;
  for (auto& kv : split(q, '&')) {
    if (kv.empty()) continue;
    size_t eq = kv.find('=');
    if (eq == std::string::npos) m[url_decode(kv)] = "";
    else m[url_decode(kv.substr(0, eq))] = url_decode(kv.substr(eq + 1));
  }
  return m;
}

// ------------------------------------------------------------------------------ crc32c (Castagnoli)
static uint32_t g_crc_table[8][256];
static std::once_flag g_crc_once;
static void crc_init() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_crc_table[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i)
      g_crc_table[t][i] = (g_crc_table[t - 1][i] >> 8) ^ g_crc_table[0][g_crc_table[t - 1][i] & 0xff];
}
uint32_t crc32c(const void* data, size_t n, uint32_t init) {
  std::call_once(g_crc_once, crc_init);
  const uint8_t* p = (const uint8_t*)data;
  uint32_t c = ~init;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    v ^= c;
    c = g_crc_table[7][v & 0xff] ^ g_crc_table[6][(v >> 8) & 0xff] ^ g_crc_table[5][(v >> 16) & 0xff] ^
        g_crc_table[4][(v >> 24) & 0xff] ^ g_crc_table[3][(v >> 32) & 0xff] ^ g_crc_table[2][(v >> 40) & 0xff] ^
        g_crc_table[1][(v >> 48) & 0xff] ^ g_crc_table[0][(v >> 56) & 0xff];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_crc_table[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return ~c;
}

void until(const std::function<void()>& fn, int64_t period_ms, StopToken& stop) {
  while (!stop.stopped()) {
    try {
      fn();
    } catch (const std::exception& e) {
      TFK_LOG(Error, std::string("recovered from exception in loop: ") + e.what());
    }
    if (stop.wait_for(period_ms)) break;
  }
}

}  // namespace tfk
