#include "yaml.h"

#include <cctype>
#include <cstdlib>
#include <stdexcept>

namespace tfk {

namespace {

struct Line {
  int indent;
  std::string text;  // content with indentation and trailing comment removed
  int no;            // 1-based source line
};

[[noreturn]] void fail(int no, const std::string& msg) {
  throw std::runtime_error("yaml: line " + std::to_string(no) + ": " + msg);
}

// Strip a trailing " # comment" that is outside quotes.
std::string strip_comment(const std::string& s) {
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (q) {
      if (c == '\\' && q == '"') { ++i; continue; }
      if (c == q) q = 0;
    } else if (c == '\'' || c == '"') {
      q = c;
    } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
      return s.substr(0, i);
    }
  }
  return s;
}

std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}

std::string ltrim(const std::string& s) {
  size_t i = 0;
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
  return s.substr(i);
}

std::string unquote_double(const std::string& s, int no) {
  std::string out;
  for (size_t i = 1; i + 1 < s.size(); ++i) {
    char c = s[i];
    if (c != '\\') { out += c; continue; }
    if (++i + 1 > s.size() - 1) fail(no, "dangling escape");
    switch (s[i]) {
      case 'n': out += '\n'; break;
      case 't': out += '\t'; break;
      case 'r': out += '\r'; break;
      case '0': out += '\0'; break;
      case '"': out += '"'; break;
      case '/': out += '/'; break;
      case '\\': out += '\\'; break;
      case 'x': {
        if (i + 2 >= s.size()) fail(no, "bad \\x escape");
        out += (char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16);
        i += 2;
        break;
      }
      case 'u': {
        if (i + 4 >= s.size()) fail(no, "bad \\u escape");
        long cp = strtol(s.substr(i + 1, 4).c_str(), nullptr, 16);
        i += 4;
        if (cp < 0x80) out += (char)cp;
        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
        break;
      }
      default: out += s[i];
    }
  }
  return out;
}

bool is_int(const std::string& s) {
  size_t i = (s[0] == '-' || s[0] == '+') ? 1 : 0;
  if (i >= s.size()) return false;
  for (; i < s.size(); ++i)
    if (!isdigit((unsigned char)s[i])) return false;
  return true;
}

bool is_float(const std::string& s) {
  char* end = nullptr;
  strtod(s.c_str(), &end);
  bool digit = false;
  for (char c : s) digit |= isdigit((unsigned char)c) != 0;
  return digit && end && *end == 0;
}

Json flow(const std::string& s, int no);

Json scalar(const std::string& raw, int no) {
  std::string s = rtrim(ltrim(raw));
  if (s.empty()) return Json();
  if (s[0] == '&' || s[0] == '*') fail(no, "anchors/aliases are not supported");
  if (s[0] == '!') fail(no, "tags are not supported");
  if (s[0] == '[' || s[0] == '{') return flow(s, no);
  if (s[0] == '"') {
    if (s.size() < 2 || s.back() != '"') fail(no, "unterminated double-quoted string");
    return Json(unquote_double(s, no));
  }
  if (s[0] == '\'') {
    if (s.size() < 2 || s.back() != '\'') fail(no, "unterminated single-quoted string");
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      out += s[i];
      if (s[i] == '\'' && s[i + 1] == '\'') ++i;
    }
    return Json(out);
  }
  if (s == "~" || s == "null" || s == "Null" || s == "NULL") return Json();
  if (s == "true" || s == "True" || s == "TRUE") return Json(true);
  if (s == "false" || s == "False" || s == "FALSE") return Json(false);
  if (is_int(s)) return Json((long long)strtoll(s.c_str(), nullptr, 10));
  if (s.size() > 2 && s[0] == '0' && (s[1] == 'x' || s[1] == 'o')) {
    return Json((long long)strtoll(s.c_str() + 2, nullptr, s[1] == 'x' ? 16 : 8));
  }
  if (is_float(s)) return Json(strtod(s.c_str(), nullptr));
  return Json(s);
}

// Split a flow collection body on top-level commas.
std::vector<std::string> split_flow(const std::string& body, int no) {
  std::vector<std::string> out;
  int depth = 0;
  char q = 0;
  std::string cur;
  for (size_t i = 0; i < body.size(); ++i) {
    char c = body[i];
    if (q) {
      cur += c;
      if (c == '\\' && q == '"' && i + 1 < body.size()) { cur += body[++i]; continue; }
      if (c == q) q = 0;
      continue;
    }
    if (c == '\'' || c == '"') q = c;
    else if (c == '[' || c == '{') ++depth;
    else if (c == ']' || c == '}') --depth;
    if (c == ',' && depth == 0) { out.push_back(cur); cur.clear(); continue; }
    cur += c;
  }
  if (q || depth) fail(no, "unbalanced flow collection");
  if (!ltrim(rtrim(cur)).empty()) out.push_back(cur);
  return out;
}

// Position of the "key: value" separator (": " or trailing ":") outside quotes/brackets, or npos.
size_t key_sep(const std::string& s) {
  char q = 0;
  int depth = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (q) {
      if (c == '\\' && q == '"') { ++i; continue; }
      if (c == q) q = 0;
      continue;
    }
    if ((c == '\'' || c == '"') && i == 0) { q = c; continue; }
    if (c == '[' || c == '{') ++depth;
    if (c == ']' || c == '}') --depth;
    if (c == ':' && depth == 0 && (i + 1 == s.size() || s[i + 1] == ' ' || s[i + 1] == '\t')) return i;
  }
  return std::string::npos;
}

std::string key_text(const std::string& k, int no) {
  Json j = scalar(k, no);
  if (j.is_string()) return j.str();
  return rtrim(ltrim(k));  // numbers/bools as keys keep their spelling
}

Json flow(const std::string& s, int no) {
  char open = s[0], close = open == '[' ? ']' : '}';
  if (s.back() != close) fail(no, "unterminated flow collection");
  std::string body = s.substr(1, s.size() - 2);
  if (open == '[') {
    Json a = Json::array();
    for (auto& part : split_flow(body, no)) a.push_back(scalar(part, no));
    return a;
  }
  Json o = Json::object();
  for (auto& part : split_flow(body, no)) {
    std::string p = rtrim(ltrim(part));
    size_t c = key_sep(p);
    if (c == std::string::npos) fail(no, "flow mapping entry without ':'");
    o[key_text(p.substr(0, c), no)] = scalar(p.substr(c + 1), no);
  }
  return o;
}

class Parser {
 public:
  Parser(const std::string& text) {
    std::vector<std::string> raw;
    size_t start = 0;
    while (start <= text.size()) {
      size_t e = text.find('\n', start);
      if (e == std::string::npos) e = text.size();
      raw.push_back(text.substr(start, e - start));
      start = e + 1;
    }
    raw_ = raw;
    for (size_t i = 0; i < raw.size(); ++i) {
      std::string l = raw[i];
      if (!l.empty() && l.back() == '\r') l.pop_back();
      size_t ind = 0;
      while (ind < l.size() && l[ind] == ' ') ++ind;
      if (ind < l.size() && l[ind] == '\t') fail((int)i + 1, "tab indentation");
      std::string body = rtrim(strip_comment(l.substr(ind)));
      if (body.empty()) continue;
      if (ind == 0 && (body == "---" || body.rfind("--- ", 0) == 0)) {
        if (!lines_.empty()) fail((int)i + 1, "multiple documents (use yaml_parse_all)");
        continue;
      }
      if (ind == 0 && body.rfind("%", 0) == 0) continue;  // directives
      if (body == "...") break;
      lines_.push_back({(int)ind, body, (int)i + 1});
    }
  }

  Json parse() {
    if (lines_.empty()) return Json();
    size_t i = 0;
    Json v = block(i, lines_[0].indent);
    if (i < lines_.size()) fail(lines_[i].no, "unexpected content (bad indentation?)");
    return v;
  }

 private:
  // Block node whose first line is lines_[i] at exactly `indent`.
  Json block(size_t& i, int indent) {
    const Line& l = lines_[i];
    if (l.text == "-" || l.text.rfind("- ", 0) == 0) return sequence(i, indent);
    if (key_sep(l.text) != std::string::npos) return mapping(i, indent);
    // a multi-line plain scalar: join continuation lines with spaces
    std::string s = l.text;
    ++i;
    while (i < lines_.size() && lines_[i].indent >= indent && key_sep(lines_[i].text) == std::string::npos &&
           lines_[i].text.rfind("- ", 0) != 0) {
      s += " " + lines_[i].text;
      ++i;
    }
    return scalar(s, l.no);
  }

  // Value after "key:" or "- " that continues on following lines (nested block), or inline.
  Json value(size_t& i, const std::string& inline_text, int parent_indent, int no, bool in_seq_item) {
    std::string t = rtrim(ltrim(inline_text));
    if (t == "|" || t == ">" || t == "|-" || t == ">-" || t == "|+" || t == ">+") return block_scalar(i, t, parent_indent);
    if (!t.empty()) return scalar(t, no);
    if (i >= lines_.size()) return Json();
    const Line& n = lines_[i];
    if (n.indent > parent_indent) return block(i, n.indent);
    // "key:\n- a" : a sequence at the key's own indent is the key's value (not in a seq item)
    if (!in_seq_item && n.indent == parent_indent && (n.text == "-" || n.text.rfind("- ", 0) == 0))
      return sequence(i, n.indent);
    return Json();
  }

  Json block_scalar(size_t& i, const std::string& style, int parent_indent) {
    bool folded = style[0] == '>';
    char chomp = style.size() > 1 ? style[1] : 0;
    // block scalars keep blank lines and '#' text: read the raw source lines
    int start_no = i < lines_.size() ? lines_[i].no : (int)raw_.size() + 1;
    int ind = -1;
    std::vector<std::string> body;
    size_t r = (size_t)(i < lines_.size() ? start_no - 1 : raw_.size());
    // find the first raw line after the header line that is deeper than parent_indent
    int header_no = i > 0 ? lines_[i - 1].no : 0;
    r = (size_t)header_no;
    for (; r < raw_.size(); ++r) {
      std::string l = raw_[r];
      if (!l.empty() && l.back() == '\r') l.pop_back();
      size_t k = 0;
      while (k < l.size() && l[k] == ' ') ++k;
      if (k == l.size()) { body.push_back(""); continue; }
      if (ind < 0) {
        if ((int)k <= parent_indent) break;
        ind = (int)k;
      }
      if ((int)k < ind) break;
      body.push_back(l.substr((size_t)ind));
    }
    while (i < lines_.size() && lines_[i].no <= (int)r) ++i;
    while (!body.empty() && body.back().empty() && chomp != '+') body.pop_back();
    std::string out;
    for (size_t k = 0; k < body.size(); ++k) {
      if (k) out += (folded && !body[k].empty() && !body[k - 1].empty()) ? " " : "\n";
      out += body[k];
    }
    if (chomp != '-' && !body.empty()) out += "\n";
    return Json(out);
  }

  Json mapping(size_t& i, int indent) {
    Json o = Json::object();
    while (i < lines_.size() && lines_[i].indent == indent) {
      const Line& l = lines_[i];
      if (l.text == "-" || l.text.rfind("- ", 0) == 0) break;
      size_t c = key_sep(l.text);
      if (c == std::string::npos) fail(l.no, "expected 'key: value'");
      std::string k = key_text(l.text.substr(0, c), l.no);
      if (k == "<<") fail(l.no, "merge keys are not supported");
      ++i;
      o[k] = value(i, l.text.substr(c + 1), indent, l.no, false);
    }
    if (i < lines_.size() && lines_[i].indent > indent) fail(lines_[i].no, "bad indentation");
    return o;
  }

  Json sequence(size_t& i, int indent) {
    Json a = Json::array();
    while (i < lines_.size() && lines_[i].indent == indent &&
           (lines_[i].text == "-" || lines_[i].text.rfind("- ", 0) == 0)) {
      Line l = lines_[i];
      std::string rest = l.text.size() > 1 ? l.text.substr(2) : "";
      int item_indent = indent + 2;
      size_t lead = 0;
      while (lead < rest.size() && rest[lead] == ' ') ++lead;
      item_indent += (int)lead;
      rest = rest.substr(lead);
      ++i;
      if (rest.empty()) {
        a.push_back(value(i, "", indent, l.no, true));
      } else if (rest == "-" || rest.rfind("- ", 0) == 0 || key_sep(rest) != std::string::npos) {
        // "- key: v" / "- - x": the item is a block whose first line sits at item_indent
        lines_.insert(lines_.begin() + (long)i, Line{item_indent, rest, l.no});
        a.push_back(block(i, item_indent));
      } else {
        a.push_back(value(i, rest, indent, l.no, true));
      }
    }
    return a;
  }

  std::vector<Line> lines_;
  std::vector<std::string> raw_;
};

}  // namespace

Json yaml_parse(const std::string& text) { return Parser(text).parse(); }

std::vector<Json> yaml_parse_all(const std::string& text) {
  std::vector<Json> out;
  std::string cur;
  size_t start = 0;
  auto flush = [&] {
    bool blank = true;
    for (char c : cur) blank &= (c == ' ' || c == '\n' || c == '\r' || c == '\t');
    if (!blank) {
      Json j = yaml_parse(cur);
      if (!j.is_null()) out.push_back(j);
    }
    cur.clear();
  };
  while (start <= text.size()) {
    size_t e = text.find('\n', start);
    if (e == std::string::npos) e = text.size();
    std::string l = text.substr(start, e - start);
    if (l == "---" || l.rfind("--- ", 0) == 0 || l == "---\r") flush();
    else cur += l + "\n";
    start = e + 1;
  }
  flush();
  return out;
}

}  // namespace tfk
