#include "json.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace sdk {

namespace {
const Json kNull;

struct Parser {
  const std::string& s;
  size_t i = 0;

  explicit Parser(const std::string& text) : s(text) {}

  [[noreturn]] void fail(const std::string& what) {
    throw JsonError("JSON parse error at offset " + std::to_string(i) + ": " + what);
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }
  bool consume(const char* lit) {
    size_t n = 0;
    while (lit[n]) ++n;
    if (s.compare(i, n, lit) == 0) {
      i += n;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) {
      out += static_cast<char>(cp);
    } else if (cp < 0x800) {
      out += static_cast<char>(0xC0 | (cp >> 6));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += static_cast<char>(0xE0 | (cp >> 12));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else {
      out += static_cast<char>(0xF0 | (cp >> 18));
      out += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    }
  }
  unsigned hex4() {
    if (i + 4 > s.size()) fail("truncated \\u escape");
    unsigned v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad \\u escape");
    }
    return v;
  }
  std::string string() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i >= s.size()) fail("truncated escape");
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
          if (cp >= 0xD800 && cp <= 0xDBFF && consume("\\u")) {
            unsigned lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (i >= s.size()) fail("unterminated string");
    ++i;
    return out;
  }
  Json value() {
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      ++i;
      Json o = Json::object();
      ws();
      if (i < s.size() && s[i] == '}') { ++i; return o; }
      while (true) {
        ws();
        std::string k = string();
        ws();
        if (i >= s.size() || s[i] != ':') fail("expected ':'");
        ++i;
        o.set(k, value());
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; return o; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++i;
      Json a = Json::array();
      ws();
      if (i < s.size() && s[i] == ']') { ++i; return a; }
      while (true) {
        a.push(value());
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == ']') { ++i; return a; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') return Json(string());
    if (consume("true")) return Json(true);
    if (consume("false")) return Json(false);
    if (consume("null")) return Json();
    size_t start = i;
    if (s[i] == '-') ++i;
    while (i < s.size() && (isdigit(static_cast<unsigned char>(s[i])) || s[i] == '.' || s[i] == 'e' ||
                            s[i] == 'E' || s[i] == '+' || s[i] == '-'))
      ++i;
    if (start == i) fail("unexpected character");
    return Json(std::strtod(s.c_str() + start, nullptr));
  }
};

void escape(std::string& out, const std::string& s) {
  out += '"';
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
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += static_cast<char>(c);
        }
    }
  }
  out += '"';
}
}  // namespace

const std::string& Json::str() const {
  if (type_ != Type::String) throw JsonError("not a string");
  return s_;
}
double Json::num() const {
  if (type_ != Type::Number) throw JsonError("not a number");
  return n_;
}
bool Json::boolean() const {
  if (type_ != Type::Bool) throw JsonError("not a bool");
  return b_;
}
const Json::Array& Json::arr() const {
  static const Array empty;
  if (type_ != Type::Array) return empty;
  return *a_;
}
Json::Array& Json::arr() {
  if (type_ != Type::Array) throw JsonError("not an array");
  return *a_;
}
const Json::Object& Json::obj() const {
  static const Object empty;
  if (type_ != Type::Object) return empty;
  return *o_;
}
const Json& Json::operator[](const std::string& key) const {
  if (type_ != Type::Object) return kNull;
  for (const auto& kv : *o_)
    if (kv.first == key) return kv.second;
  return kNull;
}
bool Json::has(const std::string& key) const {
  if (type_ != Type::Object) return false;
  for (const auto& kv : *o_)
    if (kv.first == key) return true;
  return false;
}
void Json::set(const std::string& key, Json v) {
  if (type_ == Type::Null) *this = object();
  if (type_ != Type::Object) throw JsonError("not an object");
  if (!o_) o_ = std::make_shared<Object>();
  for (auto& kv : *o_)
    if (kv.first == key) {
      kv.second = std::move(v);
      return;
    }
  o_->emplace_back(key, std::move(v));
}
void Json::push(Json v) {
  if (type_ == Type::Null) *this = array();
  if (type_ != Type::Array) throw JsonError("not an array");
  if (!a_) a_ = std::make_shared<Array>();
  a_->push_back(std::move(v));
}
size_t Json::size() const {
  if (type_ == Type::Array) return a_ ? a_->size() : 0;
  if (type_ == Type::Object) return o_ ? o_->size() : 0;
  return 0;
}

Json Json::parse(const std::string& text) {
  Parser p(text);
  Json v = p.value();
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

void Json::dump_to(std::string& out, int indent, int level) const {
  auto nl = [&](int lvl) {
    if (indent < 0) return;
    out += '\n';
    out.append(static_cast<size_t>(indent * lvl), ' ');
  };
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Number: {
      char buf[40];
      if (std::fabs(n_) < 1e15 && n_ == static_cast<double>(static_cast<long long>(n_)))
        std::snprintf(buf, sizeof buf, "%lld", static_cast<long long>(n_));
      else
        std::snprintf(buf, sizeof buf, "%.17g", n_);
      out += buf;
      break;
    }
    case Type::String: escape(out, s_); break;
    case Type::Array: {
      out += '[';
      const auto& a = arr();
      for (size_t k = 0; k < a.size(); ++k) {
        if (k) out += ',';
        nl(level + 1);
        a[k].dump_to(out, indent, level + 1);
      }
      if (!a.empty()) nl(level);
      out += ']';
      break;
    }
    case Type::Object: {
      out += '{';
      const auto& o = obj();
      for (size_t k = 0; k < o.size(); ++k) {
        if (k) out += ',';
        nl(level + 1);
        escape(out, o[k].first);
        out += indent < 0 ? ":" : ": ";
        o[k].second.dump_to(out, indent, level + 1);
      }
      if (!o.empty()) nl(level);
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

}  // namespace sdk
