#include "mustache.hpp"

#include <algorithm>
#include <cctype>

namespace sdk {

namespace {

enum class Kind { Text, Var, Raw, Open, Inverted, Close, Comment };

struct Token {
  Kind kind;
  std::string text;  // literal text or tag name
  int line;
};

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

// A line that holds exactly one section/close/comment tag (plus whitespace) vanishes entirely.
std::string strip_standalone(const std::string& tpl) {
  std::string out;
  size_t pos = 0;
  while (pos <= tpl.size()) {
    size_t nl = tpl.find('\n', pos);
    bool has_nl = nl != std::string::npos;
    std::string line = tpl.substr(pos, has_nl ? nl - pos : std::string::npos);
    std::string t = trim(line);
    bool standalone = false;
    if (t.size() >= 5 && t.compare(0, 2, "{{") == 0 && t.compare(t.size() - 2, 2, "}}") == 0 &&
        (t[2] == '#' || t[2] == '^' || t[2] == '/' || t[2] == '!') && t.find("{{", 2) == std::string::npos) {
      standalone = true;
    }
    if (standalone) {
      out += t;  // the tag only: no indentation, no newline
    } else {
      out += line;
      if (has_nl) out += '\n';
    }
    if (!has_nl) break;
    pos = nl + 1;
  }
  return out;
}

std::vector<Token> tokenize(const std::string& src, const std::vector<int>& line_of) {
  std::vector<Token> toks;
  size_t i = 0;
  while (i < src.size()) {
    size_t open = src.find("{{", i);
    if (open == std::string::npos) {
      toks.push_back({Kind::Text, src.substr(i), line_of[i]});
      break;
    }
    if (open > i) toks.push_back({Kind::Text, src.substr(i, open - i), line_of[i]});
    bool triple = src.compare(open, 3, "{{{") == 0;
    size_t close = src.find(triple ? "}}}" : "}}", open + (triple ? 3 : 2));
    if (close == std::string::npos) throw MustacheError("unclosed tag at line " + std::to_string(line_of[open]));
    std::string inner = src.substr(open + (triple ? 3 : 2), close - open - (triple ? 3 : 2));
    int line = line_of[open];
    i = close + (triple ? 3 : 2);
    if (triple) {
      toks.push_back({Kind::Raw, trim(inner), line});
      continue;
    }
    std::string t = trim(inner);
    if (t.empty()) throw MustacheError("empty tag at line " + std::to_string(line));
    char c = t[0];
    std::string name = trim(t.substr(1));
    switch (c) {
      case '#': toks.push_back({Kind::Open, name, line}); break;
      case '^': toks.push_back({Kind::Inverted, name, line}); break;
      case '/': toks.push_back({Kind::Close, name, line}); break;
      case '!': toks.push_back({Kind::Comment, name, line}); break;
      case '&': toks.push_back({Kind::Raw, name, line}); break;
      default: toks.push_back({Kind::Var, t, line});
    }
  }
  return toks;
}

bool truthy(const std::map<std::string, std::string>& env, const std::string& name) {
  auto it = env.find(name);
  if (it == env.end()) return false;
  std::string v = it->second;
  std::transform(v.begin(), v.end(), v.begin(), [](unsigned char ch) { return std::tolower(ch); });
  return !v.empty() && v != "false";
}

size_t render_range(const std::vector<Token>& toks, size_t i, const std::string& until,
                    const std::map<std::string, std::string>& env, bool emit, std::string& out,
                    std::vector<MissingValue>* missing) {
  while (i < toks.size()) {
    const Token& t = toks[i];
    switch (t.kind) {
      case Kind::Text:
        if (emit) out += t.text;
        ++i;
        break;
      case Kind::Var:
      case Kind::Raw: {
        if (emit) {
          auto it = env.find(t.text);
          if (it == env.end()) {
            if (missing) missing->push_back({t.text, t.line});
          } else {
            out += t.kind == Kind::Var ? html_escape(it->second) : it->second;
          }
        }
        ++i;
        break;
      }
      case Kind::Comment:
        ++i;
        break;
      case Kind::Open:
      case Kind::Inverted: {
        bool on = truthy(env, t.text);
        if (t.kind == Kind::Inverted) on = !on;
        i = render_range(toks, i + 1, t.text, env, emit && on, out, missing);
        break;
      }
      case Kind::Close:
        if (t.text != until)
          throw MustacheError("unexpected close tag '" + t.text + "' at line " + std::to_string(t.line));
        return i + 1;
    }
  }
  if (!until.empty()) throw MustacheError("unclosed section '" + until + "'");
  return i;
}

}  // namespace

std::string html_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size());
  for (char c : s) {
    switch (c) {
      case '&': out += "&amp;"; break;
      case '<': out += "&lt;"; break;
      case '>': out += "&gt;"; break;
      case '"': out += "&quot;"; break;
      case '\'': out += "&#39;"; break;
      case '`': out += "&#x60;"; break;
      case '=': out += "&#x3D;"; break;
      default: out += c;
    }
  }
  return out;
}

std::string render_mustache(const std::string& tpl, const std::map<std::string, std::string>& env,
                            std::vector<MissingValue>* missing) {
  // line numbers refer to the original template, so compute them before stripping
  std::string src = strip_standalone(tpl);
  // map each byte of the stripped source back to an original line number: standalone lines
  // keep their relative order, so recount by walking both strings line by line
  std::vector<int> line_of(src.size() + 1, 1);
  {
    // rebuild: iterate original lines, track how many bytes each contributes to src
    int line = 1;
    size_t sp = 0, pos = 0;
    while (pos <= tpl.size() && sp <= src.size()) {
      size_t nl = tpl.find('\n', pos);
      bool has_nl = nl != std::string::npos;
      std::string l = tpl.substr(pos, has_nl ? nl - pos : std::string::npos);
      std::string t = trim(l);
      bool standalone = t.size() >= 5 && t.compare(0, 2, "{{") == 0 && t.compare(t.size() - 2, 2, "}}") == 0 &&
                        (t[2] == '#' || t[2] == '^' || t[2] == '/' || t[2] == '!') &&
                        t.find("{{", 2) == std::string::npos;
      size_t len = standalone ? t.size() : l.size() + (has_nl ? 1 : 0);
      for (size_t k = 0; k < len && sp + k < line_of.size(); ++k) line_of[sp + k] = line;
      sp += len;
      if (!has_nl) break;
      pos = nl + 1;
      ++line;
    }
    for (size_t k = sp; k < line_of.size(); ++k) line_of[k] = line;
  }
  auto toks = tokenize(src, line_of);
  std::string out;
  render_range(toks, 0, "", env, true, out, missing);
  return out;
}

}  // namespace sdk
