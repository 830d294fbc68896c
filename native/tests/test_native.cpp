// Unit tests for the native helpers (mustache, JSON, URL parsing). Built by CMake as
// `native-tests` and run from tests/test_native.py; plain asserts, non-zero exit on failure.
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "../common/http.hpp"
#include "../common/json.hpp"
#include "../common/mustache.hpp"

static int failures = 0;

#define CHECK(cond)                                                               \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::cerr << __FILE__ << ":" << __LINE__ << ": CHECK failed: " #cond << "\n"; \
      ++failures;                                                                 \
    }                                                                             \
  } while (0)

#define CHECK_EQ(a, b)                                                                                  \
  do {                                                                                                  \
    auto _a = (a);                                                                                      \
    auto _b = (b);                                                                                      \
    if (!(_a == _b)) {                                                                                  \
      std::cerr << __FILE__ << ":" << __LINE__ << ": CHECK_EQ failed: [" << _a << "] != [" << _b << "]\n"; \
      ++failures;                                                                                       \
    }                                                                                                   \
  } while (0)

static void test_mustache() {
  std::map<std::string, std::string> env = {{"A", "<x>"}, {"B", "<y>"}, {"ON", "true"}, {"OFF", "False"}};
  CHECK_EQ(sdk::render_mustache("a={{A}} b={{{B}}} c={{& B}}", env), std::string("a=&lt;x&gt; b=<y> c=<y>"));
  CHECK_EQ(sdk::render_mustache("{{#ON}}on{{/ON}}{{^ON}}off{{/ON}}", env), std::string("on"));
  CHECK_EQ(sdk::render_mustache("{{#OFF}}on{{/OFF}}{{^OFF}}off{{/OFF}}", env), std::string("off"));
  CHECK_EQ(sdk::render_mustache("{{#NOPE}}on{{/NOPE}}{{^NOPE}}off{{/NOPE}}", env), std::string("off"));
  CHECK_EQ(sdk::render_mustache("x{{! a comment }}y", env), std::string("xy"));
  // standalone section lines disappear
  CHECK_EQ(sdk::render_mustache("a\n  {{#ON}}\nb\n  {{/ON}}\nc\n", env), std::string("a\nb\nc\n"));
  std::vector<sdk::MissingValue> missing;
  CHECK_EQ(sdk::render_mustache("x\n{{A}}\n{{MISSING}}", env, &missing), std::string("x\n&lt;x&gt;\n"));
  CHECK_EQ(missing.size(), static_cast<size_t>(1));
  if (!missing.empty()) {
    CHECK_EQ(missing[0].name, std::string("MISSING"));
    CHECK_EQ(missing[0].line, 3);
  }
  CHECK_EQ(sdk::html_escape("&\"'`="), std::string("&amp;&quot;&#39;&#x60;&#x3D;"));
  bool threw = false;
  try {
    sdk::render_mustache("{{#A}}never closed", env);
  } catch (const sdk::MustacheError&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_json() {
  auto j = sdk::Json::parse(R"({"a": [1, 2.5, "x\né"], "b": {"c": true, "d": null}, "e": -3})");
  CHECK(j.is_object());
  CHECK_EQ(j["a"].size(), static_cast<size_t>(3));
  CHECK_EQ(j["a"].arr()[1].num(), 2.5);
  CHECK_EQ(j["a"].arr()[2].str(), std::string("x\n\xc3\xa9"));
  CHECK(j["b"]["c"].boolean());
  CHECK(j["b"]["d"].is_null());
  CHECK(j["missing"].is_null());
  CHECK_EQ(j["e"].dump(), std::string("-3"));
  CHECK_EQ(sdk::Json::parse(j.dump()).dump(), j.dump());
  CHECK_EQ(sdk::Json::parse("[]").dump(2), std::string("[]"));
  bool threw = false;
  try {
    sdk::Json::parse("{\"a\": }");
  } catch (const sdk::JsonError&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_url() {
  auto u = sdk::parse_url("http://127.0.0.1:8080/base");
  CHECK_EQ(u.host, std::string("127.0.0.1"));
  CHECK_EQ(u.port, 8080);
  CHECK_EQ(u.path, std::string("/base"));
  CHECK_EQ(sdk::parse_url("http://example").port, 80);
  CHECK_EQ(sdk::url_encode("a b/c"), std::string("a%20b%2Fc"));
}

int main() {
  test_mustache();
  test_json();
  test_url();
  if (failures) {
    std::cerr << failures << " check(s) failed\n";
    return 1;
  }
  std::cout << "native tests passed\n";
  return 0;
}
