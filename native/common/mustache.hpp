// Mustache renderer shared by sdk-bootstrap and the native tests.
//
// Same subset and strictness as the scheduler's renderer
// (dcos_commons_amd/specification/yaml/template_utils.py): {{var}} (HTML-escaped with the
// jmustache escape set), {{{var}}} / {{&var}} (raw), {{#sec}}..{{/sec}}, {{^inv}}..{{/inv}},
// {{! comments}}, standalone tag lines removed. Env values "false" (any case) and "" are falsy.
// Unknown variables render as "" and are reported with their 1-based line number.
#pragma once

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace sdk {

struct MissingValue {
  std::string name;
  int line;
};

class MustacheError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

std::string html_escape(const std::string& s);

// Renders `tpl` against `env`. Appends every variable with no value to `missing` (if given).
std::string render_mustache(const std::string& tpl, const std::map<std::string, std::string>& env,
                            std::vector<MissingValue>* missing = nullptr);

}  // namespace sdk
