// sdk-cli: operator CLI for a running scheduler.
//
// Reference: cli/commands.go:39-52 and cli/commands/{plan,pod,endpoints,debug,update}.go with the
// tree renderers of cli/queries/{plan,pod}.go. Talks to the scheduler's REST API directly over
// HTTP/1.1 (no DC/OS cluster configuration needed): --url (or SDK_SCHEDULER_URL) is the scheduler
// base URL; --service selects a service of a multi-service scheduler (/v1/service/<name>/...).
#include <sys/wait.h>
#include <unistd.h>

#include <cstdlib>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "../common/http.hpp"
#include "../common/json.hpp"

namespace {

struct Ctx {
  sdk::Url base;
  std::string service;
  bool json = false;
  std::map<std::string, std::string> headers;
};

const char* kUnknown = "<UNKNOWN>";

[[noreturn]] void die(const std::string& msg, int code = 1) {
  std::cerr << msg << std::endl;
  std::exit(code);
}

std::string api(const Ctx& c, const std::string& rest) {
  return (c.service.empty() ? std::string("/v1") : "/v1/service/" + sdk::url_encode(c.service)) + rest;
}

sdk::HttpResponse call(const Ctx& c, const std::string& method, const std::string& path, const std::string& body = "",
                       const std::string& content_type = "application/json") {
  auto headers = c.headers;
  if (!body.empty()) headers["Content-Type"] = content_type;
  try {
    return sdk::http_request(method, c.base, api(c, path), body, headers);
  } catch (const std::exception& e) {
    die(std::string("Failed to reach the scheduler: ") + e.what());
  }
}

// prints the body; 2xx (and 208 "already reported") succeed, anything else is an error
int emit(const sdk::HttpResponse& r, bool pretty_json = true) {
  bool ok = (r.status >= 200 && r.status < 300);
  std::string out = r.body;
  if (pretty_json && !out.empty()) {
    try {
      out = sdk::Json::parse(out).dump(2);
    } catch (...) {
    }
  }
  if (!ok) {
    std::cerr << "HTTP " << r.status << (out.empty() ? "" : ": " + out) << std::endl;
    return r.status == 404 ? 2 : 1;
  }
  if (!out.empty()) std::cout << out << std::endl;
  return 0;
}

std::string or_unknown(const sdk::Json& j) { return j.is_string() && !j.str().empty() ? j.str() : kUnknown; }

std::string plan_tree(const std::string& name, const sdk::Json& plan) {
  std::string out = name + " (" + or_unknown(plan["strategy"]) + " strategy) (" + or_unknown(plan["status"]) + ")\n";
  const auto& phases = plan["phases"].arr();
  for (size_t i = 0; i < phases.size(); ++i) {
    bool last = i + 1 == phases.size();
    const auto& ph = phases[i];
    out += std::string(last ? "└─ " : "├─ ") + or_unknown(ph["name"]) + " (" + or_unknown(ph["strategy"]) +
           " strategy) (" + or_unknown(ph["status"]) + ")\n";
    const auto& steps = ph["steps"].arr();
    for (size_t k = 0; k < steps.size(); ++k) {
      out += std::string(last ? "   " : "│  ") + (k + 1 == steps.size() ? "└─ " : "├─ ") + or_unknown(steps[k]["name"]) +
             " (" + or_unknown(steps[k]["status"]) + ")\n";
    }
  }
  const auto& errors = plan["errors"].arr();
  if (!errors.empty()) {
    out += "\nErrors:\n";
    for (const auto& e : errors) out += "- " + e.as_text() + "\n";
  }
  while (!out.empty() && out.back() == '\n') out.pop_back();
  return out;
}

void append_tasks(std::string& out, const sdk::Json& tasks, const std::string& prefix) {
  const auto& ts = tasks.arr();
  for (size_t i = 0; i < ts.size(); ++i)
    out += prefix + (i + 1 == ts.size() ? "└─ " : "├─ ") + or_unknown(ts[i]["name"]) + " (" +
           or_unknown(ts[i]["status"]) + ")\n";
}

std::string pods_tree(const sdk::Json& j) {
  std::string out = or_unknown(j["service"]) + "\n";
  const auto& pods = j["pods"].arr();
  for (size_t p = 0; p < pods.size(); ++p) {
    bool lastp = p + 1 == pods.size();
    out += std::string(lastp ? "└─ " : "├─ ") + or_unknown(pods[p]["name"]) + "\n";
    std::string cp = lastp ? "   " : "│  ";
    const auto& inst = pods[p]["instances"].arr();
    for (size_t i = 0; i < inst.size(); ++i) {
      bool lasti = i + 1 == inst.size();
      out += cp + (lasti ? "└─ " : "├─ ") + or_unknown(inst[i]["name"]) + "\n";
      append_tasks(out, inst[i]["tasks"], cp + (lasti ? "   " : "│  "));
    }
  }
  while (!out.empty() && out.back() == '\n') out.pop_back();
  return out;
}

std::string query(const std::vector<std::pair<std::string, std::string>>& kv) {
  std::string q;
  for (const auto& p : kv) {
    if (p.second.empty()) continue;
    q += (q.empty() ? "?" : "&") + p.first + "=" + sdk::url_encode(p.second);
  }
  return q;
}

std::string arg(const std::vector<std::string>& a, size_t i, const std::string& dflt = "") {
  return i < a.size() ? a[i] : dflt;
}

void usage() {
  std::cout <<
      "usage: sdk-cli [--url URL] [--service NAME] [--json] <section> <command> [args]\n\n"
      "  plan list | status [PLAN] | start PLAN [-p K=V]... | stop PLAN | pause PLAN [PHASE]\n"
      "       resume PLAN [PHASE] | force-restart PLAN [PHASE [STEP]] | force-complete PLAN [PHASE [STEP]]\n"
      "  pod  list | status [POD] | info POD | restart POD | replace POD | pause POD [-t TASK]... | resume POD [-t TASK]...\n"
      "  endpoints [NAME]\n"
      "  debug config list|show ID|target|target_id\n"
      "  debug state framework_id|properties|property NAME|refresh_cache\n"
      "  debug pod pause|resume POD [-t TASK]...\n"
      "  describe | update status|force-complete|force-restart|pause|resume [PHASE [STEP]] | health | metrics\n"
      "  aliases: plans, pods, endpoint; plan show|interrupt|continue|restart|force; debug configs|pods;\n"
      "           deprecated top-level `config ...` and `state ...` (= debug config / debug state)\n"
      "  hdfs <hdfs args...>   (hdfs services: runs bin/hdfs on name-0-node via `dcos task exec`)\n";
}

// -- framework plugins (reference: frameworks/hdfs/cli/dcos-hdfs/main.go) --------------------

// Index of `target` if it is the first non-flag argument, else -1: everything after it belongs to
// the plugin, including flags the SDK parser would otherwise consume (`hdfs dfs -ls /`).
int first_argument_index(const std::string& target, const std::vector<std::string>& args) {
  for (size_t i = 0; i < args.size(); ++i) {
    if (args[i].rfind("-", 0) == 0) continue;
    return args[i] == target ? static_cast<int>(i) : -1;
  }
  return -1;
}

std::string shell_join(const std::vector<std::string>& args) {
  std::string out;
  for (const auto& a : args) out += (out.empty() ? "" : " ") + a;
  return out;
}

// Builds `dcos task exec name-0-node bash -c "<hdfs command>"` and runs it as a child process
// (SDK_CLI_DRY_RUN=1 prints it instead). Returns the child's exit status.
int hdfs_plugin(const std::vector<std::string>& hdfs_args) {
  std::vector<std::string> cmd = {"dcos", "task", "exec", "name-0-node", "bash", "-c",
                                  "export JAVA_HOME=$(ls -d $MESOS_SANDBOX/jdk*/); $HDFS_VERSION/bin/hdfs " +
                                      shell_join(hdfs_args)};
  if (const char* dry = std::getenv("SDK_CLI_DRY_RUN"); dry != nullptr && std::string(dry) == "1") {
    for (size_t i = 0; i < cmd.size(); ++i) std::cout << (i ? "\x1f" : "") << cmd[i];
    std::cout << std::endl;
    return 0;
  }
  pid_t pid = fork();
  if (pid < 0) die("fork failed");
  if (pid == 0) {
    std::vector<char*> argv;
    for (auto& a : cmd) argv.push_back(a.data());
    argv.push_back(nullptr);
    execvp(argv[0], argv.data());
    std::cerr << "Failed to run '" << cmd[0] << "': is the DC/OS CLI installed?" << std::endl;
    _exit(127);
  }
  int status = 0;
  waitpid(pid, &status, 0);
  return WIFEXITED(status) ? WEXITSTATUS(status) : 1;
}

// Reference cli/queries/plan.go checkPlansResponse: a scheduler 404 means the plan/phase/step is
// unknown, 208 that the command is a no-op. Returns false (after printing the error) for those.
bool plan_response(const sdk::HttpResponse& r) {
  if (r.status == 404) {
    bool scheduler_404 = r.body == "Element not found" ||
                         (r.body.size() > 10 && r.body.compare(r.body.size() - 10, 10, " not found") == 0);
    if (scheduler_404) {
      std::cerr << "Plan, phase, and/or step does not exist" << std::endl;
      return false;
    }
  }
  if (r.status == 208) {
    std::cerr << "Cannot execute command. Command has already been issued or the plan has completed" << std::endl;
    return false;
  }
  if (r.status < 200 || r.status >= 300) {
    emit(r);
    return false;
  }
  return true;
}

// A plan command answered {"message": "..."} on success; anything else "could not be" done.
int plan_command(Ctx& c, const std::string& path, const std::string& target, const std::string& verb) {
  auto r = call(c, "POST", path);
  if (!plan_response(r)) return 1;
  bool valid = false;
  try {
    auto j = sdk::Json::parse(r.body);
    valid = j.is_object() && j["message"].is_string() && !j["message"].str().empty();
  } catch (...) {
  }
  std::cout << target << (valid ? " has been " : " could not be ") << verb << "." << std::endl;
  return 0;
}

// Reference command aliases (cli/commands/plan.go:61-85): show, interrupt, continue, restart, force.
std::string plan_alias(const std::string& cmd) {
  if (cmd == "show") return "status";
  if (cmd == "interrupt") return "pause";
  if (cmd == "continue") return "resume";
  if (cmd == "restart") return "force-restart";
  if (cmd == "force") return "force-complete";
  return cmd;
}

int plan_cmd(Ctx& c, const std::vector<std::string>& a) {
  std::string cmd = plan_alias(arg(a, 0));
  if (cmd == "list") return emit(call(c, "GET", "/plans"));
  if (cmd == "status") {
    std::string plan = arg(a, 1, "deploy");
    auto r = call(c, "GET", "/plans/" + sdk::url_encode(plan));
    if (r.status != 200 && r.status != 202 && r.status != 417) return emit(r);
    if (c.json) {
      std::cout << sdk::Json::parse(r.body).dump(2) << std::endl;
    } else {
      std::cout << plan_tree(plan, sdk::Json::parse(r.body)) << std::endl;
    }
    return 0;
  }
  std::string plan = arg(a, 1);
  if (plan.empty()) die("missing PLAN argument");
  std::string p = "/plans/" + sdk::url_encode(plan);
  if (cmd == "start") {
    sdk::Json params = sdk::Json::object();
    for (size_t i = 2; i < a.size(); ++i) {
      if ((a[i] == "-p" || a[i] == "--params") && i + 1 < a.size()) {
        std::string kv = a[++i];
        size_t eq = kv.find('=');
        if (eq == std::string::npos) die("parameters must be KEY=VALUE: " + kv);
        params.set(kv.substr(0, eq), sdk::Json(kv.substr(eq + 1)));
      }
    }
    auto r = call(c, "POST", p + "/start", params.dump());
    return plan_response(r) ? emit(r) : 1;
  }
  if (cmd == "stop") {
    auto r = call(c, "POST", p + "/stop");
    return plan_response(r) ? emit(r) : 1;
  }
  std::string phase = arg(a, 2), step = arg(a, 3);
  std::string q = "\"" + plan + "\" plan";
  std::string target = step.empty() ? (phase.empty() ? q : q + ": phase \"" + phase + "\"")
                                    : q + ": step \"" + step + "\" in phase \"" + phase + "\"";
  if (cmd == "pause") return plan_command(c, p + "/interrupt" + query({{"phase", phase}}), target, "paused");
  if (cmd == "resume") return plan_command(c, p + "/continue" + query({{"phase", phase}}), target, "resumed");
  if (cmd == "force-restart")
    return plan_command(c, p + "/restart" + query({{"phase", phase}, {"step", step}}), target, "restarted");
  if (cmd == "force-complete")
    return plan_command(c, p + "/forceComplete" + query({{"phase", phase}, {"step", step}}),
                        q + ": step \"" + step + "\" in phase \"" + phase + "\"", "forced to complete");
  usage();
  return 1;
}

std::string task_filter(const std::vector<std::string>& a, size_t from) {
  sdk::Json tasks = sdk::Json::array();
  for (size_t i = from; i < a.size(); ++i)
    if ((a[i] == "-t" || a[i] == "--tasks") && i + 1 < a.size()) tasks.push(sdk::Json(a[++i]));
  return tasks.size() ? tasks.dump() : "";
}

int pod_cmd(Ctx& c, const std::vector<std::string>& a) {
  std::string cmd = arg(a, 0);
  if (cmd == "list") return emit(call(c, "GET", "/pod"));
  if (cmd == "status") {
    std::string pod = arg(a, 1);
    auto r = call(c, "GET", pod.empty() ? "/pod/status" : "/pod/" + sdk::url_encode(pod) + "/status");
    if (r.status != 200 || c.json) return emit(r);
    auto j = sdk::Json::parse(r.body);
    if (pod.empty()) {
      std::cout << pods_tree(j) << std::endl;
    } else {
      std::string out = or_unknown(j["name"]) + "\n";
      append_tasks(out, j["tasks"], "");
      while (!out.empty() && out.back() == '\n') out.pop_back();
      std::cout << out << std::endl;
    }
    return 0;
  }
  std::string pod = arg(a, 1);
  if (pod.empty()) die("missing POD argument");
  std::string p = "/pod/" + sdk::url_encode(pod);
  if (cmd == "info") return emit(call(c, "GET", p + "/info"));
  if (cmd == "restart") return emit(call(c, "POST", p + "/restart"));
  if (cmd == "replace") return emit(call(c, "POST", p + "/replace"));
  if (cmd == "pause") return emit(call(c, "POST", p + "/pause", task_filter(a, 2)));
  if (cmd == "resume") return emit(call(c, "POST", p + "/resume", task_filter(a, 2)));
  usage();
  return 1;
}

int debug_cmd(Ctx& c, const std::vector<std::string>& a) {
  std::string sec = arg(a, 0), cmd = arg(a, 1);
  if (sec == "configs") sec = "config";
  if (sec == "pods") sec = "pod";
  if (sec == "config") {
    if (cmd == "list") return emit(call(c, "GET", "/configurations"));
    if (cmd == "show") return emit(call(c, "GET", "/configurations/" + sdk::url_encode(arg(a, 2))));
    if (cmd == "target") return emit(call(c, "GET", "/configurations/target"));
    if (cmd == "target_id") return emit(call(c, "GET", "/configurations/targetId"));
  } else if (sec == "state") {
    if (cmd == "framework_id") return emit(call(c, "GET", "/state/frameworkId"));
    if (cmd == "properties") return emit(call(c, "GET", "/state/properties"));
    if (cmd == "property") return emit(call(c, "GET", "/state/properties/" + sdk::url_encode(arg(a, 2))), false);
    if (cmd == "refresh_cache") return emit(call(c, "PUT", "/state/refresh"));
  } else if (sec == "pod") {
    std::vector<std::string> rest(a.begin() + 1, a.end());
    return pod_cmd(c, rest);
  } else if (sec == "plans" || sec == "offers" || sec == "taskStatuses" || sec == "reservations") {
    return emit(call(c, "GET", "/debug/" + sec));
  }
  usage();
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  Ctx c;
  std::string url = std::getenv("SDK_SCHEDULER_URL") ? std::getenv("SDK_SCHEDULER_URL") : "http://127.0.0.1:8080";
  if (const char* tok = std::getenv("DCOS_AUTH_TOKEN")) c.headers["Authorization"] = std::string("token=") + tok;
  std::vector<std::string> a;
  std::vector<std::string> raw(argv + 1, argv + argc);
  // flags of the SDK parser take a value: skip it when looking for the plugin section
  std::vector<std::string> scan;
  for (size_t i = 0; i < raw.size(); ++i) {
    if ((raw[i] == "--url" || raw[i] == "--service" || raw[i] == "--name") && i + 1 < raw.size()) {
      scan.push_back(raw[i]);
      scan.push_back("-" + raw[++i]);
    } else {
      scan.push_back(raw[i]);
    }
  }
  int plugin_at = first_argument_index("hdfs", scan);
  if (plugin_at >= 0) {
    argc = plugin_at + 1;  // the SDK parser sees only what precedes the plugin section
  }
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s == "--url" && i + 1 < argc) url = argv[++i];
    else if (s.rfind("--url=", 0) == 0) url = s.substr(6);
    else if ((s == "--service" || s == "--name") && i + 1 < argc) c.service = argv[++i];
    else if (s.rfind("--service=", 0) == 0) c.service = s.substr(10);
    else if (s == "--json") c.json = true;
    else if (s == "-h" || s == "--help") { usage(); return 0; }
    else a.push_back(s);
  }
  try {
    c.base = sdk::parse_url(url);
  } catch (const std::exception& e) {
    die(e.what());
  }
  if (plugin_at >= 0) return hdfs_plugin(std::vector<std::string>(raw.begin() + plugin_at + 1, raw.end()));
  if (a.empty()) {
    usage();
    return 1;
  }
  std::string section = a[0];
  std::vector<std::string> rest(a.begin() + 1, a.end());
  if (section == "plans") section = "plan";
  if (section == "pods") section = "pod";
  if (section == "endpoint") section = "endpoints";
  if (section == "help") {
    usage();
    return 0;
  }
  if (section == "config" || section == "state") {  // deprecated top-level forms
    rest.insert(rest.begin(), section);
    section = "debug";
  }
  try {
    if (section == "plan") return plan_cmd(c, rest);
    if (section == "pod") return pod_cmd(c, rest);
    if (section == "endpoints")
      return emit(call(c, "GET", rest.empty() ? "/endpoints" : "/endpoints/" + sdk::url_encode(rest[0])));
    if (section == "debug") return debug_cmd(c, rest);
    if (section == "describe") return emit(call(c, "GET", "/configurations/target"));
    if (section == "update" && !rest.empty() && rest[0] != "start" && rest[0] != "package-versions") {
      // update <cmd> [PHASE [STEP]] acts on the deploy plan, which is the update plan once deployed
      std::vector<std::string> r2 = {rest[0], "deploy"};
      r2.insert(r2.end(), rest.begin() + 1, rest.end());
      return plan_cmd(c, r2);
    }
    if (section == "health") return emit(call(c, "GET", "/health?verbose=true"));
    if (section == "metrics") return emit(call(c, "GET", "/metrics"));
  } catch (const sdk::JsonError& e) {
    die(std::string("Unexpected response: ") + e.what());
  }
  usage();
  return 1;
}
