// sdk-bootstrap: runs inside every task before its command.
//
// Reference behaviour: sdk/bootstrap/main.go (flags :65-98, DNS waits :188-289, CONFIG_TEMPLATE_*
// rendering :321-376, CA install :378). MI355X additions: a GPU assignment check (-gpu-check):
// when the task was given GPUs (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES) every listed device
// must exist in the KFD topology, and the device list is echoed so the task log shows exactly
// which MI355Xs the pod owns.
#include <arpa/inet.h>
#include <dirent.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <regex>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../common/mustache.hpp"

extern char** environ;

namespace {

bool g_verbose = false;

void logf(const std::string& msg) {
  std::time_t t = std::time(nullptr);
  char ts[32];
  std::strftime(ts, sizeof ts, "%Y/%m/%d %H:%M:%S", std::localtime(&t));
  std::cerr << ts << " " << msg << std::endl;
}

[[noreturn]] void fatal(const std::string& msg) {
  logf(msg);
  std::exit(1);
}

struct Args {
  bool print_env = true;
  bool insecure = false;
  bool resolve = true;
  bool self_resolve = true;
  std::string resolve_hosts = "<TASK_NAME>.<FRAMEWORK_HOST>";
  double resolve_timeout_s = 300;
  bool template_enabled = true;
  long long template_max_bytes = 1024 * 1024;
  bool install_certs = true;
  bool get_task_ip = false;
  bool gpu_check = true;
};

bool parse_bool(const std::string& v) {
  if (v == "true" || v == "1" || v == "t" || v == "T" || v == "TRUE" || v == "True") return true;
  if (v == "false" || v == "0" || v == "f" || v == "F" || v == "FALSE" || v == "False") return false;
  fatal("invalid boolean value: " + v);
}

// Go duration subset: 300ms, 5s, 2m, 1h, 1m30s, plain seconds
double parse_duration(const std::string& s) {
  if (s == "0") return 0;
  std::regex part("([0-9.]+)(ms|s|m|h)");
  double total = 0;
  size_t consumed = 0;
  for (auto it = std::sregex_iterator(s.begin(), s.end(), part); it != std::sregex_iterator(); ++it) {
    double v = std::stod((*it)[1]);
    std::string u = (*it)[2];
    total += u == "ms" ? v / 1000 : u == "s" ? v : u == "m" ? v * 60 : v * 3600;
    consumed += it->length();
  }
  if (consumed != s.size()) {
    try {
      return std::stod(s);
    } catch (...) {
      fatal("invalid duration: " + s);
    }
  }
  return total;
}

void usage() {
  std::cout << "Usage of sdk-bootstrap:\n"
               "  -print-env=BOOL          print the (filtered) environment (default true)\n"
               "  -insecure=BOOL           do not mask credential-like variables (default false)\n"
               "  -resolve=BOOL            wait for hosts to resolve (default true)\n"
               "  -self-resolve=BOOL       verify <TASK_NAME>.<FRAMEWORK_HOST> resolves to the task IP (default true)\n"
               "  -resolve-hosts=LIST      comma-separated hosts (default <TASK_NAME>.<FRAMEWORK_HOST>)\n"
               "  -resolve-timeout=DUR     total resolution budget, 0 = forever (default 5m)\n"
               "  -template=BOOL           render CONFIG_TEMPLATE_* templates (default true)\n"
               "  -template-max-bytes=N    largest template, 0 = unlimited (default 1048576)\n"
               "  -install-certs=BOOL      install $MESOS_SANDBOX/.ssl CA into $JAVA_HOME (default true)\n"
               "  -get-task-ip             print the task IP and exit\n"
               "  -gpu-check=BOOL          validate assigned GPUs against the KFD topology (default true)\n"
               "  -verbose                 verbose logging\n";
}

Args parse_args(int argc, char** argv) {
  Args a;
  bool hosts_given = false;
  for (int i = 1; i < argc; ++i) {
    std::string arg = argv[i];
    if (arg == "-h" || arg == "--help" || arg == "-help") {
      usage();
      std::exit(0);
    }
    while (!arg.empty() && arg[0] == '-') arg.erase(arg.begin());
    std::string key = arg, val;
    bool has_val = false;
    size_t eq = arg.find('=');
    if (eq != std::string::npos) {
      key = arg.substr(0, eq);
      val = arg.substr(eq + 1);
      has_val = true;
    }
    auto next_val = [&]() -> std::string {
      if (has_val) return val;
      if (i + 1 >= argc) fatal("flag needs an argument: -" + key);
      return argv[++i];
    };
    auto bool_val = [&]() { return has_val ? parse_bool(val) : true; };
    if (key == "verbose") g_verbose = bool_val();
    else if (key == "print-env") a.print_env = bool_val();
    else if (key == "insecure") a.insecure = bool_val();
    else if (key == "resolve") a.resolve = bool_val();
    else if (key == "self-resolve") a.self_resolve = bool_val();
    else if (key == "resolve-hosts") { a.resolve_hosts = next_val(); hosts_given = true; }
    else if (key == "resolve-timeout") a.resolve_timeout_s = parse_duration(next_val());
    else if (key == "template") a.template_enabled = bool_val();
    else if (key == "template-max-bytes") a.template_max_bytes = std::stoll(next_val());
    else if (key == "install-certs") a.install_certs = bool_val();
    else if (key == "get-task-ip") a.get_task_ip = bool_val();
    else if (key == "gpu-check") a.gpu_check = bool_val();
    else {
      usage();
      fatal("flag provided but not defined: -" + key);
    }
  }
  (void)hosts_given;
  return a;
}

std::map<std::string, std::string> env_map() {
  std::map<std::string, std::string> m;
  for (char** e = environ; *e; ++e) {
    std::string kv = *e;
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    m[kv.substr(0, eq)] = kv.substr(eq + 1);
  }
  return m;
}

const char* getenv_or(const char* k, const char* dflt) {
  const char* v = std::getenv(k);
  return v ? v : dflt;
}

std::vector<std::string> split_clean(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, sep)) {
    size_t b = item.find_first_not_of(" \t"), e = item.find_last_not_of(" \t");
    if (b != std::string::npos) out.push_back(item.substr(b, e - b + 1));
  }
  return out;
}

void print_env(bool insecure) {
  static const std::regex secret("(DCOS_SERVICE_ACCOUNT_CREDENTIAL|credential|password|secret|token)",
                                 std::regex::icase);
  std::vector<std::string> lines;
  for (const auto& kv : env_map()) {
    bool hide = !insecure && std::regex_search(kv.first, secret);
    lines.push_back(kv.first + "=" + (hide ? std::string("********") : kv.second));
  }
  std::string msg = "Bootstrapping with environment:";
  for (const auto& l : lines) msg += "\n" + l;
  logf(msg);
}

std::string container_ip() {
  for (const char* k : {"MESOS_CONTAINER_IP", "LIBPROCESS_IP"}) {
    const char* v = std::getenv(k);
    if (v && *v && std::string(v) != "0.0.0.0") return v;
  }
  struct ifaddrs* ifs = nullptr;
  std::string ip = "127.0.0.1";
  if (getifaddrs(&ifs) == 0) {
    for (auto* i = ifs; i; i = i->ifa_next) {
      if (!i->ifa_addr || i->ifa_addr->sa_family != AF_INET) continue;
      char buf[INET_ADDRSTRLEN];
      auto* sin = reinterpret_cast<struct sockaddr_in*>(i->ifa_addr);
      inet_ntop(AF_INET, &sin->sin_addr, buf, sizeof buf);
      if (std::string(buf).rfind("127.", 0) == 0) continue;
      ip = buf;
      break;
    }
    freeifaddrs(ifs);
  }
  return ip;
}

std::vector<std::string> lookup(const std::string& host) {
  std::vector<std::string> out;
  struct addrinfo hints;
  std::memset(&hints, 0, sizeof hints);
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0) return out;
  std::set<std::string> seen;
  for (auto* ai = res; ai; ai = ai->ai_next) {
    char buf[INET6_ADDRSTRLEN];
    void* addr = ai->ai_family == AF_INET ? static_cast<void*>(&reinterpret_cast<sockaddr_in*>(ai->ai_addr)->sin_addr)
                                           : static_cast<void*>(&reinterpret_cast<sockaddr_in6*>(ai->ai_addr)->sin6_addr);
    inet_ntop(ai->ai_family, addr, buf, sizeof buf);
    if (seen.insert(buf).second) out.push_back(buf);
  }
  freeaddrinfo(res);
  return out;
}

using Clock = std::chrono::steady_clock;

std::vector<std::string> resolve_host(const std::string& host, Clock::time_point deadline, bool bounded) {
  logf("Waiting for '" + host + "' to resolve...");
  while (true) {
    auto r = lookup(host);
    if (!r.empty()) {
      std::string joined;
      for (const auto& x : r) joined += (joined.empty() ? "" : " ") + x;
      logf("Resolved '" + host + "' => [" + joined + "]");
      return r;
    }
    if (g_verbose) logf("Lookup failed for " + host);
    if (bounded && Clock::now() > deadline)
      fatal("Time ran out while resolving '" + host +
            "'. Customize timeout with -resolve-timeout, or use -verbose to see attempts.");
    std::this_thread::sleep_for(std::chrono::seconds(1));
  }
}

std::string task_host() {
  const char* t = std::getenv("TASK_NAME");
  const char* f = std::getenv("FRAMEWORK_HOST");
  if (!t || !f) return "";
  return std::string(t) + "." + f;
}

void render_templates(long long max_bytes) {
  auto env = env_map();
  const char* sandbox = std::getenv("MESOS_SANDBOX");
  for (const auto& kv : env) {
    if (kv.first.rfind("CONFIG_TEMPLATE_", 0) != 0) continue;
    size_t comma = kv.second.find(',');
    if (comma == std::string::npos)
      fatal("Provided value for " + kv.first + " is invalid: Should be two strings separated by a comma, got: " +
            kv.second);
    if (!sandbox) fatal("Missing required envvar: MESOS_SANDBOX");
    std::string src = std::string(sandbox) + "/" + kv.second.substr(0, comma);
    std::string dst = kv.second.substr(comma + 1);
    std::string source = "envvar '" + kv.first + "'";
    struct stat st;
    if (stat(src.c_str(), &st) != 0) fatal("Path from " + source + " doesn't exist: " + src);
    if (!S_ISREG(st.st_mode)) fatal("Path from " + source + " is not a regular file: " + src);
    if (max_bytes != 0 && st.st_size > max_bytes)
      fatal("File '" + src + "' from " + source + " is " + std::to_string(st.st_size) + " bytes, exceeds maximum " +
            std::to_string(max_bytes) + " bytes");
    std::ifstream in(src, std::ios::binary);
    std::stringstream buf;
    buf << in.rdbuf();
    std::string rendered;
    try {
      rendered = sdk::render_mustache(buf.str(), env);
    } catch (const std::exception& e) {
      fatal("Failed to render template from " + source + " at '" + dst + "': " + e.what());
    }
    logf("Writing rendered '" + dst + "' from " + source + " (" + std::to_string(buf.str().size()) + " bytes -> " +
         std::to_string(rendered.size()) + " bytes)");
    std::ofstream out(dst, std::ios::binary | std::ios::trunc);
    if (!out) fatal("Failed to write rendered template from " + source + " to '" + dst + "'");
    out << rendered;
  }
}

void install_certs() {
  std::string sandbox = getenv_or("MESOS_SANDBOX", "");
  std::string ssl = sandbox + "/.ssl";
  struct stat st;
  if (stat(ssl.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) {
    logf("No $MESOS_SANDBOX/.ssl directory found. Cannot install certificate.");
    return;
  }
  std::string cert = ssl + "/ca-bundle.crt";
  if (stat(cert.c_str(), &st) != 0) {
    cert = ssl + "/ca.crt";
    if (stat(cert.c_str(), &st) != 0) {
      logf("No CA Cert found in the sandbox. Cannot install certificate. This is expected if the cluster is not in "
           "STRICT mode.");
      return;
    }
  }
  std::string java = getenv_or("JAVA_HOME", "");
  if (java.empty()) {
    logf("No JAVA_HOME provided. Cannot install certs.");
    return;
  }
  std::string cmd = "'" + java + "/bin/keytool' -importcert -noprompt -alias dcoscert -keystore '" + java +
                    "/lib/security/cacerts' -file '" + cert + "' -storepass changeit >/dev/null 2>&1";
  if (std::system(cmd.c_str()) != 0) {
    logf("Failed to install the certificate.");
    return;
  }
  logf("Successfully installed the certificate.");
}

// Count GPU nodes (simd_count > 0) in the KFD topology.
int kfd_gpu_count() {
  const char* base = "/sys/class/kfd/kfd/topology/nodes";
  DIR* d = opendir(base);
  if (!d) return -1;
  int n = 0;
  while (auto* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::ifstream in(std::string(base) + "/" + e->d_name + "/properties");
    std::string k;
    long long v;
    while (in >> k >> v) {
      if (k == "simd_count" && v > 0) {
        ++n;
        break;
      }
    }
  }
  closedir(d);
  return n;
}

void gpu_check() {
  const char* hip = std::getenv("HIP_VISIBLE_DEVICES");
  const char* rocr = std::getenv("ROCR_VISIBLE_DEVICES");
  std::string devs = hip ? hip : (rocr ? rocr : "");
  if (devs.empty()) {
    if (g_verbose) logf("No GPUs assigned to this task.");
    return;
  }
  auto ids = split_clean(devs, ',');
  int count = kfd_gpu_count();
  logf("Task was assigned GPU device(s) [" + devs + "]; KFD reports " +
       (count < 0 ? std::string("no topology") : std::to_string(count)) + " GPU node(s)");
  if (count < 0) fatal("GPUs were assigned but /sys/class/kfd is not available (amdgpu driver not loaded?)");
  for (const auto& id : ids) {
    char* end = nullptr;
    long v = std::strtol(id.c_str(), &end, 10);
    if (end && *end == '\0' && (v < 0 || v >= count))
      fatal("Assigned GPU " + id + " does not exist on this agent (" + std::to_string(count) + " GPUs)");
  }
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse_args(argc, argv);
  std::string ip = container_ip();
  setenv("LIBPROCESS_IP", ip.c_str(), 1);
  setenv("MESOS_CONTAINER_IP", ip.c_str(), 1);
  if (a.get_task_ip) {
    std::cout << ip;
    return 0;
  }
  if (a.print_env) print_env(a.insecure);
  std::vector<std::string> hosts;
  if (a.resolve) {
    if (a.resolve_hosts == "<TASK_NAME>.<FRAMEWORK_HOST>") {
      std::string th = task_host();
      if (th.empty()) {
        print_env(a.insecure);
        fatal("Missing required envvar(s) to build default -resolve-hosts value. Either specify -resolve-hosts or "
              "provide these envvars: TASK_NAME, FRAMEWORK_HOST.");
      }
      hosts.push_back(th);
    } else {
      hosts = split_clean(a.resolve_hosts, ',');
    }
    bool bounded = a.resolve_timeout_s > 0;
    auto deadline = Clock::now() + std::chrono::milliseconds(static_cast<long long>(a.resolve_timeout_s * 1000));
    for (const auto& h : hosts) resolve_host(h, deadline, bounded);
    if (a.self_resolve) {
      std::string th = task_host();
      if (th.empty())
        fatal("Missing required envvars to build task DNS address. Ensure that TASK_NAME and FRAMEWORK_HOST are both "
              "set or disable self resolution with --self-resolve=false");
      logf("Waiting for " + th + " to resolve to " + ip);
      while (true) {
        auto r = resolve_host(th, deadline, bounded);
        if (r.size() == 1 && r[0] == ip) {
          logf(th + " resolved to " + ip + " as expected.");
          break;
        }
        if (bounded && Clock::now() > deadline)
          fatal("Time ran out waiting for " + th + " to resolve to " + ip + ".");
        std::this_thread::sleep_for(std::chrono::seconds(1));
      }
    }
  } else {
    logf("Resolve disabled via -resolve=false: Skipping host resolution");
  }
  if (a.template_enabled) {
    render_templates(a.template_max_bytes);
  } else {
    logf("Template handling disabled via -template=false: Skipping any config templates");
  }
  if (a.install_certs) install_certs();
  if (a.gpu_check) gpu_check();
  logf("SDK Bootstrap successful.");
  return 0;
}
