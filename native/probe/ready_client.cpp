// amd-gpu-ready: a GPU pod's readiness-check command.
//
// Asks the node's readiness service (`amd-gpu-probed`, socket in AMD_GPU_PROBE_SOCKET or
// --socket) to probe this task's GPU, so the check costs a socket round trip plus ~60 us of GPU
// work instead of a fresh HIP runtime. This program never touches the GPU itself (it links no
// HIP library). Without a reachable service it runs the standalone probe next to it
// (`amd-gpu-probe --readiness`) as a child process and exits with its status.
//
//   amd-gpu-ready [--device N] [--socket PATH] [--json] [--no-fallback]
//
// --device is the index within the task's own visible devices (HIP_VISIBLE_DEVICES /
// ROCR_VISIBLE_DEVICES, set by the agent from the GPUs it assigned); the service is sent the
// physical index. Exit status: 0 healthy, 1 unhealthy, 2 error (usage, no service and no fallback).
#include <errno.h>
#include <limits.h>
#include <spawn.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern char** environ;

namespace {

// index `device` of the task's visible-device list -> physical GPU index; -1 if unknown
int physical_device(int device) {
  const char* vis = std::getenv("HIP_VISIBLE_DEVICES");
  if (vis == nullptr || *vis == '\0') vis = std::getenv("ROCR_VISIBLE_DEVICES");
  if (vis == nullptr || *vis == '\0') return device;
  const char* p = vis;
  for (int idx = 0; *p != '\0'; ++idx) {
    char* end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if (end == p || (*end != ',' && *end != '\0')) return -1;  // UUID lists: not mapped here
    if (idx == device) return static_cast<int>(v);
    p = (*end == ',') ? end + 1 : end;
  }
  return -1;
}

// one request to the service; the reply line in `reply`. false if the service is unreachable.
bool ask(const std::string& path, int physical, int inject, std::string& reply) {
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  if (path.empty() || path.size() >= sizeof(addr.sun_path)) return false;
  std::memcpy(addr.sun_path, path.c_str(), path.size() + 1);
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return false;
  if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0) {
    ::close(fd);
    return false;
  }
  timeval tv{30, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  char req[64];
  const int n = std::snprintf(req, sizeof req, "READY %d %d\n", physical, inject);
  if (::send(fd, req, static_cast<size_t>(n), MSG_NOSIGNAL) != n) {
    ::close(fd);
    return false;
  }
  char buf[512];
  reply.clear();
  while (reply.size() < 4096) {
    const ssize_t got = ::recv(fd, buf, sizeof buf, 0);
    if (got < 0 && errno == EINTR) continue;
    if (got <= 0) break;
    reply.append(buf, static_cast<size_t>(got));
    if (reply.back() == '\n') break;
  }
  ::close(fd);
  return !reply.empty();
}

std::string self_dir() {
  char buf[PATH_MAX];
  const ssize_t n = ::readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return ".";
  buf[n] = '\0';
  std::string s(buf);
  const size_t slash = s.rfind('/');
  return slash == std::string::npos ? "." : s.substr(0, slash);
}

// the standalone probe as a child process (this process stays GPU-free); its exit status
int run_standalone(int device, bool json) {
  const std::string exe = self_dir() + "/amd-gpu-probe";
  const std::string dev = std::to_string(device);
  std::vector<const char*> args{exe.c_str(), "--readiness", "--device", dev.c_str()};
  if (json) args.push_back("--json");
  args.push_back(nullptr);
  pid_t pid = 0;
  if (::posix_spawn(&pid, exe.c_str(), nullptr, nullptr, const_cast<char* const*>(args.data()), environ) != 0) {
    std::fprintf(stderr, "amd-gpu-ready: no probe service and cannot run %s\n", exe.c_str());
    return 2;
  }
  int status = 0;
  while (::waitpid(pid, &status, 0) < 0) {
    if (errno != EINTR) return 2;
  }
  return WIFEXITED(status) ? WEXITSTATUS(status) : 2;
}

int usage() {
  std::fprintf(stderr, "usage: amd-gpu-ready [--device N] [--socket PATH] [--json] [--no-fallback]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  int device = 0, inject = 0;
  bool json = false, fallback = true;
  const char* env_sock = std::getenv("AMD_GPU_PROBE_SOCKET");
  std::string path = env_sock != nullptr ? env_sock : "";
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--device" && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (a == "--socket" && i + 1 < argc) path = argv[++i];
    else if (a == "--json") json = true;
    else if (a == "--no-fallback") fallback = false;
    else if (a == "--inject" && i + 1 < argc) inject = std::atoi(argv[++i]);  // tests: fault injection
    else if (a == "--readiness") continue;  // accepted for command-line parity with amd-gpu-probe
    else return usage();
  }
  if (device < 0) return usage();
  const int physical = physical_device(device);
  std::string reply;
  bool reached = physical >= 0 && ask(path, physical, inject, reply);
  if (reached && reply.find("\"busy\"") != std::string::npos) {
    // the service is saturated (its in-flight cap): ask once more after a short backoff. A
    // standalone probe here would start a whole HIP runtime of its own (0.3-0.4 s) exactly when
    // the node is busiest, so a second refusal fails the check and the agent retries it at the
    // check's next interval.
    ::usleep(20 * 1000);
    reply.clear();
    reached = ask(path, physical, inject, reply);
    if (reached && reply.find("\"busy\"") != std::string::npos) {
      std::fprintf(stderr, "amd-gpu-ready: probe service busy; check fails, retried at the next interval\n");
      return 1;
    }
  }
  if (reached) {
    if (reply.find("\"error\"") == std::string::npos) {
      if (json) std::fputs(reply.c_str(), stdout);
      return reply.find("\"healthy\": true") != std::string::npos ? 0 : 1;
    }
    // the service could not probe this device (not visible to it, HIP error): say so, then
    // probe it here if allowed
    std::fprintf(stderr, "amd-gpu-ready: service: %s", reply.c_str());
    if (!fallback) return 2;
    return run_standalone(device, json);
  }
  if (!fallback) {
    std::fprintf(stderr, "amd-gpu-ready: probe service at '%s' unreachable\n", path.c_str());
    return 2;
  }
  return run_standalone(device, json);
}
