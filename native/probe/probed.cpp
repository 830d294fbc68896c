// amd-gpu-probed: node-local GPU readiness service.
//
// A pod's readiness check is a short-lived command. Run as `amd-gpu-probe --readiness`, every
// check pays for a fresh HIP runtime (device enumeration, code-object load, context and buffer
// setup): about 0.3-0.4 s on an MI355X node, for ~60 us of GPU work. This daemon keeps one HIP
// runtime per node and the fused readiness context of every device resident (the same
// `amdprobe_readiness` routine the scheduler's in-process check calls: MFMA bf16 GEMM numerics,
// dense fp32 check of every product element, 64 MiB HBM address-hash pattern; NaN-poisoned output
// and a per-call seed so stale buffers cannot pass). `amd-gpu-ready` is the readiness command
// that talks to it.
//
// Protocol (AF_UNIX stream socket, one request per connection):
//   request : "READY <device> [inject]\n"   device = physical GPU index (as in HIP_VISIBLE_DEVICES)
//   reply   : one JSON line {"device", "ordinal", "gemm_rel_err", "mem_bad_words", "healthy",
//             "probe_seconds"} or {"error": "..."}.
// The physical index is mapped to this process's ordinal through its own HIP_VISIBLE_DEVICES (or
// ROCR_VISIBLE_DEVICES) when set. `inject` (tests only) selects a fault of amdprobe_readiness.
//
// Lifetime: SIGTERM/SIGINT, `--idle-exit S` without a request, or the parent's death
// (`--parent-death`) end it; in-flight probes finish before the process exits and the socket
// file is removed.
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/prctl.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" int amdprobe_readiness(int device, unsigned seed, int inject, double* rel_err,
                                  unsigned long long* bad_words);

namespace {

constexpr double MAX_GEMM_REL_ERR = 1e-3;  // ops/gpu_health.py MAX_GEMM_REL_ERR
constexpr int MAX_INFLIGHT = 64;           // concurrent requests served (one thread each)
std::atomic<bool> g_stop{false};
std::atomic<int> g_inflight{0};
std::atomic<long long> g_last_request_ms{0};

long long now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void on_signal(int) { g_stop.store(true); }

// physical index -> ordinal of this process (its own visible-device list), -1 if not visible
int ordinal_of(int physical) {
  const char* vis = std::getenv("HIP_VISIBLE_DEVICES");
  if (vis == nullptr || *vis == '\0') vis = std::getenv("ROCR_VISIBLE_DEVICES");
  if (vis == nullptr || *vis == '\0') return physical;
  int idx = 0;
  const char* p = vis;
  while (*p != '\0') {
    char* end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if (end == p) return -1;  // non-numeric (UUID) lists are not mapped
    if (v == physical) return idx;
    ++idx;
    p = (*end == ',') ? end + 1 : end;
    if (*end != ',' && *end != '\0') return -1;
  }
  return -1;
}

std::string probe(int physical, int inject) {
  const int ordinal = ordinal_of(physical);
  char buf[512];
  if (ordinal < 0) {
    std::snprintf(buf, sizeof buf, "{\"device\": %d, \"error\": \"device not visible to the probe service\"}\n",
                  physical);
    return buf;
  }
  const auto t0 = std::chrono::steady_clock::now();
  double rel = HUGE_VAL;
  unsigned long long bad = 0;
  const int rc = amdprobe_readiness(ordinal, 4321u + static_cast<unsigned>(physical), inject, &rel, &bad);
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rc != 0) {
    std::snprintf(buf, sizeof buf, "{\"device\": %d, \"ordinal\": %d, \"error\": \"amdprobe_readiness returned %d\"}\n",
                  physical, ordinal, rc);
    return buf;
  }
  const bool healthy = std::isfinite(rel) && rel < MAX_GEMM_REL_ERR && bad == 0;
  std::snprintf(buf, sizeof buf,
                "{\"device\": %d, \"ordinal\": %d, \"gemm_rel_err\": %.3e, \"mem_bad_words\": %llu, "
                "\"healthy\": %s, \"probe_seconds\": %.6f}\n",
                physical, ordinal, std::isfinite(rel) ? rel : 1e300, bad, healthy ? "true" : "false", secs);
  return buf;
}

void write_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t n = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return;
    off += static_cast<size_t>(n);
  }
}

void serve_connection(int fd) {
  timeval tv{5, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  std::string line;
  char c;
  while (line.size() < 128) {
    const ssize_t n = ::recv(fd, &c, 1, 0);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0 || c == '\n') break;
    line.push_back(c);
  }
  int device = -1, inject = 0;
  char verb[16] = {0};
  const int got = std::sscanf(line.c_str(), "%15s %d %d", verb, &device, &inject);
  if (got < 2 || std::strcmp(verb, "READY") != 0 || device < 0 || inject < 0 || inject > 4) {
    write_all(fd, "{\"error\": \"bad request\"}\n");
  } else {
    const std::string reply = probe(device, inject);
    write_all(fd, reply);
    std::fprintf(stderr, "served READY %d: %s", device, reply.c_str());  // one line per check
  }
  ::close(fd);
  g_last_request_ms.store(now_ms());
  g_inflight.fetch_sub(1);
}

int usage() {
  std::fprintf(stderr,
               "usage: amd-gpu-probed --socket PATH [--warm] [--idle-exit SECONDS] [--parent-death]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  std::string path;
  bool warm = false, parent_death = false;
  double idle_exit_s = 0;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--socket" && i + 1 < argc) path = argv[++i];
    else if (a == "--warm") warm = true;
    else if (a == "--parent-death") parent_death = true;
    else if (a == "--idle-exit" && i + 1 < argc) idle_exit_s = std::atof(argv[++i]);
    else return usage();
  }
  if (path.empty()) return usage();
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  if (path.size() >= sizeof(addr.sun_path)) {
    std::fprintf(stderr, "socket path too long: %s\n", path.c_str());
    return 2;
  }
  std::memcpy(addr.sun_path, path.c_str(), path.size() + 1);

  if (parent_death) {
    ::prctl(PR_SET_PDEATHSIG, SIGTERM);
    if (::getppid() == 1) return 0;  // the parent is already gone
  }
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  ::sigaction(SIGTERM, &sa, nullptr);
  ::sigaction(SIGINT, &sa, nullptr);

  if (warm) {
    // one probe per visible device: the runtime, code objects and every device context are ready
    // before the first pod asks, and a bad GPU shows up in the service log at start
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
      std::fprintf(stderr, "amd-gpu-probed: no HIP devices visible\n");
      return 1;
    }
    for (int d = 0; d < n; ++d) {
      double rel = 0;
      unsigned long long bad = 0;
      const int rc = amdprobe_readiness(d, 1u, 0, &rel, &bad);
      std::fprintf(stderr, "amd-gpu-probed: warm ordinal %d rc=%d rel_err=%.2e bad_words=%llu\n", d, rc, rel, bad);
    }
  }

  const int lfd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd < 0) {
    std::perror("socket");
    return 2;
  }
  ::unlink(path.c_str());
  if (::bind(lfd, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0 || ::listen(lfd, 64) != 0) {
    std::perror("bind/listen");
    ::close(lfd);
    return 2;
  }
  std::fprintf(stderr, "amd-gpu-probed: listening on %s\n", path.c_str());
  std::fflush(stderr);
  g_last_request_ms.store(now_ms());

  while (!g_stop.load()) {
    pollfd pfd{lfd, POLLIN, 0};
    const int r = ::poll(&pfd, 1, 200);
    if (r < 0 && errno != EINTR) break;
    if (r > 0 && (pfd.revents & POLLIN)) {
      const int cfd = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (cfd >= 0 && g_inflight.load() >= MAX_INFLIGHT) {
        // more concurrent checks than a node has GPUs many times over: refuse rather than spawn
        // without bound. amd-gpu-ready asks once more after a short backoff, then fails the check
        // (exit 1) so the agent retries it at its next interval -- it does not start a standalone
        // HIP runtime while the node is saturated.
        write_all(cfd, "{\"error\": \"busy\"}\n");
        ::close(cfd);
      } else if (cfd >= 0) {
        g_inflight.fetch_add(1);
        g_last_request_ms.store(now_ms());
        std::thread(serve_connection, cfd).detach();
      }
    }
    if (idle_exit_s > 0 && g_inflight.load() == 0 &&
        now_ms() - g_last_request_ms.load() > static_cast<long long>(idle_exit_s * 1000)) {
      break;
    }
  }
  ::close(lfd);
  ::unlink(path.c_str());
  // probes in flight finish (their kernels drain) before the process exits
  const long long deadline = now_ms() + 10000;
  while (g_inflight.load() > 0 && now_ms() < deadline) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  const int left = g_inflight.load();
  if (left > 0) {
    // detached connection threads are still inside amdprobe_readiness: running static destructors
    // and the HIP runtime's teardown under them could crash at exit, so leave without either
    std::fprintf(stderr, "amd-gpu-probed: %d probe(s) still in flight after 10 s; exiting without teardown\n", left);
    std::fflush(stderr);
    std::_Exit(3);
  }
  return 0;
}
