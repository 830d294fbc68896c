// sdk-agent-launcher: starts and reaps the task processes and check commands of the local
// DC/OS stand-in's agents (dcos_commons_amd/mesos/containerizer.py, ProcessTaskBehavior).
//
// On a cluster every Mesos agent is its own native process on its own node, and starts its
// containers without waiting on anything else. The stand-in runs all agents inside the master's
// Python process; starting a process from there (fork/exec plus a waiter thread) costs ~1 ms of
// interpreter time per task, holds the interpreter lock across the fork, and every task start or
// check of every agent queues behind the one before. This helper takes the process work out of
// the interpreter: the containerizer prepares the sandbox and sends one request line; the helper
// forks, execs and reaps, and reports back. It is single-threaded (poll over the request socket
// and a signalfd for SIGCHLD), so fork() here is cheap and safe.
//
//   sdk-agent-launcher --fd N      (N: a connected stream socket, e.g. one end of a socketpair)
//
// Requests and events are newline-delimited JSON objects:
//   {"op":"launch","id":I,"argv":[...],"exe":PATH,"cwd":DIR,"env":{...},"stdout":F,"stderr":F,
//    "setup":[["d",DIR] | ["l",TARGET,LINK] ...]}
//        -> {"ev":"started","id":I,"pid":P} | {"ev":"error","id":I,"msg":M};  later {"ev":"exited","id":I,"rc":R}
//        The sandbox set-up comes first, in the helper, in order: "d" creates DIR with its parents
//        (an existing one is fine); "l" makes LINK (parents created) a symlink to TARGET unless
//        LINK exists already. A failure there is an "error".
//   {"op":"run","id":I,"argv":[...],"cwd":DIR,"env":{...},"timeout_ms":T}
//        -> {"ev":"ran","id":I,"rc":R}   (stdio on /dev/null; R = 124 when killed at the timeout)
//   {"op":"stop"}                         -> the helper exits (it never kills: the caller owns that)
// R follows Python's subprocess convention: the exit status, or -signal for a signalled process;
// 127 when the exec itself failed. Every process starts in a session of its own (setsid), so its
// process group id is its pid and the caller can signal the whole group.
// The helper exits when the socket closes (its parent is gone).
#include <poll.h>
#include <signal.h>
#include <sys/signalfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <fcntl.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "json.hpp"

namespace {

using sdk::Json;
using Clock = std::chrono::steady_clock;

struct Child {
  std::string id;
  bool run = false;                 // a "run" request: report "ran"
  bool timed_out = false;
  Clock::time_point deadline{};     // run requests with a timeout
  bool has_deadline = false;
};

int g_fd = -1;
std::map<pid_t, Child> g_children;

void send_event(const Json& ev) {
  std::string line = ev.dump() + "\n";
  size_t off = 0;
  while (off < line.size()) {
    ssize_t n = ::write(g_fd, line.data() + off, line.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      std::_Exit(0);               // the caller is gone
    }
    off += size_t(n);
  }
}

Json event(const char* ev, const std::string& id) {
  Json j = Json::object();
  j.set("ev", ev);
  j.set("id", id);
  return j;
}

std::vector<std::string> strings(const Json& a) {
  std::vector<std::string> out;
  if (a.is_array())
    for (const auto& v : a.arr()) out.push_back(v.as_text());
  return out;
}

// mkdir -p: every missing component of `path`, mode 0755. False (errno set) on a real failure.
bool make_dirs(const std::string& path) {
  if (path.empty()) return true;
  struct stat st;
  if (::stat(path.c_str(), &st) == 0) {
    if (S_ISDIR(st.st_mode)) return true;
    errno = ENOTDIR;
    return false;
  }
  size_t slash = path.find_last_of('/');
  if (slash != std::string::npos && slash > 0 && !make_dirs(path.substr(0, slash))) return false;
  if (::mkdir(path.c_str(), 0755) == 0 || errno == EEXIST) return true;
  return false;
}

// The sandbox set-up of a launch request; an empty string when it all succeeded, else what failed.
std::string prepare(const Json& req) {
  const Json& steps = req["setup"];
  if (!steps.is_array()) return "";
  for (const auto& st : steps.arr()) {
    if (!st.is_array() || st.arr().empty()) return "bad set-up entry";
    const auto& a = st.arr();
    const std::string kind = a[0].as_text();
    if (kind == "d" && a.size() == 2) {
      if (!make_dirs(a[1].as_text())) return "mkdir " + a[1].as_text() + ": " + std::strerror(errno);
    } else if (kind == "l" && a.size() == 3) {
      const std::string target = a[1].as_text(), link = a[2].as_text();
      size_t slash = link.find_last_of('/');
      if (slash != std::string::npos && slash > 0 && !make_dirs(link.substr(0, slash)))
        return "mkdir " + link.substr(0, slash) + ": " + std::strerror(errno);
      struct stat sb;
      if (::lstat(link.c_str(), &sb) == 0) continue;   // already there (a relaunch in place)
      if (::symlink(target.c_str(), link.c_str()) != 0 && errno != EEXIST)
        return "symlink " + link + ": " + std::strerror(errno);
    } else {
      return "bad set-up entry " + kind;
    }
  }
  return "";
}

// fork + exec in a new session; stdio from the given files (empty: /dev/null). Returns the pid,
// or -1 with errno set when fork failed.
pid_t spawn(const std::string& exe, const std::vector<std::string>& argv, const std::string& cwd, const Json& env,
            const std::string& out_path, const std::string& err_path) {
  std::vector<std::string> envs;
  if (env.is_object())
    for (const auto& kv : env.obj()) envs.push_back(kv.first + "=" + kv.second.as_text());
  std::vector<char*> cargv, cenv;
  for (const auto& s : argv) cargv.push_back(const_cast<char*>(s.c_str()));
  cargv.push_back(nullptr);
  for (const auto& s : envs) cenv.push_back(const_cast<char*>(s.c_str()));
  cenv.push_back(nullptr);
  const char* path = exe.empty() ? (argv.empty() ? "/bin/true" : argv[0].c_str()) : exe.c_str();

  pid_t pid = ::fork();
  if (pid != 0) return pid;
  // child: own session (pgid = pid), default signal dispositions, stdio, cwd, exec. Ignored
  // signals survive fork and execve, and the helper ignores SIGPIPE (main), so the task gets SIGPIPE
  // and SIGXFSZ back at their defaults, as subprocess's restore_signals does for the Popen path.
  ::signal(SIGPIPE, SIG_DFL);
  ::signal(SIGXFSZ, SIG_DFL);
  sigset_t none;
  sigemptyset(&none);
  ::sigprocmask(SIG_SETMASK, &none, nullptr);
  ::setsid();
  int in = ::open("/dev/null", O_RDONLY);
  int out = out_path.empty() ? ::open("/dev/null", O_WRONLY)
                             : ::open(out_path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  int err = err_path.empty() ? ::open("/dev/null", O_WRONLY)
                             : ::open(err_path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (in < 0 || out < 0 || err < 0) ::_exit(127);
  ::dup2(in, 0);
  ::dup2(out, 1);
  ::dup2(err, 2);
  if (::close_range(3, ~0U, 0) != 0)
    for (int fd = 3; fd < 1024; ++fd) ::close(fd);
  if (!cwd.empty() && ::chdir(cwd.c_str()) != 0) ::_exit(127);
  // a bare name ("bash") is looked up on the helper's PATH, as subprocess does with the caller's
  if (std::strchr(path, '/') == nullptr)
    ::execvpe(path, cargv.data(), cenv.data());
  else
    ::execve(path, cargv.data(), cenv.data());
  ::_exit(127);
}

void handle(const Json& req) {
  const std::string op = req["op"].as_text();
  if (op == "stop") std::exit(0);
  const std::string id = req["id"].as_text();
  if (op != "launch" && op != "run") {
    Json e = event("error", id);
    e.set("msg", "unknown op " + op);
    send_event(e);
    return;
  }
  const bool run = op == "run";
  std::vector<std::string> argv = strings(req["argv"]);
  if (argv.empty()) {
    Json e = event("error", id);
    e.set("msg", "empty argv");
    send_event(e);
    return;
  }
  if (!run) {
    std::string failed = prepare(req);
    if (!failed.empty()) {
      Json e = event("error", id);
      e.set("msg", failed);
      send_event(e);
      return;
    }
  }
  pid_t pid = spawn(req["exe"].is_null() ? "" : req["exe"].as_text(), argv, req["cwd"].is_null() ? "" : req["cwd"].as_text(),
                    req["env"], run ? "" : req["stdout"].as_text(), run ? "" : req["stderr"].as_text());
  if (pid < 0) {
    Json e = event(run ? "ran" : "error", id);
    if (run)
      e.set("rc", 127);
    else
      e.set("msg", std::string("fork failed: ") + std::strerror(errno));
    send_event(e);
    return;
  }
  Child c;
  c.id = id;
  c.run = run;
  if (run && req["timeout_ms"].is_number() && req["timeout_ms"].num() > 0) {
    c.has_deadline = true;
    c.deadline = Clock::now() + std::chrono::milliseconds(int64_t(req["timeout_ms"].num()));
  }
  g_children[pid] = c;
  if (!run) {
    Json e = event("started", id);
    e.set("pid", double(pid));
    send_event(e);
  }
}

void reap() {
  for (;;) {
    int status = 0;
    pid_t pid = ::waitpid(-1, &status, WNOHANG);
    if (pid <= 0) return;
    auto it = g_children.find(pid);
    if (it == g_children.end()) continue;
    int rc = WIFEXITED(status) ? WEXITSTATUS(status) : (WIFSIGNALED(status) ? -WTERMSIG(status) : -1);
    Child c = it->second;
    g_children.erase(it);
    if (c.run) {
      Json e = event("ran", c.id);
      e.set("rc", c.timed_out ? 124 : rc);
      send_event(e);
    } else {
      Json e = event("exited", c.id);
      e.set("rc", rc);
      send_event(e);
    }
  }
}

int next_timeout_ms() {
  int best = -1;
  auto now = Clock::now();
  for (auto& kv : g_children) {
    const Child& c = kv.second;
    if (!c.has_deadline || c.timed_out) continue;
    auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(c.deadline - now).count();
    int v = ms < 0 ? 0 : int(ms + 1);
    if (best < 0 || v < best) best = v;
  }
  return best;
}

void expire() {
  auto now = Clock::now();
  for (auto& kv : g_children) {
    Child& c = kv.second;
    if (c.has_deadline && !c.timed_out && c.deadline <= now) {
      c.timed_out = true;
      ::kill(-kv.first, SIGKILL);   // its session's process group
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  for (int i = 1; i + 1 < argc; ++i)
    if (std::strcmp(argv[i], "--fd") == 0) g_fd = std::atoi(argv[i + 1]);
  if (g_fd < 0) {
    std::fprintf(stderr, "usage: sdk-agent-launcher --fd N\n");
    return 2;
  }
  ::signal(SIGPIPE, SIG_IGN);
  sigset_t mask;
  sigemptyset(&mask);
  sigaddset(&mask, SIGCHLD);
  ::sigprocmask(SIG_BLOCK, &mask, nullptr);
  int sfd = ::signalfd(-1, &mask, SFD_CLOEXEC | SFD_NONBLOCK);
  if (sfd < 0) {
    std::perror("signalfd");
    return 1;
  }
  std::string buf;
  char chunk[65536];
  for (;;) {
    pollfd fds[2] = {{g_fd, POLLIN, 0}, {sfd, POLLIN, 0}};
    int n = ::poll(fds, 2, next_timeout_ms());
    if (n < 0 && errno != EINTR) return 1;
    expire();
    if (fds[1].revents & POLLIN) {
      signalfd_siginfo si;
      while (::read(sfd, &si, sizeof si) == ssize_t(sizeof si)) {
      }
      reap();
    }
    if (fds[0].revents & (POLLIN | POLLHUP | POLLERR)) {
      ssize_t r = ::read(g_fd, chunk, sizeof chunk);
      if (r == 0) return 0;   // the caller closed its end
      if (r < 0) {
        if (errno == EINTR || errno == EAGAIN) continue;
        return 1;
      }
      buf.append(chunk, size_t(r));
      size_t nl;
      while ((nl = buf.find('\n')) != std::string::npos) {
        std::string line = buf.substr(0, nl);
        buf.erase(0, nl + 1);
        if (line.empty()) continue;
        try {
          handle(Json::parse(line));
        } catch (const std::exception& e) {
          Json ev = Json::object();
          ev.set("ev", "error");
          ev.set("id", "");
          ev.set("msg", std::string("bad request: ") + e.what());
          send_event(ev);
        }
      }
    }
    reap();   // a SIGCHLD coalesced with the previous read
  }
}
