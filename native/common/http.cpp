#include "http.hpp"

#include <netdb.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace sdk {

Url parse_url(const std::string& url) {
  Url u;
  std::string rest = url;
  size_t p = rest.find("://");
  if (p != std::string::npos) {
    u.scheme = rest.substr(0, p);
    rest = rest.substr(p + 3);
  }
  if (u.scheme != "http") throw std::runtime_error("only http:// URLs are supported: " + url);
  size_t slash = rest.find('/');
  std::string hostport = slash == std::string::npos ? rest : rest.substr(0, slash);
  u.path = slash == std::string::npos ? "/" : rest.substr(slash);
  size_t colon = hostport.rfind(':');
  if (colon != std::string::npos) {
    u.host = hostport.substr(0, colon);
    u.port = std::stoi(hostport.substr(colon + 1));
  } else {
    u.host = hostport;
    u.port = 80;
  }
  if (u.host.empty()) throw std::runtime_error("missing host in URL: " + url);
  return u;
}

std::string url_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out += static_cast<char>(c);
    } else {
      out += '%';
      out += hex[c >> 4];
      out += hex[c & 15];
    }
  }
  return out;
}

namespace {

class Socket {
 public:
  explicit Socket(int fd) : fd_(fd) {}
  ~Socket() {
    if (fd_ >= 0) ::close(fd_);
  }
  int fd() const { return fd_; }

 private:
  int fd_;
};

int connect_to(const std::string& host, int port, int timeout_ms) {
  struct addrinfo hints;
  std::memset(&hints, 0, sizeof hints);
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
  if (rc != 0) throw std::runtime_error("cannot resolve " + host + ": " + gai_strerror(rc));
  int fd = -1;
  std::string last;
  for (auto* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
    if (fd < 0) continue;
    struct timeval tv;
    tv.tv_sec = timeout_ms / 1000;
    tv.tv_usec = (timeout_ms % 1000) * 1000;
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) break;
    last = std::strerror(errno);
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) throw std::runtime_error("cannot connect to " + host + ":" + std::to_string(port) + ": " + last);
  return fd;
}

void send_all(int fd, const std::string& data) {
  size_t off = 0;
  while (off < data.size()) {
    ssize_t n = ::send(fd, data.data() + off, data.size() - off, MSG_NOSIGNAL);
    if (n <= 0) throw std::runtime_error(std::string("send failed: ") + std::strerror(errno));
    off += static_cast<size_t>(n);
  }
}

std::string recv_all(int fd) {
  std::string out;
  char buf[65536];
  while (true) {
    ssize_t n = ::recv(fd, buf, sizeof buf, 0);
    if (n == 0) break;
    if (n < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("recv failed: ") + std::strerror(errno));
    }
    out.append(buf, static_cast<size_t>(n));
  }
  return out;
}

std::string dechunk(const std::string& body) {
  std::string out;
  size_t pos = 0;
  while (pos < body.size()) {
    size_t eol = body.find("\r\n", pos);
    if (eol == std::string::npos) break;
    size_t len = std::stoul(body.substr(pos, eol - pos), nullptr, 16);
    if (len == 0) break;
    out += body.substr(eol + 2, len);
    pos = eol + 2 + len + 2;
  }
  return out;
}

}  // namespace

HttpResponse http_request(const std::string& method, const Url& base, const std::string& path_and_query,
                          const std::string& body, const std::map<std::string, std::string>& headers,
                          double timeout_s) {
  Socket s(connect_to(base.host, base.port, static_cast<int>(timeout_s * 1000)));
  std::string path = path_and_query;
  std::string prefix = base.path == "/" ? "" : base.path;
  if (!prefix.empty() && prefix.back() == '/') prefix.pop_back();
  std::string req = method + " " + prefix + path + " HTTP/1.1\r\n";
  req += "Host: " + base.host + ":" + std::to_string(base.port) + "\r\n";
  req += "Connection: close\r\nUser-Agent: sdk-cli-amd/1\r\nAccept: */*\r\n";
  for (const auto& h : headers) req += h.first + ": " + h.second + "\r\n";
  if (!body.empty() || method == "POST" || method == "PUT") req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  req += "\r\n";
  req += body;
  send_all(s.fd(), req);
  std::string raw = recv_all(s.fd());
  size_t hdr_end = raw.find("\r\n\r\n");
  if (hdr_end == std::string::npos) throw std::runtime_error("malformed HTTP response");
  HttpResponse r;
  std::string head = raw.substr(0, hdr_end);
  size_t sp = head.find(' ');
  if (sp == std::string::npos) throw std::runtime_error("malformed status line");
  r.status = std::stoi(head.substr(sp + 1, 3));
  size_t pos = head.find("\r\n");
  while (pos != std::string::npos && pos < head.size()) {
    size_t next = head.find("\r\n", pos + 2);
    std::string line = head.substr(pos + 2, next == std::string::npos ? std::string::npos : next - pos - 2);
    size_t colon = line.find(':');
    if (colon != std::string::npos) {
      std::string k = line.substr(0, colon);
      for (auto& c : k) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
      std::string v = line.substr(colon + 1);
      while (!v.empty() && v.front() == ' ') v.erase(v.begin());
      r.headers[k] = v;
    }
    pos = next;
  }
  r.body = raw.substr(hdr_end + 4);
  auto te = r.headers.find("transfer-encoding");
  if (te != r.headers.end() && te->second.find("chunked") != std::string::npos) r.body = dechunk(r.body);
  return r;
}

}  // namespace sdk
