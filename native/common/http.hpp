// Tiny blocking HTTP/1.1 client over POSIX sockets (no libcurl): enough for the scheduler API.
#pragma once

#include <map>
#include <string>

namespace sdk {

struct Url {
  std::string scheme = "http";
  std::string host = "127.0.0.1";
  int port = 80;
  std::string path = "/";
};

struct HttpResponse {
  int status = 0;
  std::map<std::string, std::string> headers;  // lower-cased names
  std::string body;
};

Url parse_url(const std::string& url);

// Throws std::runtime_error on connection/protocol failure. `timeout_s` bounds connect + I/O.
HttpResponse http_request(const std::string& method, const Url& base, const std::string& path_and_query,
                          const std::string& body = "", const std::map<std::string, std::string>& headers = {},
                          double timeout_s = 30.0);

std::string url_encode(const std::string& s);

}  // namespace sdk
