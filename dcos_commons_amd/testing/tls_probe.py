"""A minimal HTTPS server and client for end-to-end checks of TLS artifacts in the local cluster
(the reference's ``test_tls_nginx`` runs NGINX with the task's PEM files and a Java client with
its truststore; this stands in for both).

    python3 -m dcos_commons_amd.testing.tls_probe serve --cert web.crt --key web.key --port P
    python3 -m dcos_commons_amd.testing.tls_probe get --ca artifacts.ca --host NAME --connect 127.0.0.1:P

``get`` verifies the server's chain against ``--ca`` and its certificate against ``--host`` (the
name a client would use, e.g. the task's autoip host) while connecting to ``--connect``, and prints
``status=<code>``.
"""
from __future__ import annotations

import argparse
import http.server
import socket
import ssl
import sys


def serve(cert: str, key: str, port: int) -> None:
    class Handler(http.server.BaseHTTPRequestHandler):
        def do_GET(self):   # noqa: N802 (http.server's naming)
            body = b"hello over TLS\n"
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *args):
            pass

    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(cert, key)
    httpd = http.server.HTTPServer(("0.0.0.0", port), Handler)
    httpd.socket = ctx.wrap_socket(httpd.socket, server_side=True)
    httpd.serve_forever()


def get(ca: str, host: str, connect: str) -> int:
    addr, _, port = connect.rpartition(":")
    ctx = ssl.create_default_context(cafile=ca)
    with socket.create_connection((addr, int(port)), timeout=10) as raw:
        with ctx.wrap_socket(raw, server_hostname=host) as s:
            s.sendall(f"GET / HTTP/1.1\r\nHost: {host}\r\nConnection: close\r\n\r\n".encode())
            data = b""
            while True:
                chunk = s.recv(4096)
                if not chunk:
                    break
                data += chunk
    code = int(data.split(b" ", 2)[1])
    print(f"status={code}")
    return 0 if code == 200 else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("serve")
    s.add_argument("--cert", required=True)
    s.add_argument("--key", required=True)
    s.add_argument("--port", type=int, required=True)
    g = sub.add_parser("get")
    g.add_argument("--ca", required=True)
    g.add_argument("--host", required=True)
    g.add_argument("--connect", required=True)
    a = ap.parse_args(argv)
    if a.cmd == "serve":
        serve(a.cert, a.key, a.port)
        return 0
    return get(a.ca, a.host, a.connect)


if __name__ == "__main__":
    sys.exit(main())
