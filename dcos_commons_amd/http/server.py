"""Threaded HTTP server for the scheduler API.

Reference: sdk/.../framework/ApiServer.java:40-210 (Jetty on ``PORT_API``, start timeout
``API_SERVER_TIMEOUT_S``, started-callback once listening, optional wait for the scheduler's
DNS name to resolve to ``LIBPROCESS_IP``). Requests are dispatched through ``api.Router``;
``/v1/metrics`` is always mounted.
"""
from __future__ import annotations

import logging
import selectors
import socket
import threading
from http.server import BaseHTTPRequestHandler
from typing import Callable, Iterable, Optional

from dcos_commons_amd.framework.process_exit import ProcessExit
from dcos_commons_amd.utils.http_server import QuietThreadingHTTPServer

from .api import Router
from .resources import MetricsResource

LOGGER = logging.getLogger(__name__)


def resolve_scheduler_dns(hostname: str, expected_address: str) -> bool:
    """ApiServer.resolveSchedulerDNS: <=2 addresses (one v4 + one v6) containing ``expected``."""
    try:
        infos = socket.getaddrinfo(hostname, None)
    except OSError:
        return False
    addrs = []
    for fam, _, _, _, sa in infos:
        if sa[0] not in [a for _, a in addrs]:
            addrs.append((fam, sa[0]))
    if len(addrs) > 2:
        return False
    if len(addrs) == 2 and addrs[0][0] == addrs[1][0]:
        return False
    return any(a == expected_address for _, a in addrs)


class _Handler(BaseHTTPRequestHandler):
    router: Router = None
    protocol_version = "HTTP/1.1"

    def log_message(self, fmt, *args):  # route through logging instead of stderr
        LOGGER.debug("%s - " + fmt, self.address_string(), *args)

    def setup(self):
        super().setup()
        # responses go out in one write (below), so nothing waits on Nagle + the client's delayed
        # ACK on a keep-alive connection (a poller reusing its connection stalled 40 ms per request)
        self.connection.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def _handle(self, method: str):
        n = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(n) if n > 0 else b""
        resp = self.router.dispatch(method, self.path, body, dict(self.headers.items()))
        payload = resp.payload()
        self.send_response(resp.status)
        self.send_header("Content-Type", resp.content_type)
        self.send_header("Content-Length", str(len(payload)))
        # status line, headers and body in one write (BaseHTTPRequestHandler.end_headers would
        # flush the headers on their own; an HTTP/0.9 request gets no header buffer at all)
        if not hasattr(self, "_headers_buffer"):
            self._headers_buffer = []
        else:
            self._headers_buffer.append(b"\r\n")
        if method != "HEAD":
            self._headers_buffer.append(payload)
        self.flush_headers()

    def do_GET(self):
        self._handle("GET")

    def do_POST(self):
        self._handle("POST")

    def do_PUT(self):
        self._handle("PUT")

    def do_DELETE(self):
        self._handle("DELETE")


class ApiServer:
    def __init__(self, port: int, resources: Iterable, host: str = "127.0.0.1"):
        self.router = Router(list(resources) + [MetricsResource()])
        handler = type("Handler", (_Handler,), {"router": self.router})
        self.httpd = QuietThreadingHTTPServer((host, port), handler)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self._thread: Optional[threading.Thread] = None
        # serve loop wake-up: stop() returns at once instead of after socketserver's poll interval
        # (serve_forever(0.2) made every scheduler stop -- failover, config-update restart -- wait
        # up to 200 ms on the API server alone)
        self._wake_r, self._wake_w = socket.socketpair()
        self._stopping = threading.Event()
        self._serving = threading.Event()
        self._stopped = threading.Event()
        # poll(2), as socketserver uses; built here, not on the serving thread inside a timed start
        self._selector = selectors.PollSelector()
        self._selector.register(self.httpd, selectors.EVENT_READ)
        self._selector.register(self._wake_r, selectors.EVENT_READ)

    def serve(self) -> None:
        """Handles requests until ``stop()``; woken by a listening-socket event or the stop pipe."""
        self._serving.set()
        sel = self._selector
        try:
            while not self._stopping.is_set():
                for key, _ in sel.select():
                    if key.fileobj is self.httpd and not self._stopping.is_set():
                        self.httpd._handle_request_noblock()  # noqa: SLF001 - socketserver's own dispatch
                self.httpd.service_actions()
        finally:
            sel.close()
            self._stopped.set()

    @staticmethod
    def start(scheduler_config, resources, started_callback: Callable[[], None], port: Optional[int] = None,
              scheduler_hostname: Optional[str] = None, wait_for_dns: bool = False) -> "ApiServer":
        # loopback unless the operator opts in to a wider bind (SDK_API_HOST)
        host = scheduler_config.env.get_optional("SDK_API_HOST", "127.0.0.1")
        srv = ApiServer(scheduler_config.api_server_port() if port is None else port, resources, host)
        timeout = scheduler_config.api_server_init_timeout_s()

        def run():
            try:
                if wait_for_dns and scheduler_hostname:
                    ev = threading.Event()
                    deadline = threading.Timer(timeout, lambda: None if ev.is_set() else
                                               ProcessExit.exit(ProcessExit.API_SERVER_ERROR))
                    deadline.daemon = True
                    deadline.start()
                    while not resolve_scheduler_dns(scheduler_hostname, scheduler_config.scheduler_ip()):
                        if ev.wait(5):
                            break
                    ev.set()
                    deadline.cancel()
                started_callback()
                srv.serve()
            except Exception as e:  # noqa: BLE001
                LOGGER.exception("API server at port %d failed", srv.port)
                ProcessExit.exit(ProcessExit.API_SERVER_ERROR, e)

        srv._thread = threading.Thread(target=run, name="ApiServer", daemon=True)
        srv._thread.start()
        LOGGER.info("API server listening on port %d", srv.port)
        return srv

    def stop(self, timeout_s: float = 5.0) -> None:
        self._stopping.set()
        try:
            self._wake_w.send(b"x")
        except OSError:
            pass
        if self._serving.is_set() and self._thread is not threading.current_thread():
            self._stopped.wait(timeout_s)
        self.httpd.server_close()
        for sock in (self._wake_r, self._wake_w):
            try:
                sock.close()
            except OSError:
                pass

    def join(self) -> None:
        if self._thread is not None:
            self._thread.join()
