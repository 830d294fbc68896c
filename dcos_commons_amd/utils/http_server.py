"""The threading HTTP server behind the scheduler API and the Mesos master stand-in.

Two departures from ``http.server.ThreadingHTTPServer``:

* no reverse DNS lookup of the bind address (``HTTPServer.server_bind`` calls ``socket.getfqdn``
  only to fill ``server_name``, which nothing here reads; on a host whose resolver goes to the
  network it is the slowest step of a scheduler's start-up);
* a client that goes away mid-request (a scheduler process killed while its call is answered, a
  poller that times out) is logged at debug level instead of printing a traceback to stderr:
  that is how a stream ends, not a server fault. Other handler errors are still logged in full.
"""
from __future__ import annotations

import logging
import socketserver
import sys
from http.server import ThreadingHTTPServer

LOGGER = logging.getLogger(__name__)


class QuietThreadingHTTPServer(ThreadingHTTPServer):
    daemon_threads = True

    def server_bind(self):
        socketserver.TCPServer.server_bind(self)
        host, port = self.server_address[:2]
        self.server_name = host
        self.server_port = port

    def handle_error(self, request, client_address):
        err = sys.exc_info()[1]
        if isinstance(err, ConnectionError):   # BrokenPipe, ConnectionReset, ConnectionAborted
            LOGGER.debug("client %s went away: %s", client_address, err)
            return
        LOGGER.exception("error serving a request from %s", client_address)
