"""``utils.http_server.QuietThreadingHTTPServer``, the server behind the scheduler API and the
Mesos master stand-in: no reverse DNS lookup at bind, client disconnects logged quietly."""
import logging
import socket
import threading
import time
import urllib.request
from http.server import BaseHTTPRequestHandler

from dcos_commons_amd.utils.http_server import QuietThreadingHTTPServer


def test_quiet_http_server_drops_client_disconnects_only(caplog):
    """The API/master HTTP server: a client that went away is a debug line, not a traceback on
    stderr; any other handler error is still logged as an error."""
    class H(BaseHTTPRequestHandler):
        def do_GET(self):
            if self.path == "/gone":
                raise BrokenPipeError("client went away")
            raise ValueError("handler bug")

        def log_message(self, *a):
            pass

    srv = QuietThreadingHTTPServer(("127.0.0.1", 0), H)
    assert srv.server_name == "127.0.0.1"               # no reverse lookup of the bind address
    t = threading.Thread(target=srv.serve_forever, kwargs={"poll_interval": 0.05}, daemon=True)
    t.start()
    try:
        with caplog.at_level(logging.DEBUG, logger="dcos_commons_amd.utils.http_server"):
            for path in ("/gone", "/bug"):
                try:
                    urllib.request.urlopen(f"http://127.0.0.1:{srv.server_address[1]}{path}", timeout=5)
                except (OSError, socket.error):
                    pass
            deadline = time.monotonic() + 5
            while len(caplog.records) < 2 and time.monotonic() < deadline:
                time.sleep(0.01)
        levels = sorted((r.levelname, r.getMessage().split(":")[0]) for r in caplog.records)
        assert [lv for lv, _ in levels] == ["DEBUG", "ERROR"], levels
    finally:
        srv.shutdown()
        srv.server_close()


def test_api_server_stops_at_once_and_frees_its_port():
    """Scheduler restarts (failover, config rollout) stop the API server: the serve loop is woken
    by a stop pipe, not by socketserver's poll interval (was ~170 ms of every stop)."""
    from dcos_commons_amd.http.server import ApiServer
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig

    started = threading.Event()
    srv = ApiServer.start(SchedulerConfig.for_testing(PORT_API="0"), [], started.set, port=0)
    assert started.wait(5)
    with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/v1/metrics", timeout=5) as r:
        assert r.status == 200
    t0 = time.perf_counter()
    srv.stop()
    assert time.perf_counter() - t0 < 0.05
    srv._thread.join(1)
    assert not srv._thread.is_alive()
    s = socket.socket()
    try:
        s.settimeout(1)
        assert s.connect_ex(("127.0.0.1", srv.port)) != 0
    finally:
        s.close()


def test_scheduler_runner_stop_is_bounded():
    from dcos_commons_amd.benchmarks.deploy_bench import DeployBench
    from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner

    stops = []
    orig = SchedulerRunner.stop

    def timed(self):
        t0 = time.perf_counter()
        orig(self)
        stops.append(time.perf_counter() - t0)
    SchedulerRunner.stop = timed
    try:
        DeployBench(1, allocation_interval_s=0.05).run_cycle()
    finally:
        SchedulerRunner.stop = orig
    assert stops and max(stops) < 0.05, stops


def test_keep_alive_requests_are_not_held_back_by_delayed_acks():
    """Each response leaves in one write with TCP_NODELAY: a client polling over one keep-alive
    connection used to stall ~40 ms per request (headers sent, body held by Nagle until the
    client's delayed ACK)."""
    import http.client

    from dcos_commons_amd.http.server import ApiServer
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig

    started = threading.Event()
    srv = ApiServer.start(SchedulerConfig.for_testing(PORT_API="0"), [], started.set, port=0)
    assert started.wait(5)
    conn = http.client.HTTPConnection("127.0.0.1", srv.port, timeout=5)
    try:
        conn.request("GET", "/v1/metrics")
        conn.getresponse().read()
        t0 = time.perf_counter()
        for _ in range(20):
            conn.request("GET", "/v1/metrics")
            r = conn.getresponse()
            assert r.status == 200 and r.read()
        assert time.perf_counter() - t0 < 0.4     # 20 x 40 ms = 0.8 s with the stall
    finally:
        conn.close()
        srv.stop()
