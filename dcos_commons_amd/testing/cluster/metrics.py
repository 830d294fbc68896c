"""The local cluster's dcos-metrics: a StatsD endpoint per container, read back per container.

On DC/OS every container gets ``STATSD_UDP_HOST`` / ``STATSD_UDP_PORT`` pointing at a socket the
agent's metrics service opened for that container alone (containers are keyed by
``mesos.local_master.container_id_for``, what the task's statuses report), so whatever a task (or a scheduler, which
is a Marathon task) emits is attributed to it, and ``/system/v1/agent/<agent>/metrics/v0/containers
[/<container>/app]`` returns it as datapoints with the container's dimensions (the reference's
``testing/sdk_metrics.py`` reads those; the scheduler pushes its registry there through
``metrics.StatsDReporter``). Here one thread serves every container's UDP socket.

StatsD lines: ``name:value|c`` (counters add up), ``|g`` (gauges: last value, ``+``/``-`` adjust),
``|ms`` / ``|h`` / ``|d`` (timers and histograms: last value); an optional ``|@rate`` scales
counters, ``|#tags`` are ignored. Several lines may share one datagram.
"""
from __future__ import annotations

import logging
import selectors
import socket
import threading
from typing import Dict, List, Optional

LOGGER = logging.getLogger(__name__)


class _Container:
    __slots__ = ("id", "agent_id", "dimensions", "sock", "values", "kinds")

    def __init__(self, cid: str, agent_id: str, dimensions: Dict[str, str], sock: socket.socket):
        self.id, self.agent_id, self.dimensions, self.sock = cid, agent_id, dict(dimensions), sock
        self.values: Dict[str, float] = {}
        self.kinds: Dict[str, str] = {}


class LocalMetrics:
    def __init__(self, host: str = "127.0.0.1"):
        self.host = host
        self._sel = selectors.DefaultSelector()
        self._lock = threading.Lock()
        self._containers: Dict[str, _Container] = {}
        self._wake_r, self._wake_w = socket.socketpair()
        self._sel.register(self._wake_r, selectors.EVENT_READ, None)
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="local-metrics", daemon=True)
        self._thread.start()

    # -- containers ---------------------------------------------------------------------------
    def container_env(self, container_id: str, agent_id: str, dimensions: Optional[Dict[str, str]] = None
                      ) -> Dict[str, str]:
        """The StatsD address of ``container_id``'s own socket (opened on first use)."""
        with self._lock:
            c = self._containers.get(container_id)
            if c is None:
                sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
                sock.bind((self.host, 0))
                sock.setblocking(False)
                c = self._containers[container_id] = _Container(container_id, agent_id, dimensions or {}, sock)
                self._sel.register(sock, selectors.EVENT_READ, c)
                self._wake_w.send(b"x")
            port = c.sock.getsockname()[1]
        return {"STATSD_UDP_HOST": self.host, "STATSD_UDP_PORT": str(port)}

    def containers(self, agent_id: Optional[str] = None) -> List[str]:
        with self._lock:
            return sorted(c.id for c in self._containers.values() if agent_id is None or c.agent_id == agent_id)

    def app(self, container_id: str) -> Optional[dict]:
        """``/metrics/v0/containers/<id>/app``: the container's datapoints and dimensions."""
        with self._lock:
            c = self._containers.get(container_id)
            if c is None:
                return None
            points = [{"name": n, "value": v, "unit": "", "tags": {}} for n, v in sorted(c.values.items())]
            return {"datapoints": points, "dimensions": dict(c.dimensions, container_id=c.id, agent_id=c.agent_id)}

    def stop(self) -> None:
        self._stop = True
        try:
            self._wake_w.send(b"x")
        except OSError:
            pass
        self._thread.join(5)
        with self._lock:
            for c in self._containers.values():
                c.sock.close()
            self._containers.clear()
        self._wake_r.close()
        self._wake_w.close()

    # -- StatsD -----------------------------------------------------------------------------
    def _loop(self) -> None:
        while not self._stop:
            for key, _ in self._sel.select(timeout=1.0):
                if key.data is None:
                    try:
                        self._wake_r.recv(4096)
                    except OSError:
                        pass
                    continue
                try:
                    data = key.fileobj.recv(65535)
                except OSError:
                    continue
                self._ingest(key.data, data.decode("utf-8", "replace"))

    def _ingest(self, c: _Container, text: str) -> None:
        with self._lock:
            for line in text.splitlines():
                try:
                    name, rest = line.strip().split(":", 1)
                    fields = rest.split("|")
                    raw, kind = fields[0], fields[1] if len(fields) > 1 else "c"
                    rate = next((float(f[1:]) for f in fields[2:] if f.startswith("@")), 1.0)
                    value = float(raw)
                except (ValueError, IndexError):
                    LOGGER.debug("not a StatsD line: %r", line)
                    continue
                if kind == "c":
                    c.values[name] = c.values.get(name, 0.0) + value / (rate or 1.0)
                elif kind == "g" and raw[:1] in "+-" and name in c.values:
                    c.values[name] += value
                else:
                    c.values[name] = value
                c.kinds[name] = kind
