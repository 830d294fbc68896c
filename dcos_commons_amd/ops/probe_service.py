"""The node-local GPU readiness service (``native/build/amd-gpu-probed``) and its client protocol.

A GPU pod's readiness check is a command the agent runs in the task's sandbox. As
``amd-gpu-probe --readiness`` every check starts a HIP runtime from nothing (about 0.3-0.4 s on an
MI355X node) to do ~60 us of GPU work. The service keeps one runtime and the fused readiness
context of every device of the node resident; the check command becomes ``amd-gpu-ready``, which
sends ``READY <physical device>`` over a Unix socket and exits 0/1 on the reply (it links no HIP
library; without a reachable service it runs ``amd-gpu-probe --readiness`` itself). The agent
hands tasks the socket in ``AMD_GPU_PROBE_SOCKET``, as it hands them ``HIP_VISIBLE_DEVICES``.

``ProbeService`` runs the daemon as a child of this process (``LocalCluster(gpu_probe_service=True)``
starts one per node); ``ask`` is the client protocol in Python.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import time
from typing import Dict, Optional

from dcos_commons_amd.ops.build import BUILD

SOCKET_ENV = "AMD_GPU_PROBE_SOCKET"
SERVICE_BINARY = os.path.join(BUILD, "amd-gpu-probed")
CLIENT_BINARY = os.path.join(BUILD, "amd-gpu-ready")


def ask(socket_path: str, device: int, inject: int = 0, timeout_s: float = 30.0) -> Dict:
    """One readiness request for physical GPU ``device``: the service's JSON reply."""
    with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
        s.settimeout(timeout_s)
        s.connect(socket_path)
        s.sendall(f"READY {int(device)} {int(inject)}\n".encode())
        buf = b""
        while not buf.endswith(b"\n"):
            chunk = s.recv(4096)
            if not chunk:
                break
            buf += chunk
    return json.loads(buf.decode() or "{}")


class ProbeService:
    """``amd-gpu-probed`` as a child process, listening on ``socket_path``. ``warm`` probes every
    visible device at start (runtime, code objects and contexts ready before the first pod);
    the daemon exits with this process (``--parent-death``) or on ``stop()``. The parent-death
    signal follows the *thread* that started it (Linux ``PR_SET_PDEATHSIG``): start the service
    from a thread that lives as long as the service should, e.g. the main thread."""

    def __init__(self, socket_path: str, binary: str = SERVICE_BINARY, warm: bool = True,
                 env: Optional[Dict[str, str]] = None, log_path: Optional[str] = None):
        self.socket_path = socket_path
        self.binary = binary
        self.warm = warm
        self.env = env
        self.log_path = log_path or socket_path + ".log"
        self.proc: Optional[subprocess.Popen] = None

    @property
    def task_env(self) -> Dict[str, str]:
        return {SOCKET_ENV: self.socket_path}

    def start(self, timeout_s: float = 120.0) -> "ProbeService":
        if not os.path.exists(self.binary):
            raise FileNotFoundError(f"{self.binary} is not built (python -c 'import __graft_entry__ as g; g.build()')")
        argv = [self.binary, "--socket", self.socket_path, "--parent-death"] + (["--warm"] if self.warm else [])
        with open(self.log_path, "ab") as log:
            self.proc = subprocess.Popen(argv, stdin=subprocess.DEVNULL, stdout=log, stderr=log,
                                         env=dict(os.environ, **(self.env or {})))
        deadline = time.monotonic() + timeout_s
        while True:
            try:
                with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
                    s.settimeout(1.0)
                    s.connect(self.socket_path)
                return self
            except OSError:
                if self.proc.poll() is not None or time.monotonic() > deadline:
                    rc = self.proc.poll()
                    self.stop()
                    raise RuntimeError(f"GPU probe service did not start (exit {rc}); see {self.log_path}")
                time.sleep(0.02)

    def served(self) -> int:
        """Checks the service has answered so far (one ``served`` log line each)."""
        try:
            with open(self.log_path, "rb") as f:
                return sum(1 for line in f if line.startswith(b"served READY"))
        except OSError:
            return 0

    def stop(self, timeout_s: float = 15.0) -> None:
        if self.proc is None:
            return
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout_s)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)
        self.proc = None
