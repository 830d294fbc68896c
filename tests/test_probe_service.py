"""The node-local GPU readiness service (``amd-gpu-probed``) and its check command (``amd-gpu-ready``).

CPU tier: the client against a scripted socket server (device translation through the task's
``HIP_VISIBLE_DEVICES``, exit codes, JSON output, fallback rules), in the release and the
ASan/UBSan build; the daemon's protocol, error replies, idle exit and signal shutdown without a
GPU. GPU tier: the resident probe's numerics and fault injection through the service, the check
command against it, and a local cluster whose GPU pod goes ready through the service."""
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SANITIZER_ENV = {"ASAN_OPTIONS": "halt_on_error=1:abort_on_error=1:detect_leaks=1",
                 "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


@pytest.fixture(scope="module", params=["release", "sanitize"])
def client(request):
    from dcos_commons_amd.ops import build

    try:
        targets = build.build_cpp_tools(sanitize=request.param == "sanitize")
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native toolchain unavailable: {e}")
    exe = [t for t in targets if t.endswith("amd-gpu-ready")][0]
    env = dict(SANITIZER_ENV) if request.param == "sanitize" else {}
    return exe, env


class FakeService:
    """A Unix-socket server that records each request line and answers with ``reply(line)``."""

    def __init__(self, path, reply):
        self.path = path
        self.reply = reply
        self.requests = []
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.bind(path)
        self.sock.listen(8)
        self.sock.settimeout(0.2)
        self._stop = False
        self.thread = threading.Thread(target=self._loop, daemon=True)
        self.thread.start()

    def _loop(self):
        while not self._stop:
            try:
                conn, _ = self.sock.accept()
            except OSError:
                continue
            with conn:
                buf = b""
                while not buf.endswith(b"\n"):
                    chunk = conn.recv(256)
                    if not chunk:
                        break
                    buf += chunk
                line = buf.decode().strip()
                self.requests.append(line)
                conn.sendall((self.reply(line) + "\n").encode())

    def close(self):
        self._stop = True
        self.thread.join(2)
        self.sock.close()


def _run(exe, env, *args, extra_env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                          "AMD_GPU_PROBE_SOCKET")}
    e.update(env)
    e.update(extra_env or {})
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=60, env=e)


def test_client_sends_the_physical_device_and_maps_the_reply(client, tmp_path):
    exe, env = client
    healthy = {"device": 7, "ordinal": 7, "gemm_rel_err": 1e-6, "mem_bad_words": 0, "healthy": True}
    svc = FakeService(str(tmp_path / "s.sock"), lambda line: json.dumps(healthy))
    try:
        # the task's second visible device is physical GPU 7
        r = _run(exe, env, "--device", "1", "--json",
                 extra_env={"AMD_GPU_PROBE_SOCKET": svc.path, "HIP_VISIBLE_DEVICES": "5,7"})
        assert r.returncode == 0, r.stderr
        assert svc.requests[-1] == "READY 7 0"
        assert json.loads(r.stdout)["healthy"] is True
        # --socket overrides the environment; ROCR_VISIBLE_DEVICES is the second source
        r = _run(exe, env, "--socket", svc.path, "--readiness", extra_env={"ROCR_VISIBLE_DEVICES": "3"})
        assert r.returncode == 0 and svc.requests[-1] == "READY 3 0"
        # no visible-device list: the index is the physical device
        r = _run(exe, env, "--socket", svc.path, "--device", "2", "--inject", "1")
        assert r.returncode == 0 and svc.requests[-1] == "READY 2 1"
    finally:
        svc.close()


def test_client_exit_codes(client, tmp_path):
    exe, env = client
    answers = {"unhealthy": json.dumps({"device": 0, "healthy": False, "mem_bad_words": 3}),
               "error": json.dumps({"device": 0, "error": "device not visible to the probe service"})}
    mode = {"v": "unhealthy"}
    svc = FakeService(str(tmp_path / "s.sock"), lambda line: answers[mode["v"]])
    try:
        r = _run(exe, env, "--socket", svc.path)
        assert r.returncode == 1
        mode["v"] = "error"
        r = _run(exe, env, "--socket", svc.path, "--no-fallback")
        assert r.returncode == 2 and "not visible" in r.stderr
    finally:
        svc.close()
    # unreachable service, no fallback: an error, never a pass
    r = _run(exe, env, "--socket", str(tmp_path / "missing.sock"), "--no-fallback")
    assert r.returncode == 2 and "unreachable" in r.stderr
    # bad usage
    assert _run(exe, env, "--bogus").returncode == 2
    assert _run(exe, env, "--device", "-1").returncode == 2
    # a device index beyond the task's visible list is not guessed at
    r = _run(exe, env, "--socket", str(tmp_path / "missing.sock"), "--device", "3", "--no-fallback",
             extra_env={"HIP_VISIBLE_DEVICES": "0"})
    assert r.returncode == 2


def test_client_busy_service_retries_once_then_fails_without_a_standalone_probe(client, tmp_path):
    """a saturated service answers ``busy``; the client asks once more after a short
    backoff and then fails the check (exit 1: the agent retries at the next interval). It does not
    start ``amd-gpu-probe`` -- a fresh HIP runtime per refused check would add load exactly when
    the node is busiest."""
    exe, env = client
    healthy = json.dumps({"device": 0, "healthy": True})
    mode = {"busy": 2}

    def reply(line):
        if mode["busy"] > 0:
            mode["busy"] -= 1
            return json.dumps({"error": "busy"})
        return healthy
    svc = FakeService(str(tmp_path / "s.sock"), reply)
    try:
        # busy twice: exit 1, exactly two requests, no fallback message
        r = _run(exe, env, "--socket", svc.path)
        assert r.returncode == 1 and len(svc.requests) == 2, (r.returncode, svc.requests, r.stderr)
        assert "busy" in r.stderr and "standalone" not in r.stderr
        # busy once: the retry gets the answer
        mode["busy"] = 1
        r = _run(exe, env, "--socket", svc.path)
        assert r.returncode == 0 and len(svc.requests) == 4
    finally:
        svc.close()


def test_client_falls_back_to_the_standalone_probe(client, tmp_path):
    """Without a service the check runs ``amd-gpu-probe --readiness`` next to it as a child: on a
    host without a GPU that probe reports unhealthy (1), so the check fails rather than passing."""
    exe, env = client
    probe = os.path.join(os.path.dirname(exe), "amd-gpu-probe")
    if not os.path.exists(probe):
        pytest.skip("standalone probe not built next to the client")
    r = _run(exe, env, "--socket", str(tmp_path / "missing.sock"))
    assert r.returncode in (0, 1), r.stderr
    if not _has_gpu():
        assert r.returncode == 1


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


@pytest.fixture(scope="module")
def daemon_binary():
    from dcos_commons_amd.ops import build

    try:
        return build.build_probe_service()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"hipcc unavailable: {e}")


@pytest.mark.skipif(_has_gpu(), reason="error-path checks need a host without a GPU")
def test_daemon_protocol_and_lifecycle_without_gpu(daemon_binary, tmp_path):
    from dcos_commons_amd.ops.probe_service import ProbeService, ask

    path = str(tmp_path / "p.sock")
    svc = ProbeService(path, binary=daemon_binary, warm=False).start(timeout_s=30)
    try:
        rep = ask(path, 0)
        assert "error" in rep and rep["device"] == 0          # no device: an error reply, never healthy
        with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
            s.connect(path)
            s.sendall(b"HELLO\n")
            assert json.loads(s.recv(256).decode()) == {"error": "bad request"}
        assert svc.served() == 1
    finally:
        svc.stop()
    assert not os.path.exists(path)                           # SIGTERM removes the socket


def test_daemon_idle_exit_and_visible_device_mapping(daemon_binary, tmp_path):
    from dcos_commons_amd.ops.probe_service import ask

    path = str(tmp_path / "p.sock")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="4,6")
    p = subprocess.Popen([daemon_binary, "--socket", path, "--idle-exit", "0.5"], env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        deadline = time.monotonic() + 30
        while not os.path.exists(path):
            assert time.monotonic() < deadline and p.poll() is None
            time.sleep(0.02)
        # physical 5 is not among the service's devices; physical 6 is its ordinal 1
        assert ask(path, 5)["error"] == "device not visible to the probe service"
        rep = ask(path, 6)
        assert rep["ordinal"] == 1
        assert p.wait(30) == 0                                # idle for 0.5 s: exits by itself
    finally:
        if p.poll() is None:
            p.send_signal(signal.SIGKILL)
            p.wait(5)
    assert not os.path.exists(path)


@pytest.mark.gpu
def test_service_probe_numerics_and_fault_injection(daemon_binary, tmp_path):
    from dcos_commons_amd.ops.probe_service import ProbeService, ask

    path = str(tmp_path / "p.sock")
    svc = ProbeService(path, binary=daemon_binary, warm=True).start(timeout_s=120)
    try:
        rep = ask(path, 0)
        assert rep["healthy"] is True and rep["mem_bad_words"] == 0 and rep["gemm_rel_err"] < 1e-3, rep
        for inject in (1, 2, 3, 4):                           # lost tile, bad word, no GEMM, no write
            bad = ask(path, 0, inject=inject)
            assert bad["healthy"] is False, (inject, bad)
        times = []
        for _ in range(20):
            t0 = time.perf_counter()
            assert ask(path, 0)["healthy"] is True
            times.append(time.perf_counter() - t0)
        times.sort()
        assert times[len(times) // 2] < 0.05, times           # resident runtime: no per-check HIP start
    finally:
        svc.stop()


@pytest.mark.gpu
def test_ready_command_uses_the_service(daemon_binary, tmp_path):
    from dcos_commons_amd.ops import build
    from dcos_commons_amd.ops.probe_service import ProbeService

    exe = [t for t in build.build_cpp_tools() if t.endswith("amd-gpu-ready")][0]
    path = str(tmp_path / "p.sock")
    svc = ProbeService(path, binary=daemon_binary).start(timeout_s=120)
    try:
        t0 = time.perf_counter()
        r = _run(exe, {}, "--json", "--no-fallback", extra_env={"AMD_GPU_PROBE_SOCKET": path,
                                                                 "HIP_VISIBLE_DEVICES": "0"})
        dt = time.perf_counter() - t0
        assert r.returncode == 0, r.stderr
        assert json.loads(r.stdout)["healthy"] is True
        assert svc.served() == 1                              # answered by the service (warm-up not counted)
        r = _run(exe, {}, "--inject", "1", "--no-fallback", extra_env={"AMD_GPU_PROBE_SOCKET": path})
        assert r.returncode == 1 and svc.served() == 2
        assert dt < 1.0
    finally:
        svc.stop()


@pytest.mark.gpu
def test_cluster_gpu_pod_goes_ready_through_the_service():
    """helloworld gpu.yml on the local DC/OS stand-in (scheduler process, v1 HTTP API, ZooKeeper,
    real task processes) with the node's readiness service: the pod's check is ``amd-gpu-ready
    --no-fallback``, so deploy, restart and replace only complete if the service probed the GPU."""
    from dcos_commons_amd.benchmarks.cluster_bench import ClusterBench
    from dcos_commons_amd.ops.probe_service import CLIENT_BINARY

    bench = ClusterBench(1, probe_cmd=CLIENT_BINARY + " --no-fallback", probe_service=True, timeout_s=90)
    try:
        r = bench.run_cycle()
        assert bench.cluster.probe_service.served() >= 3      # deploy, restart, replace
    finally:
        bench.close()
    assert r["deploy_s"] < 10 and r["mttr_restart_s"] < 10 and r["mttr_replace_s"] < 10, r


def test_cluster_probe_service_needs_process_executor():
    from dcos_commons_amd.testing.cluster import LocalCluster

    with pytest.raises(ValueError):
        LocalCluster(agents=1, executor="synthetic", gpu_probe_service=True)


@pytest.mark.skipif(_has_gpu(), reason="needs a host where the service cannot start")
def test_cluster_start_failure_shuts_down_what_started(daemon_binary):
    """The service cannot start without a GPU: start() raises and leaves no ZooKeeper, master or
    work directory behind."""
    from dcos_commons_amd.testing.cluster import LocalCluster

    c = LocalCluster(agents=1, gpus_per_agent=1, gpu_probe_service=True, zk_process=True)
    with pytest.raises(RuntimeError, match="GPU probe service did not start"):
        c.start()
    assert c.zk.proc.poll() is not None                       # the ZooKeeper process was stopped
    assert not os.path.exists(c.work_dir)
    assert not c.master._thread.is_alive()
