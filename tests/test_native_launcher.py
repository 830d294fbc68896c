"""``sdk-agent-launcher`` (``native/agent/launcher.cpp``) through its client
``mesos.containerizer.NativeLauncher``: the local DC/OS stand-in's agents start task processes and
check commands through it instead of forking from the master's interpreter.

Covered: a launch reports its pid before it runs and its exit status when reaped; stdout/stderr go
to the sandbox files; the environment and working directory are exactly the ones sent; every
process leads its own session (so the containerizer can signal the whole task); a signalled
process reports ``-signal`` as ``subprocess`` does; ``run`` returns a command's exit code, 124 at
its timeout (the process group is killed) and 127 when the program does not exist; the helper
exits when its client goes away. Runs against the release and the ASan/UBSan builds.
"""
import os
import signal
import threading
import time

import pytest

from dcos_commons_amd.mesos.containerizer import NativeLauncher


@pytest.fixture(scope="module", params=["release", "sanitize"])
def binary(request):
    from dcos_commons_amd.ops import build

    try:
        targets = build.build_cpp_tools(sanitize=request.param == "sanitize")
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native toolchain unavailable: {e}")
    return [t for t in targets if t.endswith("sdk-agent-launcher")][0]


@pytest.fixture
def launcher(binary, monkeypatch):
    monkeypatch.setenv("ASAN_OPTIONS", "halt_on_error=1:detect_leaks=1")
    nl = NativeLauncher(binary)
    yield nl
    nl.close()


ENV = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"), "GREETING": "hello there", "MULTI": "a\nb"}


def _launch(nl, tmp_path, cmd):
    exits = []
    done = threading.Event()

    def on_exit(proc, rc):
        exits.append((proc.pid, rc))
        done.set()
    p = nl.launch(["mesos-default-executor", "-c", cmd + "\nexit $?"], "/bin/bash", str(tmp_path), ENV,
                  str(tmp_path / "stdout"), str(tmp_path / "stderr"), on_exit)
    return p, exits, done


def test_launch_reports_pid_output_environment_and_exit(launcher, tmp_path):
    p, exits, done = _launch(launcher, tmp_path, 'echo "$GREETING|$MULTI|$(pwd)"; echo err >&2; exit 7')
    assert p.pid > 0
    assert done.wait(10)
    assert exits == [(p.pid, 7)] and p.wait(0) == 7 and p.poll() == 7
    assert (tmp_path / "stdout").read_text() == f"hello there|a\nb|{tmp_path}\n"
    assert (tmp_path / "stderr").read_text() == "err\n"


def test_task_leads_its_own_session_and_reports_the_signal(launcher, tmp_path):
    p, exits, done = _launch(launcher, tmp_path, "sleep 30 & wait")
    deadline = time.time() + 5
    while os.getsid(p.pid) != p.pid and time.time() < deadline:   # setsid runs right after fork
        time.sleep(0.01)
    assert os.getsid(p.pid) == p.pid and os.getpgid(p.pid) == p.pid
    os.killpg(p.pid, signal.SIGTERM)      # the whole task, its background sleep included
    assert done.wait(10)
    assert exits[0][1] == -signal.SIGTERM


def test_run_exit_codes_timeout_and_missing_program(launcher, tmp_path):
    assert launcher.run(["bash", "-c", "exit 3"], str(tmp_path), ENV, 5) == 3
    assert launcher.run(["bash", "-c", 'test "$GREETING" = "hello there"'], str(tmp_path), ENV, 5) == 0
    t0 = time.perf_counter()
    assert launcher.run(["bash", "-c", "sleep 30"], str(tmp_path), ENV, 0.2) == 124
    assert time.perf_counter() - t0 < 5
    assert launcher.run(["/no/such/program"], str(tmp_path), ENV, 5) == 127


def test_many_concurrent_runs(launcher, tmp_path):
    out = [None] * 32

    def one(i):
        out[i] = launcher.run(["bash", "-c", f"exit {i % 5}"], str(tmp_path), ENV, 10)
    ts = [threading.Thread(target=one, args=(i,)) for i in range(32)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(20)
    assert out == [i % 5 for i in range(32)]


def test_helper_exits_when_its_client_goes_away(binary):
    import socket

    nl = NativeLauncher(binary)
    nl._ours.shutdown(socket.SHUT_RDWR)    # the master process died: its end of the socket is gone
    assert nl.proc.wait(5) == 0


def test_unwaited_launch_sets_up_the_sandbox_first(launcher, tmp_path):
    """The containerizer's launch: the helper creates the sandbox and the volume directories,
    links the volumes at their container paths, then forks; the caller does not wait for the pid."""
    sandbox = tmp_path / "agent" / "frameworks" / "fw" / "tasks" / "t1"
    volume = tmp_path / "agent" / "volumes" / "v1"
    (tmp_path / "existing").mkdir()
    exits, errors, done = [], [], threading.Event()

    def on_exit(proc, rc):
        exits.append(rc)
        done.set()
    p = launcher.launch(["mesos-default-executor", "-c", "ls data/ >/dev/null && echo ok > data/f\nexit $?"], "/bin/bash",
                        str(sandbox), ENV, str(sandbox / "stdout"), str(sandbox / "stderr"), on_exit,
                        setup=[("d", str(sandbox)), ("d", str(volume)), ("l", str(volume), str(sandbox / "data")),
                               ("l", str(tmp_path / "existing"), str(sandbox / "a" / "b")),
                               ("d", str(sandbox / "data"))],     # in order: the link is there first
                        on_error=lambda proc, msg: errors.append(msg))
    assert p.wait_started(10) > 0
    assert done.wait(10) and exits == [0] and errors == []
    assert (volume / "f").read_text() == "ok\n"
    assert os.path.islink(sandbox / "data") and os.readlink(sandbox / "a" / "b") == str(tmp_path / "existing")
    # a relaunch in place: the links exist already and are kept
    done.clear()
    launcher.launch(["x", "-c", "cat data/f"], "/bin/bash", str(sandbox), ENV, str(sandbox / "stdout2"), "",
                    on_exit, setup=[("d", str(sandbox)), ("l", str(volume), str(sandbox / "data"))],
                    on_error=lambda proc, msg: errors.append(msg))
    assert done.wait(10) and errors == [] and (sandbox / "stdout2").read_text() == "ok\n"


def test_unwaited_launch_reports_a_failed_set_up(launcher, tmp_path):
    blocker = tmp_path / "file"
    blocker.write_text("not a directory")
    failed, done = [], threading.Event()

    def on_error(proc, msg):
        failed.append((proc.pid, msg))
        done.set()
    p = launcher.launch(["x", "-c", "true"], "/bin/bash", str(blocker / "sandbox"), ENV, "", "",
                        lambda proc, rc: None, setup=[("d", str(blocker / "sandbox"))], on_error=on_error)
    assert done.wait(10)
    assert failed[0][0] == 0 and "mkdir" in failed[0][1]
    assert p.wait_started(1) == 0 and p.poll() == 127
