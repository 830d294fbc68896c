"""``sdk-agent-launcher`` (``native/agent/launcher.cpp``) through its client
``mesos.containerizer.NativeLauncher``: the local DC/OS stand-in's agents start task processes and
check commands through it instead of forking from the master's interpreter.

Covered: a launch reports its pid before it runs and its exit status when reaped; stdout/stderr go
to the sandbox files; the environment and working directory are exactly the ones sent; every
process leads its own session (so the containerizer can signal the whole task); a signalled
process reports ``-signal`` as ``subprocess`` does; ``run`` returns a command's exit code, 124 at
its timeout (the process group is killed) and 127 when the program does not exist; the helper
exits when its client goes away. An unwaited launch runs its sandbox set-up (directories, volume
links, in order) in the helper, and a failed set-up is reported instead of a start; through the
containerizer, STARTING is scheduled on the helper's started event and a sandbox the helper cannot
create fails the container. Runs against the release and the ASan/UBSan builds.
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


def test_tasks_get_default_sigpipe_and_sigxfsz(launcher, tmp_path):
    """The helper ignores SIGPIPE for itself; its children must not inherit that: a
    task's SigIgn mask has neither bit, and a pipeline's producer dies of SIGPIPE as under Popen."""
    p, exits, done = _launch(launcher, tmp_path, "grep SigIgn /proc/self/status; "
                                                 "yes | head -1 > /dev/null; echo \"${PIPESTATUS[0]}\"")
    assert done.wait(10) and exits[0][1] == 0
    sigign_line, producer_rc = (tmp_path / "stdout").read_text().split("\n")[:2]
    mask = int(sigign_line.split()[1], 16)
    assert not mask & (1 << (signal.SIGPIPE - 1)) and not mask & (1 << (signal.SIGXFSZ - 1))
    assert int(producer_rc) == 128 + signal.SIGPIPE


def test_send_failure_after_the_helper_died_is_reported_once(binary, tmp_path):
    """The helper dies between a launch's registration and its send: the read loop reports it
    through ``on_error``; the launch then returns instead of raising a second failure."""
    nl = NativeLauncher(binary)
    errors = []
    orig = nl._send

    def send_after_death(msg):
        nl.proc.kill()
        nl.proc.wait(5)
        deadline = time.time() + 5
        while not nl.closed and time.time() < deadline:   # the read loop saw EOF and failed the entry
            time.sleep(0.01)
        orig(msg)
    nl._send = send_after_death
    try:
        p = nl.launch(["x", "-c", "true"], "/bin/bash", str(tmp_path), ENV, "", "", lambda proc, rc: None,
                      on_error=lambda proc, msg: errors.append(msg))
        assert len(errors) == 1 and p.pid == 0
    except OSError:
        # the entry was still registered when the send failed: raising is then the only report
        assert errors == []
    finally:
        nl.close()


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


class _FakeMaster:
    """What ProcessTaskBehavior.launch needs of LocalMaster: ``_schedule`` and the callbacks it names."""

    def __init__(self):
        self.calls = []
        self.event = threading.Event()

    def _schedule(self, delay, fn, *args):
        self.calls.append((fn.__name__, args))
        self.event.set()

    def _lifecycle_starting(self, *a):
        pass

    def _container_failed(self, *a):
        pass

    def _process_exited(self, *a):
        pass

    def wait_for(self, name, timeout=10):
        deadline = time.time() + timeout
        while time.time() < deadline:
            hit = [args for fn, args in self.calls if fn == name]
            if hit:
                return hit[0]
            self.event.wait(0.05)
            self.event.clear()
        raise AssertionError(f"{name} not scheduled: {self.calls}")


def _task_and_agent(cmd, volume_path="data"):
    from types import SimpleNamespace

    from dcos_commons_amd.mesos import protos as P

    info = P.TaskInfo(name="hello-0-server")
    info.task_id.value = "svc__hello-0-server__1"
    info.command.value = cmd
    r = info.resources.add(name="disk", type=P.Value.SCALAR)
    r.scalar.value = 10
    r.disk.persistence.id = "vol-1"
    r.disk.volume.container_path = volume_path
    task = SimpleNamespace(info=info, framework_id="fw", executor_id="", epoch=1, gpu_devices=[])
    agent = SimpleNamespace(spec=SimpleNamespace(hostname="10.0.0.1"), id="agent-1", executors={})
    return task, agent


def test_containerizer_launches_through_the_helper_and_reports_start_then_exit(binary, tmp_path, monkeypatch):
    from dcos_commons_amd.mesos import containerizer as C

    monkeypatch.setattr(C, "native_launcher_binary", lambda: binary)
    beh = C.ProcessTaskBehavior(str(tmp_path / "work"))
    master = _FakeMaster()
    task, agent = _task_and_agent("echo hi > data/out")
    try:
        beh.launch(master, task, agent)
        master.wait_for("_lifecycle_starting")          # reported once the helper has forked
        args = master.wait_for("_process_exited")
        assert args[2] == 0                             # rc
        sandbox = beh.sandbox_of(task.info.task_id.value)
        assert os.path.islink(os.path.join(sandbox, "data"))
        assert open(os.path.join(beh.volume_dir("10.0.0.1", "vol-1"), "out")).read() == "hi\n"
    finally:
        beh.shutdown()


def test_containerizer_reports_a_sandbox_the_helper_cannot_create(binary, tmp_path, monkeypatch):
    from dcos_commons_amd.mesos import containerizer as C

    monkeypatch.setattr(C, "native_launcher_binary", lambda: binary)
    beh = C.ProcessTaskBehavior(str(tmp_path / "work"))
    (tmp_path / "work" / "10.0.0.1").write_text("a file where the agent directory should be")
    master = _FakeMaster()
    task, agent = _task_and_agent("true")
    try:
        beh.launch(master, task, agent)
        args = master.wait_for("_container_failed")
        assert "mkdir" in args[2]
        assert not [fn for fn, _ in master.calls if fn == "_lifecycle_starting"]
        # a kill of the task that never started signals nothing (no process group 0)
        assert beh.kill(master, task) is False
    finally:
        beh.shutdown()


def test_a_dead_helper_is_replaced_and_its_running_processes_are_watched(binary, tmp_path, monkeypatch):
    from dcos_commons_amd.mesos import containerizer as C

    monkeypatch.setattr(C, "native_launcher_binary", lambda: binary)
    beh = C.ProcessTaskBehavior(str(tmp_path / "work"))
    try:
        first = beh._native_launcher()
        exits, done = [], threading.Event()

        def on_exit(proc, rc):
            exits.append(rc)
            done.set()
        p = first.launch(["x", "-c", "sleep 0.3"], "/bin/bash", str(tmp_path), ENV, "", "", on_exit,
                         on_error=lambda proc, msg: None)
        assert p.wait_started(10) > 0
        first.proc.kill()                        # the helper dies under a running process
        first.proc.wait(5)
        assert done.wait(10)                     # its end is still reported (as a kill: the status is lost)
        assert exits == [-signal.SIGKILL]
        deadline = time.time() + 5
        while not first.closed and time.time() < deadline:
            time.sleep(0.01)
        second = beh._native_launcher()          # the next launch gets a new helper
        assert second is not first and not second.closed
        assert second.run(["bash", "-c", "exit 5"], str(tmp_path), ENV, 5) == 5
    finally:
        beh.shutdown()
