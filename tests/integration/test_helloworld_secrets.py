"""helloworld secrets and container-feature scenarios on the local cluster.

Reference: frameworks/helloworld/tests/{test_secrets.py, test_seccomp.py, test_shm.py,
test_share_pid_namespace.py}. Secrets from the cluster's secret store reach tasks as environment
variables, as files at a given path, or as files at the secret's own path; a changed secret is
seen after a pod restart, a config update pointing at other secrets rolls the pods; secrets
outside the service's DCOS_SPACE are refused, so the deploy never completes. Pods carry their
seccomp, shared-memory and shared-PID-namespace settings into the executor and task containers.
"""
import pytest

from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks, sdk_utils)
from tests.integration import hw_config as config

pytestmark = pytest.mark.usefixtures("local_cluster")

NUM_HELLO, NUM_WORLD = 2, 3
DEFAULT = "hello-world-secret-data"
ALTERNATIVE = DEFAULT + "-alternative"


def _options(prefix):
    return {"service": {"yaml": "secrets"},
            "hello": {"count": NUM_HELLO, "secret1": f"{prefix}secret1", "secret2": f"{prefix}secret2"},
            "world": {"count": NUM_WORLD, "secret1": f"{prefix}secret1", "secret2": f"{prefix}secret2",
                      "secret3": f"{prefix}secret3"}}


def _secrets(op, prefix, content=DEFAULT):
    for i in (1, 2, 3):
        value = f" --value={content}" if op != "delete" else ""
        sdk_cmd.run_cli(f"security secrets {op}{value} {prefix}secret{i}")


def _read(task, cmd):
    @sdk_utils.retry(timeout_s=30, interval_s=0.5)
    def read():
        rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, task, cmd)
        lines = [l.strip() for l in out.splitlines() if l.strip().startswith(DEFAULT)]
        assert rc == 0 and lines, (cmd, out)
        return lines[0]
    return read()


def _verify(content):
    assert _read("world-0-server", "echo $WORLD_SECRET1_ENV") == content       # env-key only
    assert _read("world-0-server", "cat WORLD_SECRET2_FILE") == content         # file only
    assert _read("world-0-server", f"cat {config.SERVICE_NAME}/secret3") == content   # default path
    assert _read("hello-0-server", "echo $HELLO_SECRET1_ENV") == content
    assert _read("hello-0-server", "cat secrets/secret1") == content           # env and file
    assert _read("hello-0-server", "cat secrets/secret2") == content


@pytest.fixture
def secrets_service():
    _secrets("create", f"{config.SERVICE_NAME}/")
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, NUM_HELLO + NUM_WORLD,
                        additional_options=_options(f"{config.SERVICE_NAME}/"))
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
    _secrets("delete", f"{config.SERVICE_NAME}/")
    _secrets("delete", "")


def test_secrets_basic(secrets_service):
    # the pod info carries references only: the values never pass through the scheduler
    info = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/pod/hello-0/info").json()[0]["info"]
    assert DEFAULT not in str(info)
    env = {v["name"]: v for v in info["command"]["environment"]["variables"]}
    assert env["HELLO_SECRET1_ENV"]["secret"]["reference"]["name"] == f"{config.SERVICE_NAME}/secret1"
    # restarts and replaces keep working
    for pod in ("hello-0", "world-0"):
        ids = sdk_tasks.get_task_ids(config.SERVICE_NAME, pod)
        rc, _, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, config.SERVICE_NAME, f"pod replace {pod}")
        assert rc == 0
        sdk_tasks.check_tasks_updated(config.SERVICE_NAME, pod, ids)
        sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
    sdk_tasks.check_running(config.SERVICE_NAME, NUM_HELLO + NUM_WORLD)


def test_secrets_verify(secrets_service):
    sdk_tasks.check_running(config.SERVICE_NAME, NUM_HELLO + NUM_WORLD)
    _verify(DEFAULT)


def test_secrets_update(secrets_service):
    _secrets("update", f"{config.SERVICE_NAME}/", ALTERNATIVE)
    # running tasks keep what they were launched with until they restart
    assert _read("world-0-server", "echo $WORLD_SECRET1_ENV") == DEFAULT
    for pod in ("hello-0", "world-0"):
        ids = sdk_tasks.get_task_ids(config.SERVICE_NAME, pod)
        rc, _, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, config.SERVICE_NAME, f"pod restart {pod}")
        assert rc == 0
        sdk_tasks.check_tasks_updated(config.SERVICE_NAME, pod, ids)
    sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
    sdk_tasks.check_running(config.SERVICE_NAME, NUM_HELLO + NUM_WORLD)
    _verify(ALTERNATIVE)


def test_secrets_config_update(secrets_service):
    # secrets with the same names directly under the root: a config update points the pods at them
    _secrets("create", "", ALTERNATIVE)
    _verify(DEFAULT)
    ids = sdk_tasks.get_task_ids(config.SERVICE_NAME, "")
    cfg = sdk_marathon.get_config(config.SERVICE_NAME)
    for k in ("HELLO_SECRET1", "HELLO_SECRET2", "WORLD_SECRET1", "WORLD_SECRET2", "WORLD_SECRET3"):
        cfg["env"][k] = cfg["env"][k].split("/")[-1]
    sdk_marathon.update_app(cfg)
    sdk_tasks.check_tasks_updated(config.SERVICE_NAME, "", ids)
    sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
    sdk_tasks.check_running(config.SERVICE_NAME, NUM_HELLO + NUM_WORLD)
    assert _read("world-0-server", "echo $WORLD_SECRET1_ENV") == ALTERNATIVE
    assert _read("world-0-server", "cat WORLD_SECRET2_FILE") == ALTERNATIVE
    assert _read("world-0-server", "cat secret3") == ALTERNATIVE
    assert _read("hello-0-server", "cat secrets/secret2") == ALTERNATIVE


def test_secrets_dcos_space():
    # secrets below the service's own path are not readable from its DCOS_SPACE (/hello-world)
    prefix = f"{config.SERVICE_NAME}/somePath/"
    _secrets("create", prefix)
    before = len(sdk_tasks.get_all_status_history("hello-0-server"))   # (earlier services' tasks)
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 0, additional_options=_options(prefix),
                        wait_for_deployment=False)
    try:
        with pytest.raises(Exception):
            sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME, timeout_seconds=5)

        @sdk_utils.retry(timeout_s=30, interval_s=0.5)
        def failed():
            states = [s["state"] for s in sdk_tasks.get_all_status_history("hello-0-server")[before:]]
            assert "TASK_FAILED" in states and "TASK_RUNNING" not in states, states
        failed()
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
        _secrets("delete", prefix)


# -- container features -------------------------------------------------------------------------
def _executor_container(pod):
    return sdk_cmd.service_request("GET", config.SERVICE_NAME, f"/v1/pod/{pod}/info").json()[0]["info"]["executor"][
        "container"]


def test_seccomp():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1, additional_options={"service": {"yaml": "seccomp"},
                                                                        "hello": {"seccomp-unconfined": True}})
    try:
        task = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/pod/hello-0/info").json()[0]["info"]
        assert task["container"]["linuxInfo"]["seccomp"]["unconfined"] is True
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_custom_seccomp_profile():
    """Reference test_seccomp.py: install with a named agent profile, then switch the profile
    through the scheduler's Marathon env; the pods roll to the new profile."""
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"yaml": "seccomp"}, "hello": {"seccomp-profile-name": "default.json"}})
    try:
        info = lambda: sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/pod/hello-0/info").json()[0]["info"]
        assert info()["container"]["linuxInfo"]["seccomp"]["profileName"] == "default.json"
        app = sdk_marathon.get_config(config.SERVICE_NAME)
        app["env"]["HELLO_SECCOMP_PROFILE_NAME"] = "test_profile.json"
        sdk_marathon.update_app(app)
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        assert info()["container"]["linuxInfo"]["seccomp"]["profileName"] == "test_profile.json"
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_shm():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1, additional_options={"service": {"yaml": "shm"}})
    try:
        linux = _executor_container("hello-0")["linuxInfo"]
        assert linux["ipcMode"] == "PRIVATE" and int(linux["shmSize"]) == 128
        rc, out, _ = sdk_cmd.run_cli("task log hello-0-server")
        assert rc == 0 and "/dev/shm" in out
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_share_pid_namespace():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"yaml": "share_pid_namespace"}})
    try:
        plan = sdk_plan.get_deployment_plan(config.SERVICE_NAME)
        assert [p["name"] for p in plan["phases"]] == ["server", "inspect"]
        assert plan["status"] == "COMPLETE"
        # the ONCE task saw the server's process (one PID namespace per pod) and finished
        assert [s["state"] for s in sdk_tasks.get_all_status_history("hello-0-inspect")][-1] == "TASK_FINISHED"
        tasks = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/pod/hello-0/info").json()
        for t in tasks:
            assert t["info"]["container"]["linuxInfo"]["sharePidNamespace"] is True, t["info"]["name"]
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
