"""Sidecar plans on the local cluster: ONCE-goal tasks launched by operator plans next to a
running server pod, sharing its ROOT volume.

Reference: frameworks/helloworld/tests/test_sidecar.py. One service (``sidecar.yml``, two hello
pods) serves the module: an option change reaches the server's environment and survives a pod
restart; the deploy plan's shape; a sidecar plan run, with and without a plan parameter; a failing
ONCE task that never triggers recovery, not even after a scheduler restart.
"""
import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks, sdk_upgrade
from tests.integration import hw_config as config
from tests.integration.conftest import needs_cli

PKG = config.PACKAGE_NAME
SVC = "hello-sidecar"


@pytest.fixture(scope="module", autouse=True)
def sidecar_service(local_cluster):
    sdk_install.install(PKG, SVC, 2, additional_options={"service": {"yaml": "sidecar"}, "hello": {"count": 2}})
    yield
    sdk_install.uninstall(PKG, SVC)


def _completed(task_name):
    return [t.id for t in sdk_tasks.get_summary(with_completed=True, task_name=task_name) if t.is_completed]


def _server_env():
    rc, out, _ = sdk_cmd.service_task_exec(SVC, "hello-0-server", "env")
    assert rc == 0
    return dict(line.split("=", 1) for line in out.strip().splitlines() if "=" in line)


def test_envvar_accross_restarts():
    """service.sleep reaches the server as CONFIG_SLEEP_DURATION and is still there after a
    pod restart (the relaunch keeps the task's rendered environment)."""
    sdk_upgrade.update_or_upgrade_or_downgrade(PKG, SVC, to_version=None,
                                               to_options={"service": {"name": SVC, "sleep": 9999, "yaml": "sidecar"},
                                                           "hello": {"count": 2}},
                                               expected_running_tasks=2, wait_for_deployment=True)
    assert _server_env()["CONFIG_SLEEP_DURATION"] == "9999"
    old = sdk_tasks.get_task_ids(SVC, "hello-0-server")
    sdk_cmd.svc_cli(PKG, SVC, "pod restart hello-0")
    sdk_tasks.check_tasks_updated(SVC, "hello-0-server", old)
    sdk_plan.wait_for_completed_recovery(SVC)
    assert _server_env()["CONFIG_SLEEP_DURATION"] == "9999"


def test_deploy():
    sdk_plan.wait_for_completed_deployment(SVC)
    plan = sdk_plan.get_deployment_plan(SVC)
    assert [p["name"] for p in plan["phases"]] == ["server"]
    assert [s["name"] for s in plan["phases"][0]["steps"]] == ["hello-0:[server]", "hello-1:[server]"]


def _run_sidecar(params=None):
    before = {i: len(_completed(f"hello-{i}-verify")) for i in (0, 1)}
    sdk_plan.start_plan(SVC, "sidecar", params)
    plan = sdk_plan.get_plan(SVC, "sidecar")
    assert [p["name"] for p in plan["phases"]] == ["backup", "verify"]
    assert all(len(p["steps"]) == 2 for p in plan["phases"])
    sdk_plan._poll(lambda: all(len(_completed(f"hello-{i}-verify")) > before[i] for i in (0, 1)), 60,
                   "both pods' verify sidecars")
    sdk_plan.wait_for_completed_plan(SVC, "sidecar")


def test_sidecar():
    servers = sdk_tasks.get_task_ids(SVC, "hello")
    _run_sidecar()
    for i in (0, 1):
        rc, out, _ = sdk_cmd.service_task_exec(SVC, f"hello-{i}-server",
                                               "test -f shared-data/backup.tgz && cat shared-data/backup-tag")
        assert rc == 0 and out.strip() == "untagged"
    sdk_tasks.check_tasks_not_updated(SVC, "hello-0-server", [x for x in servers if "hello-0-server" in x])


@needs_cli
def test_sidecar_parameterized():
    """A plan parameter reaches the sidecar tasks' environment (``plan start -p``)."""
    rc, _, err = sdk_cmd.svc_cli(PKG, SVC, "plan start sidecar -p BACKUP_TAG=parameterized")
    assert rc == 0, err
    sdk_plan.wait_for_completed_plan(SVC, "sidecar")
    for i in (0, 1):
        rc, out, _ = sdk_cmd.service_task_exec(SVC, f"hello-{i}-server", "cat shared-data/backup-tag")
        assert rc == 0 and out.strip() == "parameterized"


def test_toxic_sidecar_doesnt_trigger_recovery():
    """A failed ONCE task never triggers recovery, not even after a scheduler restart."""
    servers = sdk_tasks.get_task_ids(SVC, "hello-0-server")
    assert sdk_plan.get_plan(SVC, "recovery")["status"] == "COMPLETE"
    sdk_plan.start_plan(SVC, "sidecar-toxic")
    sdk_plan._poll(lambda: sdk_cmd.service_task_exec(SVC, "hello-0-server", "cat shared-data/toxic-output")[1]
                   .strip().startswith("toxic"), 60, "toxic sidecar ran")
    sdk_marathon.restart_app(SVC)
    sdk_plan.wait_for_completed_deployment(SVC)
    recovery = sdk_plan.get_plan(SVC, "recovery")
    assert recovery["status"] == "COMPLETE" and recovery["phases"] == []
    sdk_tasks.check_tasks_not_updated(SVC, "hello-0-server", servers)
