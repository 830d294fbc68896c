"""Plan and goal-state scenarios on the local cluster.

Reference: frameworks/helloworld/tests/{test_multistep_plan.py,
test_custom_plan.py, test_uninstall.py, test_decommission.py}. Each scenario
installs its own service from one of the helloworld specs, drives it with the CLI / HTTP API the
way an operator would, and checks what really ran in the task sandboxes.
"""
import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks, sdk_upgrade
from tests.integration import hw_config as config
from tests.integration.conftest import needs_cli

PKG = config.PACKAGE_NAME
pytestmark = pytest.mark.usefixtures("local_cluster")


def completed_ids(task_name):
    return [t.id for t in sdk_tasks.get_summary(with_completed=True, task_name=task_name) if t.is_completed]


def test_multistep_plan_shared_resource_set():
    svc = "hello-multistep"
    sdk_install.install(PKG, svc, 3, additional_options={"service": {"yaml": "multistep_plan"}})
    try:
        tasks = {t.name: t for t in sdk_tasks.get_service_tasks(svc)}
        assert set(tasks) == {"hello-0-first", "hello-0-second", "hello-0-third"}
        # the pod's tasks, launched by separate steps, share the pod's agent
        assert tasks["hello-0-first"].host == tasks["hello-0-second"].host == tasks["hello-0-third"].host
        third = sdk_tasks.get_task_ids(svc, "hello-0-third")
        others = sdk_tasks.get_task_ids(svc, "hello-0-first") + sdk_tasks.get_task_ids(svc, "hello-0-second")
        sdk_plan.start_plan(svc, "maintenance")
        sdk_tasks.check_tasks_updated(svc, "hello-0-third", third)
        sdk_plan.wait_for_completed_plan(svc, "maintenance")
        assert sdk_tasks.get_task_ids(svc, "hello-0-first") + sdk_tasks.get_task_ids(svc, "hello-0-second") == others
    finally:
        sdk_install.uninstall(PKG, svc)


def test_custom_plan_scenario_reverses_steps():
    svc = "hello-custom-plan"
    sdk_install.install(PKG, svc, 3, additional_options={"service": {"scenario": "CUSTOM_PLAN"}})
    try:
        plan = sdk_plan.get_deployment_plan(svc)
        world_steps = plan["phases"][1]["steps"]
        assert [s["name"] for s in world_steps] == ["world-1:[server]", "world-0:[server]"]
    finally:
        sdk_install.uninstall(PKG, svc)


def test_uninstall_via_marathon_env(local_cluster):
    """The SDK uninstall: SDK_UNINSTALL on the scheduler app kills every task, releases every
    reservation and deregisters; the (uninstall) deploy plan then reports COMPLETE."""
    svc = "hello-uninstall"
    sdk_install.install(PKG, svc, config.DEFAULT_TASK_COUNT)
    try:
        config.check_running(svc)
        assert local_cluster.reserved_resources("hello-uninstall-role")
        cfg = sdk_marathon.get_config(svc)
        cfg["env"]["SDK_UNINSTALL"] = "w00t"
        sdk_marathon.update_app(cfg)
        sdk_plan.wait_for_completed_deployment(svc)
        sdk_tasks.check_running(svc, 0, allow_more=False)
        sdk_plan._poll(lambda: not local_cluster.reserved_resources("hello-uninstall-role"), 30,
                       "reservations released")
        sdk_plan._poll(lambda: not [f for f in local_cluster.frameworks() if f["name"] == svc], 30,
                       "framework removed")
    finally:
        sdk_install.uninstall(PKG, svc)


def test_custom_decommission():
    svc = "/test/integration/hello-decommission"
    opts = {"service": {"scenario": "CUSTOM_DECOMMISSION"}}
    sdk_upgrade.test_upgrade(PKG, svc, config.DEFAULT_TASK_COUNT, from_options=opts, to_options=opts)
    try:
        for _ in range(2):   # decommission, scale back up, decommission again
            cfg = sdk_marathon.get_config(svc)
            cfg["env"]["WORLD_COUNT"] = "1"
            sdk_marathon.update_app(cfg)
            sdk_plan.wait_for_completed_deployment(svc)
            sdk_plan.wait_for_completed_plan(svc, "decommission")
            plan = sdk_plan.get_decommission_plan(svc)
            assert plan["phases"][0]["steps"][0]["name"] == "custom_decommission_step"
            sdk_tasks.check_running(svc, 2, allow_more=False)
            cfg = sdk_marathon.get_config(svc)
            cfg["env"]["WORLD_COUNT"] = "2"
            sdk_marathon.update_app(cfg)
            sdk_plan.wait_for_completed_deployment(svc)
            sdk_tasks.check_running(svc, 3, allow_more=False)
    finally:
        sdk_install.uninstall(PKG, svc)
