"""helloworld multi-service and plan-toggle scenarios on the local cluster.

Reference: frameworks/helloworld/tests/{test_multiservice_dynamic.py, test_mono_to_multi_migrate.py,
test_enable_disable.py, test_parallel_plans.py}. A scheduler started without a YAML serves
``/v1/multi``: services added there deploy, survive scheduler restarts (ServiceStore) and are
uninstalled on DELETE. A single-service scheduler updated to run several YAMLs migrates its state
into the multi-service layout without relaunching its tasks, unless their config changed. A
config switch that drops tasks from the deploy plan kills them, and switching it back relaunches
them. Manual plans started together deploy their pods side by side.
"""
import pytest

from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks, sdk_upgrade,
                                          sdk_utils)
from tests.integration import hw_config as config

pytestmark = pytest.mark.usefixtures("local_cluster")


# -- dynamic multi-service -----------------------------------------------------------------------
@pytest.fixture
def multi_scheduler(local_cluster):
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 0, additional_options={"service": {"yaml": ""}},
                        wait_for_deployment=False)
    yamls = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/multi/yaml").json()
    assert "svc" in yamls and "simple" in yamls
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def _services():
    return sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/multi").json()


def _wait_for_service_count(count):
    @sdk_utils.retry(timeout_s=60, interval_s=0.5)
    def check():
        services = _services()
        assert len(services) == count, services
        return services
    return check()


def _add(name, yaml):
    sdk_cmd.service_request("POST", config.SERVICE_NAME, f"/v1/multi/{name}?yaml={yaml}",
                            json={"FRAMEWORK_NAME": name})


SVC_STEPS = ["hello-0:[server]", "world-0:[server]", "world-1:[server]"]


def test_add_deploy_restart_remove(multi_scheduler):
    _add("test1", "svc")
    (service,) = _services()
    assert (service["service"], service["yaml"], service["uninstall"]) == ("test1", "svc", False)
    sdk_plan.wait_for_plan_status(config.SERVICE_NAME, "deploy", "COMPLETE", multiservice_name="test1")

    old = sdk_tasks.get_task_ids("marathon", config.SERVICE_NAME)[0]
    sdk_marathon.restart_app(config.SERVICE_NAME)
    sdk_tasks.check_scheduler_relaunched(config.SERVICE_NAME, old)
    (service,) = _wait_for_service_count(1)
    assert (service["service"], service["yaml"], service["uninstall"]) == ("test1", "svc", False)
    plan = sdk_plan.wait_for_plan_status(config.SERVICE_NAME, "deploy", "COMPLETE", multiservice_name="test1")
    assert sdk_plan.get_all_step_names(plan) == SVC_STEPS

    sdk_cmd.service_request("DELETE", config.SERVICE_NAME, "/v1/multi/test1")
    for service in _services():
        assert (service["service"], service["yaml"], service["uninstall"]) == ("test1", "svc", True)
    _wait_for_service_count(0)
    # its reservations are gone
    assert not sdk_install._cluster().reserved_resources("test1-role")


def test_add_multiple_uninstall(multi_scheduler):
    _add("test1", "svc")
    _add("test2", "simple")
    services = {s["service"]: s for s in _services()}
    assert set(services) == {"test1", "test2"}
    assert services["test1"]["yaml"] == "svc" and services["test2"]["yaml"] == "simple"
    assert not any(s["uninstall"] for s in services.values())
    plan = sdk_plan.wait_for_plan_status(config.SERVICE_NAME, "deploy", "COMPLETE", multiservice_name="test1")
    assert sdk_plan.get_all_step_names(plan) == SVC_STEPS
    plan = sdk_plan.wait_for_plan_status(config.SERVICE_NAME, "deploy", "COMPLETE", multiservice_name="test2")
    assert sdk_plan.get_all_step_names(plan) == ["hello-0:[server]"]

    sdk_cmd.service_request("DELETE", config.SERVICE_NAME, "/v1/multi/test2")
    for s in _services():
        assert s["service"] in ("test1", "test2") and s["uninstall"] == (s["service"] == "test2")
    sdk_marathon.restart_app(config.SERVICE_NAME)
    _wait_for_service_count(1)
    plan = sdk_plan.wait_for_plan_status(config.SERVICE_NAME, "deploy", "COMPLETE", multiservice_name="test1")
    assert sdk_plan.get_all_step_names(plan) == SVC_STEPS
    sdk_cmd.service_request("DELETE", config.SERVICE_NAME, "/v1/multi/test1")
    _wait_for_service_count(0)


# -- single service -> multi-service migration ----------------------------------------------------
@pytest.fixture
def mono_service():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 3, additional_options={"service": {"yaml": "svc"}})
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def _migrate(extra=None):
    opts = {"service": {"yaml": "", "yamls": "svc,foobar_service_name"}}
    opts.update(extra or {})
    sdk_upgrade.update_or_upgrade_or_downgrade(config.PACKAGE_NAME, config.SERVICE_NAME, to_version=None,
                                               to_options=opts, expected_running_tasks=4, wait_for_deployment=False)
    sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME, multiservice_name="foobar")


def test_old_tasks_not_relaunched(mono_service):
    hello = sdk_tasks.get_task_ids(config.SERVICE_NAME, "hello")
    _migrate()
    sdk_tasks.check_task_not_relaunched(config.SERVICE_NAME, "hello-0-server", hello[-1],
                                        multiservice_name=config.SERVICE_NAME)
    assert len(sdk_tasks.get_task_ids(config.SERVICE_NAME, "foo")) == 1
    # the state now lives in the multi-service layout: Services/<name>/...
    zk = sdk_install._cluster().zk_children(f"/dcos-service-{config.SERVICE_NAME}")
    assert "Services" in zk and sdk_cmd.cluster_request("GET", "/mesos/frameworks").ok


def test_old_tasks_get_relaunched_with_new_config(mono_service):
    hello = sdk_tasks.get_task_ids(config.SERVICE_NAME, "hello")
    _migrate({"hello": {"cpus": 0.2}})
    sdk_tasks.check_task_relaunched("hello-0-server", hello[-1])
    assert len(sdk_tasks.get_task_ids(config.SERVICE_NAME, "foo")) == 1


# -- enable / disable plan steps ------------------------------------------------------------------
def _set_test_boolean(value):
    cfg = sdk_marathon.get_config(config.SERVICE_NAME)
    cfg["env"]["TEST_BOOLEAN"] = value
    sdk_marathon.update_app(cfg)


def test_disable_then_enable():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 6,
                        additional_options={"service": {"yaml": "enable-disable"}, "hello": {"count": 3}})
    try:
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        assert sdk_plan.recovery_plan_is_empty(config.SERVICE_NAME)
        sdk_tasks.check_running(config.SERVICE_NAME, 6, timeout_seconds=30, allow_more=False)
        b_ids = sdk_tasks.get_task_ids(config.SERVICE_NAME, "hello-0-server-b")

        _set_test_boolean("false")
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        sdk_tasks.check_running(config.SERVICE_NAME, 3, timeout_seconds=30, allow_more=False)
        assert all(t.name.endswith("server-b") for t in sdk_tasks.get_service_tasks(config.SERVICE_NAME))
        assert sdk_plan.recovery_plan_is_empty(config.SERVICE_NAME)   # killed on purpose: nothing to recover
        sdk_tasks.check_tasks_not_updated(config.SERVICE_NAME, "hello-0-server-b", b_ids)

        _set_test_boolean("true")
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        sdk_tasks.check_running(config.SERVICE_NAME, 6, timeout_seconds=30, allow_more=False)
        # (the restarted scheduler may hand a killed server-a to the recovery plan before the deploy
        # plan claims its pod: either way every plan ends COMPLETE with each task launched once)
        sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
        assert len(sdk_tasks.get_task_ids(config.SERVICE_NAME, "hello-0-server-a")) == 1
        # server-a came back on the pod's volume, next to the untouched server-b
        rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, "hello-0-server-a", "cat shared/output")
        assert rc == 0 and out.split().count("server-a") == 2, out
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


# -- parallel manual plans ------------------------------------------------------------------------
def test_all_tasks_are_launched():
    name = sdk_utils.get_foldered_name(config.SERVICE_NAME)
    sdk_install.install(config.PACKAGE_NAME, name, 0, additional_options={"service": {"yaml": "plan"}},
                        wait_for_deployment=False)
    try:
        plans = ["manual-plan-0", "manual-plan-1", "manual-plan-2"]
        for plan in plans:
            sdk_plan.start_plan(name, plan)
        for plan in plans:
            sdk_plan.wait_for_completed_plan(name, plan)
        for pod in ("custom-pod-A-0", "custom-pod-B-0", "custom-pod-C-0"):
            for t in sdk_cmd.service_request("GET", name, f"/v1/pod/{pod}/info").json():
                info, status = t["info"], t.get("status")
                if status:
                    assert info["taskId"]["value"] == status["taskId"]["value"] and info["taskId"]["value"]
                else:
                    assert not info["taskId"]["value"]
        sdk_plan.wait_for_completed_deployment(name)
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, name)
