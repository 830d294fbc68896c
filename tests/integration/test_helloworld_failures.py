"""helloworld failure-handling scenarios on the local cluster.

Reference: frameworks/helloworld/tests/{test_backoff.py, test_fast_failure.py,
test_nonessential_tasks.py, test_taskcfg.py}: launch backoff keeps a crash-looping deploy (and
later recovery) plan DELAYED with offers suppressed; a non-recoverable install trips the
task-failure limit of the plan waits; killing an essential task relaunches its whole pod on a
fresh executor while killing a non-essential one relaunches only that task next to the running
essential one; a service missing its TASKCFG_* settings crash-loops until they are added.
"""
import json

import pytest

from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_install, sdk_marathon, sdk_metrics, sdk_plan, sdk_tasks,
                                          sdk_utils)
from tests.integration import hw_config as config
from tests.integration.conftest import needs_cli

pytestmark = pytest.mark.usefixtures("local_cluster")
FOLDERED = sdk_utils.get_foldered_name(config.SERVICE_NAME)
# short backoff so the DELAYED -> STARTED -> DELAYED cycle fits a unit-test budget
CRASH_LOOP = {"service": {"yaml": "crash-loop", "sleep": 1,
                          "task_failure_backoff": {"enabled": True, "initial_backoff": 2, "backoff_factor": 1.15,
                                                   "max_launch_delay": 3}}}


def _check_delayed_and_suppressed(plan):
    sdk_plan.wait_for_plan_status(FOLDERED, plan, "DELAYED")
    sdk_metrics.wait_for_scheduler_gauge_value(FOLDERED, "is_suppressed",
                                               lambda v: isinstance(v, bool) and v)


def test_default_plan_backoff():
    sdk_install.install(config.PACKAGE_NAME, FOLDERED, 0, additional_options=CRASH_LOOP, wait_for_deployment=False,
                        wait_for_all_conditions=False)
    try:
        _check_delayed_and_suppressed("deploy")
        sdk_plan.wait_for_plan_status(FOLDERED, "deploy", "STARTED")
        _check_delayed_and_suppressed("deploy")
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, FOLDERED)


def test_recovery_backoff():
    sdk_install.install(config.PACKAGE_NAME, FOLDERED, 0, additional_options=CRASH_LOOP, wait_for_deployment=False,
                        wait_for_all_conditions=False)
    try:
        _check_delayed_and_suppressed("deploy")
        sdk_plan.force_complete_step(FOLDERED, "deploy", "crash", "hello-0:[server]")
        # deploy is done: the crash loop now belongs to the recovery plan
        sdk_plan.wait_for_plan_status(FOLDERED, "recovery", "STARTED")
        _check_delayed_and_suppressed("recovery")
        sdk_plan.wait_for_plan_status(FOLDERED, "recovery", "STARTED")
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, FOLDERED)


def test_finish_install_on_failure():
    with pytest.raises(sdk_plan.TaskFailuresExceededException):
        sdk_install.install(config.PACKAGE_NAME, FOLDERED, 1, additional_options={
            "service": {"name": FOLDERED, "yaml": "non_recoverable_state",
                        "task_failure_backoff": {"enabled": False}}})   # crash-loop as fast as possible
    sdk_install.uninstall(config.PACKAGE_NAME, FOLDERED)


@pytest.fixture
def nonessential():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 2,
                        additional_options={"service": {"yaml": "nonessential_tasks"}})
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def _verify_shared_executor(pod, expected=("essential", "nonessential"), delete=True):
    """Both tasks of the pod run on one executor and see the same volume contents."""
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, config.SERVICE_NAME, f"pod info {pod}", print_output=False)
    assert rc == 0, "pod info failed"
    tasks = json.loads(out)
    assert len(tasks) == 2, out
    assert tasks[0]["info"]["executor"] == tasks[1]["info"]["executor"]
    names = [t["info"]["name"] for t in tasks]
    for name in names:
        files = sdk_cmd.run_cli(f"task ls {name} shared-volume/")[1].split()
        assert set(expected) == set(files), (name, files)
    if delete:
        sdk_cmd.service_task_exec(config.SERVICE_NAME, names[0],
                                  "rm " + " ".join(f"shared-volume/{f}" for f in expected))


@needs_cli
def test_kill_essential(nonessential):
    _verify_shared_executor("hello-0")
    old = sdk_tasks.get_service_tasks(config.SERVICE_NAME, "hello-0")
    assert len(old) == 2
    sdk_cmd.kill_task_with_pattern("shared-volume/essential", "nobody", agent_host=old[0].host)
    sdk_tasks.check_tasks_updated(config.SERVICE_NAME, "hello-0", [t.id for t in old])
    sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
    # both tasks relaunched, so both files are back
    _verify_shared_executor("hello-0", delete=False)


@needs_cli
def test_kill_nonessential(nonessential):
    _verify_shared_executor("hello-0")
    old = sdk_tasks.get_service_tasks(config.SERVICE_NAME, "hello-0")
    essential = next(t for t in old if t.name == "hello-0-essential")
    helper = next(t for t in old if t.name == "hello-0-nonessential")
    sdk_cmd.kill_task_with_pattern("shared-volume/nonessential", "nobody", agent_host=helper.host)
    sdk_tasks.check_tasks_updated(config.SERVICE_NAME, "hello-0-nonessential", [helper.id])
    sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
    sdk_tasks.check_tasks_not_updated(config.SERVICE_NAME, "hello-0-essential", [essential.id])
    # only the non-essential task ran again
    _verify_shared_executor("hello-0", expected=("nonessential",))


def test_taskcfg_deploy():
    # (launch backoff shortened from the 60 s default: the failures come back-to-back)
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 0,
                        {"service": {"yaml": "taskcfg", "task_failure_backoff": {"initial_backoff": 1,
                                                                                 "max_launch_delay": 2}}},
                        wait_for_deployment=False)
    try:
        sdk_plan.wait_for_kicked_off_deployment(config.SERVICE_NAME)
        # without TASKCFG_ALL_OUTPUT_FILENAME / _SLEEP_DURATION the tasks cannot start
        before = len(sdk_tasks.get_all_status_history("hello-0-server"))

        @sdk_utils.retry(timeout_s=120, interval_s=0.5)
        def failed_again():
            added = [s["state"] for s in sdk_tasks.get_all_status_history("hello-0-server")][before:]
            assert "TASK_FAILED" in added, added
        failed_again()
        cfg = sdk_marathon.get_config(config.SERVICE_NAME)
        del cfg["env"]["SLEEP_DURATION"]
        cfg["env"]["TASKCFG_ALL_OUTPUT_FILENAME"] = "output"
        cfg["env"]["TASKCFG_ALL_SLEEP_DURATION"] = "1000"
        sdk_marathon.update_app(cfg)
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        config.check_running()
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
