"""Canary rollout on the local cluster (serial-canary hello phase, parallel-canary world phase).

Reference: frameworks/helloworld/tests/test_canary_strategy.py -- the exact step statuses after each
``plan continue`` (first canary step, no-op continue of the plan, second phase, the rest), a count
increase that waits for a continue, and a cpu bump that rolls two canary steps one at a time.
"""
import json
import time

import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks
from tests.integration import hw_config as config
from tests.integration.conftest import needs_cli

pytestmark = needs_cli
SVC = "hello-world-canary"


@pytest.fixture(scope="module", autouse=True)
def configure_package(local_cluster):
    # due to canary: no tasks launch until the operator continues the plan
    sdk_install.install(config.PACKAGE_NAME, SVC, 0,
                        additional_options={"service": {"yaml": "canary"}, "hello": {"count": 4},
                                            "world": {"count": 4}},
                        wait_for_deployment=False)
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, SVC)


def pod_list():
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, SVC, "pod list")
    assert rc == 0, "Pod list failed"
    return json.loads(out)


def cli(cmd):
    rc, _, err = sdk_cmd.svc_cli(config.PACKAGE_NAME, SVC, cmd)
    assert rc == 0, err


def assert_plan(pl, status, phase_statuses):
    """``phase_statuses``: [(phase status, [step statuses])] in phase order."""
    assert pl["status"] == status, sdk_plan.plan_string("deploy", pl)
    assert [(p["status"], [s["status"] for s in p["steps"]]) for p in pl["phases"]] == phase_statuses, \
        sdk_plan.plan_string("deploy", pl)


def assert_no_more_tasks(expected, settle_s=1.0):
    time.sleep(settle_s)   # give the scheduler time to (wrongly) launch something
    sdk_tasks.check_running(SVC, len(expected), allow_more=False, timeout_seconds=5)
    assert pod_list() == expected


def test_canary_init():
    sdk_plan._poll(lambda: pod_list() == [], 60, "no pods")
    pl = sdk_plan.wait_for_plan_status(SVC, "deploy", "WAITING")
    assert_plan(pl, "WAITING", [("WAITING", ["WAITING", "WAITING", "PENDING", "PENDING"]),
                                ("WAITING", ["WAITING", "WAITING", "PENDING", "PENDING"])])


def test_canary_first():
    cli("plan continue deploy hello-deploy")
    sdk_tasks.check_running(SVC, 1)
    assert pod_list() == ["hello-0"]
    pl = sdk_plan.wait_for_completed_step(SVC, "deploy", "hello-deploy", "hello-0:[server]")
    assert_plan(pl, "WAITING", [("WAITING", ["COMPLETE", "WAITING", "PENDING", "PENDING"]),
                                ("WAITING", ["WAITING", "WAITING", "PENDING", "PENDING"])])


def test_canary_plan_continue_noop():
    # the plan itself is not interrupted (only shown WAITING): continuing it changes nothing
    cli("plan continue deploy")
    assert_no_more_tasks(["hello-0"])


def test_canary_second():
    cli("plan continue deploy world-deploy")
    sdk_plan.wait_for_step_status(SVC, "deploy", "world-deploy", "world-0:[server]", "PENDING")
    # the plan is serial: the world phase only clears its wait bit, nothing launches
    assert_no_more_tasks(["hello-0"])
    pl = sdk_plan.get_deployment_plan(SVC)
    assert_plan(pl, "WAITING", [("WAITING", ["COMPLETE", "WAITING", "PENDING", "PENDING"]),
                                ("PENDING", ["PENDING", "WAITING", "PENDING", "PENDING"])])


def test_canary_third():
    cli("plan continue deploy hello-deploy")
    expected = ["hello-0", "hello-1", "hello-2", "hello-3", "world-0"]
    sdk_tasks.check_running(SVC, len(expected))
    assert pod_list() == expected
    pl = sdk_plan.wait_for_completed_phase(SVC, "deploy", "hello-deploy")
    pl = sdk_plan.wait_for_completed_step(SVC, "deploy", "world-deploy", "world-0:[server]")
    assert_plan(pl, "WAITING", [("COMPLETE", ["COMPLETE"] * 4),
                                ("WAITING", ["COMPLETE", "WAITING", "PENDING", "PENDING"])])


def test_canary_fourth():
    cli("plan continue deploy world-deploy")
    expected = [f"hello-{i}" for i in range(4)] + [f"world-{i}" for i in range(4)]
    sdk_tasks.check_running(SVC, len(expected))
    assert pod_list() == expected
    pl = sdk_plan.wait_for_completed_plan(SVC, "deploy")
    assert_plan(pl, "COMPLETE", [("COMPLETE", ["COMPLETE"] * 4), ("COMPLETE", ["COMPLETE"] * 4)])


def test_increase_count():
    sdk_marathon.bump_task_count_config(SVC, "HELLO_COUNT")
    expected = [f"hello-{i}" for i in range(4)] + [f"world-{i}" for i in range(4)]
    pl = sdk_plan.wait_for_plan_status(SVC, "deploy", "WAITING")
    assert_no_more_tasks(expected)
    assert_plan(pl, "WAITING", [("WAITING", ["COMPLETE"] * 4 + ["WAITING"]), ("COMPLETE", ["COMPLETE"] * 4)])

    cli("plan continue deploy hello-deploy")
    expected = [f"hello-{i}" for i in range(5)] + [f"world-{i}" for i in range(4)]
    sdk_tasks.check_running(SVC, len(expected))
    assert pod_list() == expected
    pl = sdk_plan.wait_for_plan_status(SVC, "deploy", "COMPLETE")
    assert_plan(pl, "COMPLETE", [("COMPLETE", ["COMPLETE"] * 5), ("COMPLETE", ["COMPLETE"] * 4)])


def test_increase_cpu():
    hello_0_ids = sdk_tasks.get_task_ids(SVC, "hello-0-server")
    config.bump_hello_cpus(SVC)
    pl = sdk_plan.wait_for_plan_status(SVC, "deploy", "WAITING")
    assert_plan(pl, "WAITING", [("WAITING", ["WAITING", "WAITING", "PENDING", "PENDING", "PENDING"]),
                                ("COMPLETE", ["COMPLETE"] * 4)])
    expected = [f"hello-{i}" for i in range(5)] + [f"world-{i}" for i in range(4)]
    sdk_tasks.check_running(SVC, len(expected))
    assert pod_list() == expected
    assert hello_0_ids == sdk_tasks.get_task_ids(SVC, "hello-0-server")

    cli("plan continue deploy hello-deploy")
    sdk_tasks.check_tasks_updated(SVC, "hello-0-server", hello_0_ids)
    sdk_tasks.check_running(SVC, len(expected))
    pl = sdk_plan.wait_for_step_status(SVC, "deploy", "hello-deploy", "hello-0:[server]", "COMPLETE")
    assert_plan(pl, "WAITING", [("WAITING", ["COMPLETE", "WAITING", "PENDING", "PENDING", "PENDING"]),
                                ("COMPLETE", ["COMPLETE"] * 4)])

    hello_1_ids = sdk_tasks.get_task_ids(SVC, "hello-1-server")
    cli("plan continue deploy hello-deploy")
    sdk_tasks.check_tasks_updated(SVC, "hello-1-server", hello_1_ids)
    pl = sdk_plan.wait_for_completed_deployment(SVC)
    assert_plan(pl, "COMPLETE", [("COMPLETE", ["COMPLETE"] * 5), ("COMPLETE", ["COMPLETE"] * 4)])
