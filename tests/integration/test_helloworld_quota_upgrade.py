"""Quota upgrade: a service on its legacy role moves to the quota group's role.

Reference: frameworks/helloworld/tests/test_quota_upgrade.py. The tests run in order on one
service (the reference chains them with ``pytest.mark.dependency``): install the previous package
version in a group without an enforced role (legacy role), update the scheduler to the group role
with role migration (it subscribes with both roles, pods stay put), replace every pod onto the new
role, add pods (new role), turn migration off (single role), add more pods.
"""
import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks, sdk_upgrade
from tests.integration import hw_config as config
from tests.integration.quota_common import (ENFORCED_ROLE, LEGACY_ROLE, SERVICE_NAME, assert_multi_role,
                                            assert_single_role, roles, start_cluster)

PKG = config.PACKAGE_NAME


@pytest.fixture(scope="module", autouse=True)
def quota_cluster():
    c = start_cluster()
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": False})
    yield c
    sdk_install.uninstall(PKG, SERVICE_NAME)
    sdk_marathon.delete_group(group_id=ENFORCED_ROLE)
    c.shutdown()


def test_initial_upgrade():
    sdk_upgrade.test_upgrade(PKG, SERVICE_NAME, 3, from_options={"service": {"name": SERVICE_NAME}})
    r = roles()
    assert LEGACY_ROLE in r["task-roles"].values() and ENFORCED_ROLE not in r["task-roles"].values()
    assert_single_role(r, LEGACY_ROLE)


def test_update_scheduler_role():
    sdk_upgrade.update_or_upgrade_or_downgrade(
        PKG, SERVICE_NAME, to_version=None, expected_running_tasks=3,
        to_options={"service": {"name": SERVICE_NAME, "role": ENFORCED_ROLE, "enable_role_migration": True}})
    r = roles()
    assert set(r["task-roles"].values()) == {LEGACY_ROLE}          # pods have not been replaced yet
    assert_multi_role(r)


def test_replace_pods_to_new_role():
    for pod in ("hello-0", "world-0", "world-1"):
        old_ids = sdk_tasks.get_task_ids(SERVICE_NAME, pod)
        rc, _, _ = sdk_cmd.svc_cli(PKG, SERVICE_NAME, f"pod replace {pod}")
        assert rc == 0
        sdk_tasks.check_tasks_updated(SERVICE_NAME, pod, old_ids)
        sdk_plan.wait_for_completed_recovery(SERVICE_NAME)
        sdk_plan._poll(lambda pod=pod: roles()["task-roles"].get(f"{pod}-server") == ENFORCED_ROLE, 30,
                       f"{pod} on the new role")
    r = roles()
    assert set(r["task-roles"].values()) == {ENFORCED_ROLE}
    assert_multi_role(r)
    assert not sdk_install._cluster().reserved_resources(LEGACY_ROLE)   # the legacy reservations went


def test_add_pods_post_update():
    app = sdk_marathon.get_config(SERVICE_NAME)
    app["env"]["HELLO_COUNT"], app["env"]["WORLD_COUNT"] = "2", "3"
    sdk_marathon.update_app(app)
    sdk_plan.wait_for_completed_deployment(SERVICE_NAME)
    sdk_tasks.check_running(SERVICE_NAME, 5)
    r = roles()
    assert len(r["task-roles"]) == 5 and set(r["task-roles"].values()) == {ENFORCED_ROLE}
    assert_multi_role(r)


def test_disable_legacy_role_post_update():
    sdk_upgrade.update_or_upgrade_or_downgrade(
        PKG, SERVICE_NAME, to_version=None, expected_running_tasks=5,
        to_options={"service": {"name": SERVICE_NAME, "role": ENFORCED_ROLE, "enable_role_migration": False},
                    "hello": {"count": 2}, "world": {"count": 3}})
    r = roles()
    assert len(r["task-roles"]) == 5 and set(r["task-roles"].values()) == {ENFORCED_ROLE}
    assert_single_role(r, ENFORCED_ROLE)


def test_more_pods_disable_legacy_role_post_update():
    app = sdk_marathon.get_config(SERVICE_NAME)
    app["env"]["HELLO_COUNT"], app["env"]["WORLD_COUNT"] = "3", "4"
    sdk_marathon.update_app(app)
    sdk_plan.wait_for_completed_deployment(SERVICE_NAME)
    sdk_tasks.check_running(SERVICE_NAME, 7)
    r = roles()
    assert len(r["task-roles"]) == 7 and set(r["task-roles"].values()) == {ENFORCED_ROLE}
    assert_single_role(r, ENFORCED_ROLE)
