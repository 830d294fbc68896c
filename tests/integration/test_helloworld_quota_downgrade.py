"""Quota downgrade: a service on the quota group's enforced role goes back to its legacy role.

Reference: frameworks/helloworld/tests/test_quota_downgrade.py. In order on one service: install
under a group that enforces its role, stop enforcing it (nothing moves), update to the legacy role
(``role: slave_public``) with role migration (both roles), replace every pod onto the legacy role,
turn migration off (single legacy role), add pods, and downgrade the scheduler to the previous
package version.
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
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": True})
    yield c
    sdk_install.uninstall(PKG, SERVICE_NAME)
    sdk_marathon.delete_group(group_id=ENFORCED_ROLE)
    c.shutdown()


def test_initial_install():
    sdk_install.install(PKG, SERVICE_NAME, 3, additional_options={"service": {"name": SERVICE_NAME}})
    r = roles()
    assert set(r["task-roles"].values()) == {ENFORCED_ROLE}
    assert_single_role(r, ENFORCED_ROLE)


def test_disable_enforce_role():
    sdk_marathon.update_group(group_id=ENFORCED_ROLE, options={"enforceRole": False})
    r = roles()
    assert set(r["task-roles"].values()) == {ENFORCED_ROLE}       # nothing moves by itself
    assert_single_role(r, ENFORCED_ROLE)


def test_switch_to_legacy_role():
    sdk_upgrade.update_or_upgrade_or_downgrade(
        PKG, SERVICE_NAME, to_version=None, expected_running_tasks=3,
        to_options={"service": {"name": SERVICE_NAME, "role": "slave_public", "enable_role_migration": True}})
    r = roles()
    assert set(r["task-roles"].values()) == {ENFORCED_ROLE}
    assert_multi_role(r)


def test_replace_pods_to_legacy_role():
    for pod in ("hello-0", "world-0", "world-1"):
        old_ids = sdk_tasks.get_task_ids(SERVICE_NAME, pod)
        rc, _, _ = sdk_cmd.svc_cli(PKG, SERVICE_NAME, f"pod replace {pod}")
        assert rc == 0
        sdk_tasks.check_tasks_updated(SERVICE_NAME, pod, old_ids)
        sdk_plan.wait_for_completed_recovery(SERVICE_NAME)
        sdk_plan._poll(lambda pod=pod: roles()["task-roles"].get(f"{pod}-server") == LEGACY_ROLE, 30,
                       f"{pod} on the legacy role")
    r = roles()
    assert set(r["task-roles"].values()) == {LEGACY_ROLE}
    assert_multi_role(r)


def test_disable_quota_role():
    sdk_upgrade.update_or_upgrade_or_downgrade(
        PKG, SERVICE_NAME, to_version=None, expected_running_tasks=3,
        to_options={"service": {"name": SERVICE_NAME, "role": "slave_public", "enable_role_migration": False}})
    r = roles()
    assert len(r["task-roles"]) == 3 and set(r["task-roles"].values()) == {LEGACY_ROLE}
    assert_single_role(r, LEGACY_ROLE)


def test_add_pods_post_update():
    app = sdk_marathon.get_config(SERVICE_NAME)
    app["env"]["HELLO_COUNT"], app["env"]["WORLD_COUNT"] = "2", "3"
    sdk_marathon.update_app(app)
    sdk_plan.wait_for_completed_deployment(SERVICE_NAME)
    sdk_tasks.check_running(SERVICE_NAME, 5)
    r = roles()
    assert len(r["task-roles"]) == 5 and set(r["task-roles"].values()) == {LEGACY_ROLE}
    assert_single_role(r, LEGACY_ROLE)


def test_downgrade_scheduler():
    sdk_upgrade.test_downgrade(PKG, SERVICE_NAME, 5, to_options={"service": {"name": SERVICE_NAME},
                                                                 "hello": {"count": 2}, "world": {"count": 3}})
    r = roles()
    assert len(r["task-roles"]) == 5 and set(r["task-roles"].values()) == {LEGACY_ROLE}
    assert_single_role(r, LEGACY_ROLE)
