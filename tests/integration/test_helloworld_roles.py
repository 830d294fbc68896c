"""helloworld role scenarios on the local cluster: quota groups, role migration, pre-reserved roles.

Reference: frameworks/helloworld/tests/{test_quota_deployment.py, test_pre_reserved_sidecar.py,
test_resource_refinement.py}; the upgrade and downgrade sequences are
test_helloworld_quota_{upgrade,downgrade}.py.

* Marathon groups decide the scheduler's role: a group with ``enforceRole`` makes its name the
  role of every service under it; without it a service keeps its legacy ``<name>-role`` unless
  it asks for the group role, and ``enable_role_migration`` subscribes with both roles.
* Pre-reserved roles: pods with ``pre-reserved-role: slave_public`` refine the statically reserved
  resources of every agent, a sidecar plan runs on them, and another framework's persistent volume
  on the same static reservation survives the service's install and uninstall.
"""
import threading

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalSchedulerDriver
from dcos_commons_amd.testing.cluster.cluster import DCOS_AGENT_PORTS, LocalCluster, use
from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks, sdk_upgrade,
                                          sdk_utils)
from tests.integration import hw_config as config

ENFORCED_ROLE = "quota"
SERVICE_NAME = f"/{ENFORCED_ROLE}/hello-world"
LEGACY_ROLE = "{}-role".format(SERVICE_NAME.strip("/").replace("/", "__"))
PRE_RESERVED = (("slave_public", "cpus", 2.0), ("slave_public", "mem", 2048.0), ("slave_public", "disk", 4096.0))


@pytest.fixture(scope="module")
def local_cluster():
    specs = [AgentSpec(hostname=f"10.0.0.{i + 1}", ports=DCOS_AGENT_PORTS, region="us-west-2",
                       zone=("us-west-2a", "us-west-2b", "us-west-2c")[i % 3], pre_reserved=PRE_RESERVED)
             for i in range(5)]
    c = LocalCluster(agent_specs=specs, scheduler_env={"SDK_LOCK_WAIT_S": "1"}).start()
    use(c)
    yield c
    c.shutdown()


pytestmark = pytest.mark.usefixtures("local_cluster")


@pytest.fixture
def quota_group():
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, SERVICE_NAME)
    sdk_marathon.delete_group(group_id=ENFORCED_ROLE)


def _install_and_fetch_service_roles(options, count=3):
    sdk_install.install(config.PACKAGE_NAME, SERVICE_NAME, count, additional_options=options)
    roles = sdk_utils.get_service_roles(SERVICE_NAME)
    assert len(roles["task-roles"]) > 0
    return roles, roles["task-roles"]


# -- quota deployment ----------------------------------------------------------------------------
@pytest.mark.parametrize("options", [
    {"service": {"name": SERVICE_NAME, "role": "slave_public"}},
    {"service": {"name": SERVICE_NAME}},
], ids=["explicit_slave_public", "defaults"])
def test_nonenforced_group_role_defaults(quota_group, options):
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": False})
    roles, task_roles = _install_and_fetch_service_roles(options)
    assert LEGACY_ROLE in task_roles.values() and ENFORCED_ROLE not in task_roles.values()
    assert roles["framework-roles"] is None and roles["framework-role"] == LEGACY_ROLE


def test_nonenforced_group_role_service_role_set(quota_group):
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": False})
    roles, task_roles = _install_and_fetch_service_roles({"service": {"name": SERVICE_NAME, "role": ENFORCED_ROLE}})
    assert LEGACY_ROLE not in task_roles.values() and ENFORCED_ROLE in task_roles.values()
    assert roles["framework-roles"] is None and roles["framework-role"] == ENFORCED_ROLE


def test_nonenforced_group_role_service_role_legacy_role_set(quota_group):
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": False})
    roles, task_roles = _install_and_fetch_service_roles(
        {"service": {"name": SERVICE_NAME, "role": ENFORCED_ROLE, "enable_role_migration": True}})
    assert LEGACY_ROLE not in task_roles.values() and ENFORCED_ROLE in task_roles.values()
    assert roles["framework-role"] is None and sorted(roles["framework-roles"]) == sorted([LEGACY_ROLE, ENFORCED_ROLE])


def test_enforced_group_role_defaults(quota_group):
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": True})
    roles, task_roles = _install_and_fetch_service_roles({"service": {"name": SERVICE_NAME}})
    assert LEGACY_ROLE not in task_roles.values() and ENFORCED_ROLE in task_roles.values()
    assert roles["framework-roles"] is None and roles["framework-role"] == ENFORCED_ROLE


def test_enforced_group_role_legacy_role_set(quota_group):
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": True})
    roles, task_roles = _install_and_fetch_service_roles(
        {"service": {"name": SERVICE_NAME, "enable_role_migration": True}})
    assert LEGACY_ROLE not in task_roles.values() and ENFORCED_ROLE in task_roles.values()
    assert roles["framework-role"] is None and sorted(roles["framework-roles"]) == sorted([LEGACY_ROLE, ENFORCED_ROLE])


def test_nonenforced_group_legacy_service_role_non_migration(quota_group):
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": False})
    roles, task_roles = _install_and_fetch_service_roles(
        {"service": {"name": SERVICE_NAME, "role": "slave_public", "enable_role_migration": False}})
    assert LEGACY_ROLE in task_roles.values() and ENFORCED_ROLE not in task_roles.values()
    assert roles["framework-roles"] is None and roles["framework-role"] == LEGACY_ROLE


@pytest.mark.parametrize("enforce_role", [True, False])
def test_non_migration(quota_group, enforce_role):
    sdk_marathon.create_group(group_id=ENFORCED_ROLE, options={"enforceRole": enforce_role})
    roles, task_roles = _install_and_fetch_service_roles(
        {"service": {"name": SERVICE_NAME, "role": ENFORCED_ROLE, "enable_role_migration": False}})
    assert LEGACY_ROLE not in task_roles.values() and ENFORCED_ROLE in task_roles.values()
    assert roles["framework-roles"] is None and roles["framework-role"] == ENFORCED_ROLE


# -- pre-reserved roles --------------------------------------------------------------------------
def test_pre_reserved_sidecar():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"yaml": "pre-reserved-sidecar"}})
    try:
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        # refined reservations: the static slave_public role, then the service role
        info = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/pod/hello-0/info").json()
        server = next(t["info"] for t in info if t["info"]["name"] == "hello-0-server")
        for r in server["resources"]:
            stack = [x.get("role") for x in r.get("reservations", [])]
            assert stack[:2] == ["slave_public", "slave_public/hello-world-role"], (r["name"], stack)
        sdk_plan.start_plan(config.SERVICE_NAME, "sidecar")
        plan = sdk_plan.get_plan(config.SERVICE_NAME, "sidecar")
        assert len(plan["phases"]) == 1 and len(plan["phases"][0]["steps"]) == 1
        sdk_plan.wait_for_completed_plan(config.SERVICE_NAME, "sidecar")
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
    # the refined reservations went back to the static role
    c = sdk_install._cluster()
    assert not [r for _, r in c.reserved_resources() if len(r.reservations) > 1]


class _ForeignFramework:
    """Another framework (a Marathon app with a persistent volume in the reference test): it
    creates a persistent volume on a statically reserved ``slave_public`` disk of one agent."""

    def __init__(self, cluster, role="slave_public"):
        self.cluster = cluster
        self.volume = None
        self.agent_id = None
        self._done = threading.Event()
        info = P.FrameworkInfo(name="persistent-test", user="nobody", role=role)
        self.driver = LocalSchedulerDriver(cluster.master, self, info)

    def registered(self, driver, framework_id, master_info):
        pass

    def resource_offers(self, driver, offers):
        for o in offers:
            disk = next((r for r in o.resources if r.name == "disk" and r.reservations
                         and r.reservations[-1].role == "slave_public"), None)
            if self.volume is not None or disk is None:
                driver.decline_offer(o.id)
                continue
            v = P.Resource()
            v.CopyFrom(disk)
            v.ClearField("allocation_info")
            v.scalar.value = 500.0
            v.disk.persistence.id = "persistent-test#persistent-volume#1"
            v.disk.persistence.principal = "marathon"
            v.disk.volume.container_path = "persistent-volume"
            v.disk.volume.mode = P.Volume.RW
            op = P.Offer.Operation(type=P.Offer.Operation.CREATE)
            op.create.volumes.add().CopyFrom(v)
            driver.accept_offers([o.id], [op])
            self.volume, self.agent_id = v, o.agent_id.value
            self._done.set()

    def status_update(self, driver, status):
        pass

    def __getattr__(self, name):   # other scheduler callbacks are no-ops
        return lambda *a, **kw: None

    def start(self):
        self.driver.start()
        assert self._done.wait(10), "no offer with a slave_public disk"
        return self


def test_volume_collision_with_another_framework():
    c = sdk_install._cluster()
    foreign = _ForeignFramework(c).start()
    host = next(a["hostname"] for a in c.agents() if a["id"] == foreign.agent_id)
    path = c.behavior.volume_dir(host, foreign.volume.disk.persistence.id)
    import os

    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "test"), "w") as f:
        f.write("this is a test\n")

    def foreign_volume_intact():
        vols = [r for r in c.master.persistent_volumes(foreign.agent_id)
                if r.disk.persistence.id == foreign.volume.disk.persistence.id]
        assert len(vols) == 1 and vols[0].reservations[0].role == "slave_public"
        with open(os.path.join(path, "test")) as f:
            assert f.read().strip() == "this is a test"

    foreign_volume_intact()
    options = {"service": {"yaml": "pre-reserved"}, "hello": {"count": 1}, "world": {"count": 1}}
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 2, additional_options=options)
    try:
        config.check_running(config.SERVICE_NAME)
        foreign_volume_intact()
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
    # the uninstall cleaned up only its own reservations
    foreign_volume_intact()
