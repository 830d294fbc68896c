"""Shared set-up of the quota role suites (reference frameworks/helloworld/tests/test_quota_*.py):
a cluster of five agents in three zones, the quota group's name and the service's legacy role."""
from dcos_commons_amd.mesos.local_master import AgentSpec
from dcos_commons_amd.testing.cluster.cluster import DCOS_AGENT_PORTS, LocalCluster, use
from dcos_commons_amd.testing.sdk import sdk_utils

ENFORCED_ROLE = "quota"
SERVICE_NAME = f"/{ENFORCED_ROLE}/hello-world"
LEGACY_ROLE = "{}-role".format(SERVICE_NAME.strip("/").replace("/", "__"))


def start_cluster() -> LocalCluster:
    specs = [AgentSpec(hostname=f"10.0.0.{i + 1}", ports=DCOS_AGENT_PORTS, region="us-west-2",
                       zone=("us-west-2a", "us-west-2b", "us-west-2c")[i % 3]) for i in range(5)]
    c = LocalCluster(agent_specs=specs, scheduler_env={"SDK_LOCK_WAIT_S": "1"}).start()
    use(c)
    return c


def roles():
    r = sdk_utils.get_service_roles(SERVICE_NAME)
    assert len(r["task-roles"]) > 0
    return r


def assert_single_role(r, role):
    assert r["framework-roles"] is None and r["framework-role"] == role


def assert_multi_role(r):
    assert r["framework-role"] is None and sorted(r["framework-roles"]) == sorted([LEGACY_ROLE, ENFORCED_ROLE])
