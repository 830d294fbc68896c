"""The reference's unchanged cassandra and hdfs packages, run end to end on the local DC/OS
stand-in (synthetic task payloads).

Cosmos renders each package's own ``universe/`` (its 182 / 399 options, its
``marathon.json.mustache``); Marathon fetches the package's scheduler artifact (staged from the
reference's ``src/main/dist``, ``testing.cluster.reference_packages``) and this tree's native
bootstrap, and runs the package's ``cmd`` unchanged, which starts this SDK's scheduler on the
reference ``svc.yml`` as its own process: ZooKeeper persistence, the Mesos v1 HTTP API.

Scenarios, after the reference's system tier:
* cassandra: deploy; replace the seed node ``node-0`` (``CassandraRecoveryPlanOverrider``: the
  ``permanent-node-failure-recovery`` phase relaunches it with ``-Dcassandra.replace_address``),
  frameworks/cassandra/tests/test_zzzrecovery.py:34;
* hdfs: deploy; an ``hdfs-site.xml`` change rolled out by the ``update`` plan with the scheduler
  killed in the middle of it (the restarted scheduler resumes the rollout; every node is
  relaunched, the recovery plan is untouched), frameworks/hdfs/tests/test_sanity.py:148,291.

Skipped where the reference tree is absent (the GPU box)."""
import json
import time

import pytest

from dcos_commons_amd.testing.cluster.reference_packages import (reference_packages, reference_root,
                                                                 stage_scheduler_artifacts)
from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks
from tests.integration.conftest import make_cluster

ROOT = reference_root()
pytestmark = pytest.mark.skipif(ROOT is None, reason="reference tree not present")

CASSANDRA, HDFS = "/ref/cassandra", "/ref/hdfs"
FINISH_TASKS = ("-init_system_keyspaces", "-format", "-bootstrap", "-zkfc-format")
HDFS_TASKS = 10                      # 3 journal + 2 name + 2 zkfc + 3 data
# the reference package's readiness defaults wait 30 s (journal) and 120 s (data) before a first
# check; these are its own options, shortened as the reference's CI does for data nodes
HDFS_OPTIONS = {"journal_node": {"readiness_check": {"delay": 0, "interval": 1}},
                "data_node": {"readiness_check": {"delay": 0, "interval": 1}}}
APP_CONFIG_FIELD = "TASKCFG_ALL_CLIENT_READ_SHORTCIRCUIT_STREAMS_CACHE_EXPIRY_MS"


@pytest.fixture(scope="module", autouse=True)
def reference_cluster():
    c = make_cluster(executor="synthetic", finish_tasks=FINISH_TASKS, packages=reference_packages(ROOT))
    stage_scheduler_artifacts(c, ROOT)
    yield c
    c.shutdown()


def _pod_info(svc: str, pod: str) -> list:
    return sdk_cmd.service_request("GET", svc, f"/v1/pod/{pod}/info").json()


def test_reference_cassandra_deploys_and_replaces_the_seed_node():
    sdk_install.install("cassandra", CASSANDRA, 3)
    plan = sdk_plan.get_deployment_plan(CASSANDRA)
    assert plan["status"] == "COMPLETE"
    # the reference svc.yml ran: its node pod has 13 tasks (server + the backup/restore/repair ones)
    assert len(_pod_info(CASSANDRA, "node-0")) == 13
    old = sdk_tasks.get_task_ids(CASSANDRA, "node-0-server")
    r = sdk_cmd.service_request("POST", CASSANDRA, "/v1/pod/node-0/replace")
    assert r.status_code == 200
    sdk_tasks.check_tasks_updated(CASSANDRA, "node-0-server", old)
    sdk_plan.wait_for_completed_recovery(CASSANDRA)
    recovery = sdk_plan.get_recovery_plan(CASSANDRA)
    assert recovery["phases"][0]["name"] == "permanent-node-failure-recovery", recovery
    assert [s["name"] for s in recovery["phases"][0]["steps"]] == [f"node-{i}:[server]" for i in range(3)]
    server = next(e["info"] for e in _pod_info(CASSANDRA, "node-0") if e["info"]["name"] == "node-0-server")
    assert "-Dcassandra.replace_address=" in server["command"]["value"]
    sdk_install.uninstall("cassandra", CASSANDRA)


def test_reference_hdfs_update_survives_a_scheduler_kill():
    sdk_install.install("hdfs", HDFS, HDFS_TASKS, additional_options=HDFS_OPTIONS)
    assert sorted(sdk_plan.get_deployment_plan(HDFS)["status"] for _ in [0]) == ["COMPLETE"]
    sdk_plan.wait_for_completed_recovery(HDFS)
    old_recovery = sdk_plan.get_plan(HDFS, "recovery")
    ids = {p: sdk_tasks.get_task_ids(HDFS, p) for p in ("journal", "name", "data")}

    cfg = sdk_marathon.get_config(HDFS)
    cfg["env"][APP_CONFIG_FIELD] = str(int(cfg["env"][APP_CONFIG_FIELD]) + 1)
    sdk_marathon.update_app(cfg)
    # the restarted scheduler selects the update plan; kill it once the rollout has begun
    sdk_tasks.check_tasks_updated(HDFS, "journal-0", [i for i in ids["journal"] if "journal-0-" in i])
    prefix = sdk_marathon.get_scheduler_task_prefix(HDFS)
    sched = sdk_tasks.get_task_ids("marathon", prefix)
    assert sdk_cmd.kill_task_with_pattern("./hdfs-scheduler/bin/hdfs", "nobody",
                                          agent_host=sdk_marathon.get_scheduler_host(HDFS))
    sdk_tasks.check_tasks_updated("marathon", prefix, sched)

    for p, old in ids.items():
        sdk_tasks.check_tasks_updated(HDFS, p, old)
    deadline = time.time() + 120
    while time.time() < deadline:
        plan = sdk_plan.get_deployment_plan(HDFS)
        if plan["status"] == "COMPLETE" and len(sdk_tasks.get_service_tasks(HDFS)) >= HDFS_TASKS:
            break
        time.sleep(0.2)
    plan = sdk_plan.get_deployment_plan(HDFS)
    assert plan["status"] == "COMPLETE", json.dumps(plan)[:2000]
    # the rollout is the package's update plan (serial journal phase), not its parallel deploy
    assert plan["phases"][0]["strategy"] == "serial"
    assert sdk_plan.get_plan(HDFS, "recovery") == old_recovery
    sdk_install.uninstall("hdfs", HDFS)
