"""Cassandra framework on the local cluster (synthetic task payloads: no Cassandra binaries here).

Reference: frameworks/cassandra/tests/{test_sanity.py, test_zzzrecovery.py}: the service deploys
node by node then initialises the system keyspaces, serves its endpoints and seeds, runs the
repair / cleanup / backup plans with parameters, and recovers by replacing nodes: the seed node
(the recovery overrider relaunches it with ``-Dcassandra.replace_address=<old IP>``), a node moved
off its host by a placement change, and a node whose host was shut down.
"""
import json
import re

import pytest

from dcos_commons_amd.testing.sdk import (sdk_agents, sdk_cmd, sdk_install, sdk_marathon, sdk_networks, sdk_plan,
                                          sdk_tasks)
from tests.integration.conftest import make_cluster, needs_cli

PACKAGE = "cassandra"
SVC = "/test/integration/cassandra"
DEFAULT_TASK_COUNT = 3
ONCE_TASKS = ("-init_system_keyspaces", "-repair", "-cleanup", "-backup-schema", "-snapshot", "-upload-s3",
              "-upload-azure", "-cleanup-snapshot", "-fetch-s3", "-fetch-azure", "-restore-schema",
              "-restore-snapshot")


@pytest.fixture(scope="module", autouse=True)
def cassandra_cluster():
    c = make_cluster(executor="synthetic", finish_tasks=ONCE_TASKS)
    sdk_install.install(PACKAGE, SVC, DEFAULT_TASK_COUNT)
    yield c
    sdk_install.uninstall(PACKAGE, SVC)
    c.shutdown()


def test_deploy_plan_shape():
    plan = sdk_plan.get_deployment_plan(SVC)
    assert plan["status"] == "COMPLETE"
    assert [p["name"] for p in plan["phases"]] == ["node-deploy", "keyspace-deploy"]
    assert [s["name"] for s in plan["phases"][0]["steps"]] == [f"node-{i}:[server]" for i in range(3)]
    assert [s["name"] for s in plan["phases"][1]["steps"]] == ["node-0:[init_system_keyspaces]"]
    tasks = sdk_tasks.get_service_tasks(SVC)
    assert sorted(t.name for t in tasks) == [f"node-{i}-server" for i in range(3)]
    assert len({t.host for t in tasks}) == 3          # MAX_PER hostname 1


def test_endpoints():
    names = sdk_networks.get_endpoint_names(PACKAGE, SVC)
    assert "native-client" in names
    ep = sdk_networks.get_endpoint(PACKAGE, SVC, "native-client")
    assert len(ep["address"]) == 3 and len(ep["dns"]) == 3
    assert all(d.endswith(":9042") for d in ep["dns"])


def test_seeds_resource():
    seeds = sdk_cmd.service_request("GET", SVC, "/v1/seeds").json()
    assert len(seeds["seeds"]) == 2                     # LOCAL_SEEDS_COUNT default


def test_repair_cleanup_plans_complete():
    params = {"CASSANDRA_KEYSPACE": "testspace1"}
    sdk_plan.start_plan(SVC, "cleanup", parameters={"CASSANDRA_KEYSPACES": "testspace1"})
    sdk_plan.wait_for_completed_plan(SVC, "cleanup")
    sdk_plan.start_plan(SVC, "repair", parameters=params)
    sdk_plan.wait_for_completed_plan(SVC, "repair")
    # every node ran each one-shot task once, next to its server
    for task in ("cleanup", "repair"):
        done = [t for t in sdk_tasks.get_summary(with_completed=True) if t.name.endswith(f"-{task}")]
        assert sorted(t.name for t in done) == [f"node-{i}-{task}" for i in range(3)]
        assert all(t.state == "TASK_FINISHED" for t in done)


def test_backup_plan_phases():
    sdk_plan.start_plan(SVC, "backup-s3", parameters={"SNAPSHOT_NAME": "snap1", "CASSANDRA_KEYSPACES": "ks",
                                                      "S3_BUCKET_NAME": "bucket", "AWS_ACCESS_KEY_ID": "k",
                                                      "AWS_SECRET_ACCESS_KEY": "s", "AWS_REGION": "us-west-2"})
    plan = sdk_plan.wait_for_completed_plan(SVC, "backup-s3")
    assert [p["name"] for p in plan["phases"]] == ["backup-schema", "create-snapshots", "upload-backups",
                                                    "cleanup-snapshots"]


def test_scheduler_restart_keeps_nodes():
    ids = sdk_tasks.get_task_ids(SVC, "node")
    sdk_marathon.restart_app(SVC)
    sdk_plan.wait_for_completed_deployment(SVC)
    sdk_tasks.check_tasks_not_updated(SVC, "node", ids)


@needs_cli
def test_node_replace_replaces_seed_node():
    old = sdk_tasks.get_task_ids(SVC, "node-0-server")
    rc, out, _ = sdk_cmd.svc_cli(PACKAGE, SVC, "pod replace node-0")
    assert rc == 0 and json.loads(out)["pod"] == "node-0"
    sdk_tasks.check_tasks_updated(SVC, "node-0-server", old)
    sdk_plan.wait_for_completed_recovery(SVC)
    # the overrider's replace phase relaunched the seed with the old node's address
    recovery = sdk_plan.get_recovery_plan(SVC)
    assert recovery["phases"][0]["name"] == "permanent-node-failure-recovery", recovery
    infos = json.loads(sdk_cmd.svc_cli(PACKAGE, SVC, "pod info node-0", print_output=False)[1])
    server = next(e["info"] for e in infos if e["info"]["name"] == "node-0-server")
    assert "-Dcassandra.replace_address=" in server["command"]["value"]


@needs_cli
def test_node_replace_replaces_node():
    replace_task = [t for t in sdk_tasks.get_summary() if t.name == "node-2-server"][0]
    cfg = sdk_marathon.get_config(SVC)
    original = cfg["env"]["PLACEMENT_CONSTRAINT"]
    try:
        cfg["env"]["PLACEMENT_CONSTRAINT"] = f'[["hostname", "UNLIKE", "{replace_task.host}"]]'
        sdk_marathon.update_app(cfg)
        sdk_plan.wait_for_completed_deployment(SVC)
        sdk_cmd.svc_cli(PACKAGE, SVC, "pod replace node-2", check=True)
        sdk_tasks.check_task_relaunched("node-2-server", replace_task.id)
        sdk_plan.wait_for_completed_recovery(SVC)
        new = [t for t in sdk_tasks.get_summary() if t.name == "node-2-server"][0]
        assert new.host != replace_task.host
    finally:
        cfg = sdk_marathon.get_config(SVC)
        cfg["env"]["PLACEMENT_CONSTRAINT"] = original
        sdk_marathon.update_app(cfg)
        sdk_plan.wait_for_completed_deployment(SVC)


@needs_cli
def test_shutdown_host():
    candidates = sdk_tasks.get_tasks_avoiding_scheduler(SVC, re.compile("^node-[0-9]+-server$"))
    assert len(candidates) == len({t.host for t in candidates})      # nodes never share a machine
    victim = candidates[0]
    sdk_agents.shutdown_agent(victim.host)
    sdk_install.ignore_dead_agent(victim.host)
    sdk_cmd.svc_cli(PACKAGE, SVC, f"pod replace {victim.name[:-len('-server')]}", check=True)
    sdk_tasks.check_task_relaunched(victim.name, victim.id)
    sdk_plan.wait_for_completed_recovery(SVC)
    sdk_tasks.check_running(SVC, DEFAULT_TASK_COUNT)
    new = [t for t in sdk_tasks.get_summary() if t.name == victim.name and t.id != victim.id][0]
    assert new.agent_id != victim.agent_id
