"""HDFS framework on the local cluster (synthetic task payloads: no Hadoop binaries here).

Reference: frameworks/hdfs/tests/test_sanity.py -- HA deploy (journal -> name format/bootstrap ->
zkfc format -> data), endpoints, killing journal/name/data tasks, rolling restarts of whole pod
types, a permanent and a transient name-node failure at once, config updates rolled out by the
``update`` plan (journal nodes serially, name nodes untouched by a journal change), scale-out of
data nodes, an hdfs-site change that rolls everything without touching recovery, its rollback,
and permanent replacement of name and journal nodes (the ``replace`` plan's bootstrap steps).
"""
from xml.etree import ElementTree

import pytest

from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_hosts, sdk_install, sdk_marathon, sdk_networks, sdk_plan,
                                          sdk_recovery, sdk_tasks, sdk_utils)
from tests.integration.conftest import make_cluster, needs_cli

PACKAGE = "hdfs"
SVC = "/test/integration/hdfs"
DEFAULT_TASK_COUNT = 10           # 3 journal + 2 name + 2 zkfc + 3 data
FINISH_TASKS = ("-format", "-bootstrap", "-zkfc-format")
APP_CONFIG_FIELD = "TASKCFG_ALL_CLIENT_READ_SHORTCIRCUIT_STREAMS_CACHE_EXPIRY_MS"   # the reference test_sanity.py field


@pytest.fixture(scope="module", autouse=True)
def hdfs_cluster():
    c = make_cluster(executor="synthetic", finish_tasks=FINISH_TASKS, honor_check_delays=False)
    # (data nodes pass their first readiness check after 1 s instead of the default 10 s)
    sdk_install.install(PACKAGE, SVC, DEFAULT_TASK_COUNT,
                        additional_options={"data_node": {"readiness_check": {"delay": 1, "interval": 1}}})
    yield c
    sdk_install.uninstall(PACKAGE, SVC)
    c.shutdown()


def check_healthy(count=DEFAULT_TASK_COUNT):
    sdk_plan.wait_for_completed_deployment(SVC)
    sdk_plan.wait_for_completed_recovery(SVC)
    sdk_tasks.check_running(SVC, count)


def expect_recovery():
    sdk_plan.wait_for_completed_recovery(SVC)
    check_healthy()


def test_install_plan_shape():
    plan = sdk_plan.get_deployment_plan(SVC)
    assert [p["name"] for p in plan["phases"]] == ["journal", "name", "zkfc", "data"]
    assert [s["name"] for s in plan["phases"][1]["steps"]] == ["name-0:[format]", "name-0:[node]",
                                                               "name-1:[bootstrap]", "name-1:[node]"]
    names = sorted(t.name for t in sdk_tasks.get_service_tasks(SVC))
    assert names == sorted([f"journal-{i}-node" for i in range(3)] + ["name-0-node", "name-0-zkfc", "name-1-node",
                                                                       "name-1-zkfc"]
                           + [f"data-{i}-node" for i in range(3)])
    # the one-shot formatting tasks ran and finished exactly once
    done = {t.name for t in sdk_tasks.get_summary(with_completed=True) if t.state == "TASK_FINISHED"}
    assert {"name-0-format", "name-1-bootstrap", "name-0-zkfc-format"} <= done


def _properties(xml_text, wanted):
    root = ElementTree.fromstring(xml_text)
    return {p.find("name").text: p.find("value").text for p in root.findall("property")
            if p.find("name").text in wanted}


def test_endpoints():
    assert {"core-site.xml", "hdfs-site.xml"} <= set(sdk_networks.get_endpoint_names(PACKAGE, SVC))
    expect = {"ha.zookeeper.parent-znode": f"/{sdk_utils.get_zk_path(SVC)}/hadoop-ha"}
    assert _properties(sdk_networks.get_endpoint_string(PACKAGE, SVC, "core-site.xml"), expect) == expect
    journals = ";".join(sdk_hosts.autoip_host(SVC, f"journal-{i}-node", 8485) for i in range(3))
    expect = {"dfs.namenode.shared.edits.dir": f"qjournal://{journals}/hdfs"}
    for i in range(2):
        node = f"name-{i}-node"
        expect[f"dfs.namenode.rpc-address.hdfs.{node}"] = sdk_hosts.autoip_host(SVC, node, 9001)
        expect[f"dfs.namenode.http-address.hdfs.{node}"] = sdk_hosts.autoip_host(SVC, node, 9002)
    assert _properties(sdk_networks.get_endpoint_string(PACKAGE, SVC, "hdfs-site.xml"), expect) == expect


@pytest.mark.parametrize("pod_type", ["journal", "name", "data"])
def test_kill_node(pod_type, hdfs_cluster):
    task = sdk_tasks.get_service_tasks(SVC, f"{pod_type}-0-node")[0]
    hdfs_cluster.fail_task(task.id)
    sdk_tasks.check_tasks_updated(SVC, f"{pod_type}-0-node", [task.id])
    check_healthy()


def test_kill_scheduler():
    task_ids = sdk_tasks.get_task_ids(SVC, "")
    prefix = sdk_marathon.get_scheduler_task_prefix(SVC)
    sched = sdk_tasks.get_task_ids("marathon", prefix)
    assert sdk_cmd.kill_task_with_pattern("dcos_commons_amd.models.hdfs", "nobody",
                                          agent_host=sdk_marathon.get_scheduler_host(SVC))
    sdk_tasks.check_tasks_updated("marathon", prefix, sched)
    check_healthy()
    sdk_tasks.check_tasks_not_updated(SVC, "", task_ids)


@needs_cli
@pytest.mark.parametrize("pod_type,count", [("journal", 3), ("name", 2), ("data", 3)])
def test_restart_all_pods_of_a_type(pod_type, count):
    ids = sdk_tasks.get_task_ids(SVC, pod_type)
    for i in range(count):
        sdk_cmd.svc_cli(PACKAGE, SVC, f"pod restart {pod_type}-{i}", check=True)
    expect_recovery()
    sdk_tasks.check_tasks_updated(SVC, pod_type, ids)


@needs_cli
@pytest.mark.parametrize("replace,restart", [("name-0", "name-1"), ("name-1", "name-0")])
def test_permanent_and_transient_namenode_failures(replace, restart):
    check_healthy()
    ids = {p: sdk_tasks.get_task_ids(SVC, p) for p in ("name-0", "name-1", "journal", "data")}
    sdk_cmd.svc_cli(PACKAGE, SVC, f"pod replace {replace}", check=True)
    sdk_cmd.svc_cli(PACKAGE, SVC, f"pod restart {restart}", check=True)
    sdk_tasks.check_tasks_updated(SVC, "name-0", ids["name-0"])
    sdk_tasks.check_tasks_updated(SVC, "name-1", ids["name-1"])
    expect_recovery()
    sdk_tasks.check_tasks_not_updated(SVC, "journal", ids["journal"])
    sdk_tasks.check_tasks_not_updated(SVC, "data", ids["data"])


def test_bump_journal_cpus():
    journal_ids = sdk_tasks.get_task_ids(SVC, "journal")
    name_ids = sdk_tasks.get_task_ids(SVC, "name")
    sdk_marathon.bump_cpu_count_config(SVC, "JOURNAL_CPUS")
    sdk_tasks.check_tasks_updated(SVC, "journal", journal_ids)
    # the update plan (not the parallel deploy plan) rolls journal nodes: name nodes untouched
    sdk_tasks.check_tasks_not_updated(SVC, "name", name_ids)
    plan = sdk_plan.get_deployment_plan(SVC)
    assert plan["phases"][0]["strategy"] == "serial"
    check_healthy()


def test_bump_data_nodes():
    data_ids = sdk_tasks.get_task_ids(SVC, "data")
    sdk_marathon.bump_task_count_config(SVC, "DATA_COUNT")
    check_healthy(count=DEFAULT_TASK_COUNT + 1)
    sdk_tasks.check_tasks_not_updated(SVC, "data", data_ids)


def test_modify_app_config():
    """An hdfs-site.xml change rolls every pod through the update plan and never the recovery plan."""
    sdk_plan.wait_for_completed_recovery(SVC)
    old_recovery = sdk_plan.get_plan(SVC, "recovery")
    ids = {p: sdk_tasks.get_task_ids(SVC, p) for p in ("journal", "name", "data")}
    cfg = sdk_marathon.get_config(SVC)
    cfg["env"][APP_CONFIG_FIELD] = str(int(cfg["env"][APP_CONFIG_FIELD]) + 1)
    sdk_marathon.update_app(cfg)
    for p, old in ids.items():
        sdk_tasks.check_tasks_updated(SVC, p, old)
    check_healthy(count=DEFAULT_TASK_COUNT + 1)
    assert sdk_plan.get_plan(SVC, "recovery") == old_recovery


def test_modify_app_config_rollback():
    journal_ids = sdk_tasks.get_task_ids(SVC, "journal")
    data_ids = sdk_tasks.get_task_ids(SVC, "data")
    old_config = sdk_marathon.get_config(SVC)
    expiry = int(old_config["env"][APP_CONFIG_FIELD])
    cfg = sdk_marathon.get_config(SVC)
    cfg["env"][APP_CONFIG_FIELD] = str(expiry + 1)
    # roll out, then put the old config back as soon as the journal nodes have been touched
    sdk_marathon.update_app(cfg)
    sdk_tasks.check_tasks_updated(SVC, "journal", journal_ids)
    journal_ids = sdk_tasks.get_task_ids(SVC, "journal")
    sdk_marathon.update_app(old_config)
    sdk_tasks.check_tasks_updated(SVC, "journal", journal_ids)
    check_healthy(count=DEFAULT_TASK_COUNT + 1)
    assert int(sdk_marathon.get_config(SVC)["env"][APP_CONFIG_FIELD]) == expiry


@needs_cli
def test_permanently_replace_namenodes():
    for pod in ("name-0", "name-1", "name-0"):
        sdk_recovery.check_permanent_recovery(PACKAGE, SVC, pod, recovery_timeout_s=120)


@needs_cli
def test_permanently_replace_journalnodes():
    for pod in ("journal-0", "journal-1", "journal-2"):
        sdk_recovery.check_permanent_recovery(PACKAGE, SVC, pod, recovery_timeout_s=120)
    # the replace plan's bootstrap step re-initialised each new journal node
    boots = [t for t in sdk_tasks.get_summary(with_completed=True) if t.name.startswith("journal-")
             and t.name.endswith("-bootstrap")]
    assert len(boots) >= 3 and all(t.state == "TASK_FINISHED" for t in boots)


@needs_cli
def test_namenodes_acheive_quorum_after_journalnode_replace():
    """journal-0, journal-1, then journal-0 again replaced: every recovery completes and the name
    nodes keep running (reference test_sanity.py; HDFS-10659 had the second replacement crash-loop
    the name nodes)."""
    names = sdk_tasks.get_task_ids(SVC, "name-")
    for pod in ("journal-0", "journal-1", "journal-0"):
        old = sdk_tasks.get_task_ids(SVC, f"{pod}-")
        sdk_cmd.svc_cli(PACKAGE, SVC, f"pod replace {pod}", check=True)
        sdk_tasks.check_tasks_updated(SVC, f"{pod}-", old)
        sdk_plan.wait_for_completed_recovery(SVC)
    sdk_tasks.check_tasks_not_updated(SVC, "name-", names)
    check_healthy()
