"""helloworld recovery suite on the local cluster.

Reference: frameworks/helloworld/tests/test_zzzrecovery.py -- pod restart stays on its agent, pod
replace, pause/resume (PAUSED override: sleep command, ``exit 1`` readiness check), graceful
shutdown within the kill grace period, killing the scheduler / a task / the executor / all
executors / the master / ZooKeeper, a config update while an agent is partitioned, automatic
replacement when an agent is decommissioned, and manual replacement after an agent shutdown.
Every kill hits a real process (``pkill -9 -f`` inside the task's session).
"""
import json
import re

import pytest

from dcos_commons_amd.testing.sdk import (sdk_agents, sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks,
                                          sdk_utils)
from tests.integration import hw_config as config
from tests.integration.conftest import needs_cli

pytestmark = needs_cli
SVC = config.SERVICE_NAME


def install_options_helper(kill_grace_period=0):
    sdk_install.uninstall(config.PACKAGE_NAME, SVC)
    sdk_install.install(config.PACKAGE_NAME, SVC, config.DEFAULT_TASK_COUNT + 1,
                        additional_options={"world": {"kill_grace_period": kill_grace_period, "count": 3}})


@pytest.fixture(scope="module", autouse=True)
def configure_package(local_cluster):
    install_options_helper()
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, SVC)


def check_healthy(expected_recovery_state="COMPLETE"):
    config.check_running(SVC)
    sdk_plan.wait_for_completed_deployment(SVC)
    sdk_plan.wait_for_plan_status(SVC, "recovery", expected_recovery_state)


def pod_info(pod):
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, SVC, f"pod info {pod}", print_output=False)
    assert rc == 0, "Pod info failed"
    return json.loads(out)[0]


def pod_cmd(cmd, pod):
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, SVC, f"{cmd} {pod}")
    assert rc == 0, f"{cmd} failed"
    doc = json.loads(out)
    assert doc == {"pod": pod, "tasks": [f"{pod}-server"]}


def test_pod_restart():
    hello_ids = sdk_tasks.get_task_ids(SVC, "hello-0")
    old_agent = pod_info("hello-0")["info"]["slaveId"]["value"]
    pod_cmd("pod restart", "hello-0")
    sdk_tasks.check_tasks_updated(SVC, "hello-0", hello_ids)
    check_healthy()
    assert pod_info("hello-0")["info"]["slaveId"]["value"] == old_agent


def test_pod_replace():
    world_ids = sdk_tasks.get_task_ids(SVC, "world-0")
    pod_cmd("pod replace", "world-0")
    sdk_tasks.check_tasks_updated(SVC, "world-0", world_ids)
    check_healthy()


def _plan_step(plan="deploy"):
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, SVC, f"plan status {plan} --json")
    assert rc == 0
    phase = json.loads(out)["phases"][0]
    assert phase["name"] == "hello" and phase["steps"][0]["name"] == "hello-0:[server]"
    return phase


def _pod_task_status(pod):
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, SVC, f"pod status {pod} --json")
    assert rc == 0
    doc = json.loads(out)
    assert len(doc["tasks"]) == 1 and doc["tasks"][0]["name"] == f"{pod}-server"
    return doc["tasks"][0]["status"]


def test_pod_pause_resume():
    info = pod_info("hello-0")["info"]
    old_agent, old_cmd = info["slaveId"]["value"], info["command"]["value"]
    assert _pod_task_status("hello-0") == "RUNNING"
    assert _plan_step()["steps"][0]["status"] == "COMPLETE"

    hello_ids = sdk_tasks.get_task_ids(SVC, "hello-0")
    pod_cmd("debug pod pause", "hello-0")
    sdk_tasks.check_tasks_updated(SVC, "hello-0", hello_ids)
    # the paused task's readiness check is `exit 1`: its recovery never completes
    check_healthy(expected_recovery_state=["STARTED", "IN_PROGRESS"])
    info = pod_info("hello-0")["info"]
    assert info["slaveId"]["value"] == old_agent
    assert "This task is PAUSED" in info["command"]["value"]
    assert info["check"]["command"]["command"]["value"] == "exit 1"
    assert _pod_task_status("hello-0") == "PAUSED"
    phase = _plan_step()
    assert phase["status"] == "COMPLETE" and phase["steps"][0]["status"] == "PAUSED"

    hello_ids = sdk_tasks.get_task_ids(SVC, "hello-0")
    pod_cmd("debug pod resume", "hello-0")
    sdk_tasks.check_tasks_updated(SVC, "hello-0", hello_ids)
    check_healthy()
    info = pod_info("hello-0")["info"]
    assert info["slaveId"]["value"] == old_agent and info["command"]["value"] == old_cmd
    assert _pod_task_status("hello-0") == "RUNNING"
    assert _plan_step()["steps"][0]["status"] == "COMPLETE"


def test_pods_restart_graceful_shutdown():
    install_options_helper(kill_grace_period=30)
    world_ids = sdk_tasks.get_task_ids(SVC, "world-0")
    pod_cmd("pod restart", "world-0")
    sdk_tasks.check_tasks_updated(SVC, "world-0", world_ids)
    check_healthy()
    # the SIGTERM reached the task's trap (its message, not the echo command line, is in the log)
    _, out, _ = sdk_cmd.run_cli(f"task log --completed --lines=1000 {world_ids[0]}")
    assert any("all clean" in line and "echo" not in line for line in out.splitlines()), out
    statuses = [s["state"] for s in sdk_tasks.get_all_status_history("world-0-server")]
    assert "TASK_KILLED" in statuses


def test_kill_scheduler():
    task_ids = sdk_tasks.get_task_ids(SVC, "")
    prefix = sdk_marathon.get_scheduler_task_prefix(SVC)
    scheduler_ids = sdk_tasks.get_task_ids("marathon", prefix)
    assert len(scheduler_ids) == 1, scheduler_ids
    assert sdk_cmd.kill_task_with_pattern("dcos_commons_amd.models.helloworld", "nobody",
                                          agent_host=sdk_marathon.get_scheduler_host(SVC))
    sdk_tasks.check_tasks_updated("marathon", prefix, scheduler_ids)
    sdk_tasks.wait_for_active_framework(SVC)
    config.check_running(SVC)
    sdk_tasks.check_tasks_not_updated(SVC, "", task_ids)


def test_kill_hello_task():
    hello = sdk_tasks.get_service_tasks(SVC, task_prefix="hello-0")[0]
    assert sdk_cmd.kill_task_with_pattern("hello-data/out", "nobody", agent_host=hello.host)
    sdk_tasks.check_tasks_updated(SVC, "hello-0", [hello.id])
    check_healthy()


def test_kill_world_executor():
    world = sdk_tasks.get_service_tasks(SVC, task_prefix="world-0")[0]
    assert sdk_cmd.kill_task_with_pattern("mesos-default-executor", "nobody", agent_host=world.host)
    sdk_tasks.check_tasks_updated(SVC, "world-0", [world.id])
    check_healthy()


def test_kill_all_executors():
    tasks = sdk_tasks.get_service_tasks(SVC)
    for task in tasks:
        sdk_cmd.kill_task_with_pattern("mesos-default-executor", "nobody", agent_host=task.host)
    sdk_tasks.check_tasks_updated(SVC, "", [t.id for t in tasks])
    check_healthy()


def test_kill_master():
    task_ids = sdk_tasks.get_task_ids(SVC, "")
    assert sdk_cmd.kill_task_with_pattern("mesos-master", "root")
    check_healthy()
    sdk_tasks.check_tasks_not_updated(SVC, "", task_ids)


def test_kill_zk():
    task_ids = sdk_tasks.get_task_ids(SVC, "")
    assert sdk_cmd.kill_task_with_pattern("QuorumPeerMain", "dcos_exhibitor")
    check_healthy()
    sdk_tasks.check_tasks_not_updated(SVC, "", task_ids)


def test_config_update_while_partitioned():
    world_tasks = sdk_tasks.get_service_tasks(SVC, "world")
    host = world_tasks[0].host
    sdk_agents.partition_agent(host)
    cfg = sdk_marathon.get_config(SVC)
    updated = float(cfg["env"]["WORLD_CPUS"]) + 0.1
    cfg["env"]["WORLD_CPUS"] = str(updated)
    sdk_marathon.update_app(cfg, wait_for_completed_deployment=False)
    sdk_agents.reconnect_agent(host)
    sdk_tasks.check_tasks_updated(SVC, "world", [t.id for t in world_tasks])
    check_healthy()
    running = [t for t in sdk_tasks.get_service_tasks(SVC) if t.name.startswith("world") and t.state == "TASK_RUNNING"]
    assert len(running) == config.world_task_count(SVC)
    for t in running:
        assert config.close_enough(t.resources["cpus"], updated)


def test_auto_replace_on_decommission():
    candidates = sdk_tasks.get_tasks_avoiding_scheduler(SVC, re.compile("^(hello|world)-[0-9]+-server$"))
    assert candidates
    agent_id = candidates[0].agent_id
    replaced = [t for t in candidates if t.agent_id == agent_id]
    sdk_agents.decommission_agent(candidates[0].host)
    sdk_install.ignore_dead_agent(candidates[0].host)
    # the recovery can start and finish between two polls here: wait on the tasks, then the plan
    for old in replaced:
        sdk_tasks.check_task_relaunched(old.name, old.id)
    sdk_plan.wait_for_completed_recovery(SVC)
    new_tasks = sdk_tasks.get_summary()
    for old in replaced:
        new = [t for t in new_tasks if t.name == old.name and t.id != old.id][0]
        assert new.agent_id != old.agent_id


def test_shutdown_host():
    candidates = sdk_tasks.get_tasks_avoiding_scheduler(SVC, re.compile("^(hello|world)-[0-9]+-server$"))
    assert candidates
    host = candidates[0].host
    replaced = [t for t in candidates if t.host == host]
    sdk_agents.shutdown_agent(host)
    sdk_install.ignore_dead_agent(host)
    pods = {t.name[: -len("-server")] for t in replaced}
    assert len(pods) == len(replaced)
    for pod in pods:
        sdk_cmd.svc_cli(config.PACKAGE_NAME, SVC, f"pod replace {pod}")
    for old in replaced:
        sdk_tasks.check_task_relaunched(old.name, old.id)
    sdk_plan.wait_for_completed_recovery(SVC)
    sdk_tasks.check_running(SVC, config.DEFAULT_TASK_COUNT)
    new_tasks = sdk_tasks.get_summary()
    for old in replaced:
        new = [t for t in new_tasks if t.name == old.name and t.id != old.id][0]
        assert new.agent_id != old.agent_id
