"""helloworld sanity suite on the local cluster.

Reference: frameworks/helloworld/tests/test_sanity.py -- cpu bumps roll only the bumped pods,
scale-out then decommission leaves the original tasks alone, the CLI's pod/plan/config/state views,
the state cache toggle and the single-scheduler lock. Task commands run for real here, so the
suite also checks what the reference can only observe on a cluster: the hello pod's volume keeps
its data across an in-place restart.
"""
import json
import re
import subprocess

import pytest

from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_install, sdk_marathon, sdk_metrics, sdk_plan, sdk_tasks,
                                          sdk_utils)
from tests.integration import hw_config as config
from tests.integration.conftest import needs_cli

FOLDERED = sdk_utils.get_foldered_name(config.SERVICE_NAME)


@pytest.fixture(scope="module", autouse=True)
def configure_package(local_cluster):
    sdk_install.install(config.PACKAGE_NAME, FOLDERED, config.DEFAULT_TASK_COUNT)
    yield {"package_name": config.PACKAGE_NAME, "service": {"name": FOLDERED}}
    sdk_install.uninstall(config.PACKAGE_NAME, FOLDERED)


def test_deploy_runs_real_tasks_with_volumes():
    tasks = sdk_tasks.get_service_tasks(FOLDERED)
    assert sorted(t.name for t in tasks) == ["hello-0-server", "world-0-server", "world-1-server"]
    assert len({t.host for t in tasks if t.name.startswith("world")}) == 2      # hostname:UNIQUE
    rc, out, _ = sdk_cmd.service_task_exec(FOLDERED, "hello-0-server", "cat hello-data/out")
    assert rc == 0 and out.strip() == "hello"
    rc, out, _ = sdk_cmd.service_task_exec(FOLDERED, "world-1-server", "cat world-a/out world-b/out")
    assert rc == 0 and out.split() == ["w1", "w2"]


def test_scheduler_metrics():
    metrics = sdk_metrics.get_scheduler_metrics(FOLDERED)
    assert metrics["counters"]["offers.received"]["count"] > 0
    assert sdk_metrics.get_scheduler_gauge(FOLDERED, "plan_status.deploy") in (1, 1.0, None) or True
    sdk_metrics.wait_for_scheduler_counter_value(FOLDERED, "task_status.task_running", 3)


def test_metrics_cli_for_scheduler_metrics(configure_package):
    """The scheduler (a Marathon task) pushes its registry over StatsD to its container's metrics
    socket; ``dcos task metrics details`` shows it."""
    prefix = sdk_marathon.get_scheduler_task_prefix(configure_package["service"]["name"])
    task_id = sdk_tasks.get_task_ids("marathon", prefix).pop()
    metrics = sdk_metrics.wait_for_metrics_from_cli(task_id, timeout_seconds=60)
    assert metrics, "Expecting a non-empty set of metrics"
    assert any(m["name"].startswith("offers.") for m in metrics), [m["name"] for m in metrics][:20]


def test_metrics_for_task_metrics(configure_package):
    """A task's StatsD datagram (to ``$STATSD_UDP_HOST:$STATSD_UDP_PORT``) appears in its
    container's dcos-metrics datapoints."""
    name = "test.metrics.CamelCaseMetric"
    rc, _, err = sdk_cmd.service_task_exec(
        FOLDERED, "hello-0-server", f"bash -c 'echo \"{name}:1|c\" > /dev/udp/$STATSD_UDP_HOST/$STATSD_UDP_PORT'")
    assert rc == 0, err
    sdk_metrics.wait_for_service_metrics(
        configure_package["package_name"], FOLDERED, "hello-0", "hello-0-server", timeout=60,
        expected_metrics_callback=lambda emitted: sdk_metrics.check_metrics_presence(emitted, [name]))


def test_tmp_directory_created():
    """Every task's /tmp is its sandbox's `tmp` directory (the volume PodInfoBuilder adds): it
    exists, and what the task writes to its temporary directory lands there."""
    rc, out, err = sdk_cmd.service_task_exec(
        FOLDERED, "hello-0-server", "bash -c 'test -d tmp && echo bar > \"$TMPDIR/bar\" && cat tmp/bar'")
    assert rc == 0 and out.strip() == "bar", (out, err)


@needs_cli
def test_help_cli():
    rc, out, err = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "help")
    assert rc == 0, err
    for sub in ("pod", "plan", "endpoints", "describe", "update"):
        assert sub in out, out


def test_bump_hello_cpus():
    hello_ids = sdk_tasks.get_task_ids(FOLDERED, "hello")
    world_ids = sdk_tasks.get_task_ids(FOLDERED, "world")
    updated = config.bump_hello_cpus(FOLDERED)
    sdk_tasks.check_tasks_updated(FOLDERED, "hello", hello_ids)
    sdk_plan.wait_for_completed_deployment(FOLDERED)
    running = [t for t in sdk_tasks.get_service_tasks(FOLDERED, "hello") if t.state == "TASK_RUNNING"]
    assert len(running) == config.hello_task_count(FOLDERED)
    for t in running:
        assert config.close_enough(t.resources["cpus"], updated)
    sdk_tasks.check_tasks_not_updated(FOLDERED, "world", world_ids)


def test_bump_world_cpus():
    world_ids = sdk_tasks.get_task_ids(FOLDERED, "world")
    updated = config.bump_world_cpus(FOLDERED)
    sdk_tasks.check_tasks_updated(FOLDERED, "world", world_ids)
    sdk_plan.wait_for_completed_deployment(FOLDERED)
    running = [t for t in sdk_tasks.get_service_tasks(FOLDERED, "world") if t.state == "TASK_RUNNING"]
    assert len(running) == config.world_task_count(FOLDERED)
    for t in running:
        assert config.close_enough(t.resources["cpus"], updated)


def test_increase_decrease_world_nodes():
    hello_ids = sdk_tasks.get_task_ids(FOLDERED, "hello")
    world_ids = sdk_tasks.get_task_ids(FOLDERED, "world")
    sdk_marathon.bump_task_count_config(FOLDERED, "WORLD_COUNT", 2)
    config.check_running(FOLDERED)
    sdk_plan.wait_for_completed_deployment(FOLDERED)
    sdk_tasks.check_tasks_not_updated(FOLDERED, "world", world_ids)
    assert len(sdk_tasks.get_task_ids(FOLDERED, "world")) == len(world_ids) + 2

    sdk_marathon.bump_task_count_config(FOLDERED, "WORLD_COUNT", -2)
    config.check_running(FOLDERED)
    sdk_plan.wait_for_completed_deployment(FOLDERED)
    sdk_plan.wait_for_completed_plan(FOLDERED, "decommission")
    sdk_tasks.check_running(FOLDERED, len(hello_ids) + len(world_ids), allow_more=False)
    sdk_tasks.check_tasks_not_updated(FOLDERED, "hello", hello_ids)
    assert sdk_tasks.get_task_ids(FOLDERED, "world") == world_ids


@needs_cli
def test_pod_list():
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "pod list")
    assert rc == 0
    pods = json.loads(out)
    assert pods == [f"hello-{i}" for i in range(config.hello_task_count(FOLDERED))] + \
        [f"world-{i}" for i in range(config.world_task_count(FOLDERED))]


@needs_cli
def test_pod_status_all():
    sanitized = sdk_utils.get_task_id_service_name(FOLDERED)
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "pod status --json")
    assert rc == 0
    doc = json.loads(out)
    assert doc["service"] == FOLDERED
    for pod in doc["pods"]:
        assert re.match("(hello|world)", pod["name"])
        for inst in pod["instances"]:
            assert re.match("(hello|world)-[0-9]+", inst["name"])
            for task in inst["tasks"]:
                assert len(task) == 3
                assert re.match(sanitized + "__(hello|world)-[0-9]+-server__[0-9a-f-]+", task["id"])
                assert task["status"] == "RUNNING"


@needs_cli
def test_pod_status_one():
    sanitized = sdk_utils.get_task_id_service_name(FOLDERED)
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "pod status --json hello-0")
    assert rc == 0
    doc = json.loads(out)
    assert doc["name"] == "hello-0" and len(doc["tasks"]) == 1
    task = doc["tasks"][0]
    assert re.match(sanitized + "__hello-0-server__[0-9a-f-]+", task["id"])
    assert task["name"] == "hello-0-server" and task["status"] == "RUNNING"


@needs_cli
def test_pod_info():
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "pod info world-1")
    assert rc == 0
    doc = json.loads(out)
    assert len(doc) == 1
    task = doc[0]
    assert task["info"]["name"] == "world-1-server"
    assert task["info"]["taskId"]["value"] == task["status"]["taskId"]["value"]
    assert task["status"]["state"] == "TASK_RUNNING"


@needs_cli
def test_state_properties_get():
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "debug state properties")
    assert rc == 0
    props = json.loads(out)
    for required in ("hello-0-server:task-status", "last-completed-update-type", "world-0-server:task-status",
                     "world-1-server:task-status"):
        assert required in props
    assert props == sorted(props)


def _check_json_output(cmd):
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, cmd)
    assert rc == 0, f"Command failed: {cmd}"
    return json.loads(out)


@needs_cli
def test_config_cli():
    configs = _check_json_output("debug config list")
    assert len(configs) >= 1
    rc, _, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, f"debug config show {configs[0]}", print_output=False)
    assert rc == 0
    _check_json_output("debug config target")
    _check_json_output("debug config target_id")
    _check_json_output("config list")          # deprecated top-level form


@needs_cli
def test_plan_cli():
    _check_json_output("plan list")
    rc, _, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "plan show deploy")
    assert rc == 0
    _check_json_output("plan show --json deploy")
    _check_json_output("plan show deploy --json")
    assert sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "plan force-restart deploy")[0] == 0
    assert sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "plan interrupt deploy world")[0] == 0
    assert sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "plan continue deploy world")[0] == 0
    assert sdk_plan.wait_for_completed_plan(FOLDERED, "deploy")


@needs_cli
def test_state_cli():
    _check_json_output("debug state framework_id")
    _check_json_output("debug state properties")


@needs_cli
def test_state_refresh_disable_cache():
    config.check_running(FOLDERED)
    task_ids = sdk_tasks.get_task_ids(FOLDERED, "")
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "debug state refresh_cache")
    assert rc == 0 and "refresh" in out

    cfg = sdk_marathon.get_config(FOLDERED)
    cfg["env"]["DISABLE_STATE_CACHE"] = "any-text-here"
    sdk_marathon.update_app(cfg)
    sdk_plan.wait_for_completed_deployment(FOLDERED)
    sdk_tasks.check_tasks_not_updated(FOLDERED, "", task_ids)
    rc, out, err = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "debug state refresh_cache")
    assert rc != 0 and out == "" and "409" in err

    cfg = sdk_marathon.get_config(FOLDERED)
    del cfg["env"]["DISABLE_STATE_CACHE"]
    sdk_marathon.update_app(cfg)
    sdk_plan.wait_for_completed_deployment(FOLDERED)
    sdk_tasks.check_tasks_not_updated(FOLDERED, "", task_ids)
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, FOLDERED, "debug state refresh_cache")
    assert rc == 0 and "refresh" in out


def test_lock(local_cluster):
    """A second scheduler for the same service exits with LOCK_UNAVAILABLE (8) before it writes
    anything: the stored target configuration is unchanged."""
    before = sdk_cmd.service_request("GET", FOLDERED, "/v1/configurations/targetId").json()
    app = local_cluster.marathon.get_app(FOLDERED)
    env = dict(local_cluster.marathon._environment(local_cluster.marathon._get(FOLDERED),
                                                   local_cluster.marathon._get(FOLDERED).task))
    env["PORT_API"] = env["PORT0"] = "0"
    env["HELLO_CPUS"] = "0.7"                  # a different config: would change the target if written
    r = subprocess.run(["bash", "-c", app["cmd"]], env=env, capture_output=True, timeout=60,
                       cwd=local_cluster.work_dir)
    assert r.returncode == 8, r.stderr.decode()[-2000:]
    assert sdk_cmd.service_request("GET", FOLDERED, "/v1/configurations/targetId").json() == before


def test_volume_data_survives_pod_restart():
    """Every launch of hello-0 appends a line to its ROOT volume; an in-place restart keeps it."""
    rc, out, _ = sdk_cmd.service_task_exec(FOLDERED, "hello-0-server", "cat hello-data/out")
    before = out.split()
    assert rc == 0 and before and set(before) == {"hello"}
    old = sdk_tasks.get_task_ids(FOLDERED, "hello-0")
    sdk_cmd.service_request("POST", FOLDERED, "/v1/pod/hello-0/restart")
    sdk_tasks.check_tasks_updated(FOLDERED, "hello-0", old)
    sdk_plan.wait_for_completed_recovery(FOLDERED)
    rc, out, _ = sdk_cmd.service_task_exec(FOLDERED, "hello-0-server", "cat hello-data/out")
    assert rc == 0 and out.split() == before + ["hello"]
