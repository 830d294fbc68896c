"""helloworld volume scenarios on the local cluster.

Reference: frameworks/helloworld/tests/{test_executor_volumes.py, test_host_volumes.py,
test_mount_volumes.py, test_profile_mount_volumes.py}. A pod-level (executor) volume is shared by
the pod's tasks and survives a task relaunch; host volumes expose agent paths inside the task; a
MOUNT volume takes a whole agent disk and a task relaunched in place gets the same disk and its
data back; a volume that asks for a disk profile only lands on disks of that profile.
"""
import json

import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_plan, sdk_tasks, sdk_utils
from tests.integration import hw_config as config
from tests.integration.conftest import make_cluster, needs_cli

# every agent: two plain 2 GB disks and one 1 GB disk of the "fast-nvme" profile
MOUNT_DISKS = (("/dcos/volume0", 2000.0), ("/dcos/volume1", 1000.0, "fast-nvme"), ("/dcos/volume2", 2000.0))


@pytest.fixture(scope="module")
def local_cluster():
    c = make_cluster(mount_disks=MOUNT_DISKS)
    yield c
    c.shutdown()


pytestmark = pytest.mark.usefixtures("local_cluster")


def _pod_info(pod):
    return sdk_cmd.service_request("GET", config.SERVICE_NAME, f"/v1/pod/{pod}/info").json()


def _volumes(task_info):
    """(container path, persistence id, size, source) of every persistent volume of a task info
    (its own resources and its executor's)."""
    out = []
    for r in task_info.get("resources", []) + task_info.get("executor", {}).get("resources", []):
        disk = r.get("disk", {})
        if "persistence" in disk:
            out.append((disk["volume"]["containerPath"], disk["persistence"]["id"], r["scalar"]["value"],
                        disk.get("source", {})))
    return out


def _log(task_name):
    rc, out, _ = sdk_cmd.run_cli(f"task log --lines=50 {task_name}", print_output=False)
    assert rc == 0
    return out


def test_executor_volume_shared_and_kept_across_relaunch():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 2,
                        additional_options={"service": {"yaml": "executor_volume"}, "hello": {"count": 2}})
    try:
        plan = sdk_plan.get_deployment_plan(config.SERVICE_NAME)
        assert [p["name"] for p in plan["phases"]] == ["hello"]
        assert [s["name"] for s in plan["phases"][0]["steps"]] == \
            ["hello-0:[writer]", "hello-0:[server]", "hello-1:[writer]", "hello-1:[server]"]
        # the writer (ONCE) wrote into the pod volume, the server read it from the same pod volume
        for i in range(2):
            assert "data" in _log(f"hello-{i}-server").split()
            info = {t["info"]["name"]: t["info"] for t in _pod_info(f"hello-{i}")}
            # (the writer's executor exited with its task group; the server's executor carries the
            # same reserved pod volume)
            pod_vols = [v for v in _volumes(info[f"hello-{i}-server"]) if v[0] == "pod-data"]
            assert len(pod_vols) == 1 and pod_vols[0][2] == 64
            assert [v for v in _volumes(info[f"hello-{i}-writer"]) if v[0] == "pod-data"] == pod_vols
            assert [v[0] for v in _volumes(info[f"hello-{i}-server"]) if v[0] != "pod-data"] == ["task-data"]
        old = sdk_tasks.get_service_tasks(config.SERVICE_NAME, "hello-0-server")[0]
        vols_before = sorted(_volumes(next(t["info"] for t in _pod_info("hello-0")
                                           if t["info"]["name"] == "hello-0-server")))
        assert sdk_cmd.kill_task_with_pattern("pod-data/file", agent_host=old.host)
        sdk_tasks.check_task_relaunched("hello-0-server", old.id)
        sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
        new = sdk_tasks.get_service_tasks(config.SERVICE_NAME, "hello-0-server")[0]
        assert new.host == old.host
        # relaunched in place: same volumes, and the file the writer left is still there
        assert sorted(_volumes(next(t["info"] for t in _pod_info("hello-0")
                                    if t["info"]["name"] == "hello-0-server"))) == vols_before

        @sdk_utils.retry(timeout_s=30, interval_s=0.5)
        def reread():
            assert _log("hello-0-server").split().count("data") >= 1
        reread()
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_host_volume_mounts():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"yaml": "host-volume"}})
    try:
        info = _pod_info("hello-0")[0]["info"]
        vols = {v["containerPath"]: v for v in info["container"]["volumes"]}
        assert vols["host-etc"]["hostPath"] == "/etc" and vols["host-etc"]["mode"] == "RO"
        assert vols["host-tmp"]["mode"] == "RW"

        @sdk_utils.retry(timeout_s=30, interval_s=0.5)
        def read_group():
            rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, "hello-0-server", "cat host-etc/group")
            assert rc == 0 and any(line.startswith("root:") for line in out.splitlines()), out
        read_group()
        rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, "hello-0-server", "ls host-tmp/x")
        assert rc == 0, out
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


@pytest.fixture
def pod_mount_service():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 4,
                        additional_options={"service": {"yaml": "pod-mount-volume"}, "hello": {"count": 2}})
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def _verify_shared_executor(pod):
    """Both tasks of ``pod`` run in one executor and see each other's writes to the pod volume
    (reference test_mount_volumes.py ``verify_shared_executor``)."""
    infos = [t["info"] for t in _pod_info(pod)]
    assert len(infos) == 2
    assert infos[0]["executor"] == infos[1]["executor"]
    rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, f"{pod}-agent", "sort -u mount-data/written-by")
    assert rc == 0 and out.split() == ["agent", "node"], out


@needs_cli
def test_pod_mount_volume_survives_task_kill(pod_mount_service):
    rc, out, _ = sdk_cmd.svc_cli(config.PACKAGE_NAME, config.SERVICE_NAME, "pod info hello-0", print_output=False)
    assert rc == 0
    infos = {i["info"]["name"]: i["info"] for i in json.loads(out)}
    pod_vol = [v for v in _volumes(infos["hello-0-node"]) if v[0] == "mount-data"]
    node_vol = [v for v in _volumes(infos["hello-0-node"]) if v[0] == "node-disk"]
    (_, pid, size, source), = pod_vol
    # whole plain disks, never the profiled one; the node task's own disk is the other plain one
    assert size == 2000.0 and source["type"] == "MOUNT" and "profile" not in source
    assert node_vol[0][3]["mount"]["root"] != source["mount"]["root"] and "profile" not in node_vol[0][3]
    old = sdk_tasks.get_service_tasks(config.SERVICE_NAME, "hello-0-node")[0]
    sdk_cmd.service_task_exec(config.SERVICE_NAME, "hello-0-node", "echo kept > mount-data/marker")
    assert sdk_cmd.kill_task_with_pattern("df mount-data", agent_host=old.host)
    sdk_tasks.check_task_relaunched("hello-0-node", old.id)
    sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
    relaunched = {i["info"]["name"]: i["info"] for i in _pod_info("hello-0")}
    assert [v[1] for v in _volumes(relaunched["hello-0-node"]) if v[0] == "mount-data"] == [pid]
    rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, "hello-0-node", "cat mount-data/marker")
    assert rc == 0 and out.strip() == "kept"


def _kill_one(pod, victim, survivor, pattern):
    _verify_shared_executor(pod)
    tasks = {t.name: t for t in sdk_tasks.get_service_tasks(config.SERVICE_NAME, pod)}
    assert set(tasks) == {f"{pod}-node", f"{pod}-agent"}
    assert sdk_cmd.kill_task_with_pattern(pattern, agent_host=tasks[f"{pod}-{victim}"].host)
    sdk_tasks.check_tasks_updated(config.SERVICE_NAME, f"{pod}-{victim}", [tasks[f"{pod}-{victim}"].id])
    sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
    sdk_tasks.check_tasks_not_updated(config.SERVICE_NAME, f"{pod}-{survivor}", [tasks[f"{pod}-{survivor}"].id])
    # the relaunch ran in the same executor, against the same pod volume
    _verify_shared_executor(pod)


def test_kill_node(pod_mount_service):
    """Kill the node task: only it is relaunched, in the pod's running executor."""
    _kill_one("hello-0", "node", "agent", "node-disk/written-by")


def test_kill_agent(pod_mount_service):
    """Kill the agent task: only it is relaunched, in the pod's running executor."""
    _kill_one("hello-0", "agent", "node", "agent-root/written-by")


def test_profile_mount_volume():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"yaml": "profile-mount-volume"}})
    try:
        sdk_tasks.check_running(config.SERVICE_NAME, 1)
        (path, _, size, source), = _volumes(_pod_info("hello-0")[0]["info"])
        assert path == "fast-data" and size == 1000.0
        assert source["profile"] == "fast-nvme" and source["mount"]["root"] == "/dcos/volume1"
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_testing_volumes_added_to_running_agents(local_cluster):
    """tools/create_testing_volumes.py: agents re-register with new /dcos/volume<N> disks and a
    profiled MOUNT volume deploys onto them without disturbing anything running."""
    from dcos_commons_amd.tools.create_testing_volumes import create_testing_volumes

    roots = create_testing_volumes(local_cluster, count=1, size_mb=300.0, profile="xfs")
    assert roots and all(r == "/dcos/volume3" for r in roots)   # after the module's three disks
    for aid in local_cluster.agent_ids.values():
        offered = [r for r in local_cluster.master.agent_resources(aid)
                   if r.HasField("disk") and r.disk.source.mount.root == "/dcos/volume3"]
        assert len(offered) == 1 and offered[0].disk.source.profile == "xfs" and offered[0].scalar.value == 300.0
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1, additional_options={
        "service": {"yaml": "profile-mount-volume"}})
    try:
        (path, _, size, source), = _volumes(_pod_info("hello-0")[0]["info"])
        # 500 MB asked, but only the 1 GB fast-nvme disks carry that profile: the xfs disks are ignored
        assert source["profile"] == "fast-nvme"
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
