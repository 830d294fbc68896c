"""helloworld placement and region scenarios on the local cluster.

Reference: frameworks/helloworld/tests/{test_placement.py, test_region_awareness.py}. The
placement suite runs on agents that all report one zone (as the reference's CI cluster does):
``@zone`` UNIQUE / MAX_PER / GROUP_BY constraints then deploy hello and world-0 and leave world-1
waiting for an offer that can never match, hostname UNIQUE / MAX_PER / GROUP_BY spread pods evenly
over the agents, CLUSTER pins every pod to one agent, a constraint on a missing attribute deploys
nothing, Marathon places the scheduler itself by its app constraints, and every task sees its
zone and region. The region suite adds agents of a second region: pods stay in the master's
(local) region by default, go to a configured remote region, and a region change of a deployed
service is refused until it is reverted.
"""
import pytest

from dcos_commons_amd.mesos.local_master import AgentSpec
from dcos_commons_amd.testing.cluster.cluster import DCOS_AGENT_PORTS, LocalCluster, use
from dcos_commons_amd.testing.sdk import sdk_agents, sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks
from tests.integration import hw_config as config

LOCAL_REGION, REMOTE_REGION = "us-west-2", "us-east-1"
N_AGENTS = 5


@pytest.fixture(scope="module")
def local_cluster():
    # 5 agents of the local region, all in one zone, plus 3 agents of a remote region
    specs = [AgentSpec(hostname=f"10.0.0.{i + 1}", ports=DCOS_AGENT_PORTS, region=LOCAL_REGION,
                       zone="us-west-2a", attributes={"rack_id": f"rack-{i % 2}"}) for i in range(N_AGENTS)]
    specs += [AgentSpec(hostname=f"10.1.0.{i + 1}", ports=DCOS_AGENT_PORTS, region=REMOTE_REGION,
                        zone="us-east-1a") for i in range(3)]
    c = LocalCluster(agent_specs=specs, region=LOCAL_REGION, zones=("us-west-2a",),
                     scheduler_env={"SDK_LOCK_WAIT_S": "1"}).start()
    use(c)
    yield c
    c.shutdown()


pytestmark = pytest.mark.usefixtures("local_cluster")


def _local_agents():
    return [a["hostname"] for a in sdk_agents.get_private_agents() if a["hostname"].startswith("10.0.")]


def _agent_sets():
    hello, world = [], []
    for t in sdk_tasks.get_service_tasks(config.SERVICE_NAME):
        (hello if t.name.startswith("hello-") else world).append(t.host)
    return hello, world


def _ensure_count_per_agent(hello_count, world_count):
    hello, world = _agent_sets()
    assert len(hello) == len(set(hello)) * hello_count, hello
    assert len(world) == len(set(world)) * world_count, world


def _succeed_placement(options):
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 3, additional_options=options)
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def _fail_placement(options):
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 0, additional_options=options,
                        wait_for_deployment=False)
    try:
        sdk_plan.wait_for_step_status(config.SERVICE_NAME, "deploy", "world", "world-0:[server]", "COMPLETE")
        pl = sdk_plan.get_deployment_plan(config.SERVICE_NAME)
        # everything else is stuck looking for a match
        assert pl["status"] == "IN_PROGRESS" and len(pl["phases"]) == 2
        hello, world = pl["phases"]
        assert hello["status"] == "COMPLETE" and len(hello["steps"]) == 1
        assert world["status"] == "IN_PROGRESS" and len(world["steps"]) == 2
        assert world["steps"][0]["status"] == "COMPLETE"
        assert world["steps"][1]["status"] in ("PREPARED", "PENDING")
        with pytest.raises(AssertionError):
            sdk_tasks.check_running(config.SERVICE_NAME, 3, timeout_seconds=3)
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def _zone_options(hello, world):
    return {"hello": {"placement": f'[["@zone", {hello}]]'}, "world": {"placement": f'[["@zone", {world}]]'}}


def test_scheduler_task_placement_by_marathon():
    agent = _local_agents()[2]
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 3,
                        additional_options={"service": {"constraints": [["hostname", "LIKE", agent]]}})
    try:
        summary = sdk_tasks.get_service_tasks("marathon", config.SERVICE_NAME)
        assert len(summary) == 1, summary
        assert summary[0].host == agent, "Scheduler task constraint placement failed by marathon"
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_region_zone_injection():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 3)
    try:
        for pod in ("hello-0", "world-0", "world-1"):
            info = sdk_cmd.service_request("GET", config.SERVICE_NAME, f"/v1/pod/{pod}/info").json()[0]["info"]
            env = {v["name"]: v.get("value") for v in info["command"]["environment"]["variables"]}
            assert env["ZONE"] == "us-west-2a" and env["REGION"] == LOCAL_REGION, env
            rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, f"{pod}-server", "echo $ZONE/$REGION")
            assert rc == 0 and out.strip() == f"us-west-2a/{LOCAL_REGION}"
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_rack_not_found():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 0, wait_for_deployment=False,
                        additional_options={"hello": {"placement": '[["rack_id", "LIKE", "rack-foo-.*"]]'},
                                            "world": {"placement": '[["rack_id", "LIKE", "rack-foo-.*"]]'}})
    try:
        with pytest.raises(AssertionError):
            sdk_tasks.check_running(config.SERVICE_NAME, 1, timeout_seconds=3)
        pl = sdk_plan.wait_for_plan_status(config.SERVICE_NAME, "deploy", "IN_PROGRESS")
        assert len(pl["phases"]) == 2
        hello, world = pl["phases"]
        assert hello["status"] == "IN_PROGRESS" and len(hello["steps"]) == 1
        assert hello["steps"][0]["status"] in ("PREPARED", "PENDING")
        assert world["status"] == "PENDING" and [s["status"] for s in world["steps"]] == ["PENDING", "PENDING"]
        # the offer outcomes name the failing rule
        offers = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v2/debug/offers").json()
        assert "rack_id" in str(offers) or "Placement" in str(offers) or "placement" in str(offers)
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_rack_found():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 3,
                        additional_options={"hello": {"placement": '[["rack_id", "LIKE", "rack-1"]]'},
                                            "world": {"placement": '[["rack_id", "LIKE", "rack-0"]]'}})
    try:
        racks = {a["hostname"]: a["attributes"].get("rack_id") for a in sdk_agents.get_agents()}
        for t in sdk_tasks.get_service_tasks(config.SERVICE_NAME):
            assert racks[t.host] == ("rack-1" if t.name.startswith("hello") else "rack-0"), (t, racks)
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_unique_zone_fails():
    _fail_placement(_zone_options('"UNIQUE"', '"UNIQUE"'))


def test_max_per_zone_fails():
    _fail_placement(_zone_options('"MAX_PER", "1"', '"MAX_PER", "1"'))


def test_max_per_zone_succeeds():
    _succeed_placement(_zone_options('"MAX_PER", "1"', '"MAX_PER", "2"'))


def test_group_by_zone_succeeds():
    _succeed_placement(_zone_options('"GROUP_BY", "1"', '"GROUP_BY", "1"'))


def test_group_by_zone_fails():
    _fail_placement(_zone_options('"GROUP_BY", "1"', '"GROUP_BY", "2"'))


def test_hostname_unique():
    n = N_AGENTS
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 2 * n, additional_options={
        "hello": {"count": n, "placement": '[["hostname", "UNIQUE"], ["@region", "IS", "us-west-2"]]'},
        "world": {"count": n, "placement": '[["hostname", "UNIQUE"], ["@region", "IS", "us-west-2"]]'}})
    try:
        _ensure_count_per_agent(hello_count=1, world_count=1)
        hello, world = _agent_sets()
        assert set(hello) == set(world) == set(_local_agents())
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_max_per_hostname():
    n = N_AGENTS
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 5 * n, additional_options={
        "hello": {"count": 2 * n, "placement": '[["hostname", "MAX_PER", "2"], ["@region", "IS", "us-west-2"]]'},
        "world": {"count": 3 * n, "placement": '[["hostname", "MAX_PER", "3"], ["@region", "IS", "us-west-2"]]'}})
    try:
        _ensure_count_per_agent(hello_count=2, world_count=3)
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_rr_by_hostname():
    n = N_AGENTS
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 4 * n, additional_options={
        "hello": {"count": 2 * n, "placement": f'[["hostname", "GROUP_BY", "{n}"], ["@region", "IS", "us-west-2"]]'},
        "world": {"count": 2 * n, "placement": f'[["hostname", "GROUP_BY", "{n}"], ["@region", "IS", "us-west-2"]]'}})
    try:
        _ensure_count_per_agent(hello_count=2, world_count=2)
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_cluster():
    agent = _local_agents()[-1]
    n = N_AGENTS
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, n, additional_options={
        "hello": {"count": n, "placement": f'[["hostname", "CLUSTER", "{agent}"]]'}, "world": {"count": 0}})
    try:
        _ensure_count_per_agent(hello_count=n, world_count=0)
        assert {t.host for t in sdk_tasks.get_service_tasks(config.SERVICE_NAME)} == {agent}
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


# -- region awareness ----------------------------------------------------------------------------
def _pod_region(pod):
    info = sdk_cmd.service_request("GET", config.SERVICE_NAME, f"/v1/pod/{pod}/info").json()[0]["info"]
    return next(l["value"] for l in info["labels"]["labels"] if l["key"] == "offer_region")


def _region_service(region=None):
    svc = {"scenario": "MULTI_REGION", "allow_region_awareness": True}
    if region:
        svc["region"] = region
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 3, additional_options={"service": svc})


def _change_region_config(region):
    cfg = sdk_marathon.get_config(config.SERVICE_NAME)
    if region is None:
        cfg["env"].pop("SERVICE_REGION", None)
    else:
        cfg["env"]["SERVICE_REGION"] = region
    sdk_marathon.update_app(cfg, wait_for_completed_deployment=False)


def test_nodes_deploy_to_local_region_by_default():
    _region_service()
    try:
        local = sdk_cmd.cluster_request("GET", "/mesos/state").json()["domain"]["fault_domain"]["region"]["name"]
        assert local == LOCAL_REGION
        for pod in ("hello-0", "world-0", "world-1"):
            assert _pod_region(pod) == local
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_nodes_can_deploy_to_remote_region():
    _region_service(REMOTE_REGION)
    try:
        for pod in ("hello-0", "world-0", "world-1"):
            assert _pod_region(pod) == REMOTE_REGION
        assert {t.host for t in sdk_tasks.get_service_tasks(config.SERVICE_NAME)} <= \
            {f"10.1.0.{i + 1}" for i in range(3)}
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_region_config_update_does_not_succeed():
    _region_service()
    try:
        _change_region_config(REMOTE_REGION)
        sdk_plan.wait_for_plan_status(config.SERVICE_NAME, "deploy", "ERROR", timeout_seconds=60)
        _change_region_config(None)
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME, timeout_seconds=60)
        for pod in ("hello-0", "world-0", "world-1"):
            assert _pod_region(pod) == LOCAL_REGION
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


# -- a changed placement constraint (reference test_placement.py:399-470) ----------------------
def _task_host(task_name):
    """The agent a task runs on, from its TaskInfo's offer_hostname label, checked against the
    task summary (reference ``get_task_host``)."""
    info = sdk_cmd.service_request("GET", config.SERVICE_NAME, f"/v1/pod/{task_name.rsplit('-', 1)[0]}/info").json()
    task = next(i["info"] for i in info if i["info"]["name"] == task_name)
    host = next(lb["value"] for lb in task["labels"]["labels"] if lb["key"] == "offer_hostname")
    summary = [t for t in sdk_tasks.get_service_tasks(config.SERVICE_NAME) if t.name == task_name]
    assert len(summary) == 1 and summary[0].host == host, (host, summary)
    return host


def _setup_constraint_switch():
    """hello-0 pinned to one agent, then the service's placement switched to another agent."""
    some_agent, other_agent = _local_agents()[:2]
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1, additional_options={
        "service": {"yaml": "marathon_constraint"},
        "hello": {"count": 1, "placement": f'[["hostname", "LIKE", "{some_agent}"]]'},
        "world": {"count": 0}})
    old_ids = sdk_tasks.get_task_ids(config.SERVICE_NAME, "hello")
    app = sdk_marathon.get_config(config.SERVICE_NAME)
    app["env"]["HELLO_PLACEMENT"] = f'[["hostname", "LIKE", "{other_agent}"]]'
    sdk_marathon.update_app(app)
    sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
    return some_agent, other_agent, old_ids


def test_updated_placement_constraints_no_task_change():
    """A placement change alone is not a task change: nothing relaunches or moves."""
    some_agent, _, old_ids = _setup_constraint_switch()
    try:
        sdk_tasks.check_tasks_not_updated(config.SERVICE_NAME, "hello", old_ids)
        assert _task_host("hello-0-server") == some_agent
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_updated_placement_constraints_not_applied_with_other_changes():
    """A new pod follows the new constraint; the running one stays where it is."""
    some_agent, other_agent, _ = _setup_constraint_switch()
    try:
        app = sdk_marathon.get_config(config.SERVICE_NAME)
        app["env"]["HELLO_COUNT"] = "2"
        sdk_marathon.update_app(app)
        sdk_tasks.check_running(config.SERVICE_NAME, 2)
        sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        assert _task_host("hello-0-server") == some_agent
        assert _task_host("hello-1-server") == other_agent
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_updated_placement_constraints_restarted_tasks_dont_move():
    """A restart relaunches in place, on the pod's reservations, whatever the constraint says."""
    some_agent, _, old_ids = _setup_constraint_switch()
    try:
        sdk_cmd.svc_cli(config.PACKAGE_NAME, config.SERVICE_NAME, "pod restart hello-0")
        sdk_tasks.check_tasks_updated(config.SERVICE_NAME, "hello", old_ids)
        sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
        assert _task_host("hello-0-server") == some_agent
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_updated_placement_constraints_replaced_tasks_do_move():
    """A replace is a new footprint: it is placed by the new constraint."""
    _, other_agent, old_ids = _setup_constraint_switch()
    try:
        sdk_cmd.svc_cli(config.PACKAGE_NAME, config.SERVICE_NAME, "pod replace hello-0")
        sdk_tasks.check_tasks_updated(config.SERVICE_NAME, "hello", old_ids)
        sdk_plan.wait_for_completed_recovery(config.SERVICE_NAME)
        assert _task_host("hello-0-server") == other_agent
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
