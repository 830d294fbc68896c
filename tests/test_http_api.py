"""The /v1 HTTP API against a live, deployed scheduler.

Status codes and shapes follow the reference's query/endpoint suites
(sdk/scheduler/src/test/java/com/mesosphere/sdk/http/queries/PlansQueriesTest.java,
PodQueriesTest.java, ConfigQueriesTest.java, StateQueriesTest.java, EndpointsQueriesTest.java,
ArtifactQueriesTest.java, http/endpoints/HealthResourceTest.java, http/types/PlanInfoTest.java):
plan GET 200/202/404 (417 on errors), commands answer ``{"message": "Received cmd: <cmd>"}``, 208
when the command is a no-op, 404 for unknown plans/phases/steps, 400 for an invalid request.
"""
import json
import uuid

import pytest

from dcos_commons_amd.mesos import protos as P
from test_e2e_helloworld import Cluster


@pytest.fixture(scope="module")
def deployed():
    with Cluster() as c:
        c.wait_plan("deploy")
        yield c


def _cmd_ok(r, cmd):
    assert r.status == 200, (r.status, r.body)
    assert r.json()["message"].startswith(f"Received cmd: {cmd}")


# ---------------------------------------------------------------------------------------
# plans


def test_plan_list_and_plan_info_shape(deployed):
    api = deployed.api
    r = api.get("/v1/plans")
    assert r.status == 200 and sorted(r.json()) == ["deploy", "recovery"]
    r = api.get("/v1/plans/deploy")
    assert r.status == 200
    plan = r.json()
    assert set(plan) == {"phases", "errors", "strategy", "status"}
    assert plan["status"] == "COMPLETE" and plan["errors"] == [] and plan["strategy"] == "serial"
    phase = plan["phases"][0]
    assert set(phase) == {"id", "name", "steps", "strategy", "status"}
    uuid.UUID(phase["id"])
    step = phase["steps"][0]
    assert set(step) == {"id", "status", "name", "message"}
    assert step["name"] == "hello-0:[server]" and step["status"] == "COMPLETE"
    assert "hello-0:[server]" in step["message"]


def test_unknown_plan_is_404(deployed):
    api = deployed.api
    assert api.get("/v1/plans/nope").status == 404
    for cmd in ("continue", "interrupt", "stop", "forceComplete", "restart"):
        assert api.post(f"/v1/plans/nope/{cmd}").status == 404, cmd
    assert api.post("/v1/plans/nope/start", b"{}").status == 404


def test_commands_on_complete_plan_are_already_reported(deployed):
    api = deployed.api
    assert api.post("/v1/plans/deploy/continue").status == 208
    assert api.post("/v1/plans/deploy/interrupt").status == 208
    assert api.post("/v1/plans/deploy/continue?phase=hello").status == 208
    assert api.post("/v1/plans/deploy/forceComplete?phase=hello&step=hello-0:[server]").status == 208


def test_force_complete_argument_validation(deployed):
    api = deployed.api
    assert api.post("/v1/plans/deploy/forceComplete?step=hello-0:[server]").status == 400
    assert api.post("/v1/plans/deploy/forceComplete?phase=nope&step=nope").status == 404
    assert api.post(f"/v1/plans/deploy/forceComplete?phase={uuid.uuid4()}&step={uuid.uuid4()}").status == 404
    assert api.post("/v1/plans/deploy/restart?phase=nope&step=nope").status == 404
    assert api.post("/v1/plans/deploy/continue?phase=nope").status == 404
    assert api.post("/v1/plans/deploy/interrupt?phase=nope").status == 404


def test_start_rejects_invalid_env_names(deployed):
    r = deployed.api.post("/v1/plans/deploy/start", json.dumps({"not-valid-envname": "v"}).encode())
    assert r.status == 400


def test_phase_and_step_lookup_by_id_or_name(deployed):
    api = deployed.api
    plan = api.get("/v1/plans/deploy").json()
    phase = plan["phases"][1]
    step = phase["steps"][0]
    # restart of a step by id, then by name; each restart re-runs the step to COMPLETE
    _cmd_ok(api.post(f"/v1/plans/deploy/restart?phase={phase['id']}&step={step['id']}"), "restart")
    deployed.wait_plan("deploy")
    _cmd_ok(api.post(f"/v1/plans/deploy/restart?phase={phase['name']}&step={step['name']}"), "restart")
    deployed.wait_plan("deploy")


def test_deprecated_plan_aliases(deployed):
    api = deployed.api
    r = api.get("/v1/plan")
    assert r.status == 200 and r.json()["status"] == "COMPLETE"
    assert api.post("/v1/plan/continue").status == 208
    assert api.post("/v1/plan/interrupt").status == 208


def test_operator_plan_start_stop_cycle():
    with Cluster(spec_file="sidecar.yml") as c:
        c.wait_plan("deploy")
        api = c.api
        r = api.get("/v1/plans/sidecar")
        assert r.status == 202 and r.json()["status"] in ("WAITING", "PENDING")
        _cmd_ok(api.post("/v1/plans/sidecar/interrupt?phase=backup"), "interrupt")
        assert api.post("/v1/plans/sidecar/interrupt?phase=backup").status == 208
        _cmd_ok(api.post("/v1/plans/sidecar/continue?phase=backup"), "continue")
        r = api.post("/v1/plans/sidecar/start", json.dumps({"BACKUP_TAG": "t1"}).encode())
        assert r.status == 200
        c.wait(lambda: api.get("/v1/plans/sidecar").json()["status"] in ("IN_PROGRESS", "STARTING", "STARTED"))
        r = api.post("/v1/plans/sidecar/stop")
        assert r.status == 200
        plan = api.get("/v1/plans/sidecar").json()
        assert plan["status"] in ("WAITING", "PENDING")
        # forceComplete of a whole phase, then the plan
        _cmd_ok(api.post("/v1/plans/sidecar/forceComplete?phase=backup"), "forceComplete")
        phases = {p["name"]: p for p in api.get("/v1/plans/sidecar").json()["phases"]}
        assert phases["backup"]["status"] == "COMPLETE"
        _cmd_ok(api.post("/v1/plans/sidecar/forceComplete"), "forceComplete")
        assert api.get("/v1/plans/sidecar").status == 200


# ---------------------------------------------------------------------------------------
# pods


def test_pod_list_status_info(deployed):
    api = deployed.api
    assert sorted(api.get("/v1/pod").json()) == ["hello-0", "hello-1", "world-0", "world-1"]
    allst = api.get("/v1/pod/status").json()
    assert allst["service"] == "hello-world"
    by_type = {p["name"]: p for p in allst["pods"]}
    assert sorted(by_type) == ["hello", "world"]
    inst = by_type["hello"]["instances"][0]
    assert inst["name"] == "hello-0"
    task = inst["tasks"][0]
    assert task["name"] == "hello-0-server" and task["status"] == "RUNNING" and task["id"]
    st = api.get("/v1/pod/hello-0/status").json()
    assert st["name"] == "hello-0" and st["tasks"][0]["status"] == "RUNNING"
    info = api.get("/v1/pod/hello-0/info").json()
    assert info[0]["info"]["name"] == "hello-0-server"
    assert info[0]["status"]["state"] == "TASK_RUNNING"


def test_pod_unknown_is_404(deployed):
    api = deployed.api
    assert api.get("/v1/pod/nope-0/status").status == 404
    assert api.get("/v1/pod/nope-0/info").status == 404
    for cmd in ("restart", "replace", "pause", "resume"):
        assert api.post(f"/v1/pod/nope-0/{cmd}").status == 404, cmd


def test_pod_pause_and_resume():
    with Cluster() as c:
        c.wait_plan("deploy")
        api = c.api
        r = api.post("/v1/pod/hello-1/pause")
        assert r.status == 200 and r.json() == {"pod": "hello-1", "tasks": ["hello-1-server"]}
        status = lambda: api.get("/v1/pod/hello-1/status").json()["tasks"][0]["status"]  # noqa: E731
        # PAUSING while the override is in progress, PAUSED once the paused task runs
        c.wait(lambda: status() == "PAUSED", what="PAUSED")
        # pausing again re-applies the override (no conflict, as in PodQueries.overrideGoalState)
        assert api.post("/v1/pod/hello-1/pause").status == 200
        c.wait(lambda: status() == "PAUSED", what="PAUSED again")
        # a paused task runs the pause command instead of its own
        cmd = c.store.fetch_task("hello-1-server").command.value
        assert "PAUSED" in cmd and "hello-data" not in cmd
        r = api.post("/v1/pod/hello-1/resume")
        assert r.status == 200
        c.wait(lambda: status() == "RUNNING" and "hello-data" in c.store.fetch_task("hello-1-server").command.value,
               what="resumed")
        assert api.post("/v1/pod/hello-1/resume").status == 200


def test_pod_restart_keeps_reservations_replace_does_not():
    with Cluster(agents=4) as c:
        c.wait_plan("deploy")
        api = c.api
        old = c.store.fetch_task("hello-0-server")
        r = api.post("/v1/pod/hello-0/restart")
        assert r.status == 200 and r.json() == {"pod": "hello-0", "tasks": ["hello-0-server"]}
        c.wait(lambda: c.store.fetch_task("hello-0-server").task_id.value != old.task_id.value
               and c.store.fetch_status("hello-0-server").state == P.TASK_RUNNING)
        new = c.store.fetch_task("hello-0-server")
        assert new.agent_id.value == old.agent_id.value
        rid = lambda t: sorted(l.value for r in t.resources for l in r.reservations[-1].labels.labels  # noqa: E731
                               if l.key == "resource_id")
        assert rid(new) == rid(old)


# ---------------------------------------------------------------------------------------
# configurations, state, endpoints, health, artifacts


def test_configurations(deployed):
    api = deployed.api
    ids = api.get("/v1/configurations").json()
    assert len(ids) == 1
    targets = api.get("/v1/configurations/targetId").json()   # an array, like the id list
    assert targets == ids
    target = targets[0]
    t = api.get("/v1/configurations/target").json()
    assert t["name"] == "hello-world" and [p["type"] for p in t["pod-specs"]] == ["hello", "world"]
    assert api.get(f"/v1/configurations/{target}").json() == t
    assert api.get(f"/v1/configurations/{uuid.uuid4()}").status == 404
    assert api.get("/v1/configurations/not-a-uuid").status == 400


def test_state_views(deployed):
    api = deployed.api
    fid = api.get("/v1/state/frameworkId").json()
    assert isinstance(fid, list) and len(fid) == 1 and fid[0]
    props = api.get("/v1/state/properties").json()
    assert "last-completed-update-type" in props or "deployment-completed" in json.dumps(props) or props
    assert api.get("/v1/state/properties/nope").status == 404
    # agents without a fault domain: no task has a zone
    assert api.get("/v1/state/zone/tasks").json() == {}
    assert api.get("/v1/state/zone/tasks/hello-0-server").status == 404
    assert api.get("/v1/state/zone/tasks/nope").status == 404
    assert api.put("/v1/state/refresh").status in (200, 409)


def test_state_files_round_trip(deployed):
    api = deployed.api
    body = b"hello file contents"
    boundary = "XyZ"
    mp = (f"--{boundary}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"f.txt\"\r\n"
          f"Content-Type: text/plain\r\n\r\n").encode() + body + f"\r\n--{boundary}--\r\n".encode()
    r = api.put("/v1/state/files/f.txt", mp, headers={"Content-Type": f"multipart/form-data; boundary={boundary}"})
    assert r.status == 200, r.body
    assert api.get("/v1/state/files").body == "[f.txt]"       # Java List.toString, text/plain
    got = api.get("/v1/state/files/f.txt").body
    assert (got.encode() if isinstance(got, str) else got) == body
    assert api.get("/v1/state/files/missing").status == 404


def test_endpoints(deployed):
    api = deployed.api
    r = api.get("/v1/endpoints")
    assert r.status == 200 and isinstance(r.json(), list)
    assert api.get("/v1/endpoints/nope").status == 404


def test_health(deployed):
    r = deployed.api.get("/v1/health")
    assert r.status == 200
    v = deployed.api.get("/v1/health?verbose=true")
    assert v.status == 200


def test_artifact_template_validation(deployed):
    api = deployed.api
    cid = api.get("/v1/configurations/targetId").json()[0]
    assert api.get(f"/v1/artifacts/template/not-a-uuid/hello/server/cfg").status == 400
    assert api.get(f"/v1/artifacts/template/{uuid.uuid4()}/hello/server/cfg").status == 404
    assert api.get(f"/v1/artifacts/template/{cid}/nope/server/cfg").status == 404
    assert api.get(f"/v1/artifacts/template/{cid}/hello/nope/cfg").status == 404
    assert api.get(f"/v1/artifacts/template/{cid}/hello/server/nope").status == 404


# ---------------------------------------------------------------------------------------
# debug and metrics


def test_debug_endpoints(deployed):
    api = deployed.api
    offers = api.get("/v1/debug/offers")
    assert offers.status == 200
    v2 = api.get("/v2/debug/offers").json()
    assert isinstance(v2, dict)
    plans = api.get("/v1/debug/plans").json()
    assert "deploy" in json.dumps(plans)
    statuses = api.get("/v1/debug/taskStatuses").json()
    assert "hello-0-server" in json.dumps(statuses)
    res = api.get("/v1/debug/reservations").json()
    hosts = {"host-0", "host-1", "host-2"}
    assert set(res) <= hosts and all(len(ids) >= 4 for ids in res.values())
    threads = api.get("/v1/debug/threads")
    assert threads.status == 200 and threads.body


def test_metrics(deployed):
    api = deployed.api
    m = api.get("/v1/metrics").json()
    assert "counters" in m and "timers" in m and "gauges" in m
    assert any(k.startswith("operation.") for k in m["counters"])
    assert any(k.startswith("task_status.") for k in m["counters"])
    prom = api.get("/v1/metrics/prometheus")
    text = prom.body if isinstance(prom.body, str) else prom.body.decode()
    assert prom.status == 200 and "offers" in text
