"""More OfferEvaluator scenarios: overlay ports, port env vars in checks, dynamic port ranges,
named VIPs, port changes on update, multiple and profiled volumes, executor volumes, and the
recovery target-config choice.

Mirrors the rest of the reference's evaluate suites (sdk/scheduler/src/test/java/com/mesosphere/
sdk/offer/evaluate/{PortEvaluationStageTest,OfferEvaluatorPortsTest,OfferEvaluatorVolumesTest,
OfferEvaluatorTest}.java). Fixtures are shared with ``test_offer_evaluator``.
"""
import uuid

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import resources as RU
from dcos_commons_amd.offer.recommendations import (CreateOfferRecommendation, LaunchOfferRecommendation,
                                                    ReserveOfferRecommendation, UnreserveOfferRecommendation)
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader, TaskLabelWriter, env_to_map
from dcos_commons_amd.scheduler.recovery import RecoveryType
from test_offer_evaluator import (C, L, R, U, Fixture, _executor_reserved, _reserved, _respec, complete_offer,
                                  executor_room, mount_disk, of, offer, ops, ranges, scalar, server, task_resource)


def _task_info(recs):
    return of(recs, LaunchOfferRecommendation)[0].task_info


def _env(recs):
    return env_to_map(_task_info(recs).command.environment)


def _discovery_ports(recs):
    return {p.name: p.number for p in _task_info(recs).discovery.ports.ports}


# ---------------------------------------------------------------------------------------
# overlay networks: ports are not resources there


OVERLAY = "networks:\n  dcos: {}\n"


def test_overlay_port_is_not_reserved_but_advertised_and_exported():
    f = Fixture(server(1.0, 32, extra="ports:\n  overlay-port-name:\n    port: 80\n    env-key: PORT_TEST_IGNORED\n"),
                pod_extra=OVERLAY)
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10000)))])
    assert recs
    assert not any(r.name == "ports" for r in _task_info(recs).resources)
    assert _discovery_ports(recs) == {"overlay-port-name": 80}
    assert _env(recs)["PORT_TEST_IGNORED"] == "80"
    assert not any(rec.get_operation() is not None and rec.get_operation().type == R and
                   rec.get_operation().reserve.resources[0].name == "ports" for rec in recs)


def test_overlay_dynamic_ports_come_from_the_overlay_range_and_skip_explicit_ones():
    ports = ("ports:\n  explicit-port:\n    port: 1025\n    env-key: PORT_TEST_EXPLICIT\n"
             "  dynamic-port:\n    port: 0\n    env-key: PORT_TEST_DYNAMIC\n")
    f = Fixture(server(1.0, 32, extra=ports), pod_extra=OVERLAY)
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10000)))])
    assert _discovery_ports(recs) == {"explicit-port": 1025, "dynamic-port": 1026}
    env = _env(recs)
    assert env["PORT_TEST_EXPLICIT"] == "1025" and env["PORT_TEST_DYNAMIC"] == "1026"
    assert not any(r.name == "ports" for r in _task_info(recs).resources)


def test_single_dynamic_overlay_port_is_the_first_of_the_range():
    f = Fixture(server(1.0, 32, extra="ports:\n  dyn-port-name:\n    port: 0\n    env-key: PORT_TEST_DYNAMIC_OVERLAY\n"),
                pod_extra=OVERLAY)
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    assert _discovery_ports(recs) == {"dyn-port-name": 1025}
    assert _env(recs)["PORT_TEST_DYNAMIC_OVERLAY"] == "1025"


# ---------------------------------------------------------------------------------------
# port env vars inside health and readiness checks


CHECKS = """\
ports:
  test-port:
    port: 0
    env-key: PORT_TEST
health-check:
  cmd: ./health $PORT_TEST
  interval: 5
  grace-period: 30
  max-consecutive-failures: 3
  delay: 0
  timeout: 10
readiness-check:
  cmd: ./ready $PORT_TEST
  interval: 5
  delay: 0
  timeout: 10
"""


@pytest.mark.parametrize("pod_extra", ["", OVERLAY])
def test_port_env_var_reaches_health_and_readiness_checks(pod_extra):
    f = Fixture(server(1.0, 32, extra=CHECKS), pod_extra=pod_extra)
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10100)))])
    ti = _task_info(recs)
    port = _env(recs)["PORT_TEST"]
    if pod_extra:
        assert port == "1025"
    else:
        assert 10000 <= int(port) <= 10100
    assert env_to_map(ti.health_check.command.environment)["PORT_TEST"] == port
    # the readiness check is the default executor's CheckInfo on the task
    assert ti.HasField("check")
    assert env_to_map(ti.check.command.command.environment)["PORT_TEST"] == port


# ---------------------------------------------------------------------------------------
# dynamic ports: allowed ranges, pre-reserved roles, stickiness


PR = "slave_public"


def _dyn(ranges_yaml):
    return server(1.0, 32, extra=f"ports:\n  TEST:\n    port: 0\n    env-key: PORT_TEST\n    ranges:\n{ranges_yaml}")


def _prereserved_offer(lo, hi):
    return offer(scalar("cpus", 2.0, PR), scalar("mem", 64, PR), *executor_room(PR),
                 _reserved_ports(lo, hi))


def _reserved_ports(lo, hi):
    r = ranges("ports", (lo, hi), role=PR)
    res = r.reservations.add()
    res.type = P.Resource.ReservationInfo.STATIC
    res.role = PR
    return r


@pytest.mark.parametrize("ranges_yaml,offered,expected", [
    ("      - begin: 25\n        end: 600\n", (23, 5050), 25),
    ("      - begin: 6000\n        end: 8000\n", (23, 5050), None),
    ("      - begin: 6000\n        end: 8000\n      - begin: 2\n        end: 21\n", (23, 5050), None),
    ("      - begin: 1024\n", (3000, 5050), 3000),                   # unbounded above
    ("      - end: 23\n", (23, 5050), 23),                            # inclusive upper bound
    ("      - begin: 5050\n        end: 6000\n", (23, 5050), 5050),   # inclusive lower bound
])
def test_dynamic_port_allowed_ranges_on_pre_reserved_ports(ranges_yaml, offered, expected):
    f = Fixture(_dyn(ranges_yaml), pod_extra=f"pre-reserved-role: {PR}\n")
    recs = f.evaluate([_prereserved_offer(*offered)])
    if expected is None:
        assert recs == []
    else:
        assert int(_env(recs)["PORT_TEST"]) == expected
        port = task_resource(recs, "ports")
        assert port.reservations[0].role == PR  # refined from the pre-reservation


def test_dynamic_port_needs_the_pre_reserved_role():
    f = Fixture(server(1.0, 32, extra="ports:\n  TEST:\n    port: 0\n"), pod_extra=f"pre-reserved-role: {PR}\n")
    # only unreserved ports in the offer: the pre-reserved pod cannot take them
    recs = f.evaluate([offer(scalar("cpus", 2.0, PR), scalar("mem", 64, PR), *executor_room(PR),
                             ranges("ports", (10000, 10010)))])
    assert recs == []
    recs = f.evaluate([_prereserved_offer(10000, 10010)])
    assert recs and 10000 <= int(task_resource(recs, "ports").ranges.range[0].begin) <= 10010


def test_dynamic_port_is_not_sticky_after_replacement():
    f = Fixture(server(1.0, 32, extra="ports:\n  dyn:\n    port: 0\n    env-key: MY_PORT\n"))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10000)))])
    assert _env(first)["MY_PORT"] == "10000"
    info = f.task()
    TaskLabelWriter(info).set_permanently_failed().apply()
    f.state_store.store_tasks([info])
    # the new agent offers a different port range: a permanent replacement picks from it
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (20000, 20000)),
                                      agent="agent2", host="host2")], recovery=RecoveryType.PERMANENT)
    assert recs and _env(recs)["MY_PORT"] == "20000"


def test_multiple_dynamic_ports_get_distinct_values():
    f = Fixture(server(1.0, 32, extra="ports:\n  a:\n    port: 0\n    env-key: A\n  b:\n    port: 0\n    env-key: B\n"))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10001)))])
    env = _env(recs)
    assert {env["A"], env["B"]} == {"10000", "10001"}
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10000)))]) == []


# ---------------------------------------------------------------------------------------
# named VIPs


def test_named_vip_port_is_reserved_and_labelled():
    f = Fixture(server(1.0, 32, extra="ports:\n  http:\n    port: 8080\n    vip:\n      prefix: web\n      port: 80\n"))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (8000, 9000)))])
    port = task_resource(recs, "ports")
    assert [(r.begin, r.end) for r in port.ranges.range] == [(8080, 8080)]
    (dp,) = _task_info(recs).discovery.ports.ports
    assert dp.name == "http" and dp.number == 8080
    vips = [lab.value for lab in dp.labels.labels if lab.key.startswith("VIP_")]
    assert vips == ["web:80"]
    assert dp.visibility == P.DiscoveryInfo.CLUSTER  # VIP ports default to cluster visibility


def test_dynamic_vip_port_is_labelled_with_the_vip_port():
    f = Fixture(server(1.0, 32, extra="ports:\n  http:\n    port: 0\n    vip:\n      prefix: web\n      port: 80\n"))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10000)))])
    (dp,) = _task_info(recs).discovery.ports.ports
    assert dp.number == 10000
    assert [lab.value for lab in dp.labels.labels if lab.key.startswith("VIP_")] == ["web:80"]


# ---------------------------------------------------------------------------------------
# port changes on a configuration update


def _ports_after(first, *extra):
    return offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem"),
                                                 _reserved(first, "ports")] + list(extra)))


def test_static_port_change_unreserves_the_old_and_reserves_the_new():
    f = Fixture(server(1.0, 32, extra="ports:\n  http:\n    port: 8080\n"))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (8080, 8081)))])
    g = _respec(f, server(1.0, 32, extra="ports:\n  http:\n    port: 8081\n"))
    recs = g.evaluate([_ports_after(first, ranges("ports", (8081, 8081)))])
    assert recs
    unres = [r for r in of(recs, UnreserveOfferRecommendation)
             if r.get_operation().unreserve.resources[0].name == "ports"]
    res = [r for r in of(recs, ReserveOfferRecommendation) if r.get_operation().reserve.resources[0].name == "ports"]
    assert [(x.begin, x.end) for x in unres[0].get_operation().unreserve.resources[0].ranges.range] == [(8080, 8080)]
    assert [(x.begin, x.end) for x in res[0].get_operation().reserve.resources[0].ranges.range] == [(8081, 8081)]
    assert _discovery_ports(recs) == {"http": 8081}


def test_dynamic_to_static_port_change():
    f = Fixture(server(1.0, 32, extra="ports:\n  http:\n    port: 0\n"))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10000)))])
    g = _respec(f, server(1.0, 32, extra="ports:\n  http:\n    port: 8080\n"))
    recs = g.evaluate([_ports_after(first, ranges("ports", (8080, 8080)))])
    assert recs and _discovery_ports(recs) == {"http": 8080}
    assert L in ops(recs) and U in ops(recs) and R in ops(recs)


def test_relaunch_on_expected_multiple_ports_only_launches():
    f = Fixture(server(1.0, 32, extra="ports:\n  a:\n    port: 8080\n  b:\n    port: 0\n"))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (8080, 8090)))])
    launch = of(first, LaunchOfferRecommendation)[0]
    port_resources = [r for r in launch.task_info.resources if r.name == "ports"]
    again = f.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem")]
                                + port_resources))])
    assert ops(again) == [L, None]
    assert _discovery_ports(again) == _discovery_ports(first)


# ---------------------------------------------------------------------------------------
# volumes


def test_multiple_root_volumes_each_get_created():
    vols = ("volumes:\n  data:\n    path: data\n    type: ROOT\n    size: 100\n"
            "  logs:\n    path: logs\n    type: ROOT\n    size: 200\n")
    f = Fixture(server(1.0, 32, extra=vols))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 1000))])
    created = sorted((v.disk.volume.container_path, v.scalar.value) for rec in of(recs, CreateOfferRecommendation)
                     for v in rec.get_operation().create.volumes)
    assert created == [("data", 100.0), ("logs", 200.0)]
    pids = {r.disk.persistence.id for r in _task_info(recs).resources if r.name == "disk"}
    assert len(pids) == 2 and "" not in pids
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 250))]) == []


def _profiled(size, profile, root):
    d = mount_disk(size, root)
    d.disk.source.profile = profile
    return d


def test_mount_volumes_pick_disks_by_profile():
    vols = ("volumes:\n  fast:\n    path: fast\n    type: MOUNT\n    size: 100\n    profiles: [ssd]\n"
            "  slow:\n    path: slow\n    type: MOUNT\n    size: 100\n    profiles: [hdd]\n")
    f = Fixture(server(1.0, 32, extra=vols))
    disks = [_profiled(500, "hdd", "/mnt/hdd0"), _profiled(500, "ssd", "/mnt/ssd0")]
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), *disks)])
    by_path = {v.disk.volume.container_path: (v.disk.source.profile, v.disk.source.mount.root)
               for rec in of(recs, CreateOfferRecommendation) for v in rec.get_operation().create.volumes}
    assert by_path == {"fast": ("ssd", "/mnt/ssd0"), "slow": ("hdd", "/mnt/hdd0")}
    # no disk with a matching profile -> no match
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), _profiled(500, "hdd", "/a"),
                                      _profiled(500, "hdd", "/b"))]) == []


def test_two_mount_volumes_need_two_disks():
    vols = ("volumes:\n  a:\n    path: a\n    type: MOUNT\n    size: 100\n"
            "  b:\n    path: b\n    type: MOUNT\n    size: 100\n")
    f = Fixture(server(1.0, 32, extra=vols))
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), mount_disk(1000))]) == []
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), mount_disk(1000, "/mnt/d0"),
                                      mount_disk(1000, "/mnt/d1"))])


def test_root_volume_cannot_come_from_another_resource():
    f = Fixture(server(1.0, 32, extra="volume:\n  path: data\n  type: ROOT\n  size: 500\n"))
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 1000))]) == []  # no disk at all


POD_VOLUME = "volume:\n  path: shared\n  type: ROOT\n  size: 100\n"


def test_pod_volume_lives_on_the_executor():
    f = Fixture(server(1.0, 32), pod_extra=POD_VOLUME)
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 500))])
    launch = of(recs, LaunchOfferRecommendation)[0]
    exec_vols = [r for r in launch.executor_info.resources if r.name == "disk" and r.disk.persistence.id]
    assert len(exec_vols) == 1 and exec_vols[0].disk.volume.container_path == "shared"
    assert not any(r.disk.persistence.id for r in launch.task_info.resources if r.name == "disk")
    assert C in ops(recs)


def test_relaunch_without_the_executor_volume_fails():
    f = Fixture(server(1.0, 32), pod_extra=POD_VOLUME)
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 500))])
    exec_res = [r for r in _executor_reserved(first) if not r.disk.persistence.id]
    recs = f.evaluate([offer(*(exec_res + [_reserved(first, "cpus"), _reserved(first, "mem")]))])
    assert recs == []
    assert ops(f.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"),
                                                                 _reserved(first, "mem")]))])) == [L, None]


# ---------------------------------------------------------------------------------------
# recovery: which configuration a relaunch uses (OfferEvaluator.getTargetConfig)


TWO = server(1.0, 32) + "init:\n  goal: ONCE\n  cmd: ./init\n  cpus: 0.1\n  memory: 32\n"


def _stored(f, name, config, running=True):
    t = P.TaskInfo(name=name)
    t.task_id.value = f"test-service__{name}__{uuid.uuid4()}"
    t.agent_id.value = "agent1"
    w = TaskLabelWriter(t)
    w.set_type("pod-type")
    w.set_index(0)
    if config is not None:
        w.set_target_configuration(config)
    w.apply()
    f.state_store.store_tasks([t])
    st = P.TaskStatus(task_id=t.task_id, state=P.TASK_RUNNING if running else P.TASK_FAILED)
    f.state_store.store_status(name, st)
    return t


def _this_pod(f):
    return {t.name: t for t in f.state_store.fetch_tasks()}


def test_target_config_without_recovery_is_the_current_target():
    f = Fixture(TWO)
    other = uuid.uuid4()
    _stored(f, "pod-type-0-server", other)
    req = f.requirement(recovery=RecoveryType.NONE)
    assert f.evaluator.get_target_config(req, _this_pod(f)) == f.target


def test_target_config_for_recovery_without_tasks_is_the_target():
    f = Fixture(TWO)
    req = f.requirement(tasks=["server"], recovery=RecoveryType.TRANSIENT)
    assert f.evaluator.get_target_config(req, {}) == f.target


def test_target_config_for_recovery_with_an_unlabelled_task_is_the_target():
    f = Fixture(TWO)
    _stored(f, "pod-type-0-server", None)
    req = f.requirement(tasks=["server"], recovery=RecoveryType.TRANSIENT)
    assert f.evaluator.get_target_config(req, _this_pod(f)) == f.target


def test_target_config_for_recovery_keeps_the_task_config():
    f = Fixture(TWO)
    old = uuid.uuid4()
    _stored(f, "pod-type-0-server", old)
    req = f.requirement(tasks=["server"], recovery=RecoveryType.TRANSIENT)
    assert f.evaluator.get_target_config(req, _this_pod(f)) == old


def test_target_config_ignores_tasks_not_being_launched():
    f = Fixture(TWO)
    old, other = uuid.uuid4(), uuid.uuid4()
    _stored(f, "pod-type-0-server", old)
    _stored(f, "pod-type-0-init", other)
    req = f.requirement(tasks=["server"], recovery=RecoveryType.TRANSIENT)
    assert f.evaluator.get_target_config(req, _this_pod(f)) == old


def test_target_config_prefers_the_running_goal_task_over_once_tasks():
    f = Fixture(TWO)
    server_cfg, init_cfg = uuid.uuid4(), uuid.uuid4()
    _stored(f, "pod-type-0-server", server_cfg, running=False)  # goal RUNNING (status is irrelevant)
    _stored(f, "pod-type-0-init", init_cfg, running=True)       # goal ONCE
    req = f.requirement(tasks=["server", "init"], recovery=RecoveryType.TRANSIENT)
    assert f.evaluator.get_target_config(req, _this_pod(f)) == server_cfg
    req = f.requirement(tasks=["init"], recovery=RecoveryType.TRANSIENT)
    assert f.evaluator.get_target_config(req, _this_pod(f)) == init_cfg


def test_launched_task_carries_the_recovery_config_label():
    f = Fixture(server(1.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    info = f.task()
    old = uuid.uuid4()
    TaskLabelWriter(info).set_target_configuration(old).apply()
    f.state_store.store_tasks([info])
    recs = f.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem")]))],
                      recovery=RecoveryType.TRANSIENT)
    assert str(TaskLabelReader(_task_info(recs)).get_target_configuration()) == str(old)
    assert RU.get_resource_id(task_resource(recs, "cpus")) == RU.get_resource_id(_reserved(first, "cpus"))
