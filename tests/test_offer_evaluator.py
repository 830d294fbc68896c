"""OfferEvaluator and the evaluation stages, driven directly (no scheduler, no master).

Scenarios follow the reference's evaluator suites
(sdk/scheduler/src/test/java/com/mesosphere/sdk/offer/evaluate/OfferEvaluatorTest.java,
OfferEvaluatorPortsTest.java, OfferEvaluatorVolumesTest.java, OfferEvaluatorPlacementTest.java,
MesosResourcePoolTest.java): first launch reserves executor + task resources and returns
RESERVE…/LAUNCH_GROUP/StoreTaskInfo; a relaunch on the expected reservations only launches; a
bigger spec grows the reservation in place (RESERVE of the delta under the same resource_id), a
smaller one shrinks it (UNRESERVE of the delta); pre-reserved roles produce refined reservations;
static/dynamic ports, ROOT/MOUNT volumes, GPUs, placement and multi-offer selection.
"""
import textwrap
import uuid

import pytest

from dcos_commons_amd.http.endpoint_utils import template_url_factory
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import common_id_utils
from dcos_commons_amd.offer import resources as RU
from dcos_commons_amd.offer.evaluate.offer_evaluator import OfferEvaluator
from dcos_commons_amd.offer.recommendations import (CreateOfferRecommendation, LaunchOfferRecommendation,
                                                    ReserveOfferRecommendation, StoreTaskInfoRecommendation,
                                                    UnreserveOfferRecommendation)
from dcos_commons_amd.offer.resource_pool import MesosResourcePool
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader, env_to_map, text_attribute
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement
from dcos_commons_amd.scheduler.recovery import RecoveryType
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import PodInstance
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.persistent_launch_recorder import PersistentLaunchRecorder
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister

CFG = SchedulerConfig.for_testing()
FID = "test-framework-id"


def scalar(name, v, role="*"):
    r = P.Resource(name=name, type=P.Value.SCALAR, role=role)
    r.scalar.value = v
    if role != "*":
        res = r.reservations.add()
        res.type = P.Resource.ReservationInfo.STATIC
        res.role = role
    return r


def ranges(name, *pairs, role="*"):
    r = P.Resource(name=name, type=P.Value.RANGES, role=role)
    for b, e in pairs:
        x = r.ranges.range.add()
        x.begin, x.end = b, e
    return r


def mount_disk(size, root="/mnt/disk0"):
    r = scalar("disk", size)
    r.disk.source.type = P.Resource.DiskInfo.Source.MOUNT
    r.disk.source.mount.root = root
    return r


def offer(*resources, oid="o1", host="host1", agent="agent1", attrs=()):
    o = P.Offer()
    o.id.value = oid
    o.framework_id.value = FID
    o.agent_id.value = agent
    o.hostname = host
    for r in resources:
        o.resources.add().CopyFrom(r)
    for a in attrs:
        o.attributes.add().CopyFrom(a)
    return o


def executor_room(role="*"):
    """Unreserved room for the default executor (0.1 cpus, 32 MB, 256 MB disk)."""
    return [scalar("cpus", 0.1, role), scalar("mem", 32, role), scalar("disk", 256, role)]


def complete_offer(*resources, role="*", **kw):
    return offer(*(list(resources) + executor_room(role)), **kw)


class Fixture:
    def __init__(self, task_yaml, pod_extra="", count=1, name="test-service"):
        text = (f"name: {name}\nscheduler:\n  principal: test-principal\npods:\n  pod-type:\n    count: {count}\n"
                + (textwrap.indent(textwrap.dedent(pod_extra), "    ") if pod_extra else "")
                + "    tasks:\n" + textwrap.indent(textwrap.dedent(task_yaml), "      "))
        raw = RawServiceSpec.from_string(text)
        self.spec = mappers.ServiceSpecGenerator(raw, CFG, "/tmp", {}).build()
        persister = MemPersister()
        self.framework_store = FrameworkStore(persister)
        self.framework_store.store_framework_id(P.FrameworkID(value=FID))
        self.state_store = StateStore(persister)
        self.target = uuid.uuid4()
        self.evaluator = OfferEvaluator(self.framework_store, self.state_store, self.spec.name, self.target,
                                        template_url_factory(self.spec.name, CFG), CFG)
        self.recorder = PersistentLaunchRecorder(self.state_store, self.spec)

    def requirement(self, index=0, tasks=None, recovery=RecoveryType.NONE, pod=None):
        pod = pod or self.spec.pods[0]
        return PodInstanceRequirement(PodInstance(pod, index), tasks or [t.name for t in pod.tasks],
                                      recovery_type=recovery)

    def evaluate(self, offers, **kw):
        return self.evaluator.evaluate(self.requirement(**kw), offers)

    def launch(self, offers, **kw):
        recs = self.evaluate(offers, **kw)
        assert recs, "expected a launch"
        self.recorder.record(recs)
        return recs

    def task(self, name="pod-type-0-server"):
        return self.state_store.fetch_task(name)


def server(cpus=1.0, mem=None, extra=""):
    body = f"server:\n  goal: RUNNING\n  cmd: ./server\n  cpus: {cpus}\n"
    if mem is not None:
        body += f"  memory: {mem}\n"
    return body + textwrap.indent(textwrap.dedent(extra), "  ")


def ops(recs):
    return [r.get_operation().type if r.get_operation() is not None else None for r in recs]


def of(recs, cls):
    return [r for r in recs if isinstance(r, cls)]


def task_resource(recs, name):
    launch = of(recs, LaunchOfferRecommendation)[0]
    return next(r for r in launch.task_info.resources if r.name == name)


R, L, U, C = (P.Offer.Operation.RESERVE, P.Offer.Operation.LAUNCH_GROUP, P.Offer.Operation.UNRESERVE,
              P.Offer.Operation.CREATE)


# ---------------------------------------------------------------------------------------
# scalars: reserve, relaunch, grow, shrink


def test_reserve_and_launch_scalar():
    f = Fixture(server(1.0, 32))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    # executor cpus/mem/disk, task cpus/mem, then the launch and the (op-less) state-store record
    assert ops(recs) == [R, R, R, R, R, L, None]
    reserves = of(recs, ReserveOfferRecommendation)
    task_cpu = next(r.get_operation().reserve.resources[0] for r in reserves[3:]
                    if r.get_operation().reserve.resources[0].name == "cpus")
    assert task_cpu.scalar.value == 1.0
    assert RU.get_role(task_cpu) == "test-service-role"
    assert RU.get_principal(task_cpu) == "test-principal"
    assert len(RU.get_resource_id(task_cpu)) == 36
    assert RU.get_framework_id(task_cpu) == FID
    assert not task_cpu.HasField("disk")
    launch = of(recs, LaunchOfferRecommendation)[0]
    assert RU.get_resource_id(task_resource(recs, "cpus")) == RU.get_resource_id(task_cpu)
    eid = launch.get_operation().launch_group.executor.executor_id
    assert common_id_utils.to_executor_name(eid) == "pod-type"
    assert eid.value.startswith("test-service__pod-type__")
    assert isinstance(recs[-1], StoreTaskInfoRecommendation)


def _reserved(recs, name, task=True):
    """The reserved form of one resource from a launch (what the master re-offers)."""
    if task:
        return task_resource(recs, name)
    launch = of(recs, LaunchOfferRecommendation)[0]
    return next(r for r in launch.executor_info.resources if r.name == name)


def _executor_reserved(recs):
    launch = of(recs, LaunchOfferRecommendation)[0]
    return list(launch.get_operation().launch_group.executor.resources)


def test_relaunch_on_expected_resources_only_launches():
    f = Fixture(server(1.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    again = f.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem")]))])
    assert ops(again) == [L, None]
    assert RU.get_resource_id(task_resource(again, "cpus")) == RU.get_resource_id(_reserved(first, "cpus"))


def test_increase_reservation_reserves_the_delta_under_the_same_id():
    f = Fixture(server(1.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    rid = RU.get_resource_id(_reserved(first, "cpus"))
    bigger = Fixture(server(2.0, 32))
    bigger.state_store = f.state_store
    bigger.evaluator = OfferEvaluator(f.framework_store, f.state_store, f.spec.name, f.target,
                                      template_url_factory(f.spec.name, CFG), CFG)
    recs = bigger.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem"),
                                                                  scalar("cpus", 1.0)]))])
    assert ops(recs) == [R, L, None]
    grow = recs[0].get_operation().reserve.resources[0]
    assert grow.name == "cpus" and grow.scalar.value == 1.0 and RU.get_resource_id(grow) == rid
    assert task_resource(recs, "cpus").scalar.value == 2.0
    assert RU.get_resource_id(task_resource(recs, "cpus")) == rid


def _respec(f, task_yaml):
    g = Fixture(task_yaml)
    g.framework_store, g.state_store, g.target = f.framework_store, f.state_store, f.target
    g.evaluator = OfferEvaluator(f.framework_store, f.state_store, g.spec.name, f.target,
                                 template_url_factory(g.spec.name, CFG), CFG)
    return g


def test_decrease_reservation_unreserves_the_delta():
    f = Fixture(server(2.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    rid = RU.get_resource_id(_reserved(first, "cpus"))
    g = _respec(f, server(1.0, 32))
    recs = g.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem")]))])
    assert ops(recs) == [U, L, None]
    shrink = recs[0].get_operation().unreserve.resources[0]
    assert shrink.scalar.value == 1.0 and RU.get_resource_id(shrink) == rid
    assert task_resource(recs, "cpus").scalar.value == 1.0


def test_increase_fails_without_room():
    f = Fixture(server(2.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    small = _reserved(first, "cpus")
    small.scalar.value = 1.0
    recs = f.evaluate([offer(*(_executor_reserved(first) + [small, _reserved(first, "mem")]))])
    assert recs == []


def test_insufficient_offer_is_rejected_and_outcome_is_tracked():
    from dcos_commons_amd.offer.history import OfferOutcomeTracker

    f = Fixture(server(4.0, 32))
    f.evaluator.offer_outcome_tracker = OfferOutcomeTracker()
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))]) == []
    tracked = f.evaluator.offer_outcome_tracker.to_json()
    text = str(tracked)
    assert "pod-type-0:[server]" in text and "FAIL" in text and "cpus" in text


def test_launch_uses_first_sufficient_offer():
    f = Fixture(server(1.0, 32))
    small = complete_offer(scalar("cpus", 0.5), scalar("mem", 64), oid="small", agent="a-small")
    big = complete_offer(scalar("cpus", 2.0), scalar("mem", 64), oid="big", agent="a-big")
    recs = f.evaluate([small, big])
    assert recs and all(r.offer.id.value == "big" for r in recs)
    assert of(recs, LaunchOfferRecommendation)[0].task_info.agent_id.value == "a-big"


# ---------------------------------------------------------------------------------------
# labels and environment on the launched TaskInfo


def test_launch_embeds_offer_attributes_and_identity_labels():
    f = Fixture(server(1.0, 32))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), host="h7",
                                      attrs=[text_attribute("rack", "r1"), text_attribute("zone", "a")])])
    ti = of(recs, LaunchOfferRecommendation)[0].task_info
    r = TaskLabelReader(ti)
    assert r.get_hostname() == "h7"
    assert r.get_offer_attribute_strings() == ["rack:r1", "zone:a"]
    assert r.get_type() == "pod-type" and r.get_index() == 0
    assert str(r.get_target_configuration()) == str(f.target)
    env = env_to_map(ti.command.environment)
    assert env["TASK_NAME"] == "pod-type-0-server"
    assert env["POD_INSTANCE_INDEX"] == "0"
    assert ti.task_id.value.startswith("test-service__pod-type-0-server__")
    assert ti.name == "pod-type-0-server"


def test_stored_task_info_is_recorded_with_staging_status():
    f = Fixture(server(1.0, 32))
    f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    ti = f.task()
    assert ti is not None and ti.task_id.value
    st = f.state_store.fetch_status("pod-type-0-server")
    assert st.state == P.TASK_STAGING and st.task_id.value == ti.task_id.value


# ---------------------------------------------------------------------------------------
# pre-reserved roles (reservation refinement)


def test_pre_reserved_role_produces_refined_reservation():
    f = Fixture(server(1.0, 32), pod_extra="pre-reserved-role: slave_public\n")
    pr = "slave_public"
    recs = f.evaluate([offer(scalar("cpus", 2.0, pr), scalar("mem", 64, pr), *executor_room(pr))])
    assert recs, "pre-reserved resources must be consumable"
    cpu = task_resource(recs, "cpus")
    assert [x.role for x in cpu.reservations][0] == pr
    assert cpu.reservations[-1].type == P.Resource.ReservationInfo.DYNAMIC
    assert cpu.reservations[-1].role.startswith(pr + "/")


def test_missing_pre_reservation_fails():
    f = Fixture(server(1.0, 32), pod_extra="pre-reserved-role: slave_public\n")
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))]) == []
    other = "other_role"
    assert f.evaluate([offer(scalar("cpus", 2.0, other), scalar("mem", 64, other), *executor_room(other))]) == []


# ---------------------------------------------------------------------------------------
# ports


def test_static_port_reserved_and_exported():
    f = Fixture(server(1.0, 32, extra="ports:\n  http:\n    port: 8080\n"))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (8000, 9000)))])
    port = task_resource(recs, "ports")
    assert [(r.begin, r.end) for r in port.ranges.range] == [(8080, 8080)]
    ti = of(recs, LaunchOfferRecommendation)[0].task_info
    # no env-key in the spec: the port is only advertised through DiscoveryInfo
    assert [(p.name, p.number) for p in ti.discovery.ports.ports] == [("http", 8080)]
    assert not any(k.startswith("PORT") for k in env_to_map(ti.command.environment))


def test_static_port_outside_offer_fails():
    f = Fixture(server(1.0, 32, extra="ports:\n  http:\n    port: 8080\n"))
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (9000, 9100)))]) == []


def test_dynamic_port_picks_from_offer_and_is_sticky_on_relaunch():
    f = Fixture(server(1.0, 32, extra="ports:\n  dyn:\n    port: 0\n    env-key: MY_PORT\n"))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (10000, 10010)))])
    port = task_resource(first, "ports")
    chosen = port.ranges.range[0].begin
    assert 10000 <= chosen <= 10010 and port.ranges.range[0].end == chosen
    env = env_to_map(of(first, LaunchOfferRecommendation)[0].task_info.command.environment)
    assert env["MY_PORT"] == str(chosen)
    again = f.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem"),
                                                              _reserved(first, "ports")]))])
    assert ops(again) == [L, None]
    assert task_resource(again, "ports").ranges.range[0].begin == chosen


def test_multiple_ports_and_ranges():
    f = Fixture(server(1.0, 32, extra="ports:\n  a:\n    port: 8080\n  b:\n    port: 8081\n  c:\n    port: 0\n"))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), ranges("ports", (8080, 8082)))])
    assert recs
    got = sorted(r.begin for res in of(recs, LaunchOfferRecommendation)[0].task_info.resources
                 if res.name == "ports" for r in res.ranges.range)
    assert got == [8080, 8081, 8082]


# ---------------------------------------------------------------------------------------
# volumes


def test_root_volume_reserves_and_creates():
    f = Fixture(server(1.0, 32, extra="volume:\n  path: data\n  type: ROOT\n  size: 500\n"))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 1000))])
    creates = of(recs, CreateOfferRecommendation)
    assert len(creates) == 1
    vol = creates[0].get_operation().create.volumes[0]
    assert vol.scalar.value == 500
    assert vol.disk.volume.container_path == "data"
    assert vol.disk.persistence.id
    # the volume in the launched task is the created one
    disk = task_resource(recs, "disk")
    assert disk.disk.persistence.id == vol.disk.persistence.id
    assert ops(recs).index(C) > ops(recs).index(R)


def test_root_volume_too_big_fails():
    f = Fixture(server(1.0, 32, extra="volume:\n  path: data\n  type: ROOT\n  size: 5000\n"))
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 1000))]) == []


def test_mount_volume_consumes_whole_disk():
    f = Fixture(server(1.0, 32, extra="volume:\n  path: data\n  type: MOUNT\n  size: 500\n"))
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), mount_disk(2000))])
    assert recs
    vol = of(recs, CreateOfferRecommendation)[0].get_operation().create.volumes[0]
    assert vol.scalar.value == 2000                      # MOUNT disks are atomic
    assert vol.disk.source.type == P.Resource.DiskInfo.Source.MOUNT
    assert vol.disk.source.mount.root == "/mnt/disk0"


def test_mount_volume_too_small_fails():
    f = Fixture(server(1.0, 32, extra="volume:\n  path: data\n  type: MOUNT\n  size: 5000\n"))
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), mount_disk(2000))]) == []


def test_relaunch_reuses_persistent_volume():
    f = Fixture(server(1.0, 32, extra="volume:\n  path: data\n  type: ROOT\n  size: 500\n"))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 1000))])
    vol = task_resource(first, "disk")
    again = f.evaluate([offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem"),
                                                              vol]))])
    assert ops(again) == [L, None]
    assert task_resource(again, "disk").disk.persistence.id == vol.disk.persistence.id


# ---------------------------------------------------------------------------------------
# GPUs, multi-task pods, recovery


def test_gpu_resource_is_reserved():
    f = Fixture(server(1.0, 32, extra="gpus: 1\n"))
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))]) == []
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("gpus", 8))])
    gpu = task_resource(recs, "gpus")
    assert gpu.scalar.value == 1 and RU.get_resource_id(gpu)


def test_multiple_tasks_share_one_executor():
    two = server(1.0, 32) + "worker:\n  goal: RUNNING\n  cmd: ./worker\n  cpus: 0.5\n  memory: 32\n"
    f = Fixture(two)
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    launches = of(recs, LaunchOfferRecommendation)
    assert sorted(l.task_info.name for l in launches) == ["pod-type-0-server", "pod-type-0-worker"]
    eids = {l.get_operation().launch_group.executor.executor_id.value for l in launches}
    assert len(eids) == 1
    # executor resources are reserved once
    assert sum(1 for r in of(recs, ReserveOfferRecommendation)
               if r.get_operation().reserve.resources[0].name == "disk") == 1


def test_launch_one_task_of_pod_keeps_sibling_resources_reserved():
    two = server(1.0, 32) + "worker:\n  goal: RUNNING\n  cmd: ./worker\n  cpus: 0.5\n  memory: 32\n"
    f = Fixture(two)
    recs = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))], tasks=["server"])
    launches = of(recs, LaunchOfferRecommendation)
    assert [l.task_info.name for l in launches] == ["pod-type-0-server"]
    stored = sorted(r.task_info.name for r in of(recs, StoreTaskInfoRecommendation))
    assert stored == ["pod-type-0-server", "pod-type-0-worker"]


def test_transient_relaunch_reuses_reservations_permanent_gets_new_ones():
    f = Fixture(server(1.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    rid = RU.get_resource_id(_reserved(first, "cpus"))
    # TASK_FAILED: transient recovery relaunches on the same reservations
    st = P.TaskStatus(state=P.TASK_FAILED)
    st.task_id.CopyFrom(f.task().task_id)
    f.state_store.store_status("pod-type-0-server", st)
    reoffer = offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem")]))
    t = f.evaluate([reoffer], recovery=RecoveryType.TRANSIENT)
    assert ops(t) == [L, None]
    assert RU.get_resource_id(task_resource(t, "cpus")) == rid
    # PERMANENT: a fresh footprint with new resource ids, on a fresh offer
    p = f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), oid="o2", agent="agent2")],
                   recovery=RecoveryType.PERMANENT)
    assert L in ops(p) and R in ops(p)
    assert RU.get_resource_id(task_resource(p, "cpus")) != rid


def test_placement_rule_gates_offer():
    f = Fixture(server(1.0, 32), pod_extra="placement: 'hostname:LIKE:good-.*'\n")
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), host="bad-1")]) == []
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), host="good-1")])


def test_unique_placement_against_recorded_siblings():
    f = Fixture(server(1.0, 32), pod_extra="placement: 'hostname:UNIQUE'\n", count=2)
    f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), host="h1")], index=0)
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), host="h1", oid="o2")], index=1) == []
    assert f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), host="h2", oid="o3",
                                      agent="agent2")], index=1)


def test_evaluation_requires_registered_framework():
    f = Fixture(server(1.0, 32))
    f.framework_store.clear_framework_id()
    with pytest.raises(RuntimeError):
        f.evaluate([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])


# ---------------------------------------------------------------------------------------
# MesosResourcePool


def test_resource_pool_merges_unreserved_and_tracks_reserved():
    r1 = scalar("cpus", 1.0)
    r2 = scalar("cpus", 2.5)
    o = offer(r1, r2, ranges("ports", (1, 5)), ranges("ports", (10, 12)), mount_disk(100))
    pool = MesosResourcePool(o, "role")
    merged = pool.unreserved_merged_pool()
    assert merged["cpus"].scalar.value == pytest.approx(3.5)
    assert sorted((r.begin, r.end) for r in merged["ports"].ranges.range) == [(1, 5), (10, 12)]
    assert "disk" not in merged                       # MOUNT disk lives in the atomic pool


def test_resource_pool_consume_reserved_by_id():
    f = Fixture(server(1.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    cpu = _reserved(first, "cpus")
    pool = MesosResourcePool(offer(cpu), "test-service-role")
    rid = RU.get_resource_id(cpu)
    assert pool.get_reserved_resource_by_id(rid) is not None
    v = P.Value(type=P.Value.SCALAR)
    v.scalar.value = 1.0
    assert pool.consume_reserved("cpus", v, rid) is not None
    assert pool.consume_reserved("cpus", v, rid) is None       # consumed once


# ---------------------------------------------------------------------------------------
# write-ahead footprint marker (launch_new_footprint) and same-cycle placement


def test_recorder_marks_only_launches_that_create_their_footprint():
    f = Fixture(server(1.0, 32, extra="volume:\n  path: data\n  type: ROOT\n  size: 10\n"))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64), scalar("disk", 64))])
    assert TaskLabelReader(f.task()).is_launch_new_footprint()
    # relaunch in place on the reservations + volume the first launch created
    reserved = _executor_reserved(first) + [r for r in of(first, LaunchOfferRecommendation)[0].task_info.resources]
    again = f.launch([offer(*reserved)])
    assert ops(again) == [L, None]
    assert not TaskLabelReader(f.task()).is_launch_new_footprint()


class _Step:
    def __init__(self, req):
        self.req, self.recs, self.started = req, None, False

    def is_pending(self):
        return not self.started

    def is_prepared(self):
        return False

    def start(self):
        self.started = True

    def get_pod_instance_requirement(self):
        return self.req

    def update_offer_status(self, recs):
        self.recs = recs

    def get_name(self):
        return f"step-{self.req.pod_instance.index}"


def test_same_cycle_placement_sees_pods_matched_earlier_in_the_cycle():
    """MAX_PER rack 1 with two pods in one offer cycle: the second step must see the first
    step's pod (the reference evaluates both against the pre-cycle task set and can stack them)."""
    from dcos_commons_amd.scheduler.plan.plan_scheduler import PlanScheduler

    f = Fixture(server(1.0, 32), pod_extra='placement: \'[["rack", "MAX_PER", "1"]]\'\n', count=2)
    offers = [complete_offer(scalar("cpus", 2.0), scalar("mem", 64), oid=f"o{i}", host=f"host{i}",
                             agent=f"agent{i}", attrs=[text_attribute("rack", rack)])
              for i, rack in ((1, "r1"), (2, "r1"), (3, "r2"))]
    steps = [_Step(f.requirement(index=i)) for i in (0, 1)]
    recs = PlanScheduler(f.evaluator, f.state_store).resource_offers(offers, steps)
    launches = of(recs, LaunchOfferRecommendation)
    assert len(launches) == 2
    assert sorted(TaskLabelReader(l.task_info).get_offer_attribute_strings()[0] for l in launches) == \
        ["rack:r1", "rack:r2"]


def test_in_place_relaunch_skips_offers_without_its_reservations():
    """An offer lacking a reservation the existing pipeline consumes by ID fails without running
    the stages (one ``ReservationPrecheck`` outcome is tracked); the offer that carries them is
    evaluated as usual, whatever its position."""
    from dcos_commons_amd.offer.history import OfferOutcomeTracker

    f = Fixture(server(1.0, 32))
    first = f.launch([complete_offer(scalar("cpus", 2.0), scalar("mem", 64))])
    f.evaluator.offer_outcome_tracker = OfferOutcomeTracker()
    other_agent = complete_offer(scalar("cpus", 8.0), scalar("mem", 640), oid="other", agent="a-other")
    partial = offer(*(_executor_reserved(first) + [_reserved(first, "cpus")]), oid="partial")
    assert f.evaluate([other_agent, partial]) == []
    text = str(f.evaluator.offer_outcome_tracker.to_json())
    assert text.count("ReservationPrecheck") == 2 and "lacks 2 of the 2" in text and "lacks 1 of the 2" in text
    full = offer(*(_executor_reserved(first) + [_reserved(first, "cpus"), _reserved(first, "mem")]), oid="full")
    again = f.evaluate([other_agent, full])
    assert ops(again) == [L, None] and again[0].offer.id.value == "full"


def _instance_templates(evaluator):
    """The evaluator's per-instance templates (its cache also keeps one per pod type, keyed
    without the index, to move to other instances)."""
    return {k: v for k, v in evaluator._templates.items() if isinstance(k[0], int)}


def test_pod_templates_are_reused_across_evaluations_without_leaking_offer_state():
    """The evaluator keeps one untouched PodInfoBuilder template per (pod instance, target config,
    requirement env, goal overrides) and each evaluation works on a copy: task IDs, agent IDs,
    port env vars and reservations of one evaluation never reach the next."""
    f = Fixture(server(extra="ports:\n  http:\n    port: 0\n    env-key: PORT_HTTP\n"))
    o1 = complete_offer(scalar("cpus", 1.0), ranges("ports", (5000, 5000)), agent="a1", oid="o1")
    o2 = complete_offer(scalar("cpus", 1.0), ranges("ports", (6000, 6000)), agent="a2", oid="o2")
    first = of(f.evaluate([o1]), LaunchOfferRecommendation)[0].task_info
    assert len(_instance_templates(f.evaluator)) == 1
    tpl = next(iter(_instance_templates(f.evaluator).values()))[1]
    second = of(f.evaluate([o2]), LaunchOfferRecommendation)[0].task_info
    assert len(_instance_templates(f.evaluator)) == 1
    assert next(iter(_instance_templates(f.evaluator).values()))[1] is tpl
    assert first.task_id.value != second.task_id.value
    assert (first.agent_id.value, second.agent_id.value) == ("a1", "a2")
    assert env_to_map(first.command.environment)["PORT_HTTP"] == "5000"
    assert env_to_map(second.command.environment)["PORT_HTTP"] == "6000"
    untouched = tpl.get_task_builder("server")
    assert not untouched.task_id.value and not untouched.resources and "PORT_HTTP" not in env_to_map(
        untouched.command.environment)
    # another pod index, requirement environment or target config is another template
    f.evaluator.evaluate(PodInstanceRequirement(PodInstance(f.spec.pods[0], 0), ["server"],
                                                environment={"EXTRA": "1"}), [o1])
    assert len(_instance_templates(f.evaluator)) == 2


def test_other_instances_of_a_pod_are_moved_from_its_first_template(monkeypatch):
    """Index 1 of a pod whose index 0 was evaluated with the same inputs gets index 0's template
    moved to it (PodInfoBuilder.for_instance) instead of a fresh build; what it launches is what
    a fresh build launches (tests/test_template_instances.py checks the templates byte for byte)."""
    from dcos_commons_amd.offer.evaluate import pod_info_builder as PIB

    f = Fixture(server())
    o1 = complete_offer(scalar("cpus", 1.0), agent="a1", oid="o1")
    f.evaluate([o1])
    builds = []
    orig = PIB.PodInfoBuilder.__init__

    def counting(self, *a, **k):
        builds.append(1)
        orig(self, *a, **k)
    monkeypatch.setattr(PIB.PodInfoBuilder, "__init__", counting)
    rec = of(f.evaluator.evaluate(PodInstanceRequirement(PodInstance(f.spec.pods[0], 1), ["server"]), [o1]),
             LaunchOfferRecommendation)[0].task_info
    assert not builds
    assert rec.name == f"{f.spec.pods[0].type}-1-server"
    env = env_to_map(rec.command.environment)
    assert env["POD_INSTANCE_INDEX"] == "1" and env["TASK_NAME"] == rec.name and env[rec.name] == "true"
