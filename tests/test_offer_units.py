"""Offer-layer units: the per-offer resource pool, range math, the resource builder in both
reservation modes, foreign-reservation filtering, the offer accepter and accepted-offer filtering,
and UNRESERVE operations for volumes.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/offer/{MesosResourcePoolTest,RangeUtilsTest,
ResourceBuilderTest,ResourceUtilsTest,OfferAccepterTest,OfferUtilsTest,
UnreserveOfferRecommendationTest}.java. "Legacy" reservations (the deprecated ``role`` +
``reservation`` fields) are what a cluster without RESERVATION_REFINEMENT gets; "refined" ones are
the ``reservations`` stack (pre-reserved STATIC role, then our DYNAMIC one).
"""
import uuid

import pytest

import testutils as U
from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.framework import driver
from dcos_commons_amd.framework.offer_processing import OfferAccepter, filter_out_accepted
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import values as V
from dcos_commons_amd.offer.recommendations import (DestroyOfferRecommendation, OfferRecommendation,
                                                    StoreTaskInfoRecommendation, UnreserveOfferRecommendation)
from dcos_commons_amd.offer.resource_pool import MesosResourcePool
from dcos_commons_amd.offer.resources import MesosResource, ResourceBuilder, is_processable
from dcos_commons_amd.offer.taskdata import labels as L
from dcos_commons_amd.specification.specs import ANY_ROLE, ResourceSpec, VolumeSpec
from dcos_commons_amd.testing.harness import RecordingDriver

FRAMEWORK_ID = "01234567-890a-bcde-f012-34567890abcd"
CPU_VALUE = U.scalar_value(1.0)


@pytest.fixture(params=["refined", "legacy"])
def mode(request):
    saved = capabilities.get_instance()
    capabilities.override_capabilities(capabilities.Capabilities().with_overrides(
        supports_pre_reserved_resources=request.param == "refined"))
    yield request.param
    capabilities.override_capabilities(saved)


@pytest.fixture
def refined():
    saved = capabilities.get_instance()
    capabilities.override_capabilities(capabilities.Capabilities())
    yield
    capabilities.override_capabilities(saved)


# ---------------------------------------------------------------------------------------
# MesosResourcePool


def _pool(*resources):
    return MesosResourcePool(U.get_offer(resources), ANY_ROLE)


def test_pool_without_atomic_resources(refined):
    assert _pool(U.unreserved_cpus(1.0)).unreserved_atomic_pool == {}


def test_pool_with_one_mount_disk(refined):
    pool = _pool(U.unreserved_mount_volume(1000))
    assert list(pool.unreserved_atomic_pool) == ["disk"] and len(pool.unreserved_atomic_pool["disk"]) == 1


def test_pool_reserved_mount_disk_goes_to_the_reserved_pool(refined):
    r = U.reserved_mount_volume(1000)
    pool = _pool(r)
    assert pool.unreserved_atomic_pool == {}
    assert list(pool.reserved_pool) == [MesosResource(r).resource_id]
    assert pool.reserved_pool[U.RESOURCE_ID].resource == r


def test_pool_with_two_mount_disks(refined):
    r = U.unreserved_mount_volume(1000)
    pool = _pool(r, r)
    assert len(pool.unreserved_atomic_pool) == 1 and len(pool.unreserved_atomic_pool["disk"]) == 2


def _mount_spec(size, profiles):
    return VolumeSpec.create_mount_volume(size, U.CONTAINER_PATH, profiles, U.ROLE, ANY_ROLE, U.PRINCIPAL)


@pytest.mark.parametrize("offer_profile,spec_profiles,consumed", [
    (None, [], True),
    ("bar", ["foo", "bar"], True),
    ("bar", ["foo"], False),
    (None, ["foo", "bar"], False),
    ("bar", [], False),
])
def test_consume_mount_disk_by_profile(refined, offer_profile, spec_profiles, consumed):
    r = U.unreserved_mount_volume(1000, offer_profile)
    pool = _pool(r)
    got = pool.consume_atomic("disk", _mount_spec(1000, spec_profiles))
    if consumed:
        assert got.resource == r and pool.unreserved_atomic_pool == {}
    else:
        assert got is None and len(pool.unreserved_atomic_pool["disk"]) == 1


def test_consume_reserved_resource(refined):
    r = U.reserved_cpus(1.0, U.RESOURCE_ID)
    pool = _pool(r)
    assert len(pool.reserved_pool) == 1
    assert pool.consume_reserved("cpus", V.get_value(r), U.RESOURCE_ID).resource == r
    assert pool.reserved_pool == {}


def test_consume_part_of_a_reserved_resource_keeps_the_rest(refined):
    r = U.reserved_cpus(3.0, U.RESOURCE_ID)
    pool = _pool(r)
    pool.consume_reserved("cpus", U.scalar_value(1.0), U.RESOURCE_ID)
    assert V.get_value(pool.reserved_pool[U.RESOURCE_ID].resource).scalar.value == 2.0


def test_consume_unreserved_merged_resource(refined):
    r = U.unreserved_cpus(1.0)
    pool = _pool(r)
    assert pool.unreserved_merged_pool()["cpus"].scalar.value == 1.0
    assert pool.consume_reservable_merged("cpus", V.get_value(r), ANY_ROLE).resource == r
    assert pool.unreserved_merged_pool()["cpus"] == V.get_zero(P.Value.SCALAR)


def test_consume_insufficient_unreserved_resource(refined):
    pool = _pool(U.unreserved_cpus(1.0))
    assert pool.consume_reservable_merged("cpus", U.scalar_value(2.0), ANY_ROLE) is None


def test_no_unreserved_resources(refined):
    assert _pool(U.reserved_cpus(1.0, str(uuid.uuid4()))).unreserved_merged_pool() == {}


def test_merged_ranges_and_pre_reserved_pool(refined):
    pool = _pool(U.unreserved_ports(1000, 1001), U.unreserved_ports(1002, 1005), U.prereserved_port(2000, 2001, "base"))
    assert [(r.begin, r.end) for r in pool.unreserved_merged_pool()["ports"].ranges.range] == [(1000, 1005)]
    got = pool.consume_reservable_merged("ports", U.ranges_value((2000, 2000)), "base")
    assert got is not None and got.resource.reservations[0].role == "base"


def test_free_returns_resources_to_the_pool(refined):
    pool = _pool(U.unreserved_cpus(2.0))
    got = pool.consume_reservable_merged("cpus", U.scalar_value(2.0), ANY_ROLE)
    pool.free(got)
    assert pool.unreserved_merged_pool()["cpus"].scalar.value == 2.0


# ---------------------------------------------------------------------------------------
# RangeUtils


def _r(*pairs):
    return V.ranges_to_intervals(U.ranges_value(*pairs).ranges.range)


@pytest.mark.parametrize("a,b,merged", [
    ([(1, 3)], [(2, 4)], [(1, 4)]),
    ([(1, 3)], [(5, 7)], [(1, 3), (5, 7)]),
    ([(1, 5)], [(2, 4)], [(1, 5)]),
    ([(1, 3)], [(4, 7)], [(1, 7)]),  # adjacent ranges join
])
def test_merge_ranges(a, b, merged):
    assert V.merge_intervals(_r(*a), _r(*b)) == merged


@pytest.mark.parametrize("a,b,diff", [
    ([(1, 3), (5, 7)], [(1, 3)], [(5, 7)]),
    ([(2, 3)], [(1, 5)], []),
    ([(1, 10)], [(4, 6)], [(1, 3), (7, 10)]),
])
def test_subtract_ranges(a, b, diff):
    assert V.subtract_intervals(_r(*a), _r(*b)) == diff


def test_is_in_any():
    r1 = U.ranges_value((1, 3), (5, 7)).ranges.range
    assert [V.is_in_any(r1, v) for v in range(9)] == [False, True, True, True, False, True, True, True, False]
    r2 = U.ranges_value((2, 2)).ranges.range
    assert [V.is_in_any(r2, v) for v in (1, 2, 3)] == [False, True, False]


# ---------------------------------------------------------------------------------------
# ResourceBuilder


def test_unreserved_resource(mode):
    r = ResourceBuilder.from_unreserved_value("cpus", CPU_VALUE).build()
    assert (r.name, r.type, r.scalar.value, r.role) == ("cpus", P.Value.SCALAR, 1.0, ANY_ROLE)
    assert not r.HasField("reservation") and len(r.reservations) == 0


def _validate_scalar(r, mode, resource_id=None, namespace=None, framework_id=None):
    if mode == "refined":
        assert r.role == ANY_ROLE and not r.HasField("reservation")
        res = r.reservations[-1]
        assert (res.principal, res.role) == (U.PRINCIPAL, U.ROLE)
    else:
        assert r.role == U.ROLE and r.HasField("reservation") and len(r.reservations) == 0
        res = r.reservation
        assert res.principal == U.PRINCIPAL and not res.HasField("role")
    labels = L.labels_to_map(res.labels)
    if resource_id is not None:
        assert labels["resource_id"] == resource_id
    else:
        assert len(labels["resource_id"]) == 36
    assert labels.get("namespace") == namespace
    assert labels.get("framework_id") == framework_id
    assert len(labels) == 1 + (namespace is not None) + (framework_id is not None)


def _cpu_spec(pre_reserved_role=ANY_ROLE):
    return ResourceSpec(name="cpus", value=CPU_VALUE, role=U.ROLE, principal=U.PRINCIPAL,
                        pre_reserved_role=pre_reserved_role)


NAMESPACES = [(None, None), ("/path/to/namespace", FRAMEWORK_ID)]


@pytest.mark.parametrize("namespace,framework_id", NAMESPACES)
def test_new_resource_from_spec(mode, namespace, framework_id):
    r = ResourceBuilder.from_spec(_cpu_spec(), None, namespace, framework_id).build()
    _validate_scalar(r, mode, None, namespace, framework_id)


@pytest.mark.parametrize("namespace,framework_id", NAMESPACES)
def test_existing_resource_from_spec(mode, namespace, framework_id):
    rid = str(uuid.uuid4())
    r = ResourceBuilder.from_spec(_cpu_spec(), rid, namespace, framework_id).build()
    _validate_scalar(r, mode, rid, namespace, framework_id)


@pytest.mark.parametrize("namespace,framework_id", [(None, None), ("foo", FRAMEWORK_ID)])
def test_refine_static_resource(refined, namespace, framework_id):
    r = ResourceBuilder.from_spec(_cpu_spec(U.PRE_RESERVED_ROLE), None, namespace, framework_id).build()
    assert len(r.reservations) == 2
    _validate_scalar(r, "refined", None, namespace, framework_id)
    assert r.reservations[0].type == P.Resource.ReservationInfo.STATIC
    assert r.reservations[0].role == U.PRE_RESERVED_ROLE


def _validate_disk(r, mode, resource_id=None, namespace=None, framework_id=None):
    assert r.HasField("disk") and r.disk.HasField("persistence")
    assert len(r.disk.persistence.id) == 36 and r.disk.persistence.principal == U.PRINCIPAL
    assert r.disk.volume.container_path == U.CONTAINER_PATH and r.disk.volume.mode == P.Volume.RW
    _validate_scalar(r, mode, resource_id, namespace, framework_id)


def _root(size=10):
    return VolumeSpec.create_root_volume(size, U.CONTAINER_PATH, U.ROLE, ANY_ROLE, U.PRINCIPAL)


@pytest.mark.parametrize("namespace,framework_id", NAMESPACES)
@pytest.mark.parametrize("kind", ["root", "mount"])
def test_volume_from_spec(mode, kind, namespace, framework_id):
    spec, source = (_root(), None) if kind == "root" else (_mount_spec(10, []), U.MOUNT_DISK_SOURCE)
    r = ResourceBuilder.from_volume_spec(spec, None, namespace, None, None, source, framework_id).build()
    _validate_disk(r, mode, None, namespace, framework_id)
    if source is not None:
        assert r.disk.source == U.MOUNT_DISK_SOURCE
    rid, pid = str(uuid.uuid4()), str(uuid.uuid4())
    r = ResourceBuilder.from_volume_spec(spec, rid, namespace, pid, None, source, framework_id).build()
    _validate_disk(r, mode, rid, namespace, framework_id)
    assert r.disk.persistence.id == pid


@pytest.mark.parametrize("namespace,framework_id", NAMESPACES)
@pytest.mark.parametrize("kind", ["scalar", "root", "mount"])
def test_from_existing_resource_round_trips(mode, kind, namespace, framework_id):
    rid, pid = str(uuid.uuid4()), str(uuid.uuid4())
    if kind == "scalar":
        original = ResourceBuilder.from_spec(_cpu_spec(), rid, namespace, framework_id).build()
    elif kind == "root":
        original = ResourceBuilder.from_volume_spec(_root(), rid, namespace, pid, None, None, framework_id).build()
    else:
        original = ResourceBuilder.from_volume_spec(_mount_spec(10, []), rid, namespace, pid, None,
                                                    U.MOUNT_DISK_SOURCE, framework_id).build()
    assert ResourceBuilder.from_existing_resource(original).build() == original


def test_from_existing_rejects_foreign_resources(refined):
    with pytest.raises(ValueError):
        ResourceBuilder.from_existing_resource(U.unreserved_cpus(1.0))


# ---------------------------------------------------------------------------------------
# ResourceUtils.isProcessable


UNEXPECTED_1 = U.reserved_root_volume(1000.0, "unexpected-volume-id-1", "unexpected-volume-id-1")
UNEXPECTED_2 = U.reserved_root_volume(1000.0, "unexpected-volume-id-2", "unexpected-volume-id-2",
                                      "unknown-framework-id")
EXPECTED_1 = U.reserved_root_volume(1000.0, "expected-volume-id-1", "expected-volume-id-1", U.FRAMEWORK_ID.value)


@pytest.mark.parametrize("resource,roles,ok", [
    (UNEXPECTED_1, [], False),
    (UNEXPECTED_1, ["different-role"], False),
    (UNEXPECTED_1, ["different-role-0", "different-role-1"], False),
    (UNEXPECTED_1, [U.ROLE], True),
    (UNEXPECTED_1, [U.ROLE, "another-role"], True),
    (UNEXPECTED_2, [U.ROLE], False),   # reserved by another framework
    (EXPECTED_1, [U.ROLE], True),
])
def test_is_processable(refined, resource, roles, ok):
    assert is_processable(resource, roles, U.FRAMEWORK_ID.value) is ok


def test_partial_role_subset_is_not_processable(refined):
    alien = P.Resource()
    alien.CopyFrom(UNEXPECTED_1)
    alien.role = "alien-role"
    assert not is_processable(alien, [U.ROLE, "another-role"], U.FRAMEWORK_ID.value)


# ---------------------------------------------------------------------------------------
# OfferAccepter / accepted-offer filtering


def _offer(host, agent, oid, fid):
    o = P.Offer(hostname=host)
    o.agent_id.value = agent
    o.id.value = oid
    o.framework_id.value = fid
    return o


OFFER_A = _offer("hostA", "agentA", "offerA", "fwkA")
OFFER_B = _offer("hostB", "agentB", "offerB", "fwkB")
EXEC = P.ExecutorInfo()
EXEC.executor_id.CopyFrom(U.EXECUTOR_ID)
TASK = P.TaskInfo(name=U.TASK_NAME)
TASK.task_id.CopyFrom(U.TASK_ID)
TASK.agent_id.CopyFrom(U.AGENT_ID)


@pytest.fixture
def recs(refined):
    destroy_a = DestroyOfferRecommendation(OFFER_A, U.unreserved_cpus(1.0))
    destroy_b = DestroyOfferRecommendation(OFFER_B, U.unreserved_cpus(2.0))
    store_a = StoreTaskInfoRecommendation(OFFER_A, TASK, EXEC)
    store_b = StoreTaskInfoRecommendation(OFFER_B, TASK, EXEC)
    unreserve_a = UnreserveOfferRecommendation(OFFER_A, U.unreserved_cpus(1.1))
    unreserve_b = UnreserveOfferRecommendation(OFFER_B, U.unreserved_cpus(2.1))
    return [destroy_a, destroy_b, store_a, store_b, unreserve_a, unreserve_b]


@pytest.fixture
def drv():
    d = RecordingDriver()
    driver.set_driver(d)
    yield d
    driver.set_driver(None)


def test_accept_nothing(drv):
    OfferAccepter().accept([])
    assert drv.accepts == []


def test_group_by_agent(recs):
    groups = OfferAccepter.group_by_agent(recs)
    assert groups == {"agentA": [recs[0], recs[2], recs[4]], "agentB": [recs[1], recs[3], recs[5]]}


def test_one_accept_per_agent(drv, recs):
    OfferAccepter().accept(recs)
    assert [a.offer_ids for a in drv.accepts] == [["offerA"], ["offerB"]]  # deduplicated, agent order
    # stored TaskInfos have no operation: only DESTROY and UNRESERVE reach the master
    assert drv.accepts[0].operations == [recs[0].get_operation(), recs[4].get_operation()]
    assert drv.accepts[1].operations == [recs[1].get_operation(), recs[5].get_operation()]


class Rec(OfferRecommendation):
    def __init__(self, offer, with_operation):
        super().__init__(offer, P.Offer.Operation() if with_operation else None)


def _offers():
    out = []
    for oid in ("no-operation", "with-without-operation", "with-operation", "no-recommendation"):
        o = U.get_offer([U.unreserved_cpus(2), U.unreserved_mem(1000), U.unreserved_disk(10000)])
        o.id.value = oid
        out.append(o)
    return out


def _ids(offers):
    return [o.id.value for o in offers]


def test_filter_accepted_offers():
    offers = _offers()
    recs = [Rec(offers[0], False), Rec(offers[1], False), Rec(offers[1], True), Rec(offers[2], True)]
    assert _ids(filter_out_accepted(offers, [recs[2]])) == ["no-operation", "with-operation", "no-recommendation"]
    assert _ids(filter_out_accepted(offers, [])) == _ids(offers)
    assert _ids(filter_out_accepted(offers, recs)) == ["no-operation", "no-recommendation"]
    other = _offers()[:2]
    other[0].id.value, other[1].id.value = "abc", "def"
    assert _ids(filter_out_accepted(offers, [Rec(other[0], False), Rec(other[1], True)])) == _ids(offers)


# ---------------------------------------------------------------------------------------
# UnreserveOfferRecommendation


def test_unreserve_root_disk_drops_the_volume(refined):
    r = U.reserved_root_volume(1)
    op = UnreserveOfferRecommendation(U.get_offer([r]), r).get_operation()
    assert len(op.unreserve.resources) == 1
    got = op.unreserve.resources[0]
    assert not got.HasField("disk") and not got.HasField("revocable")
    expected = P.Resource()
    expected.CopyFrom(r)
    expected.ClearField("disk")
    assert got == expected


def test_unreserve_mount_disk_keeps_only_the_source(refined):
    r = U.reserved_mount_volume(1)
    op = UnreserveOfferRecommendation(U.get_offer([r]), r).get_operation()
    got = op.unreserve.resources[0]
    assert got.HasField("disk") and got.disk.HasField("source") and not got.HasField("revocable")
    expected = P.Resource()
    expected.CopyFrom(r)
    expected.disk.Clear()
    expected.disk.source.CopyFrom(r.disk.source)
    assert got == expected


@pytest.mark.parametrize("pre_reserved", [ANY_ROLE, "slave_public"])
@pytest.mark.parametrize("namespace", [None, "ns"])
def test_wire_template_reservations_equal_the_builder(refined, pre_reserved, namespace):
    """``new_reservation`` / ``new_root_volume`` (the per-spec wire templates the evaluator uses for
    new reservations on plain chunks) build exactly what ResourceBuilder builds for the same ids."""
    from dcos_commons_amd.offer.resources import get_persistence_id, get_resource_id, new_reservation, new_root_volume

    spec = ResourceSpec(name="cpus", value=CPU_VALUE, role=U.ROLE,
                        principal=U.PRINCIPAL, pre_reserved_role=pre_reserved)
    for _ in range(2):   # template built, then reused
        r, rid = new_reservation(spec, namespace, "fw-id")
        assert get_resource_id(r) == rid
        assert r == ResourceBuilder.from_spec(spec, rid, namespace, "fw-id").build()
    vol = VolumeSpec.create_root_volume(64, U.CONTAINER_PATH, U.ROLE, pre_reserved, U.PRINCIPAL)
    for _ in range(2):
        r, rid = new_reservation(vol, namespace, "fw-id")
        v = new_root_volume(vol, rid, namespace, "fw-id")
        pid = get_persistence_id(v)
        assert get_resource_id(v) == rid and pid and pid != rid
        assert v == ResourceBuilder.from_volume_spec(vol, rid, namespace, pid, None, None, "fw-id").build()


def test_env_template_merges_like_a_sorted_map():
    """``labels.EnvTemplate`` (a task spec's environment encoded once; per-instance variables
    merged in name order as byte slices) is byte-identical to encoding the merged, sorted map."""
    import random

    from dcos_commons_amd.offer.taskdata import labels as L

    rnd = random.Random(7)
    names = [f"{rnd.choice('ABCDEFGHIJ')}{rnd.choice('_XYZ0')}{i}" for i in range(60)]
    for trial in range(200):
        static = {n: f"v{rnd.randrange(5)}" for n in rnd.sample(names, rnd.randrange(0, 40))}
        extra = {n: f"x{rnd.randrange(5)}" for n in rnd.sample(names + ["AAA", "zzz", "M"], rnd.randrange(0, 12))}
        got = L.EnvTemplate(static).encode(extra)
        assert got == L.env_bytes_from_map({**static, **extra}), (static, extra)
    assert L.env_template(static) is L.env_template(static)      # cached per spec map
    env = P.Environment()
    env.MergeFromString(L.EnvTemplate({"B": "2", "D": "4"}).encode({"A": "1", "D": "x", "E": "5"}))
    assert [(v.name, v.value) for v in env.variables] == [("A", "1"), ("B", "2"), ("D", "x"), ("E", "5")]
