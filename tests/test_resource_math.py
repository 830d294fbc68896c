"""The local master's resource arithmetic (``mesos.resource_math``) and its operation application:
RESERVE/UNRESERVE are all-or-nothing per operation, as Mesos applies each offer operation."""
import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import LocalMaster
from dcos_commons_amd.mesos.resource_math import InsufficientResources, ResourceBag, pop_reservation


def _scalar(name, value, role=None, rid=None):
    r = P.Resource(name=name, type=P.Value.SCALAR)
    r.scalar.value = value
    if role:
        res = r.reservations.add(role=role, type=P.Resource.ReservationInfo.DYNAMIC, principal="p")
        res.labels.labels.add(key="resource_id", value=rid or "id")
    return r


def _ports(begin, end):
    r = P.Resource(name="ports", type=P.Value.RANGES)
    r.ranges.range.add(begin=begin, end=end)
    return r


def _state(bag):
    return sorted((bag._proto[k].name, len(bag._proto[k].reservations), v if isinstance(v, float) else tuple(v))
                  for k, v in bag._q.items())


def test_subtract_checks_containment_for_scalars_and_ranges():
    bag = ResourceBag([_scalar("cpus", 2.0), _ports(1000, 1010)])
    bag.subtract(_scalar("cpus", 0.5))
    bag.subtract(_ports(1000, 1004))
    assert _state(bag) == [("cpus", 0, 1.5), ("ports", 0, ((1005, 1010),))]
    with pytest.raises(InsufficientResources):
        bag.subtract(_scalar("cpus", 1.6))
    with pytest.raises(InsufficientResources):
        bag.subtract(_ports(1004, 1006))
    with pytest.raises(InsufficientResources):
        bag.subtract(_scalar("mem", 1.0))
    assert _state(bag) == [("cpus", 0, 1.5), ("ports", 0, ((1005, 1010),))]
    bag.subtract(_scalar("cpus", 1.5))                # to zero: the entry goes away
    assert _state(bag) == [("ports", 0, ((1005, 1010),))]


def test_reserve_operation_is_all_or_nothing():
    bag = ResourceBag([_scalar("cpus", 1.0), _scalar("mem", 100.0)])
    before = _state(bag)
    op = P.Offer.Operation(type=P.Offer.Operation.RESERVE)
    op.reserve.resources.extend([_scalar("cpus", 0.5, "svc-role", "a"), _scalar("mem", 200.0, "svc-role", "b")])
    with pytest.raises(InsufficientResources):
        LocalMaster._swap_in_place(bag, [(pop_reservation(r), r) for r in op.reserve.resources])
    assert _state(bag) == before                       # the cpus reservation was rolled back
    ok = [(pop_reservation(r), r) for r in (_scalar("cpus", 0.5, "svc-role", "a"),
                                             _scalar("mem", 60.0, "svc-role", "b"))]
    LocalMaster._swap_in_place(bag, ok)
    assert _state(bag) == [("cpus", 0, 0.5), ("cpus", 1, 0.5), ("mem", 0, 40.0), ("mem", 1, 60.0)]
    # UNRESERVE of more than is reserved changes nothing either
    back = [(_scalar("cpus", 0.5, "svc-role", "a"), _scalar("cpus", 0.5)),
            (_scalar("mem", 61.0, "svc-role", "b"), _scalar("mem", 61.0))]
    snapshot = _state(bag)
    with pytest.raises(InsufficientResources):
        LocalMaster._swap_in_place(bag, back)
    assert _state(bag) == snapshot

