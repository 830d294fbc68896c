"""Mesos resource multiset arithmetic used by the local master/agents.

A ``ResourceBag`` maps a resource *identity* (the Resource message with its quantity fields
cleared: name, type, reservation stack incl. labels, disk persistence/source) to a quantity
(float for SCALAR, an interval list for RANGES). Adding/subtracting whole ``P.Resource``
messages then mirrors Mesos' ``Resources`` arithmetic closely enough for reservation
bookkeeping: RESERVE pushes a reservation onto an unreserved chunk, UNRESERVE pops it,
CREATE/DESTROY toggle ``disk.persistence``.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Tuple, Union

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.values import _normalize, subtract_intervals

EPS = 5e-4  # Mesos scalars are fixed-point with 3 decimal digits
Quantity = Union[float, List[Tuple[int, int]]]


class InsufficientResources(Exception):
    pass


_IDENTITY_CACHE: Dict[bytes, bytes] = {}
_IDENTITY_CACHE_MAX = 8192


def identity(r: P.Resource) -> bytes:
    """The resource's identity bytes, memoized on its full wire form: the same resources go
    through every ACCEPT several times (RESERVE, then the LAUNCH that consumes them), and the
    copy + clear + deterministic serialize costs ~4x a plain serialize + dict hit."""
    full = r.SerializeToString()
    k = _IDENTITY_CACHE.get(full)
    if k is None:
        k = _identity(r)
        if len(_IDENTITY_CACHE) >= _IDENTITY_CACHE_MAX:
            _IDENTITY_CACHE.clear()
        _IDENTITY_CACHE[full] = k
    return k


def _identity(r: P.Resource) -> bytes:
    c = P.Resource()
    c.CopyFrom(r)
    c.ClearField("scalar")
    c.ClearField("ranges")
    c.ClearField("set")
    c.ClearField("allocation_info")
    c.ClearField("role")  # deprecated pre-refinement field; the reservation stack is authoritative
    return c.SerializeToString(deterministic=True)


def _quantity(r: P.Resource) -> Quantity:
    if r.type == P.Value.SCALAR:
        return float(r.scalar.value)
    if r.type == P.Value.RANGES:
        return _normalize((int(x.begin), int(x.end)) for x in r.ranges.range)
    raise ValueError(f"Unsupported resource type for {r.name}: {r.type}")


def _is_empty(q: Quantity) -> bool:
    return (q <= EPS) if isinstance(q, float) else not q


class ResourceBag:
    def __init__(self, resources: Iterable[P.Resource] = ()):
        self._q: Dict[bytes, Quantity] = {}
        self._proto: Dict[bytes, P.Resource] = {}
        for r in resources:
            self.add(r)

    def copy(self) -> "ResourceBag":
        b = ResourceBag()
        b._q = {k: (list(v) if isinstance(v, list) else v) for k, v in self._q.items()}
        b._proto = dict(self._proto)
        return b

    def add(self, r: P.Resource) -> None:
        k = identity(r)
        q = _quantity(r)
        if k not in self._proto:
            p = P.Resource()
            p.ParseFromString(k)
            self._proto[k] = p
        cur = self._q.get(k)
        if cur is None:
            self._q[k] = q
        elif isinstance(q, float):
            self._q[k] = round((cur + q) * 1000.0) / 1000.0
        else:
            self._q[k] = _normalize(list(cur) + list(q))

    def add_all(self, rs: Iterable[P.Resource]) -> None:
        for r in rs:
            self.add(r)

    def contains(self, r: P.Resource) -> bool:
        k = identity(r)
        cur = self._q.get(k)
        if cur is None:
            return False
        q = _quantity(r)
        if isinstance(q, float):
            return cur + EPS >= q
        return subtract_intervals(q, cur) == []

    def subtract(self, r: P.Resource) -> None:
        k = identity(r)
        cur = self._q.get(k)
        q = _quantity(r)
        if isinstance(q, float):
            if cur is None or cur + EPS < q:
                raise InsufficientResources(f"{r.name} {q} not available (have {cur})")
            nv = round((cur - q) * 1000.0) / 1000.0
        else:
            if cur is None or subtract_intervals(q, cur) != []:
                raise InsufficientResources(f"{r.name} {q} not available (have {cur})")
            nv = subtract_intervals(cur, q)
        if _is_empty(nv):
            del self._q[k]
        else:
            self._q[k] = nv

    def subtract_all(self, rs: Iterable[P.Resource]) -> None:
        for r in rs:
            self.subtract(r)

    def is_empty(self) -> bool:
        return not self._q

    def to_resources(self) -> List[P.Resource]:
        out = []
        for k, q in self._q.items():
            r = P.Resource()
            r.CopyFrom(self._proto[k])
            if isinstance(q, float):
                r.scalar.value = round(q, 3)
            else:
                for b, e in q:
                    r.ranges.range.add(begin=b, end=e)
            out.append(r)
        return out

    def scalar(self, name: str) -> float:
        return sum(q for k, q in self._q.items() if isinstance(q, float) and self._proto[k].name == name)

    def take_all(self) -> List[P.Resource]:
        out = self.to_resources()
        self._q.clear()
        self._proto.clear()
        return out


def effective_role(r: P.Resource) -> str:
    if len(r.reservations):
        return r.reservations[-1].role
    return r.role if r.HasField("role") and r.role else "*"


def pop_reservation(r: P.Resource) -> P.Resource:
    c = P.Resource()
    c.CopyFrom(r)
    if len(c.reservations):
        del c.reservations[-1]
    c.ClearField("allocation_info")
    return c


def strip_volume(r: P.Resource) -> P.Resource:
    c = P.Resource()
    c.CopyFrom(r)
    c.ClearField("allocation_info")
    if c.HasField("disk"):
        c.disk.ClearField("persistence")
        c.disk.ClearField("volume")
        if not c.disk.ListFields():
            c.ClearField("disk")
    return c
