"""Scalar / range arithmetic on Mesos ``Value`` messages.

Reference: sdk/.../offer/{ValueUtils,RangeUtils}.java. Ranges are inclusive ``[begin, end]``
and are normalized (sorted, merged, adjacent intervals coalesced) after every operation.
"""
from __future__ import annotations

from typing import Iterable, List, Tuple

from dcos_commons_amd.mesos import protos as P

Interval = Tuple[int, int]


def _normalize(intervals: Iterable[Interval]) -> List[Interval]:
    out: List[Interval] = []
    for a, b in sorted(intervals):
        if a > b:
            continue
        if out and a <= out[-1][1] + 1:
            if b > out[-1][1]:
                out[-1] = (out[-1][0], b)
        else:
            out.append((a, b))
    return out


def ranges_to_intervals(ranges) -> List[Interval]:
    return [(int(r.begin), int(r.end)) for r in ranges]


def merge_intervals(a: List[Interval], b: List[Interval]) -> List[Interval]:
    return _normalize(list(a) + list(b))


def subtract_intervals(minuend: List[Interval], subtrahend: List[Interval]) -> List[Interval]:
    result = _normalize(minuend)
    for sa, sb in _normalize(subtrahend):
        nxt = []
        for a, b in result:
            if sb < a or sa > b:
                nxt.append((a, b))
                continue
            if a < sa:
                nxt.append((a, sa - 1))
            if sb < b:
                nxt.append((sb + 1, b))
        result = nxt
    return result


def is_in_any(ranges, value: int) -> bool:
    return any(r.begin <= value <= r.end for r in ranges)


def intervals_to_value(intervals: List[Interval]) -> P.Value:
    v = P.Value(type=P.Value.RANGES)
    v.ranges.SetInParent()
    for a, b in intervals:
        v.ranges.range.add(begin=a, end=b)
    return v


def get_value(resource: P.Resource) -> P.Value:
    t = resource.type
    v = P.Value(type=t)
    if t == P.Value.SCALAR:
        v.scalar.CopyFrom(resource.scalar)
    elif t == P.Value.RANGES:
        v.ranges.CopyFrom(resource.ranges)
    elif t == P.Value.SET:
        v.set.CopyFrom(resource.set)
    else:
        raise ValueError(f"Unsupported value type {t} in resource {resource.name}")
    return v


def get_zero(t: int) -> P.Value:
    if t == P.Value.SCALAR:
        v = P.Value(type=t)
        v.scalar.value = 0.0
        return v
    if t == P.Value.RANGES:
        return intervals_to_value([])
    raise ValueError(f"Unsupported type {t} for zero value")


def fixed(x: float) -> float:
    """Mesos scalar precision: values are fixed-point with three decimal digits, so 0.3 - 0.1 is
    0.2 (not 0.19999999999999998) and a merged 0.1 + 0.2 cpus still fits a 0.2 request."""
    return round(x * 1000.0) / 1000.0


def _check_types(a: P.Value, b: P.Value, op: str) -> None:
    if a.type != b.type:
        raise ValueError(f"Values to {op} do not have matching type: {a.type} vs {b.type}")


def add(a: P.Value, b: P.Value) -> P.Value:
    _check_types(a, b, "add")
    if a.type == P.Value.SCALAR:
        v = P.Value(type=a.type)
        v.scalar.value = fixed(a.scalar.value + b.scalar.value)
        return v
    if a.type == P.Value.RANGES:
        return intervals_to_value(merge_intervals(ranges_to_intervals(a.ranges.range),
                                                  ranges_to_intervals(b.ranges.range)))
    raise ValueError(f"Unsupported type {a.type} when adding")


def subtract(a: P.Value, b: P.Value) -> P.Value:
    _check_types(a, b, "subtract")
    if a.type == P.Value.SCALAR:
        v = P.Value(type=a.type)
        v.scalar.value = fixed(a.scalar.value - b.scalar.value)
        return v
    if a.type == P.Value.RANGES:
        return intervals_to_value(subtract_intervals(ranges_to_intervals(a.ranges.range),
                                                     ranges_to_intervals(b.ranges.range)))
    raise ValueError(f"Unsupported type {a.type} when subtracting")


def compare(a: P.Value, b: P.Value) -> int:
    _check_types(a, b, "compare")
    if a.type == P.Value.SCALAR:
        x, y = fixed(a.scalar.value), fixed(b.scalar.value)
        return -1 if x < y else (1 if x > y else 0)
    if a.type == P.Value.RANGES:
        ia = _normalize(ranges_to_intervals(a.ranges.range))
        ib = _normalize(ranges_to_intervals(b.ranges.range))
        if ia == ib:
            return 0
        if not subtract_intervals(ia, ib):
            return -1
        return 1
    raise ValueError(f"Unsupported type {a.type} when comparing")


def equal(a: P.Value, b: P.Value) -> bool:
    return compare(a, b) == 0


def sufficient(desired, available) -> bool:
    """MesosResourcePool.sufficientValue: desired - available <= 0."""
    if desired is None:
        return True
    if available is None:
        return False
    if desired.type == P.Value.SCALAR and available.type == P.Value.SCALAR:
        # the common case (cpus/mem/disk/gpus) without building intermediate Value protos
        return fixed(desired.scalar.value - available.scalar.value) <= 0
    return compare(subtract(desired, available), get_zero(desired.type)) <= 0


def to_string(v: P.Value) -> str:
    if v.type == P.Value.SCALAR:
        return f"scalar {{ value: {v.scalar.value} }}"
    if v.type == P.Value.RANGES:
        return "ranges [" + ", ".join(f"{r.begin}-{r.end}" for r in v.ranges.range) + "]"
    return P.to_text(v)
