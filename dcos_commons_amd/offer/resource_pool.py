"""Per-offer consumable resource pool.

Reference: sdk/.../offer/MesosResourcePool.java:24-456. An offer's resources are split into
* an unreserved *atomic* pool (MOUNT disks: consumed whole),
* a *reserved* pool keyed by ``resource_id`` (our prior reservations),
* an unreserved *merged* pool keyed by role (scalars summed, ranges merged).
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional

from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.specification.specs import ANY_ROLE, VolumeSpec

from . import values as V
from .resources import MesosResource, ResourceBuilder, get_disk_source, unreserved_resource

LOGGER = logging.getLogger(__name__)


def _consumable(pod_role: Optional[str], resource: P.Resource) -> bool:
    if pod_role is None or not resource.HasField("allocation_info") or not resource.allocation_info.HasField("role"):
        return True
    return pod_role == resource.allocation_info.role


class MesosResourcePool:
    def __init__(self, offer: P.Offer, role: Optional[str] = None):
        self.offer = offer
        resources = [MesosResource(r) for r in offer.resources if _consumable(role, r)]
        self.unreserved_atomic_pool: Dict[str, List[MesosResource]] = {}
        self.reserved_pool: Dict[str, MesosResource] = {}
        self.merged_pool_by_role: Dict[str, Dict[str, P.Value]] = {}
        for mr in resources:
            rid = mr.resource_id
            if rid is not None:
                self.reserved_pool[rid] = mr
            elif mr.is_atomic():
                self.unreserved_atomic_pool.setdefault(mr.name, []).append(mr)
            else:
                pool = self.merged_pool_by_role.setdefault(mr.role, {})
                cur = pool.get(mr.name)
                pool[mr.name] = mr.value if cur is None else V.add(cur, mr.value)

    # -- views -------------------------------------------------------------------------
    def unreserved_merged_pool(self) -> Dict[str, P.Value]:
        return self.merged_pool_by_role.get(ANY_ROLE, {})

    def unreserved_merged_pool_by_role(self, role: str) -> Dict[str, P.Value]:
        return self.merged_pool_by_role.get(role, {})

    def get_reserved_resource_by_id(self, rid: str) -> Optional[MesosResource]:
        return self.reserved_pool.get(rid)

    # -- consumption -------------------------------------------------------------------
    def consume_reserved(self, name: str, value: P.Value, resource_id: str) -> Optional[MesosResource]:
        mr = self.reserved_pool.get(resource_id)
        if mr is None:
            LOGGER.debug("Failed to find reserved %s resource with resource id %s", name, resource_id)
            return None
        if mr.is_atomic():
            if V.sufficient(value, mr.value):
                del self.reserved_pool[resource_id]
            else:
                LOGGER.warning("Reserved atomic quantity of %s is insufficient: desired %s, reserved %s",
                               name, V.to_string(value), V.to_string(mr.value))
                return None
        else:
            available = mr.value
            if V.compare(available, value) > 0:
                remaining = ResourceBuilder.from_existing_resource(mr.resource).set_value(
                    V.subtract(available, value)).build()
                self.reserved_pool[resource_id] = MesosResource(remaining)
            else:
                del self.reserved_pool[resource_id]
        return mr

    def consume_atomic(self, name: str, spec: VolumeSpec) -> Optional[MesosResource]:
        atomic = self.unreserved_atomic_pool.get(name)
        found = None
        remaining = []
        for mr in atomic or []:
            src = get_disk_source(mr.resource)
            profile = src.profile if src is not None and src.HasField("profile") else None
            profile_ok = (profile in spec.profiles) if profile is not None else not spec.profiles
            if found is None and V.sufficient(spec.value, mr.value) and profile_ok:
                found = mr
            else:
                remaining.append(mr)
        if remaining:
            self.unreserved_atomic_pool[name] = remaining
        else:
            self.unreserved_atomic_pool.pop(name, None)
        return found

    def consume_reservable_merged(self, name: str, desired: P.Value, pre_reserved_role: str) -> Optional[MesosResource]:
        pool = self.merged_pool_by_role.get(pre_reserved_role)
        if pool is None:
            LOGGER.debug("No unreserved resources available for role '%s'", pre_reserved_role)
            return None
        available = pool.get(name)
        if not V.sufficient(desired, available):
            return None
        pool[name] = V.subtract(available, desired)
        r = unreserved_resource(name, desired)
        if capabilities.get_instance().supports_pre_reserved_resources and pre_reserved_role != ANY_ROLE:
            r.reservations.add(role=pre_reserved_role, type=P.Resource.ReservationInfo.STATIC)
        return MesosResource(r)

    def free(self, mr: MesosResource) -> None:
        if mr.is_atomic():
            r = P.Resource()
            r.CopyFrom(mr.resource)
            r.ClearField("reservation")
            r.role = ANY_ROLE
            if r.HasField("disk"):
                r.disk.ClearField("persistence")
                r.disk.ClearField("volume")
            self.unreserved_atomic_pool.setdefault(mr.name, []).append(MesosResource(r))
            return
        rid = mr.resource_id
        if rid is not None:
            self.reserved_pool.pop(rid, None)
        prev = mr.previous_role
        pool = self.merged_pool_by_role.setdefault(prev, {})
        cur = pool.get(mr.name)
        pool[mr.name] = V.add(cur if cur is not None else V.get_zero(mr.type), mr.value)
