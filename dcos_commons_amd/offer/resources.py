"""Resource helpers: ``MesosResource``, ``ResourceUtils`` and ``ResourceBuilder``.

Reference: sdk/.../offer/{MesosResource,ResourceUtils,ResourceBuilder}.java. Reserved resources
carry the labels ``resource_id``, ``framework_id`` and ``namespace`` on their (last, refined)
``ReservationInfo``; a pre-reserved role adds a STATIC reservation beneath the DYNAMIC one.
"""
from __future__ import annotations

from typing import Iterable, List, Optional

from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.taskdata import labels as L
from dcos_commons_amd.specification.specs import (
    ANY_ROLE,
    DISK_RESOURCE_TYPE,
    ResourceSpec,
    VolumeSpec,
    VolumeType,
)
from dcos_commons_amd.utils.ids import uuid4_str

from . import values as V

MOUNT = P.Resource.DiskInfo.Source.MOUNT


# ---------------------------------------------------------------------------------------
# ResourceUtils


def get_reservation(resource: P.Resource) -> Optional[P.Resource.ReservationInfo]:
    if len(resource.reservations) > 0:
        return resource.reservations[-1]
    if resource.HasField("reservation"):
        return resource.reservation
    return None


def get_resource_id(resource: P.Resource) -> Optional[str]:
    r = get_reservation(resource)
    return L.get_resource_id(r) if r is not None else None


def has_resource_id(resource: P.Resource) -> bool:
    return get_resource_id(resource) is not None


def get_framework_id(resource: P.Resource) -> Optional[str]:
    r = get_reservation(resource)
    return L.get_framework_id(r) if r is not None else None


def get_namespace(resource: P.Resource) -> Optional[str]:
    r = get_reservation(resource)
    return L.get_resource_namespace(r) if r is not None else None


def get_principal(resource: P.Resource) -> Optional[str]:
    r = get_reservation(resource)
    return r.principal if r is not None else None


def get_persistence_id(resource: P.Resource) -> Optional[str]:
    if resource.HasField("disk") and resource.disk.HasField("persistence"):
        return resource.disk.persistence.id
    return None


def is_mount_volume(resource: P.Resource) -> bool:
    return (resource.HasField("disk") and resource.disk.HasField("source")
            and resource.disk.source.HasField("type") and resource.disk.source.type == MOUNT)


def get_disk_source(resource: P.Resource) -> Optional[P.Resource.DiskInfo.Source]:
    return resource.disk.source if is_mount_volume(resource) else None


def get_role(resource: P.Resource) -> str:
    return MesosResource(resource).role


def get_all_resources(task_info: P.TaskInfo) -> List[P.Resource]:
    out = list(task_info.resources)
    if task_info.HasField("executor"):
        out.extend(task_info.executor.resources)
    return out


def get_all_resources_of(task_infos: Iterable[P.TaskInfo]) -> List[P.Resource]:
    out: List[P.Resource] = []
    for t in task_infos:
        out.extend(get_all_resources(t))
    return out


def get_resource_ids(resources: Iterable[P.Resource]) -> List[str]:
    seen, out = set(), []
    for r in resources:
        rid = get_resource_id(r)
        if rid is not None and rid not in seen:
            seen.add(rid)
            out.append(rid)
    return out


def _dynamic_reservations(resource: P.Resource):
    res = list(resource.reservations)
    if resource.HasField("reservation"):
        res.append(resource.reservation)
    return [r for r in res if r.HasField("type") and r.type == P.Resource.ReservationInfo.DYNAMIC]


def is_processable(resource: P.Resource, our_roles, framework_id: Optional[str]) -> bool:
    """Filters foreign dynamic reservations out of incoming offers (ResourceUtils.isProcessable)."""
    dyn = _dynamic_reservations(resource)
    if not dyn:
        return True
    roles = {r.role for r in dyn}
    if resource.HasField("role"):
        roles.add(resource.role)
    roles.discard(ANY_ROLE)
    resource_id_present = has_resource_id(resource)
    reservation_is_ours = roles <= set(our_roles)
    fid = get_framework_id(resource)
    fid_present = fid is not None and framework_id is not None
    fid_processable = (not fid_present) or fid == framework_id
    return resource_id_present and reservation_is_ours and fid_processable


# ---------------------------------------------------------------------------------------
# MesosResource


class MesosResource:
    __slots__ = ("resource",)

    def __init__(self, resource: P.Resource):
        self.resource = resource

    def is_atomic(self) -> bool:
        return is_mount_volume(self.resource)

    @property
    def name(self) -> str:
        return self.resource.name

    @property
    def type(self) -> int:
        return self.resource.type

    @property
    def resource_id(self) -> Optional[str]:
        return get_resource_id(self.resource)

    def has_resource_id(self) -> bool:
        return self.resource_id is not None

    @property
    def value(self) -> P.Value:
        return V.get_value(self.resource)

    @property
    def role(self) -> str:
        if len(self.resource.reservations) > 0:
            return self.resource.reservations[-1].role
        return ANY_ROLE

    @property
    def previous_role(self) -> str:
        n = len(self.resource.reservations)
        if n > 0:
            if n <= 1:
                return self.resource.role
            return self.resource.reservations[n - 2].role
        return ANY_ROLE

    @property
    def principal(self) -> Optional[str]:
        if self.resource.HasField("reservation") and self.resource.reservation.HasField("principal"):
            return self.resource.reservation.principal
        return None

    def __repr__(self):
        return f"MesosResource({self.resource.name}={V.to_string(self.value)}, id={self.resource_id})"


# ---------------------------------------------------------------------------------------
# ResourceBuilder


def _set_value(r: P.Resource, value: P.Value, fresh: bool = False) -> None:
    r.type = value.type
    if not fresh:
        r.ClearField("scalar")
        r.ClearField("ranges")
        r.ClearField("set")
    if value.type == P.Value.SCALAR:
        r.scalar.CopyFrom(value.scalar)
    elif value.type == P.Value.RANGES:
        r.ranges.CopyFrom(value.ranges)
    elif value.type == P.Value.SET:
        r.set.CopyFrom(value.set)
    else:
        raise ValueError(f"Unsupported spec value type: {value.type}")


def unreserved_resource(name: str, value: P.Value) -> P.Resource:
    """``ResourceBuilder.from_unreserved_value(name, value).build()`` without the builder: an
    unreserved ``*`` resource (the pool's view of what a consumption took from an offer)."""
    r = P.Resource(name=name, role=ANY_ROLE)
    _set_value(r, value, True)
    return r


class ResourceBuilder:
    def __init__(self, name: str, value: P.Value, pre_reserved_role: str = ANY_ROLE):
        self.name = name
        self.value = value
        self.pre_reserved_role = pre_reserved_role or ANY_ROLE
        self.role: Optional[str] = None
        self.principal: Optional[str] = None
        self.resource_id: Optional[str] = None
        self.resource_namespace: Optional[str] = None
        self.disk_container_path: Optional[str] = None
        self.disk_persistence_id: Optional[str] = None
        self.provider_id = None
        self.disk_source = None
        self.mesos_resource: Optional[MesosResource] = None
        self.framework_id: Optional[str] = None
        self.built_resource_id: Optional[str] = None  # the id ``build`` wrote into the reservation

    @staticmethod
    def from_spec(spec: ResourceSpec, resource_id: Optional[str] = None, resource_namespace: Optional[str] = None,
                  framework_id: Optional[str] = None) -> "ResourceBuilder":
        b = ResourceBuilder(spec.name, spec.value, spec.pre_reserved_role)
        b.role = spec.role
        b.principal = spec.principal
        b.resource_id = resource_id
        b.resource_namespace = resource_namespace
        b.framework_id = framework_id
        return b

    @staticmethod
    def from_volume_spec(spec: VolumeSpec, resource_id: Optional[str], resource_namespace: Optional[str],
                         persistence_id: Optional[str], provider_id, disk_source,
                         framework_id: Optional[str]) -> "ResourceBuilder":
        b = ResourceBuilder.from_spec(spec, resource_id, resource_namespace, framework_id)
        b.provider_id = provider_id
        if spec.type == VolumeType.ROOT:
            if disk_source is not None:
                raise ValueError("Source must not be set on a ROOT volume")
            return b.set_root_volume(spec.container_path, persistence_id)
        if spec.type == VolumeType.MOUNT:
            if disk_source is None:
                raise ValueError("Source must be set on a MOUNT volume")
            return b.set_mount_volume(spec.container_path, persistence_id, disk_source)
        raise ValueError(f"Unexpected disk type: {spec.type}")

    @staticmethod
    def _existing_roles(resource: P.Resource):
        """(role, pre-reserved role) of a resource we reserved. A legacy reservation (no
        ``reservations`` stack) carries our role in ``resource.role``; the reference reads only
        the stack and so rebuilds legacy resources as ``*`` (ResourceBuilder.java:139-161)."""
        if len(resource.reservations) == 0 and resource.HasField("reservation"):
            return resource.role or ANY_ROLE, ANY_ROLE
        return get_role(resource), resource.role or ANY_ROLE

    @staticmethod
    def from_existing_resource(resource: P.Resource) -> "ResourceBuilder":
        role, pre_reserved_role = ResourceBuilder._existing_roles(resource)
        if not resource.HasField("disk"):
            if not has_resource_id(resource):
                raise ValueError("Cannot generate resource spec from resource which has not been reserved by the SDK.")
            spec = ResourceSpec(name=resource.name, value=V.get_value(resource), role=role,
                                principal=get_principal(resource) or "", pre_reserved_role=pre_reserved_role)
            return ResourceBuilder.from_spec(spec, get_resource_id(resource), get_namespace(resource),
                                             get_framework_id(resource))
        disk = resource.disk
        if disk.HasField("source"):
            profiles = [disk.source.profile] if disk.source.HasField("profile") else []
            spec = VolumeSpec(name=DISK_RESOURCE_TYPE, value=V.get_value(resource), role=role,
                              principal=disk.persistence.principal, pre_reserved_role=pre_reserved_role,
                              type=VolumeType.MOUNT, container_path=disk.volume.container_path,
                              profiles=tuple(profiles))
        else:
            spec = VolumeSpec(name=DISK_RESOURCE_TYPE, value=V.get_value(resource), role=role,
                              principal=disk.persistence.principal, pre_reserved_role=pre_reserved_role,
                              type=VolumeType.ROOT, container_path=disk.volume.container_path)
        return ResourceBuilder.from_volume_spec(
            spec, get_resource_id(resource), get_namespace(resource), get_persistence_id(resource),
            resource.provider_id if resource.HasField("provider_id") else None, get_disk_source(resource),
            get_framework_id(resource))

    @staticmethod
    def from_unreserved_value(name: str, value: P.Value) -> "ResourceBuilder":
        return ResourceBuilder(name, value, ANY_ROLE)

    def set_value(self, value: P.Value) -> "ResourceBuilder":
        self.value = value
        return self

    def set_resource_id(self, rid: str) -> "ResourceBuilder":
        self.resource_id = rid
        return self

    def set_root_volume(self, container_path: str, persistence_id: Optional[str]) -> "ResourceBuilder":
        if self.name != DISK_RESOURCE_TYPE:
            raise ValueError("Refusing to set disk information against resource of type: " + self.name)
        self.disk_container_path = container_path
        self.disk_persistence_id = persistence_id
        return self

    def set_mount_volume(self, container_path: str, persistence_id: Optional[str], disk_source) -> "ResourceBuilder":
        self.set_root_volume(container_path, persistence_id)
        if disk_source.type != MOUNT:
            raise ValueError(f"Expecting disk source to be of type MOUNT: {disk_source}")
        self.disk_source = disk_source
        return self

    def set_mesos_resource(self, mr: MesosResource) -> "ResourceBuilder":
        self.mesos_resource = mr
        return self

    def _reservation_labels(self, labels: P.Labels) -> None:
        """resource_id / framework_id / namespace labels, in the key order ``map_to_labels`` writes
        (sorted: framework_id < namespace < resource_id)."""
        rid = self.resource_id or uuid4_str()
        self.built_resource_id = rid
        if self.framework_id is not None:
            labels.labels.add(key=L.FRAMEWORK_ID_RESERVATION_LABEL, value=self.framework_id)
        if self.resource_namespace is not None:
            labels.labels.add(key=L.NAMESPACE_RESERVATION_LABEL, value=self.resource_namespace)
        labels.labels.add(key=L.RESOURCE_ID_RESERVATION_LABEL, value=rid)

    def _reservation(self) -> P.Resource.ReservationInfo:
        r = P.Resource.ReservationInfo(role=self.role, type=P.Resource.ReservationInfo.DYNAMIC,
                                       principal=self.principal or "")
        self._reservation_labels(r.labels)
        return r

    def build(self) -> P.Resource:
        r = P.Resource()
        fresh = self.mesos_resource is None
        if not fresh:
            r.CopyFrom(self.mesos_resource.resource)
            r.ClearField("allocation_info")
        r.name = self.name
        r.role = ANY_ROLE
        r.type = self.value.type
        caps = capabilities.get_instance()
        pre_reserved_supported = caps.supports_pre_reserved_resources
        if self.role is not None and not has_resource_id(r):
            if pre_reserved_supported:
                if self.pre_reserved_role != ANY_ROLE and self.mesos_resource is None:
                    r.reservations.add(role=self.pre_reserved_role, type=P.Resource.ReservationInfo.STATIC)
                res = r.reservations.add(role=self.role, type=P.Resource.ReservationInfo.DYNAMIC,
                                         principal=self.principal or "")
                self._reservation_labels(res.labels)
            else:
                r.reservation.principal = self.principal or ""
                self._reservation_labels(r.reservation.labels)
        if self.role is not None and not pre_reserved_supported:
            r.role = self.role
        elif pre_reserved_supported and len(r.reservations) > 0:
            r.ClearField("role")
        if self.provider_id is not None:
            r.provider_id.CopyFrom(self.provider_id)
        if self.disk_container_path is not None:
            r.disk.volume.container_path = self.disk_container_path
            r.disk.volume.mode = P.Volume.RW
            r.disk.persistence.principal = self.principal or ""
            r.disk.persistence.id = self.disk_persistence_id or uuid4_str()
            if self.disk_source is not None:
                r.disk.source.CopyFrom(self.disk_source)
        _set_value(r, self.value, fresh)
        return r


# A placeholder resource_id of the length of every generated one (str(uuid4()): 36 characters),
# swapped for the real id in the serialized template.
_ID_PLACEHOLDER = "rrrrrrrr-rrrr-4rrr-8rrr-rrrrrrrrrrrr"
_NEW_RESERVATIONS: dict = {}


def new_reservation(spec: ResourceSpec, namespace: Optional[str], framework_id: Optional[str]):
    """``ResourceBuilder.from_spec(spec, None, namespace, framework_id).build()`` for a new
    reservation of a plain offered chunk, and its generated resource id, from a per-spec wire
    template: every pod of a pod type reserves the same cpus/mem/disk/gpus with the same role,
    principal and labels, so only the resource id differs. The template is built once with a
    placeholder id of the same length, which is replaced in the serialized bytes; the result is
    parsed in C instead of assembled field by field in Python (about 8 resources per pod launch)."""
    pre = capabilities.get_instance().supports_pre_reserved_resources
    key = (id(spec), namespace, framework_id, pre)
    hit = _NEW_RESERVATIONS.get(key)
    if hit is None or hit[0] is not spec:
        b = ResourceBuilder.from_spec(spec, _ID_PLACEHOLDER, namespace, framework_id)
        data = b.build().SerializeToString()
        if data.count(_ID_PLACEHOLDER.encode()) != 1:
            hit = (spec, None)
        else:
            hit = (spec, data)
        if len(_NEW_RESERVATIONS) > 4096:
            _NEW_RESERVATIONS.clear()
        _NEW_RESERVATIONS[key] = hit
    rid = uuid4_str()
    if hit[1] is None:   # a layout the template cannot stand for: build it the long way
        b = ResourceBuilder.from_spec(spec, rid, namespace, framework_id)
        return b.build(), rid
    return P.Resource.FromString(hit[1].replace(_ID_PLACEHOLDER.encode(), rid.encode(), 1)), rid


_PERSISTENCE_PLACEHOLDER = "pppppppp-pppp-4ppp-8ppp-pppppppppppp"
_NEW_ROOT_VOLUMES: dict = {}


def new_root_volume(spec: VolumeSpec, resource_id: str, namespace: Optional[str],
                    framework_id: Optional[str]) -> P.Resource:
    """``ResourceBuilder.from_volume_spec(spec, resource_id, namespace, None, None, None,
    framework_id).build()`` of a new ROOT volume on a plain disk chunk (a fresh persistence id),
    from a per-spec wire template with placeholder resource and persistence ids (see
    ``new_reservation``)."""
    pre = capabilities.get_instance().supports_pre_reserved_resources
    key = (id(spec), namespace, framework_id, pre)
    hit = _NEW_ROOT_VOLUMES.get(key)
    if hit is None or hit[0] is not spec:
        b = ResourceBuilder.from_volume_spec(spec, _ID_PLACEHOLDER, namespace, _PERSISTENCE_PLACEHOLDER, None, None,
                                             framework_id)
        data = b.build().SerializeToString()
        ok = data.count(_ID_PLACEHOLDER.encode()) == 1 and data.count(_PERSISTENCE_PLACEHOLDER.encode()) == 1
        hit = (spec, data if ok else None)
        if len(_NEW_ROOT_VOLUMES) > 4096:
            _NEW_ROOT_VOLUMES.clear()
        _NEW_ROOT_VOLUMES[key] = hit
    if hit[1] is None:
        return ResourceBuilder.from_volume_spec(spec, resource_id, namespace, None, None, None, framework_id).build()
    data = hit[1].replace(_ID_PLACEHOLDER.encode(), resource_id.encode(), 1)
    return P.Resource.FromString(data.replace(_PERSISTENCE_PLACEHOLDER.encode(), uuid4_str().encode(), 1))
