"""Shared builders for unit suites: constants, resources, offers, tasks, statuses.

The reference keeps the same helpers under sdk/scheduler/src/test/java/com/mesosphere/sdk/testutils/
({TestConstants,ResourceTestUtils,OfferTestUtils,TaskTestUtils}.java). Names follow them so a
reference test reads across one to one; values (IDs, hostnames, roles) are the reference's too.
"""
from __future__ import annotations

import random
from typing import Iterable, List, Optional, Sequence

from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.common_id_utils import to_executor_id, to_task_id
from dcos_commons_amd.offer.resources import ResourceBuilder
from dcos_commons_amd.offer.taskdata import labels as L
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.specification.specs import ANY_ROLE, VolumeSpec
from dcos_commons_amd.utils.ids import uuid4_str  # noqa: F401 (re-exported for suites)

# ---------------------------------------------------------------------------------------
# TestConstants

SERVICE_NAME = "service-name"
SERVICE_USER = "service-user"
CONTAINER_PATH = "test-container-path"
EXECUTOR_NAME = "test-executor-name"
HOSTNAME = "test-hostname"
PERSISTENCE_ID = "test-persistence-id"
PRINCIPAL = "test-principal"
ROLE = "test-role"
PRE_RESERVED_ROLE = "base-role"
TASK_NAME = "test-task-name"
TASK_TYPE = "test-task-type"
TASK_INDEX = 0
POD_TYPE = "pod-type"
RESOURCE_ID = "test-resource-id"
RESOURCE_SET_ID = "test-resource-set-id"
PORT_ENV_NAME = "TEST_PORT_NAME"
PORT_API_VALUE = 8080
ZONE = "zone"
LOCAL_REGION = "local"
REMOTE_REGION = "remote"

OFFER_ID = P.OfferID(value="test-offer-id")
AGENT_ID = P.AgentID(value="test-slave-id")
FRAMEWORK_ID = P.FrameworkID(value="test-framework-id")
EXECUTOR_ID = to_executor_id(SERVICE_NAME, EXECUTOR_NAME)
TASK_ID = to_task_id(SERVICE_NAME, TASK_NAME)

MOUNT_DISK_SOURCE = P.Resource.DiskInfo.Source(
    type=P.Resource.DiskInfo.Source.MOUNT, mount=P.Resource.DiskInfo.Source.Mount(root="/mnt/source"))


def domain_info(region: str) -> P.DomainInfo:
    d = P.DomainInfo()
    d.fault_domain.zone.name = ZONE
    d.fault_domain.region.name = region
    return d


LOCAL_DOMAIN_INFO = domain_info(LOCAL_REGION)
REMOTE_DOMAIN_INFO = domain_info(REMOTE_REGION)


# ---------------------------------------------------------------------------------------
# ResourceTestUtils


def _unreserved(name: str, value: P.Value, role: str = ANY_ROLE) -> P.Resource:
    r = P.Resource(name=name, type=value.type, role=role)
    if role != ANY_ROLE:
        r.reservations.add(role=role, principal=PRINCIPAL)
    if value.type == P.Value.SCALAR:
        r.scalar.CopyFrom(value.scalar)
    elif value.type == P.Value.RANGES:
        r.ranges.CopyFrom(value.ranges)
    else:
        r.set.CopyFrom(value.set)
    return r


def scalar_value(v: float) -> P.Value:
    return P.Value(type=P.Value.SCALAR, scalar=P.Value.Scalar(value=v))


def ranges_value(*pairs) -> P.Value:
    val = P.Value(type=P.Value.RANGES)
    for b, e in pairs:
        val.ranges.range.add(begin=b, end=e)
    return val


def unreserved_cpus(v: float, pre_reserved_role: str = ANY_ROLE) -> P.Resource:
    return _unreserved("cpus", scalar_value(v), pre_reserved_role)


def unreserved_mem(v: float, pre_reserved_role: str = ANY_ROLE) -> P.Resource:
    return _unreserved("mem", scalar_value(v), pre_reserved_role)


def unreserved_disk(v: float, pre_reserved_role: str = ANY_ROLE) -> P.Resource:
    return _unreserved("disk", scalar_value(v), pre_reserved_role)


def unreserved_ports(begin: int, end: int) -> P.Resource:
    return _unreserved("ports", ranges_value((begin, end)))


def prereserved_port(begin: int, end: int, pre_reserved_role: str) -> P.Resource:
    return _unreserved("ports", ranges_value((begin, end)), pre_reserved_role)


def unreserved_mount_volume(size: float, profile: Optional[str] = None) -> P.Resource:
    r = unreserved_disk(size)
    r.disk.source.CopyFrom(MOUNT_DISK_SOURCE)
    if profile is not None:
        r.disk.source.profile = profile
    return r


def add_reservation(r: P.Resource, resource_id: str) -> P.Resource:
    """ResourceTestUtils.addReservation: the labels go on the refined (last) reservation when the
    cluster supports pre-reserved resources, else on the legacy ``reservation`` field."""
    if capabilities.get_instance().supports_pre_reserved_resources:
        res = r.reservations.add(role=ROLE, principal=PRINCIPAL)
    else:
        r.role = ROLE
        res = r.reservation
        res.principal = PRINCIPAL
    L.set_reservation_label(res, L.RESOURCE_ID_RESERVATION_LABEL, resource_id)
    L.set_reservation_label(res, L.NAMESPACE_RESERVATION_LABEL, SERVICE_NAME)
    L.set_reservation_label(res, L.FRAMEWORK_ID_RESERVATION_LABEL, FRAMEWORK_ID.value)
    return r


def reserved_cpus(v: float, resource_id: str) -> P.Resource:
    return add_reservation(unreserved_cpus(v), resource_id)


def reserved_mem(v: float, resource_id: str) -> P.Resource:
    return add_reservation(unreserved_mem(v), resource_id)


def reserved_disk(v: float, resource_id: str) -> P.Resource:
    return add_reservation(unreserved_disk(v), resource_id)


def reserved_ports(begin: int, end: int, resource_id: str) -> P.Resource:
    return add_reservation(unreserved_ports(begin, end), resource_id)


def reserved_mount_volume(size: float, profile: Optional[str] = None, resource_id: str = RESOURCE_ID,
                          persistence_id: str = PERSISTENCE_ID) -> P.Resource:
    r = unreserved_mount_volume(size, profile)
    r.disk.persistence.id = persistence_id
    r.disk.persistence.principal = PRINCIPAL
    r.disk.volume.container_path = CONTAINER_PATH
    r.disk.volume.mode = P.Volume.RW
    return add_reservation(r, resource_id)


def reserved_root_volume(size: float, resource_id: str = RESOURCE_ID, persistence_id: str = PERSISTENCE_ID,
                         framework_id: Optional[str] = None) -> P.Resource:
    spec = VolumeSpec.create_root_volume(size, CONTAINER_PATH, ROLE, ANY_ROLE, PRINCIPAL)
    return ResourceBuilder.from_volume_spec(spec, resource_id, None, persistence_id, None, None,
                                            framework_id).build()


# ---------------------------------------------------------------------------------------
# OfferTestUtils


def empty_offer(offer_id: P.OfferID = OFFER_ID, hostname: str = HOSTNAME) -> P.Offer:
    o = P.Offer(hostname=hostname)
    o.id.CopyFrom(offer_id)
    o.framework_id.CopyFrom(FRAMEWORK_ID)
    o.agent_id.CopyFrom(AGENT_ID)
    return o


def get_offer(resources: Iterable[P.Resource] = (), **kw) -> P.Offer:
    o = empty_offer(**kw)
    o.resources.extend(resources)
    return o


def executor_resources(pre_reserved_role: str = ANY_ROLE) -> List[P.Resource]:
    return [unreserved_cpus(0.1, pre_reserved_role), unreserved_mem(256, pre_reserved_role),
            unreserved_disk(512, pre_reserved_role)]


def complete_offer(resources: Iterable[P.Resource] = (), pre_reserved_role: str = ANY_ROLE, **kw) -> P.Offer:
    o = empty_offer(**kw)
    o.resources.extend(executor_resources(pre_reserved_role))
    o.resources.extend(resources)
    return o


# ---------------------------------------------------------------------------------------
# TaskTestUtils


def get_task_info(resources: Sequence[P.Resource] = (), index: Optional[int] = None, name: str = TASK_NAME,
                  task_id: Optional[P.TaskID] = None) -> P.TaskInfo:
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(task_id if task_id is not None else TASK_ID)
    t.agent_id.CopyFrom(AGENT_ID)
    t.command.value = "echo test"
    t.container.type = P.ContainerInfo.MESOS
    w = TaskLabelWriter(t)
    w.set_type(TASK_TYPE)
    w.set_index(random.randrange(1 << 31) if index is None else index)
    t.labels.CopyFrom(w.to_proto())
    for r in resources:
        if r.name == "ports":
            res = r.reservations[-1] if len(r.reservations) else r.reservation
            if L.get_resource_id(res):
                t.command.environment.variables.add(name=PORT_ENV_NAME, value=str(r.ranges.range[0].begin))
    t.resources.extend(resources)
    return t


def executor_info(resources: Sequence[P.Resource] = (), executor_id: str = "") -> P.ExecutorInfo:
    e = P.ExecutorInfo(name=EXECUTOR_NAME)
    e.executor_id.value = executor_id
    e.command.SetInParent()
    e.resources.extend(resources)
    return e


def generate_status(task_id: P.TaskID, state: int, ready: Optional[bool] = None) -> P.TaskStatus:
    s = P.TaskStatus(state=state)
    s.task_id.CopyFrom(task_id)
    if ready is not None:
        s.labels.labels.add(key=L.READINESS_CHECK_PASSED_LABEL, value=str(ready).lower())
    return s


def with_labels(task: P.TaskInfo, fn) -> P.TaskInfo:
    """Applies ``fn(TaskLabelWriter)`` to a copy of ``task`` and returns it."""
    c = P.TaskInfo()
    c.CopyFrom(task)
    w = TaskLabelWriter(c)
    fn(w)
    c.labels.CopyFrom(w.to_proto())
    return c


def with_failed_flag(task: P.TaskInfo) -> P.TaskInfo:
    return with_labels(task, lambda w: w.set_permanently_failed())
