"""Map the resources already on a TaskInfo / ExecutorInfo back onto the current specs.

Reference: sdk/.../offer/evaluate/{TaskResourceMapper,ExecutorResourceMapper,ResourceMapperUtils,
ResourceLabels,TaskPortLookup}.java. Matching resources become *update* stages (reuse the
reservation, grow/shrink it), unmatched specs become *create* stages, and unmatched resources
are *orphans* to be unreserved (and destroyed, for executor volumes).
"""
from __future__ import annotations

from typing import Collection, List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer import values as V
from dcos_commons_amd.offer.resources import (
    get_disk_source,
    get_framework_id,
    get_namespace,
    get_persistence_id,
    get_resource_id,
)
from dcos_commons_amd.specification.specs import NamedVIPSpec, PortSpec, ResourceSpec, VolumeSpec

from .stages import (
    NamedVIPEvaluationStage,
    PortEvaluationStage,
    ResourceEvaluationStage,
    VolumeEvaluationStage,
)


class ResourceLabels:
    __slots__ = ("original", "updated", "resource_id", "namespace", "persistence_id", "provider_id",
                 "disk_source", "framework_id")

    def __init__(self, original, updated, resource_id, namespace, persistence_id=None, provider_id=None,
                 disk_source=None, framework_id=None):
        self.original = original
        self.updated = updated
        self.resource_id = resource_id
        self.namespace = namespace
        self.persistence_id = persistence_id
        self.provider_id = provider_id
        self.disk_source = disk_source
        self.framework_id = framework_id


def _label_if_matches(task_value: Optional[str], ours: Optional[str]) -> Optional[str]:
    if task_value is None:
        return None
    if ours is None or ours != task_value:
        return None
    return task_value


def find_matching_disk_spec(resource: P.Resource, specs: List[ResourceSpec], namespace) -> Optional[ResourceLabels]:
    rid = get_resource_id(resource)
    if rid is None:
        return None
    for s in specs:
        if isinstance(s, VolumeSpec) and resource.disk.volume.container_path == s.container_path:
            return ResourceLabels(
                s, s.with_disk_size(resource.scalar.value), rid,
                _label_if_matches(get_namespace(resource), namespace), get_persistence_id(resource),
                resource.provider_id if resource.HasField("provider_id") else None, get_disk_source(resource),
                get_framework_id(resource))
    return None


def find_matching_resource_spec(resource: P.Resource, specs: List[ResourceSpec], namespace,
                                framework_id) -> Optional[ResourceLabels]:
    rid = get_resource_id(resource)
    if rid is None:
        return None
    for s in specs:
        if s.name == resource.name:
            return ResourceLabels(s, s, rid, _label_if_matches(get_namespace(resource), namespace),
                                  framework_id=_label_if_matches(get_framework_id(resource), framework_id))
    return None


def _remove_identity(lst: List, item) -> bool:
    for i, x in enumerate(lst):
        if x is item:
            del lst[i]
            return True
    return False


def _to_stage(task_names, spec, resource_id, namespace, persistence_id, provider_id, disk_source, framework_id):
    if isinstance(spec, NamedVIPSpec):
        return NamedVIPEvaluationStage(spec, task_names, resource_id, namespace, framework_id)
    if isinstance(spec, PortSpec):
        return PortEvaluationStage(spec, task_names, resource_id, namespace, framework_id)
    if isinstance(spec, VolumeSpec):
        return VolumeEvaluationStage.get_existing(spec, task_names, resource_id, namespace, persistence_id,
                                                  provider_id, disk_source, framework_id)
    return ResourceEvaluationStage(spec, task_names, resource_id, namespace, framework_id)


class TaskResourceMapper:
    def __init__(self, task_spec_names: Collection[str], resource_set, task_info: P.TaskInfo, namespace, framework_id):
        self.namespace = namespace
        self.framework_id = framework_id
        self.task_spec_names = list(task_spec_names)
        self.resource_specs: List[ResourceSpec] = list(resource_set.resources) + list(resource_set.volumes)
        self.prior_ports = {p.name: int(p.number) for p in task_info.discovery.ports.ports if p.name}
        self.resources = list(task_info.resources)
        self.orphaned_resources: List[P.Resource] = []
        self.evaluation_stages = self._stages()

    def _find_port(self, resource: P.Resource, specs) -> Optional[ResourceLabels]:
        ranges = resource.ranges.range
        if len(ranges) != 1 or ranges[0].end != ranges[0].begin:
            return None
        rid = get_resource_id(resource)
        if rid is None:
            return None
        for s in specs:
            if not isinstance(s, PortSpec):
                continue
            if s.port == 0:
                prior = self.prior_ports.get(s.port_name)
                if prior is None:
                    continue
                if V.is_in_any(ranges, prior):
                    return ResourceLabels(s, s, rid, _label_if_matches(get_namespace(resource), self.namespace),
                                          framework_id=_label_if_matches(get_framework_id(resource),
                                                                         self.framework_id))
            elif V.is_in_any(ranges, s.port):
                return ResourceLabels(s, s, rid, _label_if_matches(get_namespace(resource), self.namespace),
                                      framework_id=_label_if_matches(get_framework_id(resource), self.framework_id))
        return None

    def _stages(self):
        remaining = list(self.resource_specs)
        matching: List[ResourceLabels] = []
        for r in self.resources:
            if r.name == constants.DISK_RESOURCE_TYPE:
                m = find_matching_disk_spec(r, remaining, self.namespace)
            elif r.name == constants.PORTS_RESOURCE_TYPE:
                m = self._find_port(r, remaining)
            else:
                m = find_matching_resource_spec(r, remaining, self.namespace, self.framework_id)
            if m is not None:
                if not _remove_identity(remaining, m.original):
                    raise ValueError(f"Didn't find {m.original} in {remaining}")
                matching.append(m)
            else:
                self.orphaned_resources.append(r)
        stages = []
        for m in matching:
            stages.append(_to_stage(self.task_spec_names, m.updated, m.resource_id, m.namespace, m.persistence_id,
                                    m.provider_id, m.disk_source, m.framework_id))
        for spec in remaining:
            stages.append(_to_stage(self.task_spec_names, spec, None, self.namespace, None, None, None,
                                    self.framework_id))
        return stages


class ExecutorResourceMapper:
    def __init__(self, pod_spec, resource_specs, executor_resources, namespace, framework_id):
        self.volume_specs = list(pod_spec.volumes)
        self.resource_specs = list(resource_specs)
        self.executor_resources = list(executor_resources)
        self.namespace = namespace
        self.framework_id = framework_id
        self.orphaned_resources: List[P.Resource] = []
        self.evaluation_stages = self._stages()

    def _stages(self):
        remaining: List[ResourceSpec] = list(self.volume_specs) + list(self.resource_specs)
        matching: List[ResourceLabels] = []
        for r in self.executor_resources:
            if r.name == constants.DISK_RESOURCE_TYPE and r.HasField("disk"):
                m = find_matching_disk_spec(r, remaining, self.namespace)
            else:
                m = find_matching_resource_spec(r, remaining, self.namespace, self.framework_id)
            if m is not None:
                if not _remove_identity(remaining, m.original):
                    raise ValueError(f"Didn't find {m.original} in {remaining}")
                matching.append(m)
            elif r.HasField("disk"):
                self.orphaned_resources.append(r)
        stages = []
        for m in matching:
            if isinstance(m.updated, VolumeSpec):
                stages.append(VolumeEvaluationStage.get_existing(m.updated, [], m.resource_id, m.namespace,
                                                                 m.persistence_id, m.provider_id, m.disk_source,
                                                                 m.framework_id))
            else:
                stages.append(ResourceEvaluationStage(m.updated, [], m.resource_id, m.namespace, m.framework_id))
        for spec in remaining:
            if isinstance(spec, VolumeSpec):
                stages.append(VolumeEvaluationStage.get_new(spec, [], self.namespace, self.framework_id))
            else:
                stages.append(ResourceEvaluationStage(spec, [], None, self.namespace, self.framework_id))
        return stages
