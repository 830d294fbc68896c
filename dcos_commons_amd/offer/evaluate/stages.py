"""Offer evaluation pipeline stages.

Reference: sdk/.../offer/evaluate/{OfferEvaluationStage,ExecutorEvaluationStage,
PlacementRuleEvaluationStage,ResourceEvaluationStage,PortEvaluationStage,NamedVIPEvaluationStage,
VolumeEvaluationStage,LaunchEvaluationStage,UnreserveEvaluationStage,DestroyEvaluationStage,
OfferEvaluationUtils}.java. Each stage consumes from the per-offer ``MesosResourcePool`` and
mutates the ``PodInfoBuilder``; its ``EvaluationOutcome`` carries RESERVE/CREATE/LAUNCH_GROUP/...
recommendations.
"""
from __future__ import annotations

import logging
from typing import Collection, Optional

from dcos_commons_amd.dcos import constants as dcos
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import common_id_utils
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer import values as V
from dcos_commons_amd.offer.recommendations import (
    CreateOfferRecommendation,
    DestroyOfferRecommendation,
    LaunchOfferRecommendation,
    ReserveOfferRecommendation,
    StoreTaskInfoRecommendation,
    UnreserveOfferRecommendation,
)
from dcos_commons_amd.offer.resource_pool import MesosResourcePool
from dcos_commons_amd.offer.resources import (
    MesosResource,
    ResourceBuilder,
    get_disk_source,
    get_resource_id,
    new_reservation,
    new_root_volume,
)
from dcos_commons_amd.offer.taskdata import labels as L
from dcos_commons_amd.specification.specs import (
    NamedVIPSpec,
    PortSpec,
    ResourceSpec,
    VolumeSpec,
    VolumeType,
    ranges_value,
)

from .outcome import EvaluationOutcome
from .pod_info_builder import PodInfoBuilder

LOGGER = logging.getLogger(__name__)


class OfferEvaluationStage:
    def evaluate(self, pool: MesosResourcePool, builder: PodInfoBuilder) -> EvaluationOutcome:
        raise NotImplementedError


# ---------------------------------------------------------------------------------------
# OfferEvaluationUtils


class ReserveEvaluationOutcome:
    """``resource``: for a brand-new reservation of exactly the spec's value, the reserved
    resource as built from the spec (the task carries the same resource, so it is not rebuilt)."""

    __slots__ = ("outcome", "resource_id", "resource")

    def __init__(self, outcome: EvaluationOutcome, resource_id: Optional[str], resource=None):
        self.outcome = outcome
        self.resource_id = resource_id
        self.resource = resource


def evaluate_simple_resource(stage, spec: ResourceSpec, resource_id: Optional[str], namespace: Optional[str],
                             pool: MesosResourcePool, framework_id: Optional[str]) -> ReserveEvaluationOutcome:
    if resource_id is None:
        mr = pool.consume_reservable_merged(spec.name, spec.value, spec.pre_reserved_role)
    else:
        mr = pool.consume_reserved(spec.name, spec.value, resource_id)
    if mr is None:
        if resource_id is None:
            return ReserveEvaluationOutcome(EvaluationOutcome.fail(
                stage, "Offer lacks sufficient unreserved '%s' with role '%s' for new reservation: '%s'",
                spec.name, spec.pre_reserved_role, spec), None)
        return ReserveEvaluationOutcome(EvaluationOutcome.fail(
            stage, "Offer lacks previously reserved '%s' with resourceId: '%s' for resource: '%s'",
            spec.name, resource_id, spec), None)
    if resource_id is None:
        # a new reservation: consume_reservable_merged hands out exactly the spec's value
        # an offered chunk that carried nothing beyond name/type/value builds to exactly what
        # ResourceBuilder.from_spec(spec, new_id) produces, so it is built fresh (from the spec's
        # wire template) and the task carries the same resource
        plain = not (mr.resource.HasField("disk") or mr.resource.HasField("provider_id")
                     or len(mr.resource.reservations) or mr.resource.HasField("reservation"))
        if plain:
            resource, new_id = new_reservation(spec, namespace, framework_id)
        else:
            b = ResourceBuilder.from_spec(spec, None, namespace, framework_id)
            resource = b.set_mesos_resource(mr).build()
            new_id = b.built_resource_id
        rec = ReserveOfferRecommendation(pool.offer, resource)
        return ReserveEvaluationOutcome(EvaluationOutcome.pass_(
            stage, "Offer contains sufficient unreserved '%s', generated new resourceId: '%s' "
                   "for new reservation: '%s'", spec.name, new_id, spec,
            recommendations=[rec], mesos_resource=mr), new_id, resource if plain else None)
    if V.equal(mr.value, spec.value):
        return ReserveEvaluationOutcome(EvaluationOutcome.pass_(
            stage, "Offer contains previously reserved '%s' with resourceId: '%s' for resource: '%s'",
            spec.name, resource_id, spec, mesos_resource=mr), resource_id)
    difference = V.subtract(spec.value, mr.value)
    if V.compare(difference, V.get_zero(difference.type)) > 0:
        extra = pool.consume_reservable_merged(spec.name, difference, spec.pre_reserved_role)
        if extra is None:
            return ReserveEvaluationOutcome(EvaluationOutcome.fail(
                stage, "Insufficient resources to increase reservation of existing '%s' resource '%s' with "
                       "resourceId '%s': needed %s", spec.name, spec, resource_id, V.to_string(difference)), None)
        resource = ResourceBuilder.from_spec(spec, resource_id, namespace, framework_id).set_value(extra.value).build()
        rec = ReserveOfferRecommendation(pool.offer, resource)
        return ReserveEvaluationOutcome(EvaluationOutcome.pass_(
            stage, "Offer contains sufficient '%s' to increase desired resource by %s: resourceId: '%s': '%s'",
            spec.name, V.to_string(difference), resource_id, spec, recommendations=[rec], mesos_resource=extra),
            get_resource_id(resource))
    unreserve = V.subtract(mr.value, spec.value)
    resource = ResourceBuilder.from_spec(spec, resource_id, namespace, framework_id).set_value(unreserve).build()
    rec = UnreserveOfferRecommendation(pool.offer, resource)
    return ReserveEvaluationOutcome(EvaluationOutcome.pass_(
        stage, "Decreased '%s' by %s for desired resource with resourceId: '%s': %s",
        spec.name, V.to_string(unreserve), resource_id, spec, recommendations=[rec], mesos_resource=mr),
        get_resource_id(resource))


def set_protos(builder: PodInfoBuilder, resource: P.Resource, task_name: Optional[str]) -> None:
    if task_name is not None:
        builder.get_task_builder(task_name).resources.add().CopyFrom(resource)
    else:
        builder.get_executor_builder().resources.add().CopyFrom(resource)


def is_running_executor(builder: PodInfoBuilder, offer: P.Offer) -> bool:
    e = builder.get_executor_builder()
    if e is None:
        return False
    return any(x.value == e.executor_id.value for x in offer.executor_ids)


def get_role(pod_spec) -> Optional[str]:
    for t in pod_spec.tasks:
        for r in t.resource_set.resources:
            return r.role
    return None


# ---------------------------------------------------------------------------------------
# stages


class ExecutorEvaluationStage(OfferEvaluationStage):
    def __init__(self, service_name: str, executor_id: Optional[P.ExecutorID]):
        self.service_name = service_name
        self.executor_id = executor_id

    def evaluate(self, pool, builder):
        e = builder.get_executor_builder()
        if e is None:
            return EvaluationOutcome.pass_(self, "No executor requirement defined")
        id_str = self.executor_id.value if self.executor_id is not None else ""
        if self.executor_id is not None and not any(x.value == id_str for x in pool.offer.executor_ids):
            return EvaluationOutcome.fail(self, "Offer does not contain the needed Executor ID: '%s'", id_str)
        if self.executor_id is not None:
            e.executor_id.CopyFrom(self.executor_id)
            return EvaluationOutcome.pass_(self, "Offer contains the matching Executor ID: '%s'", id_str)
        eid = common_id_utils.to_executor_id(self.service_name, e.name)
        e.executor_id.CopyFrom(eid)
        return EvaluationOutcome.pass_(self, "No Executor ID required, generated: '%s'", eid.value)


class PlacementRuleEvaluationStage(OfferEvaluationStage):
    def __init__(self, deployed_tasks, placement_rule):
        self.deployed_tasks = list(deployed_tasks)
        self.placement_rule = placement_rule

    def evaluate(self, pool, builder):
        if self.placement_rule is None:
            return EvaluationOutcome.pass_(self, "No placement rule defined")
        return self.placement_rule.filter(pool.offer, builder.pod_instance, self.deployed_tasks)


class ResourceEvaluationStage(OfferEvaluationStage):
    def __init__(self, spec: ResourceSpec, task_names: Collection[str], resource_id: Optional[str],
                 namespace: Optional[str], framework_id: Optional[str]):
        self.spec = spec
        self.task_names = list(task_names)
        self.resource_id = resource_id
        self.namespace = namespace
        self.framework_id = framework_id

    def evaluate(self, pool, builder):
        if not self.task_names and self.resource_id is not None and is_running_executor(builder, pool.offer):
            set_protos(builder, ResourceBuilder.from_spec(self.spec, self.resource_id, self.namespace,
                                                          self.framework_id).build(), None)
            return EvaluationOutcome.pass_(self, "Including running executor's '%s' resource with resourceId: '%s': %s",
                                           self.spec.name, self.resource_id, self.spec)
        res = evaluate_simple_resource(self, self.spec, self.resource_id, self.namespace, pool, self.framework_id)
        if not res.outcome.passing:
            return res.outcome
        resource = res.resource if res.resource is not None else \
            ResourceBuilder.from_spec(self.spec, res.resource_id, self.namespace, self.framework_id).build()
        for t in self.task_names:
            set_protos(builder, resource, t)
        if not self.task_names:
            set_protos(builder, resource, None)
        return res.outcome


def _requires_host_ports(network_names) -> bool:
    if not network_names:
        return True
    return any(dcos.network_supports_port_mapping(n) for n in network_names)


def _ports_in_resource(r: P.Resource):
    if r.name != constants.PORTS_RESOURCE_TYPE:
        return set()
    out = set()
    for rg in r.ranges.range:
        out.update(p for p in range(int(rg.begin), int(rg.end) + 1) if p != 0)
    return out


class PortEvaluationStage(OfferEvaluationStage):
    def __init__(self, spec: PortSpec, task_names: Collection[str], resource_id: Optional[str],
                 namespace: Optional[str], framework_id: Optional[str]):
        self.spec = spec
        self.task_names = list(task_names)
        self.resource_id = resource_id
        self.namespace = namespace
        self.framework_id = framework_id
        self.use_host_ports = _requires_host_ports(spec.network_names)

    def evaluate(self, pool, builder):
        requested = int(self.spec.value.ranges.range[0].begin)
        assigned = requested
        if requested == 0:
            prior = None
            for t in self.task_names:
                prior = builder.get_prior_port_for_task(t, self.spec)
                if prior is not None:
                    break
            if prior is not None:
                assigned = prior
            else:
                role = builder.pod_instance.pod.pre_reserved_role
                dyn = (self._select_dynamic_port(pool, builder, role) if self.use_host_ports
                       else self._select_overlay_port(builder))
                if dyn is None:
                    return EvaluationOutcome.fail(
                        self, "No ports were available for dynamic claim in offer, and no matching port %s was "
                              "present in prior %s", self.spec.port_name,
                        "executor" if not self.task_names else f"tasks: {self.task_names}")
                assigned = dyn
        updated = self.spec.with_value(ranges_value([(assigned, assigned)]))
        if self.use_host_ports:
            res = evaluate_simple_resource(self, updated, self.resource_id, self.namespace, pool, self.framework_id)
            if not res.outcome.passing:
                return res.outcome
            self.set_protos(builder, ResourceBuilder.from_spec(updated, res.resource_id, self.namespace,
                                                               self.framework_id).build())
            return EvaluationOutcome.pass_(
                self, "Offer contains required %sport: '%s' with resourceId: '%s'",
                "previously reserved " if self.resource_id else "", assigned, self.resource_id,
                recommendations=res.outcome.get_offer_recommendations(), mesos_resource=res.outcome.mesos_resource)
        self.set_protos(builder, ResourceBuilder.from_spec(updated, self.resource_id, self.namespace,
                                                           self.framework_id).build())
        return EvaluationOutcome.pass_(
            self, "Port %s doesn't require resource reservation, ignoring resource requirements and using port %d",
            self.spec.port_name, assigned)

    def set_protos(self, builder: PodInfoBuilder, resource: P.Resource) -> None:
        port = int(resource.ranges.range[0].begin)
        key = self.spec.env_key
        val = str(port)
        for tname in self.task_names:
            t = builder.get_task_builder(tname)
            if not t.HasField("discovery"):
                t.discovery.visibility = constants.DEFAULT_TASK_DISCOVERY_VISIBILITY
                t.discovery.name = t.name
            t.discovery.ports.ports.add(number=port, visibility=self.spec.visibility,
                                        protocol=dcos.DEFAULT_IP_PROTOCOL, name=self.spec.port_name)
            if key is not None:
                t.command.environment.CopyFrom(L.with_env_var(t.command.environment, key, val))
                if t.HasField("health_check"):
                    t.health_check.command.environment.CopyFrom(
                        L.with_env_var(t.health_check.command.environment, key, val))
                if t.HasField("check"):
                    t.check.command.command.environment.CopyFrom(
                        L.with_env_var(t.check.command.command.environment, key, val))
                if L.TaskLabelReader(t).has_readiness_check_label():
                    L.TaskLabelWriter(t).set_readiness_check_envvar(key, val).apply()
            if self.use_host_ports:
                t.resources.add().CopyFrom(resource)
        if not self.task_names:
            e = builder.get_executor_builder()
            if key is not None:
                e.command.environment.CopyFrom(L.with_env_var(e.command.environment, key, val))
            if self.use_host_ports:
                e.resources.add().CopyFrom(resource)

    def _select_dynamic_port(self, pool, builder, role) -> Optional[int]:
        consumed = set()
        for t in builder.pod_instance.pod.tasks:
            for r in t.resource_set.resources:
                if isinstance(r, PortSpec) and r.port != 0:
                    consumed.add(r.port)
        for r in builder.get_task_resources():
            consumed |= _ports_in_resource(r)
        for r in builder.get_executor_resources():
            consumed |= _ports_in_resource(r)
        available = pool.unreserved_merged_pool_by_role(role).get(constants.PORTS_RESOURCE_TYPE)
        if available is None:
            return None
        allowed = None
        if self.spec.ranges:
            allowed = set()
            for rg in self.spec.ranges:
                allowed.update(range(rg.begin, rg.end + 1))
        for rg in available.ranges.range:
            for p in range(int(rg.begin), int(rg.end) + 1):
                if p in consumed:
                    continue
                if allowed is not None and p not in allowed:
                    continue
                return p
        return None

    @staticmethod
    def _select_overlay_port(builder) -> Optional[int]:
        for p in range(dcos.OVERLAY_DYNAMIC_PORT_RANGE_START, dcos.OVERLAY_DYNAMIC_PORT_RANGE_END + 1):
            if not builder.is_assigned_overlay_port(p):
                builder.add_assigned_overlay_port(p)
                return p
        return None


class NamedVIPEvaluationStage(PortEvaluationStage):
    def set_protos(self, builder, resource):
        super().set_protos(builder, resource)
        spec: NamedVIPSpec = self.spec
        port_entry = None
        for tname in self.task_names:
            matches = [p for p in builder.get_task_builder(tname).discovery.ports.ports if p.name == spec.port_name]
            if len(matches) == 1:
                port_entry = matches[0]
                break
        if port_entry is None:
            raise ValueError(f"Unable to find port entry with name {spec.port_name} in tasks: {self.task_names}")
        port_entry.protocol = spec.protocol
        L.set_vip_labels(port_entry, spec.vip_name, spec.vip_port, spec.network_names,
                         dcos.network_supports_port_mapping)


class VolumeEvaluationStage(OfferEvaluationStage):
    def __init__(self, spec: VolumeSpec, task_names: Collection[str], resource_id: Optional[str],
                 namespace: Optional[str], persistence_id: Optional[str], provider_id, disk_source,
                 framework_id: Optional[str]):
        self.spec = spec
        self.task_names = list(task_names)
        self.resource_id = resource_id
        self.namespace = namespace
        self.persistence_id = persistence_id
        self.provider_id = provider_id
        self.disk_source = disk_source
        self.framework_id = framework_id

    @staticmethod
    def get_new(spec, task_names, namespace, framework_id) -> "VolumeEvaluationStage":
        return VolumeEvaluationStage(spec, task_names, None, namespace, None, None, None, framework_id)

    @staticmethod
    def get_existing(spec, task_names, resource_id, namespace, persistence_id, provider_id, disk_source,
                     framework_id) -> "VolumeEvaluationStage":
        return VolumeEvaluationStage(spec, task_names, resource_id, namespace, persistence_id, provider_id,
                                     disk_source, framework_id)

    def evaluate(self, pool, builder):
        recs = []
        if (not self.task_names and self.resource_id is not None and self.persistence_id is not None
                and is_running_executor(builder, pool.offer)):
            builder.set_executor_volume(self.spec)
            vol = PodInfoBuilder.get_existing_executor_volume(
                self.spec, self.resource_id, self.namespace, self.persistence_id, self.provider_id,
                self.disk_source, self.framework_id)
            builder.get_executor_builder().resources.add().CopyFrom(vol)
            return EvaluationOutcome.pass_(
                self, "Setting info for already running Executor with existing volume with resourceId: '%s' and "
                      "persistenceId: '%s'", self.resource_id, self.persistence_id)
        if self.spec.type == VolumeType.ROOT:
            res = evaluate_simple_resource(self, self.spec, self.resource_id, self.namespace, pool, self.framework_id)
            if not res.outcome.passing:
                return res.outcome
            recs.extend(res.outcome.get_offer_recommendations())
            mr = res.outcome.mesos_resource
            if res.resource is not None and self.persistence_id is None and len(res.resource_id or "") == 36:
                # a new volume on a plain chunk: the reservation was built fresh, so is the volume
                resource = new_root_volume(self.spec, res.resource_id, self.namespace, self.framework_id)
            else:
                resource = ResourceBuilder.from_volume_spec(
                    self.spec, res.resource_id, self.namespace, self.persistence_id, None, None,
                    self.framework_id).set_mesos_resource(mr).build()
        else:
            if self.resource_id is None:
                mr = pool.consume_atomic(constants.DISK_RESOURCE_TYPE, self.spec)
            else:
                mr = pool.get_reserved_resource_by_id(self.resource_id)
            if mr is None:
                return EvaluationOutcome.fail(self, "Failed to find MOUNT volume for '%s'.", self.spec)
            r = mr.resource
            resource = ResourceBuilder.from_volume_spec(
                self.spec, self.resource_id, self.namespace, self.persistence_id,
                r.provider_id if r.HasField("provider_id") else None, get_disk_source(r),
                self.framework_id).set_value(mr.value).set_mesos_resource(mr).build()
            if self.resource_id is None:
                recs.append(ReserveOfferRecommendation(pool.offer, resource))
        if self.persistence_id is None:
            recs.append(CreateOfferRecommendation(pool.offer, resource))
        for t in self.task_names:
            set_protos(builder, resource, t)
        if not self.task_names:
            set_protos(builder, resource, None)
            builder.set_executor_volume(self.spec)
        if self.resource_id is not None:
            return EvaluationOutcome.pass_(
                self, "Offer contains previously reserved 'disk' with resourceId: '%s' and persistenceId: '%s' "
                      "for resource: '%s'", self.resource_id, self.persistence_id, self.spec,
                recommendations=recs, mesos_resource=mr)
        return EvaluationOutcome.pass_(
            self, "Offer contains sufficient unreserved 'disk', generated new resourceId: '%s' for new "
                  "reservation: '%s'", get_resource_id(resource), self.spec, recommendations=recs, mesos_resource=mr)


def _update_fault_domain_env(t: P.TaskInfo, offer: P.Offer) -> None:
    if not (offer.HasField("domain") and offer.domain.HasField("fault_domain")) or not t.HasField("command"):
        return
    t.command.environment.variables.add(name=L.REGION_TASKENV, value=offer.domain.fault_domain.region.name)
    t.command.environment.variables.add(name=L.ZONE_TASKENV, value=offer.domain.fault_domain.zone.name)


class LaunchEvaluationStage(OfferEvaluationStage):
    def __init__(self, service_name: str, task_spec_name: str, should_launch: bool):
        self.service_name = service_name
        self.task_spec_name = task_spec_name
        self.should_launch = should_launch

    def evaluate(self, pool, builder):
        e = builder.get_executor_builder()
        offer = pool.offer
        t = builder.get_task_builder(self.task_spec_name)
        if self.should_launch:
            t.task_id.CopyFrom(common_id_utils.to_task_id(self.service_name, t.name))
        else:
            t.task_id.value = ""
        t.agent_id.CopyFrom(offer.agent_id)
        w = L.TaskLabelWriter(t).set_offer_attributes(offer).set_type(builder.type).set_index(builder.index)
        w.set_hostname(offer)
        if offer.HasField("domain") and offer.domain.HasField("fault_domain"):
            w.set_region(offer.domain.fault_domain.region.name).set_zone(offer.domain.fault_domain.zone.name)
        w.apply()
        _update_fault_domain_env(t, offer)
        # no snapshot copies: the builder belongs to this one offer's evaluation, and no stage
        # after a task's launch stage touches that task or the executor (executor, pod-volume and
        # TLS stages run first; each later resource-set stage writes only its own tasks). The
        # LAUNCH_GROUP operation copies both, and the store recommendation copies them when the
        # launch is recorded.
        snapshot, exec_snapshot = t, e
        if self.should_launch:
            return EvaluationOutcome.pass_(
                self, "Added launch operation for %s", self.task_spec_name,
                recommendations=[LaunchOfferRecommendation(offer, snapshot, exec_snapshot),
                                 StoreTaskInfoRecommendation(offer, snapshot, exec_snapshot)])
        return EvaluationOutcome.pass_(self, "Added metadata update for %s", self.task_spec_name,
                                       recommendations=[StoreTaskInfoRecommendation(offer, snapshot, exec_snapshot)])


class UnreserveEvaluationStage(OfferEvaluationStage):
    def __init__(self, resource: P.Resource):
        self.resource = resource

    def evaluate(self, pool, builder):
        pool.free(MesosResource(self.resource))
        return EvaluationOutcome.pass_(self, "Unreserving orphaned resource: %s", P.to_text(self.resource),
                                       recommendations=[UnreserveOfferRecommendation(pool.offer, self.resource)])


class DestroyEvaluationStage(OfferEvaluationStage):
    def __init__(self, resource: P.Resource):
        self.resource = resource

    def evaluate(self, pool, builder):
        return EvaluationOutcome.pass_(self, "Destroying orphaned resource: %s", P.to_text(self.resource),
                                       recommendations=[DestroyOfferRecommendation(pool.offer, self.resource)],
                                       mesos_resource=MesosResource(self.resource))


# ---------------------------------------------------------------------------------------
# TLSEvaluationStage


class TLSEvaluationStage(OfferEvaluationStage):
    """Provisions the task's TLS artifacts as secrets and mounts them read-only in the container.

    Reference: offer/evaluate/TLSEvaluationStage.java:110-190. Artifacts are (re)generated only when
    a secret is missing (e.g. the SANs changed); each transport-encryption entry mounts
    ``<name>.crt/.key/.ca`` (TLS) or ``<name>.keystore/.truststore`` (KEYSTORE) as SECRET volumes.
    """

    class Builder:
        def __init__(self, service_name: str, scheduler_config, updater=None):
            self.service_name = service_name
            self.scheduler_config = scheduler_config
            self.namespace = scheduler_config.secrets_namespace(service_name)
            if updater is None:
                from dcos_commons_amd.dcos.clients import CertificateAuthorityClient, DcosHttpExecutor, SecretsClient
                from dcos_commons_amd.offer.evaluate.security import TLSArtifactsGenerator, TLSArtifactsUpdater

                executor = DcosHttpExecutor(scheduler_config.dcos_auth_token_provider())
                updater = TLSArtifactsUpdater(service_name, SecretsClient(executor),
                                              TLSArtifactsGenerator(CertificateAuthorityClient(executor)))
            self.updater = updater

        def build(self, task_name: str) -> "TLSEvaluationStage":
            return TLSEvaluationStage(self.service_name, task_name, self.namespace, self.updater,
                                      self.scheduler_config)

        __call__ = build

    def __init__(self, service_name: str, task_name: str, namespace: str, updater, scheduler_config):
        self.service_name = service_name
        self.task_name = task_name
        self.namespace = namespace
        self.updater = updater
        self.scheduler_config = scheduler_config

    def evaluate(self, pool: MesosResourcePool, builder: PodInfoBuilder) -> EvaluationOutcome:
        from dcos_commons_amd.offer.evaluate.security import CertificateNamesGenerator, TLSArtifactPaths

        pi = builder.pod_instance
        task_spec = next(t for t in pi.pod.tasks if t.name == self.task_name)
        if not task_spec.transport_encryption:
            return EvaluationOutcome.pass_(self, "No TLS specs found for task")
        names = CertificateNamesGenerator(self.service_name, task_spec, pi, self.scheduler_config)
        paths = TLSArtifactPaths(self.namespace, common_id_utils.get_task_instance_name(pi, task_spec),
                                 names.sans_hash())
        task = builder.get_task_builder(self.task_name)
        for te in task_spec.transport_encryption:
            try:
                self.updater.update(paths, names, te.name)
            except Exception as e:  # noqa: BLE001
                LOGGER.error("Failed to process certificates for %s: %s", self.task_name, e)
                return EvaluationOutcome.fail(
                    self, "Failed to store TLS artifacts for task %s because of exception: %s", self.task_name, e)
            existing = {(v.container_path, v.source.secret.reference.name) for v in task.container.volumes}
            for entry in paths.get_paths_for_type(te.type.value, te.name):
                if (entry.mount_path, entry.secret_store_path) in existing:
                    continue
                v = task.container.volumes.add(container_path=entry.mount_path, mode=P.Volume.RO)
                v.source.type = P.Volume.Source.SECRET
                v.source.secret.type = P.Secret.REFERENCE
                v.source.secret.reference.name = entry.secret_store_path
        return EvaluationOutcome.pass_(self, "TLS certificate created and added to the task")
