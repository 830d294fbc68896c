"""Configuration validators run on every scheduler start against the prior target config.

Reference: sdk/.../config/validate/*.java (DefaultConfigValidators.java:18-47). Each validator is a
callable ``validate(old_config: Optional[ServiceSpec], new_config: ServiceSpec) -> [ConfigValidationError]``;
fatal errors stop the scheduler, non-fatal ones keep the previous target and surface as deploy-plan
errors.
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional

from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.dcos import constants as dcos
from dcos_commons_amd.http.endpoint_utils import remove_slashes
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.evaluate import placement as pl
from dcos_commons_amd.offer.task_utils import has_tasks_with_tls, volumes_equal
from dcos_commons_amd.specification.specs import ANY_ROLE

LOGGER = logging.getLogger(__name__)


class ConfigValidationError:
    __slots__ = ("config_field", "old_value", "new_value", "message", "fatal")

    def __init__(self, config_field, old_value, new_value, message, fatal=False):
        self.config_field = config_field
        self.old_value = old_value
        self.new_value = new_value
        self.message = message
        self.fatal = fatal

    @staticmethod
    def value_error(field, value, message, fatal=False):
        return ConfigValidationError(field, None, value, message, fatal)

    @staticmethod
    def transition_error(field, old, new, message, fatal=False):
        return ConfigValidationError(field, old, new, message, fatal)

    def is_fatal(self) -> bool:
        return self.fatal

    def __str__(self):
        if self.old_value is not None:
            return (f"Field: '{self.config_field}'; Transition: '{self.old_value}' => '{self.new_value}'; "
                    f"Message: '{self.message}'; Fatal: {str(self.fatal).lower()}")
        return (f"Field: '{self.config_field}'; Value: '{self.new_value}'; Message: '{self.message}'; "
                f"Fatal: {str(self.fatal).lower()}")

    __repr__ = __str__


class ConfigValidator:
    def validate(self, old_config, new_config) -> List[ConfigValidationError]:
        raise NotImplementedError

    def __call__(self, old_config, new_config):
        return self.validate(old_config, new_config)


def _pods_by_type(spec) -> Optional[Dict[str, object]]:
    out = {}
    for p in spec.pods:
        if p.type in out:
            return None
        out[p.type] = p
    return out


class ServiceNameCannotContainDoubleUnderscores(ConfigValidator):
    def validate(self, old, new):
        if "__" in new.name:
            return [ConfigValidationError.value_error(
                "ServiceName", new.name, f"Service name may not contain double underscores: {new.name}")]
        return []


class PodSpecsCannotShrink(ConfigValidator):
    def validate(self, old, new):
        if old is None:
            return []
        new_pods = _pods_by_type(new)
        if new_pods is None:
            return [ConfigValidationError.value_error("PodSpecs", "null", "Duplicate pod types detected.")]
        errors = []
        for op in old.pods:
            np_ = new_pods.get(op.type)
            if np_ is None:
                if not op.allow_decommission:
                    errors.append(ConfigValidationError.transition_error(
                        f"PodSpec[name:{op.type}]", str(op.count), "null",
                        f"New config is missing PodSpec named '{op.type}' (expected present with >= {op.count} tasks)"))
                continue
            if np_.count < op.count and not np_.allow_decommission:
                errors.append(ConfigValidationError.transition_error(
                    f"PodSpec[name:{np_.type}]", str(op.count), str(np_.count),
                    f"New config's PodSpec named '{np_.type}' has {np_.count} tasks, expected >={op.count} tasks"))
        return errors


def pod_requests_gpu_resources(pod) -> bool:
    if dcos.DEFAULT_GPU_POLICY:
        return True
    return any(r.name == constants.GPUS_RESOURCE_TYPE and r.value.scalar.value >= 1
               for t in pod.tasks for r in t.resource_set.resources)


def service_requests_gpu_resources(spec) -> bool:
    return any(pod_requests_gpu_resources(p) for p in spec.pods)


class PodSpecsCannotUseUnsupportedFeatures(ConfigValidator):
    def validate(self, old, new):
        caps = capabilities.get_instance()
        errors = []
        for pod in new.pods:
            def err(field, msg):
                errors.append(ConfigValidationError.value_error("pod:" + pod.type, field, msg))
            if not caps.supports_gpu_resource and pod_requests_gpu_resources(pod):
                err(constants.GPUS_RESOURCE_TYPE, "This DC/OS cluster does not support GPU resources")
            if not caps.supports_pre_reserved_resources and pod.pre_reserved_role != ANY_ROLE:
                err("pre-reserved-role", "This DC/OS cluster does not support consuming pre-reserved resources.")
            if not caps.supports_rlimits and pod.rlimits:
                err("rlimits", "This DC/OS cluster does not support setting rlimits")
            requests_cni = any(n.port_mappings for n in pod.networks) or any(
                r.name == "ports" for t in pod.tasks for r in t.resource_set.resources)
            if not caps.supports_cni_port_mapping and requests_cni:
                err("network", "This DC/OS cluster does not support CNI port mapping")
            if not caps.supports_env_based_secrets and any(s.env_key for s in pod.secrets):
                err("secrets:env", "This DC/OS cluster does not support environment-based secrets")
            if not caps.supports_file_based_secrets and any(s.file_path or not s.env_key for s in pod.secrets):
                err("secrets:file", "This DC/OS cluster does not support file-based secrets")
            if not caps.supports_shm and (pod.shared_memory is not None or pod.shared_memory_size is not None):
                err("shm", "This DC/OS cluster does not support shared memory")
            if not caps.supports_seccomp and (pod.seccomp_unconfined or pod.seccomp_profile_name):
                LOGGER.warning("Seccomp is not supported in this cluster.")
        return errors


class PodSpecsCannotChangeNetworkRegime(ConfigValidator):
    @staticmethod
    def _uses_host_ports(pod) -> bool:
        if not pod.networks:
            return True
        return any(dcos.network_supports_port_mapping(n.name) for n in pod.networks)

    def validate(self, old, new):
        if old is None:
            return []
        new_pods = _pods_by_type(new)
        if new_pods is None:
            return [ConfigValidationError.value_error("PodSpecs", "null", "Duplicate pod types detected.")]
        old_pods = {p.type: p for p in old.pods}
        errors = []
        for t, np_ in new_pods.items():
            bad = [n.name for n in np_.networks if not dcos.network_supports_port_mapping(n.name) and n.port_mappings]
            if bad:
                errors.append(ConfigValidationError.transition_error(
                    f"PodSpec[name:{t}]", "null", str(np_.networks),
                    f"New config has pod {t} that indicates port mapping for virtual network(s) {', '.join(bad)}, "
                    "that do not support port mapping."))
            op = old_pods.get(t)
            if op is not None and self._uses_host_ports(op) != self._uses_host_ports(np_):
                errors.append(ConfigValidationError.transition_error(
                    f"PodSpec[name:{op.type}]", str(op.networks), str(np_.networks),
                    f"New config has pod {t} moving networks from {op.networks} to {np_.networks}, changing its "
                    f"host ports requirements from {self._uses_host_ports(op)} to {self._uses_host_ports(np_)}, "
                    "not allowed."))
        return errors


class PreReservationCannotChange(ConfigValidator):
    def validate(self, old, new):
        if old is None:
            return []
        new_pods = {p.type: p for p in new.pods}
        errors = []
        for op in old.pods:
            np_ = new_pods.get(op.type)
            if np_ is None:
                continue
            if np_.pre_reserved_role != op.pre_reserved_role:
                errors.append(ConfigValidationError.transition_error(
                    f"PodSpec[pre-reserved-role:{op.pre_reserved_role}]", op.pre_reserved_role, np_.pre_reserved_role,
                    f"New config has changed the pre-reserved-role of PodSpec named '{op.type}' (expected it to "
                    f"stay '{op.pre_reserved_role}')"))
        return errors


class UserCannotChange(ConfigValidator):
    def validate(self, old, new):
        if old is None:
            return []
        errors = []
        if old.user is not None and old.user != new.user:
            errors.append(ConfigValidationError.transition_error(
                "user", old.user, new.user,
                f"INVALID CONFIGURATION UPDATE. Cannot change user of deployed service from '{old.user}' to "
                f"'{new.user}'.\nRevert to previous user '{old.user}' to proceed. Current set of configuration "
                "updates will NOT be applied.", True))
        old_pods = {p.type: p for p in old.pods}
        for np_ in new.pods:
            op = old_pods.get(np_.type)
            if op is not None and op.user != np_.user:
                ou, nu = op.user or "null", np_.user or "null"
                errors.append(ConfigValidationError.transition_error(
                    "user", ou, nu,
                    f"INVALID CONFIGURATION UPDATE. Cannot change existing pod type user from '{ou}' to '{nu}'.\n"
                    f"Pod type user must remain the same across deployments. Revert to previous user '{ou}' to "
                    "proceed. Current set of configuration updates will NOT be applied.", True))
        return errors


class TLSRequiresServiceAccount(ConfigValidator):
    def __init__(self, scheduler_config):
        self.scheduler_config = scheduler_config

    def validate(self, old, new):
        if not has_tasks_with_tls(new):
            return []
        try:
            self.scheduler_config.dcos_auth_token_provider()  # construction only; no login happens here
        except Exception:  # noqa: BLE001
            return [ConfigValidationError.value_error(
                "transport-encryption", "",
                "Scheduler is missing a service account that is required for provisioning TLS artifacts. "
                "Please configure in order to continue.")]
        return []


class DomainCapabilityValidator(ConfigValidator):
    def validate(self, old, new):
        if capabilities.get_instance().supports_domains:
            return []
        errors = []
        # (the reference formats this message with its two arguments swapped,
        # DomainCapabilityValidator.java:37-52; here the pod type and the field are in place)
        tmpl = "The PlacementRule for PodSpec '%s' may not reference %s prior to DC/OS 1.11."
        for pod in new.pods:
            if pod.placement_rule is None:
                continue
            if pl.references_zone(pod):
                errors.append(ConfigValidationError.value_error("PlacementRule", str(pod.placement_rule),
                                                                tmpl % (pod.type, "Zones")))
            if pl.references_region(pod):
                errors.append(ConfigValidationError.value_error("PlacementRule", str(pod.placement_rule),
                                                                tmpl % (pod.type, "Regions")))
        return errors


class PlacementRuleIsValid(ConfigValidator):
    def _valid(self, rule) -> bool:
        if isinstance(rule, (pl.OrRule, pl.AndRule)):
            return all(self._valid(r) for r in rule.rules)
        return not isinstance(rule, pl.InvalidPlacementRule)

    def validate(self, old, new):
        return [ConfigValidationError.value_error(
            "PlacementRule", str(p.placement_rule),
            f"The PlacementRule for PodSpec '{p.type}' had invalid constraints")
            for p in new.pods if p.placement_rule is not None and not self._valid(p.placement_rule)]


class RegionCannotChange(ConfigValidator):
    def validate(self, old, new):
        if old is None:
            return []
        if old.region != new.region:
            return [ConfigValidationError.transition_error(
                "region", str(old.region), str(new.region),
                "Region for old service must remain the same across deployments.")]
        return []


class ServiceNameCannotBreakDNS(ConfigValidator):
    MAX = 63

    def validate(self, old, new):
        too_long = len(remove_slashes(new.name)) > self.MAX
        if old is not None:
            if too_long:
                LOGGER.warning("The service name (without slashes) exceeds the maximum size allowed in a DNS "
                               "subdomain.")
            return []
        if too_long:
            return [ConfigValidationError.value_error(
                "service.name", new.name,
                "Service name (without slashes) exceeds 63 characters. In order for service DNS to work correctly, "
                "the service name (without slashes) must not exceed 63 characters")]
        return []


class TaskSpecsCannotUseUnsupportedFeatures(ConfigValidator):
    def validate(self, old, new):
        if capabilities.get_instance().supports_shm:
            return []
        return [ConfigValidationError.value_error("task:" + t.name, "shm",
                                                  "This DC/OS cluster does not support shared memory")
                for p in new.pods for t in p.tasks
                if t.shared_memory is not None or t.shared_memory_size is not None]


class ServiceRoleCannotChangeOnIncompleteDeployment(ConfigValidator):
    def validate(self, old, new):
        if old is None or old.role == new.role:
            return []
        return [ConfigValidationError.transition_error(
            "role", old.role, new.role,
            "Detected service role change on an incomplete previous deployment!\nScheduler will not continue "
            "with deployment!\nResolve previous deployment issues before issuing role change.\nDowngrade the "
            "service to the previous version if the issue persists.\n", True)]


class TaskVolumesCannotChange(ConfigValidator):
    @staticmethod
    def _tasks(spec, errors):
        out = {}
        for p in spec.pods:
            for t in p.tasks:
                key = f"{p.type}-{t.name}"
                if key in out:
                    errors.append(ConfigValidationError.value_error(
                        "TaskSpecifications", t.name,
                        f"Duplicate TaskSpecifications named '{t.name}' in Service '{spec.name}'"))
                out[key] = t
        return out

    def validate(self, old, new):
        errors: List[ConfigValidationError] = []
        old_tasks = self._tasks(old, errors) if old is not None else {}
        new_tasks = self._tasks(new, errors)
        for k, ot in old_tasks.items():
            nt = new_tasks.get(k)
            if nt is None:
                continue
            if not volumes_equal(ot, nt):
                errors.append(ConfigValidationError.transition_error(
                    f"TaskVolumes[taskname:{nt.name}]", str(list(ot.resource_set.volumes)),
                    str(list(nt.resource_set.volumes)), "Volumes must be equal."))
        return errors


class TaskEnvCannotChange(ConfigValidator):
    ALLOW_UNSET_TO_SET = "ALLOW_UNSET_TO_SET"
    ALLOW_SET_TO_UNSET = "ALLOW_SET_TO_UNSET"

    def __init__(self, pod_type: str, task_name: str, env_name: str, *rules: str):
        self.pod_type = pod_type
        self.task_name = task_name
        self.env_name = env_name
        self.rules = set(rules)

    def validate(self, old, new):
        if old is None:
            return []
        op = old.pod(self.pod_type)
        ot = op.task(self.task_name) if op else None
        if ot is None or ot.command is None:
            return []
        np_ = new.pod(self.pod_type)
        nt = np_.task(self.task_name) if np_ else None
        if nt is None:
            raise ValueError(f"Unable to find requested pod={self.pod_type}, task={self.task_name} in config")
        if nt.command is None:
            raise ValueError(f"Requested pod={self.pod_type}, task={self.task_name} in config lacks a command")
        ov = ot.command.env.get(self.env_name)
        nv = nt.command.env.get(self.env_name)
        field = f"{self.pod_type}.{self.task_name}.env.{self.env_name}"
        if not (ov or "").strip():
            if not (nv or "").strip() or self.ALLOW_UNSET_TO_SET in self.rules:
                return []
            return [ConfigValidationError.transition_error(
                field, ov, nv, f"Env value {self.env_name} cannot change from unset to set")]
        if not (nv or "").strip():
            if self.ALLOW_SET_TO_UNSET in self.rules:
                return []
            return [ConfigValidationError.transition_error(
                field, ov, nv, f"Env value {self.env_name} cannot be unset after being set")]
        if ov == nv:
            return []
        return [ConfigValidationError.transition_error(field, ov, nv, f"Env value {self.env_name} cannot change")]


def zone_validate(old, new, *pod_types) -> List[ConfigValidationError]:
    """ZoneValidator: a pod's placement may not start/stop referencing zones."""
    errors = []
    for pt in pod_types:
        if old is None:
            continue
        op = old.pod(pt)
        if op is None:
            continue
        np_ = new.pod(pt)
        if np_ is None:
            raise ValueError(f"Unable to find requested pod={pt}, in config")
        if pl.references_zone(op) != pl.references_zone(np_):
            errors.append(ConfigValidationError.transition_error(
                f"{pt}.PlacementRule", str(op.placement_rule), str(np_.placement_rule),
                f"PlacementRule cannot change from {op.placement_rule} to {np_.placement_rule}"))
    return errors


class ZoneValidator(ConfigValidator):
    def __init__(self, *pod_types: str):
        self.pod_types = pod_types

    def validate(self, old, new):
        return zone_validate(old, new, *self.pod_types)


def get_validators(scheduler_config) -> List[ConfigValidator]:
    return [
        ServiceNameCannotContainDoubleUnderscores(),
        PodSpecsCannotShrink(),
        PodSpecsCannotUseUnsupportedFeatures(),
        PodSpecsCannotChangeNetworkRegime(),
        PreReservationCannotChange(),
        UserCannotChange(),
        TLSRequiresServiceAccount(scheduler_config),
        DomainCapabilityValidator(),
        PlacementRuleIsValid(),
        RegionCannotChange(),
        ServiceNameCannotBreakDNS(),
        TaskSpecsCannotUseUnsupportedFeatures(),
    ]


def get_role_validators(has_role_changed: bool, has_completed_deployment: bool) -> List[ConfigValidator]:
    if has_role_changed and has_completed_deployment:
        return []
    if has_role_changed:
        return [ServiceRoleCannotChangeOnIncompleteDeployment()]
    return [TaskVolumesCannotChange()]
