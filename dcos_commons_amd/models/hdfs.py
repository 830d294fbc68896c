"""HDFS (HA) service: scheduler entry point and HDFS-specific behaviour.

Reference: frameworks/hdfs/src/main/java/com/mesosphere/sdk/hdfs/scheduler/{Main.java,
HdfsRecoveryPlanOverrider.java, HdfsRecoveryPlanOverriderFactory.java, HDFSZoneValidator.java,
HDFSUserAuthMapperBuilder.java, HDFSAuthEnvContainer.java}.

* Placement: journal and name pods avoid each other's types (and their own); data pods avoid
  other data pods -- ANDed with any user placement constraint.
* Replacement: a PERMANENT failure of ``journal-<i>`` or ``name-<i>`` is recovered with the
  ``replace`` plan's ``[bootstrap]`` (PERMANENT) then ``[node...]`` (TRANSIENT) step pair for that
  index, as phase ``permanent-<type>-failure-recovery``. Data nodes use the default recovery.
* Endpoints: ``/v1/endpoints/hdfs-site.xml`` and ``core-site.xml`` serve client configs rendered
  from the task templates with the ALL-pods ``TASKCFG_*`` env.
* Kerberos: ``auth_to_local`` rules (user rules from base64 ``TASKCFG_ALL_AUTH_TO_LOCAL`` plus
  one default rule per HDFS task host) go to every pod as ``DECODED_AUTH_TO_LOCAL``.

Run: ``python -m dcos_commons_amd.models.hdfs frameworks/hdfs/specs/svc.yml``.
"""
from __future__ import annotations

import base64
import dataclasses
import logging
import os
import sys
from typing import Dict, List, Mapping, Optional

from dcos_commons_amd.config.task_env_router import TaskEnvRouter
from dcos_commons_amd.config.validate import ConfigValidator, zone_validate
from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.offer.evaluate import placement as pl
from dcos_commons_amd.scheduler.plan.elements import DefaultPhase
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement, RecoveryType
from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy
from dcos_commons_amd.scheduler.recovery import RecoveryPlanOverrider, RecoveryPlanOverriderFactory, RecoveryStep
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.specification.yaml.template_utils import render_mustache_throw_if_missing
from dcos_commons_amd.storage.zk_persister import get_service_root_path

LOGGER = logging.getLogger(__name__)

JOURNAL, NAME, DATA = "journal", "name", "data"
JOURNAL_NODE_COUNT, NAME_NODE_COUNT = 3, 2
SERVICE_ZK_ROOT_TASKENV = "SERVICE_ZK_ROOT"
HDFS_SITE_XML, CORE_SITE_XML = "hdfs-site.xml", "core-site.xml"
REPLACE_PLAN_NAME = "replace"
PHASE_NAME_TEMPLATE = "permanent-{}-failure-recovery"

AUTH_TO_LOCAL = "AUTH_TO_LOCAL"
PRIMARY_ENV_KEY = "TASKCFG_ALL_SECURITY_KERBEROS_PRIMARY"
REALM_ENV_KEY = "TASKCFG_ALL_SECURITY_KERBEROS_REALM"
FRAMEWORK_USER_ENV_KEY = "TASKCFG_ALL_TASK_USER"
DECODED_AUTH_TO_LOCAL = "DECODED_" + AUTH_TO_LOCAL
TASKCFG_ALL_AUTH_TO_LOCAL = "TASKCFG_ALL_" + AUTH_TO_LOCAL
_DEFAULT_RULE = "RULE:[2:$1/$2@$0]({primary}/{task}.{host}@{realm})s/.*/{user}/"


class HDFSAuthEnvContainer:
    def __init__(self, env: Mapping[str, str]):
        missing = [k for k in (PRIMARY_ENV_KEY, REALM_ENV_KEY, FRAMEWORK_USER_ENV_KEY) if k not in env]
        if missing:
            raise RuntimeError(f"The following environment keys are missing {', '.join(missing)}")
        self.primary = env[PRIMARY_ENV_KEY]
        self.realm = env[REALM_ENV_KEY]
        self.framework_user = env[FRAMEWORK_USER_ENV_KEY]
        raw = env.get(TASKCFG_ALL_AUTH_TO_LOCAL)
        self.env_auth_mapping = base64.b64decode(raw).decode("utf-8") if raw else ""


class HDFSUserAuthMapperBuilder:
    def __init__(self, env: Mapping[str, str], framework_host: str):
        self.framework_host = framework_host
        self.env = HDFSAuthEnvContainer(env)
        self.mappings: List[str] = []

    def add_user_auth_mapping_from_env(self) -> "HDFSUserAuthMapperBuilder":
        self.mappings.append(self.env.env_auth_mapping)
        return self

    def add_default_user_auth_mapping(self, pod_type: str, task: str, count: int) -> "HDFSUserAuthMapperBuilder":
        for i in range(count):
            self.mappings.append(_DEFAULT_RULE.format(primary=self.env.primary, task=f"{pod_type}-{i}-{task}",
                                                      host=self.framework_host, realm=self.env.realm,
                                                      user=self.env.framework_user))
        return self

    def build(self) -> str:
        return "\n".join(m for m in self.mappings if m and m.strip())


class HDFSZoneValidator(ConfigValidator):
    def validate(self, old, new):
        return zone_validate(old, new, NAME, JOURNAL, DATA)


class HdfsRecoveryPlanOverrider(RecoveryPlanOverrider):
    def __init__(self, state_store, replace_plan):
        self.state_store = state_store
        self.replace_plan = replace_plan

    def override(self, stopped: PodInstanceRequirement) -> Optional[DefaultPhase]:
        pod_type = stopped.pod_instance.pod.type
        if pod_type == DATA or stopped.recovery_type != RecoveryType.PERMANENT:
            LOGGER.info("No overrides necessary. Pod is not a journal or name node or it isn't a permanent failure.")
            return None
        index = stopped.pod_instance.index
        limit = NAME_NODE_COUNT if pod_type == NAME else JOURNAL_NODE_COUNT
        if pod_type not in (NAME, JOURNAL) or index >= limit:
            LOGGER.error("Encountered unexpected index: %d, falling back to default recovery plan manager.", index)
            return None
        LOGGER.info("Returning replacement plan for %snode %d.", pod_type, index)
        return self._recovery_phase(index, pod_type)

    def _recovery_phase(self, index: int, phase_name: str) -> DefaultPhase:
        phase = next((p for p in self.replace_plan.get_children() if p.get_name() == phase_name), None)
        if phase is None:
            raise RuntimeError(f"Expected phase name {phase_name} does not exist in the service spec plan")
        steps = phase.get_children()
        boot, node = steps[index * 2], steps[index * 2 + 1]
        breq, nreq = boot.get_pod_instance_requirement(), node.get_pod_instance_requirement()
        return DefaultPhase(PHASE_NAME_TEMPLATE.format(phase_name), [
            RecoveryStep(boot.get_name(), PodInstanceRequirement(breq.pod_instance, breq.tasks_to_launch,
                                                                 recovery_type=RecoveryType.PERMANENT),
                         self.state_store),
            RecoveryStep(node.get_name(), PodInstanceRequirement(nreq.pod_instance, nreq.tasks_to_launch,
                                                                 recovery_type=RecoveryType.TRANSIENT),
                         self.state_store),
        ], SerialStrategy(), [])


class HdfsRecoveryPlanOverriderFactory(RecoveryPlanOverriderFactory):
    def create(self, state_store, plans) -> HdfsRecoveryPlanOverrider:
        plan = next((p for p in plans if p.get_name() == REPLACE_PLAN_NAME), None)
        if plan is None:
            raise RuntimeError(f"Failed to find plan: {REPLACE_PLAN_NAME}")
        return HdfsRecoveryPlanOverrider(state_store, plan)


def with_placement_rules(spec):
    """Journal/name avoid each other and themselves; data avoids data (Main.setPlacementRules)."""
    rules = {
        JOURNAL: pl.AndRule([pl.TaskTypeRule.avoid(JOURNAL), pl.TaskTypeRule.avoid(NAME)]),
        NAME: pl.AndRule([pl.TaskTypeRule.avoid(NAME), pl.TaskTypeRule.avoid(JOURNAL)]),
        DATA: pl.TaskTypeRule.avoid(DATA),
    }
    pods = []
    for t in (JOURNAL, NAME, DATA):
        pod = spec.pod(t)
        if pod is None:
            raise ValueError(f"Missing required pod named '{t}' in service spec")
        rule = rules[t] if pod.placement_rule is None else pl.AndRule([rules[t], pod.placement_rule])
        pods.append(dataclasses.replace(pod, placement_rule=rule))
    return dataclasses.replace(spec, pods=tuple(pods))


def render_client_config(path: str, service_name: str, scheduler_config, user_auth_mapping: str,
                         env: Mapping[str, str]) -> str:
    """Client-side hdfs-site/core-site for the endpoints API (Main.renderTemplate)."""
    with open(path, "r", encoding="utf-8") as f:
        text = f.read()
    values: Dict[str, str] = dict(TaskEnvRouter(env).get_config("ALL"))
    values.update({
        "FRAMEWORK_HOST": endpoint_utils.to_auto_ip_domain(service_name, scheduler_config),
        "FRAMEWORK_NAME": service_name,
        "SCHEDULER_API_HOSTNAME": endpoint_utils.to_scheduler_auto_ip_hostname(service_name, scheduler_config),
        "SCHEDULER_API_PORT": str(scheduler_config.api_server_port()),
        "MESOS_SANDBOX": "sandboxpath",
        SERVICE_ZK_ROOT_TASKENV: get_service_root_path(service_name),
        DECODED_AUTH_TO_LOCAL: user_auth_mapping,
    })
    return render_mustache_throw_if_missing(os.path.basename(path), text, values)


def create_scheduler_builder(yaml_path: str, scheduler_config: Optional[SchedulerConfig] = None,
                             env: Optional[Dict[str, str]] = None, persister=None) -> SchedulerBuilder:
    env = dict(os.environ if env is None else env)
    cfg = scheduler_config or SchedulerConfig.from_env()
    config_dir = os.path.dirname(os.path.abspath(yaml_path))
    raw = RawServiceSpec.new_builder(yaml_path).set_env(env).build()
    if str(env.get("TASKCFG_ALL_SECURITY_KERBEROS_ENABLED", "")).lower() == "true":
        host = endpoint_utils.to_auto_ip_domain(raw.name, cfg)
        mapping = (HDFSUserAuthMapperBuilder(env, host).add_user_auth_mapping_from_env()
                   .add_default_user_auth_mapping(JOURNAL, "node", JOURNAL_NODE_COUNT)
                   .add_default_user_auth_mapping(NAME, "zkfc", NAME_NODE_COUNT)
                   .add_default_user_auth_mapping(NAME, "node", NAME_NODE_COUNT)
                   .add_default_user_auth_mapping(DATA, "node", int(env.get("DATA_COUNT", "0")))
                   .build())
    else:
        mapping = ""
    gen = ServiceSpecGenerator(raw, cfg, config_dir, env)
    gen.set_all_pods_env(SERVICE_ZK_ROOT_TASKENV, get_service_root_path(raw.name))
    gen.set_all_pods_env(DECODED_AUTH_TO_LOCAL, mapping)
    spec = gen.build()
    builder = SchedulerBuilder(with_placement_rules(spec), cfg, persister)
    builder.set_recovery_manager_factory(HdfsRecoveryPlanOverriderFactory()).set_plans_from(raw)
    for name in (HDFS_SITE_XML, CORE_SITE_XML):
        builder.set_endpoint_producer(name, render_client_config(os.path.join(config_dir, name), spec.name, cfg,
                                                                 mapping, env))
    return builder.set_custom_config_validators([HDFSZoneValidator()]).with_single_region_constraint()


def main(argv=None) -> int:
    from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner

    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 1:
        raise SystemExit(f"Expected one file argument, got: {argv}")
    from dcos_commons_amd.utils import logging_utils

    logging_utils.configure()
    from dcos_commons_amd.models import resolve_spec

    SchedulerRunner.from_scheduler_builder(create_scheduler_builder(resolve_spec(argv[0], "hdfs"))).run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
