"""Apache Cassandra service: scheduler entry point and Cassandra-specific behaviour.

Reference: frameworks/cassandra/src/main/java/com/mesosphere/sdk/cassandra/{scheduler/Main.java,
scheduler/CassandraRecoveryPlanOverrider.java, scheduler/CassandraRecoveryPlanOverriderFactory.java,
scheduler/CassandraSeedUtils.java, scheduler/CassandraZoneValidator.java, api/SeedsResource.java}.

* Seeds: the first ``LOCAL_SEEDS_COUNT`` (default 2) nodes' autoip hostnames, injected into every
  pod as ``LOCAL_SEEDS``; ``GET /v1/seeds`` also lists ``TASKCFG_ALL_REMOTE_SEEDS`` (multi-DC).
* Replace-node recovery: a PERMANENT failure of ``node-<i>`` is recovered with the ``replace``
  plan's step whose server command gains ``-Dcassandra.replace_address=<old IP>`` (taken from the
  ``<task>:task-status`` property the scheduler keeps), so the new node streams the dead node's
  token ranges. Replacing a *seed* also restarts every other node so they pick up the new seed IP.
* Validation: zones cannot be toggled in the placement rule (``CassandraZoneValidator``) and the
  data center / rack env of ``node.server`` may only go from unset to set.
* ``AUTHENTICATION_CUSTOM_YAML_BLOCK`` is decoded from ``TASKCFG_ALL_AUTHENTICATION_CUSTOM_YAML_BLOCK_BASE64``.

Run: ``python -m dcos_commons_amd.models.cassandra frameworks/cassandra/specs/svc.yml``.
"""
from __future__ import annotations

import base64
import dataclasses
import logging
import os
import sys
from typing import Dict, List, Mapping, Optional

from dcos_commons_amd.config.validate import ConfigValidator, TaskEnvCannotChange, zone_validate
from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.http.api import Route, json_ok
from dcos_commons_amd.offer.common_id_utils import get_task_instance_name
from dcos_commons_amd.scheduler.plan.elements import DefaultPhase
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement, RecoveryType
from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy
from dcos_commons_amd.scheduler.recovery import RecoveryPlanOverrider, RecoveryPlanOverriderFactory, RecoveryStep
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import CommandSpec, PodInstance
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state import state_store_utils

LOGGER = logging.getLogger(__name__)

POD_TYPE = "node"
SERVER_TASK = "server"
REPLACE_PLAN_NAME = "replace"
RECOVERY_PHASE_NAME = "permanent-node-failure-recovery"
AUTH_YAML_BASE64_ENV = "TASKCFG_ALL_AUTHENTICATION_CUSTOM_YAML_BLOCK_BASE64"


def seeds_count(env: Optional[Mapping[str, str]] = None) -> int:
    return int((env if env is not None else os.environ).get("LOCAL_SEEDS_COUNT") or 2)


def get_local_seeds(service_name: str, scheduler_config, count: int) -> List[str]:
    return [endpoint_utils.to_auto_ip_hostname(service_name, f"{POD_TYPE}-{i}-{SERVER_TASK}", scheduler_config)
            for i in range(count)]


def is_seed_node(index: int, count: int) -> bool:
    return index < count


class SeedsResource:
    """``GET /v1/seeds`` -> ``{"seeds": [...]}``."""

    def __init__(self, configured_seeds: List[str]):
        self.seeds = list(dict.fromkeys(configured_seeds))

    def routes(self):
        return [Route("GET", "/v1/seeds", lambda req: json_ok({"seeds": list(self.seeds)}))]


class CassandraZoneValidator(ConfigValidator):
    def validate(self, old, new):
        return zone_validate(old, new, POD_TYPE)


class CassandraRecoveryPlanOverrider(RecoveryPlanOverrider):
    def __init__(self, state_store, replace_plan, seed_count: int = 2):
        self.state_store = state_store
        self.replace_plan = replace_plan
        self.seed_count = seed_count

    def override(self, stopped: PodInstanceRequirement) -> Optional[DefaultPhase]:
        if stopped.pod_instance.pod.type != POD_TYPE or stopped.recovery_type != RecoveryType.PERMANENT:
            LOGGER.info("No overrides necessary. Pod is not a node or it isn't a permanent failure.")
            return None
        index = stopped.pod_instance.index
        LOGGER.info("Returning replacement plan for node %d.", index)
        return self._node_recovery_phase(index)

    def _node_recovery_phase(self, index: int) -> Optional[DefaultPhase]:
        phase = self.replace_plan.get_children()[0]
        launch_step = phase.get_children()[index]
        launch_step.start()
        req = launch_step.get_pod_instance_requirement()
        pi = req.pod_instance
        pod = pi.pod
        server = next(t for t in pod.tasks if t.name == SERVER_TASK)
        status = state_store_utils.get_task_status_from_property(self.state_store, get_task_instance_name(pi, server))
        if status is None or not len(status.container_status.network_infos) or \
                not len(status.container_status.network_infos[0].ip_addresses):
            LOGGER.error("No previously stored TaskStatus to pull IP address from in Cassandra recovery")
            return None
        replace_ip = status.container_status.network_infos[0].ip_addresses[0].ip_address
        cmd = server.command
        new_cmd = CommandSpec(f"{cmd.value.strip()} -Dcassandra.replace_address={replace_ip} "
                              f"-Dcassandra.consistent.rangemovement=false\n", cmd.environment)
        new_server = dataclasses.replace(server, command=new_cmd)
        new_pod = dataclasses.replace(pod, tasks=tuple(new_server if t.name == SERVER_TASK else t for t in pod.tasks))
        replace_req = PodInstanceRequirement(PodInstance(new_pod, index), req.tasks_to_launch,
                                             recovery_type=RecoveryType.PERMANENT)
        steps = [RecoveryStep(launch_step.get_name(), replace_req, self.state_store)]
        if is_seed_node(index, self.seed_count):
            LOGGER.info("Scheduling restart of all nodes other than 'node-%d' to refresh seed node address.", index)
            for step in phase.get_children():
                sreq = step.get_pod_instance_requirement()
                if sreq.pod_instance.index == index:
                    continue
                steps.append(RecoveryStep(step.get_name(), PodInstanceRequirement(
                    sreq.pod_instance, sreq.tasks_to_launch, recovery_type=RecoveryType.TRANSIENT), self.state_store))
        return DefaultPhase(RECOVERY_PHASE_NAME, steps, SerialStrategy(), [])


class CassandraRecoveryPlanOverriderFactory(RecoveryPlanOverriderFactory):
    def __init__(self, seed_count: Optional[int] = None):
        self.seed_count = seed_count

    def create(self, state_store, plans) -> CassandraRecoveryPlanOverrider:
        plan = next((p for p in plans if p.get_name() == REPLACE_PLAN_NAME), None)
        if plan is None:
            raise RuntimeError(f"Failed to find plan: {REPLACE_PLAN_NAME}")
        return CassandraRecoveryPlanOverrider(state_store, plan,
                                              self.seed_count if self.seed_count is not None else seeds_count())


def custom_validators() -> List[ConfigValidator]:
    return [CassandraZoneValidator(),
            TaskEnvCannotChange(POD_TYPE, SERVER_TASK, "CASSANDRA_LOCATION_DATA_CENTER",
                                TaskEnvCannotChange.ALLOW_UNSET_TO_SET),
            TaskEnvCannotChange(POD_TYPE, SERVER_TASK, "CASSANDRA_LOCATION_RACK",
                                TaskEnvCannotChange.ALLOW_UNSET_TO_SET)]


def create_scheduler_builder(yaml_path: str, scheduler_config: Optional[SchedulerConfig] = None,
                             env: Optional[Dict[str, str]] = None, persister=None) -> SchedulerBuilder:
    env = dict(os.environ if env is None else env)
    cfg = scheduler_config or SchedulerConfig.from_env()
    raw = RawServiceSpec.new_builder(yaml_path).set_env(env).build()
    count = seeds_count(env)
    local_seeds = get_local_seeds(raw.name, cfg, count)
    gen = ServiceSpecGenerator(raw, cfg, os.path.dirname(os.path.abspath(yaml_path)), env)
    gen.set_all_pods_env("LOCAL_SEEDS", ",".join(local_seeds))
    yaml_b64 = env.get(AUTH_YAML_BASE64_ENV)
    if yaml_b64:
        gen.set_all_pods_env("AUTHENTICATION_CUSTOM_YAML_BLOCK", base64.b64decode(yaml_b64).decode("utf-8"))
    configured = list(local_seeds)
    remote = env.get("TASKCFG_ALL_REMOTE_SEEDS")
    if remote:
        configured.extend(s for s in remote.split(",") if s)
    return (SchedulerBuilder(gen.build(), cfg, persister)
            .set_custom_config_validators(custom_validators())
            .set_plans_from(raw)
            .set_custom_resources([SeedsResource(configured)])
            .set_recovery_manager_factory(CassandraRecoveryPlanOverriderFactory(count))
            .with_single_region_constraint())


def main(argv=None) -> int:
    from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner

    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 1:
        raise SystemExit(f"Expected one file argument, got: {argv}")
    from dcos_commons_amd.utils import logging_utils

    logging_utils.configure()
    from dcos_commons_amd.models import resolve_spec

    SchedulerRunner.from_scheduler_builder(create_scheduler_builder(resolve_spec(argv[0], "cassandra"))).run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
