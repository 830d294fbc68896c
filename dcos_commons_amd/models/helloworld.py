"""The hello-world reference service: entry modes, scenarios and example customizations.

Reference: frameworks/helloworld/src/main/java/com/mesosphere/sdk/helloworld/scheduler/{Main.java,
Scenario.java, ReversePhasesCustomizer.java, DecommissionCustomizer.java,
ExampleMultiServiceResource.java}.

Entry modes (``python -m dcos_commons_amd.models.helloworld [yaml[,yaml...]]``):
* ``SCENARIOS`` contains ``JAVA`` -> a service spec built in code (``sample_service_spec``);
* one YAML file -> a single-service scheduler;
* several YAML files -> one framework running each file as a namespaced service;
* no YAML -> dynamic multi-service: services are added/removed at runtime through
  ``/v1/multi`` (``ExampleMultiServiceResource``) and survive scheduler restarts (``ServiceStore``).

Scenarios (``SCENARIOS=YAML,CUSTOM_PLAN,...``): ``MULTI_REGION`` (single-region placement),
``CUSTOM_PLAN`` (deploy phases run their steps in reverse), ``CUSTOM_DECOMMISSION`` (every
decommission phase starts with an extra no-op step). YAML names resolve against
``frameworks/helloworld/specs`` (``HELLO_WORLD_SPEC_DIR`` overrides).
"""
from __future__ import annotations

import enum
import json
import logging
import os
import sys
from typing import Dict, Iterable, List, Mapping, Optional

from dcos_commons_amd.http.api import Route, json_ok, plain
from dcos_commons_amd.scheduler.plan.customizer import PlanCustomizer
from dcos_commons_amd.scheduler.plan.elements import AbstractStep, DefaultPhase, DefaultPlan
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.specification.specs import (
    CommandSpec,
    GoalState,
    PodSpec,
    ResourceSetBuilder,
    ServiceSpec,
    TaskSpec,
)
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec

LOGGER = logging.getLogger(__name__)

SPEC_DIR = os.environ.get("HELLO_WORLD_SPEC_DIR") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "frameworks", "helloworld", "specs")
YAML_EXT = ".yml"
CUSTOM_DECOMMISSION_STEP_NAME = "custom_decommission_step"


class Scenario(enum.Enum):
    YAML = "YAML"
    JAVA = "JAVA"
    CUSTOM_PLAN = "CUSTOM_PLAN"
    CUSTOM_DECOMMISSION = "CUSTOM_DECOMMISSION"
    MULTI_REGION = "MULTI_REGION"


def get_scenarios(env: Mapping[str, str]) -> List[Scenario]:
    out = []
    for raw in (env.get("SCENARIOS") or Scenario.YAML.value).split(","):
        raw = raw.strip()
        try:
            out.append(Scenario(raw.upper()))
        except ValueError:
            raise ValueError(f"Unable to parse SCENARIOS value '{raw}'. Expected one of: "
                             f"{[s.value for s in Scenario]}") from None
    return out


class ReversePhasesCustomizer(PlanCustomizer):
    """Runs every deploy phase's steps in reverse order."""

    def update_plan(self, plan):
        if plan.is_deploy_plan():
            for phase in plan.get_children():
                phase.get_children().reverse()
        return plan


class _CustomStep(AbstractStep):
    def __init__(self, namespace: Optional[str]):
        super().__init__(CUSTOM_DECOMMISSION_STEP_NAME, namespace)

    def start(self) -> None:
        self._set_status(Status.COMPLETE)


class DecommissionCustomizer(PlanCustomizer):
    """Prepends a custom step to every phase of the decommission plan."""

    def __init__(self, namespace: Optional[str] = None):
        self.namespace = namespace

    def update_plan(self, plan):
        if not plan.is_decommission_plan():
            return plan
        phases = [DefaultPhase(ph.get_name(), [_CustomStep(self.namespace)] + list(ph.get_children()),
                               SerialStrategy(), ph.get_errors()) for ph in plan.get_children()]
        return DefaultPlan(plan.get_name(), phases)


def customize(builder: SchedulerBuilder, namespace: Optional[str], scenarios: Iterable[Scenario]) -> SchedulerBuilder:
    for s in scenarios:
        if s == Scenario.MULTI_REGION:
            builder.with_single_region_constraint()
        elif s == Scenario.CUSTOM_PLAN:
            builder.set_plan_customizer(ReversePhasesCustomizer())
        elif s == Scenario.CUSTOM_DECOMMISSION:
            builder.set_plan_customizer(DecommissionCustomizer(namespace))
    return builder


def sample_service_spec(env: Mapping[str, str]) -> ServiceSpec:
    """The service Main builds in code for the JAVA scenario (createSampleServiceSpec)."""
    from dcos_commons_amd.config.task_env_router import TaskEnvRouter

    rs = ResourceSetBuilder("hello-world-role", "*", "hello-world-principal")
    rs.id = "hello-resources"
    rs.cpus(float(env["HELLO_CPUS"])).memory(256.0).add_volume("ROOT", 5000.0, "hello-container-path")
    task = TaskSpec(name="hello", goal=GoalState.RUNNING, resource_set=rs.build(),
                    command=CommandSpec.build("echo hello >> hello-container-path/output && sleep 1000",
                                              TaskEnvRouter(env).get_config("hello"), None))
    pod = PodSpec(type="hello", count=int(env["HELLO_COUNT"]), tasks=(task,))
    return ServiceSpec.create("hello-world", [pod], principal="hello-world-principal",
                              zookeeper_connection="master.mesos:2181")


def yaml_file(name: str) -> str:
    return os.path.join(SPEC_DIR, name + YAML_EXT) if not name.endswith(YAML_EXT) else name


# -- dynamic multi-service -------------------------------------------------------------------
class ExampleMultiServiceResource:
    """``/v1/multi``: list services / available YAMLs, add a service from a YAML + env overrides,
    trigger a service's uninstall. Service contexts are persisted by ``ServiceStore`` so a restarted
    scheduler recovers them (``recover``)."""

    def __init__(self, scheduler_config, framework_config, persister, scenarios, manager, env=None):
        from dcos_commons_amd.scheduler.multi import ServiceStore

        self.manager = manager
        self.base_env = dict(os.environ if env is None else env)

        def factory(context: bytes):
            data = json.loads(context.decode("utf-8"))
            params = dict(self.base_env)
            params.update({p["key"]: p["value"] for p in data.get("params", [])})
            path = yaml_file(data["yaml"])
            raw = RawServiceSpec.new_builder(path).set_env(params).build()
            spec = (ServiceSpecGenerator(raw, scheduler_config, os.path.dirname(path), params)
                    .set_multi_service_framework_config(framework_config).build())
            builder = (SchedulerBuilder(spec, scheduler_config, persister).set_plans_from(raw)
                       .enable_multi_service(framework_config.framework_name))
            return customize(builder, framework_config.framework_name, scenarios).build()

        self.store = ServiceStore(persister, factory)

    @staticmethod
    def serialize(name: str, yaml_name: str, env_override: Mapping[str, str]) -> bytes:
        params = [{"key": k, "value": v} for k, v in sorted(env_override.items())]
        return json.dumps({"name": name, "yaml": yaml_name, "params": params}).encode("utf-8")

    def routes(self):
        return [Route("GET", "/v1/multi/yaml", self.list_yamls), Route("GET", "/v1/multi", self.list_services),
                Route("POST", "/v1/multi/{name}", self.add), Route("DELETE", "/v1/multi/{name}", self.uninstall)]

    def list_yamls(self, req):
        return json_ok(sorted(f[:-len(YAML_EXT)] for f in os.listdir(SPEC_DIR) if f.endswith(YAML_EXT)))

    def list_services(self, req):
        from dcos_commons_amd.scheduler.uninstall import UninstallScheduler

        out = []
        for name in self.manager.get_service_names():
            svc = self.manager.get_service(name)
            if svc is None:
                continue
            entry = {"service": name, "uninstall": isinstance(svc, UninstallScheduler)}
            ctx = self.store.get(name)
            if ctx is not None:
                entry["yaml"] = json.loads(ctx.decode("utf-8"))["yaml"]
            out.append(entry)
        return json_ok(out)

    def add(self, req):
        name, yaml_name = req.params["name"], req.q("yaml")
        try:
            override = req.json() or {}
            if not yaml_name or not os.path.exists(yaml_file(yaml_name)):
                raise ValueError(f"unknown yaml '{yaml_name}'")
            service = self.store.put(self.serialize(name, yaml_name, {str(k): str(v) for k, v in override.items()}))
        except Exception as e:  # noqa: BLE001
            LOGGER.error("Failed to generate or persist service: %s", e)
            return plain(f"Failed to generate or persist service: {e}", 400)
        self.manager.put_service(service)
        return json_ok({"name": service.service_spec.name, "yaml": yaml_name})

    def uninstall(self, req):
        self.manager.uninstall_service(req.params["name"])
        return plain(f"Triggered removal of service: {req.params['name']}")

    def recover(self) -> None:
        for service in self.store.recover():
            self.manager.put_service(service)

    def uninstall_callback(self):
        return self.store.uninstall_callback()


# -- entry point ----------------------------------------------------------------------------
def run(args: List[str], env: Optional[Dict[str, str]] = None, scheduler_config=None, persister=None,
        driver_factory=None, block: bool = True):
    """Starts the scheduler for ``args`` (comma/space separated YAML names); returns the runner."""
    from dcos_commons_amd.framework.env_store import EnvStore
    from dcos_commons_amd.framework.framework_config import FrameworkConfig
    from dcos_commons_amd.scheduler.multi import MultiServiceEventClient, MultiServiceManager, MultiServiceRunner
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
    from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner
    from dcos_commons_amd.storage.factory import persister_for_service

    env = dict(os.environ if env is None else env)
    cfg = scheduler_config or SchedulerConfig.from_env()
    scenarios = get_scenarios(env)
    LOGGER.info("Using scenarios: %s", [s.value for s in scenarios])
    if Scenario.JAVA in scenarios:
        builder = SchedulerBuilder(sample_service_spec(env), cfg, persister)
        runner = SchedulerRunner.from_scheduler_builder(customize(builder, None, scenarios),
                                                        driver_factory=driver_factory)
        runner.run(block=block)
        return runner
    yamls = [yaml_file(y.strip()) for a in args for y in a.split(",") if y.strip()]
    if len(yamls) == 1:
        raw = RawServiceSpec.new_builder(yamls[0]).set_env(env).build()
        spec = ServiceSpecGenerator(raw, cfg, os.path.dirname(yamls[0]), env).build()
        builder = SchedulerBuilder(spec, cfg, persister).set_plans_from(raw)
        runner = SchedulerRunner.from_scheduler_builder(customize(builder, None, scenarios),
                                                        driver_factory=driver_factory)
        runner.run(block=block)
        return runner
    fc = FrameworkConfig.from_env_store(EnvStore(env))
    if persister is None:
        persister = persister_for_service(type("S", (), {"name": fc.framework_name,
                                                         "zookeeper_connection": fc.zookeeper_host_port})(), cfg)
    manager = MultiServiceManager()
    if yamls:
        from dcos_commons_amd.storage.persister_utils import check_and_migrate

        check_and_migrate(fc.framework_name, persister)
        for path in yamls:
            raw = RawServiceSpec.new_builder(path).set_env(env).build()
            spec = (ServiceSpecGenerator(raw, cfg, os.path.dirname(path), env)
                    .set_multi_service_framework_config(fc).build())
            builder = (SchedulerBuilder(spec, cfg, persister).set_plans_from(raw)
                       .enable_multi_service(fc.framework_name))
            manager.put_service(customize(builder, fc.framework_name, scenarios).build())
        client = MultiServiceEventClient(fc.framework_name, cfg, manager, persister,
                                         uninstall_callback=lambda n: LOGGER.info("Service completed uninstall: %s", n))
    else:
        resource = ExampleMultiServiceResource(cfg, fc, persister, scenarios, manager, env)
        resource.recover()
        client = MultiServiceEventClient(fc.framework_name, cfg, manager, persister, custom_endpoints=[resource],
                                         uninstall_callback=resource.uninstall_callback())
    runner = MultiServiceRunner(cfg, fc, persister, client,
                                using_gpus=str(env.get("FRAMEWORK_GPUS", "")).lower() == "true",
                                driver_factory=driver_factory)
    runner.run(block=block)
    return runner


def main(argv=None) -> int:
    from dcos_commons_amd.utils import logging_utils

    logging_utils.configure()
    run(sys.argv[1:] if argv is None else argv)
    return 0


if __name__ == "__main__":
    sys.exit(main())
