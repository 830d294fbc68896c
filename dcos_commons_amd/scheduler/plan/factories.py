"""Step / phase / plan factories and the YAML ``plans:`` generator.

Reference: sdk/.../scheduler/plan/{DefaultStepFactory,DefaultPhaseFactory,DeployPlanFactory}.java
and sdk/.../specification/PlanGenerator.java:39-302.
"""
from __future__ import annotations

import logging
import traceback
from typing import Dict, List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader
from dcos_commons_amd.specification.specs import GoalState, PodInstance, PodSpec, ServiceSpec

from .deployment_step import DeploymentStep
from .elements import DefaultPhase, DefaultPlan
from .pod_instance_requirement import PodInstanceRequirement
from .status import Status
from .strategy import (
    CanaryStrategy,
    DependencyStrategy,
    DependencyStrategyHelper,
    SerialStrategy,
    phase_strategy_generator,
    plan_strategy_generator,
    serial_generator,
)

LOGGER = logging.getLogger(__name__)
DEFAULT_POD_INDEX_LABEL = "default"
PARALLEL_STRATEGY_TYPES = ("parallel", "parallel-canary")


def step_name(pod_instance: PodInstance, tasks: List[str]) -> str:
    return f"{pod_instance.name}:[{', '.join(tasks)}]"


class DefaultStepFactory:
    def __init__(self, config_target_store, state_store, namespace: Optional[str] = None):
        self.config_target_store = config_target_store
        self.state_store = state_store
        self.namespace = namespace

    def get_step(self, pod_instance: PodInstance, tasks_to_launch: List[str]) -> DeploymentStep:
        try:
            self._validate(pod_instance, tasks_to_launch)
            infos = []
            for t in pod_instance.pod.tasks:
                if t.name in tasks_to_launch:
                    info = self.state_store.fetch_task_shared(f"{pod_instance.name}-{t.name}")
                    if info is not None:
                        infos.append(info)
            status = Status.PENDING if not infos else self._status(pod_instance, infos)
            return DeploymentStep(step_name(pod_instance, tasks_to_launch),
                                  PodInstanceRequirement(pod_instance, tasks_to_launch),
                                  self.state_store, self.namespace).update_initial_status(status)
        except Exception as e:  # noqa: BLE001
            LOGGER.error("Failed to generate Step: %s", e)
            return DeploymentStep(pod_instance.name, PodInstanceRequirement(pod_instance, []), self.state_store,
                                  self.namespace).add_error("".join(traceback.format_exception(e)))

    @staticmethod
    def _validate(pod_instance: PodInstance, tasks: List[str]) -> None:
        specs = [t for t in pod_instance.pod.tasks if t.name in tasks]
        rs_ids = [t.resource_set.id for t in specs]
        if len(set(rs_ids)) < len(rs_ids):
            raise ValueError(
                f"Attempted to simultaneously launch tasks: {tasks} in pod: {pod_instance.name} using the same "
                f"resource set id: {rs_ids}. These tasks should either be run in separate steps or use different "
                "resource set ids")
        prefixes = [t.discovery.prefix for t in specs if t.discovery is not None and t.discovery.prefix]
        if len(set(prefixes)) < len(prefixes):
            raise ValueError(
                f"Attempted to simultaneously launch tasks: {tasks} in pod: {pod_instance.name} using the same DNS "
                f"name: {prefixes}. These tasks should either be run in separate steps or use different DNS names")

    def _status(self, pod_instance: PodInstance, infos: List[P.TaskInfo]) -> Status:
        from dcos_commons_amd.offer.task_utils import get_goal_state, is_permanently_failed

        target = self.config_target_store.get_target_config()
        for info in infos:
            goal = get_goal_state(pod_instance, info.name)
            reached = self.has_reached_goal_state(info, goal, target)
            if not (reached or is_permanently_failed(info)):
                return Status.PENDING
        return Status.COMPLETE

    def has_reached_goal_state(self, info: P.TaskInfo, goal: GoalState, target_config_id) -> bool:
        status = self.state_store.fetch_status(info.name)
        if status is None:
            return False
        reader = TaskLabelReader(info)
        if goal == GoalState.RUNNING:
            if status.state != P.TASK_RUNNING:
                return False
            return reader.get_target_configuration() == target_config_id and \
                reader.is_readiness_check_succeeded(status)
        if goal == GoalState.FINISH:
            return status.state == P.TASK_FINISHED and reader.get_target_configuration() == target_config_id
        if goal == GoalState.ONCE:
            return status.state == P.TASK_FINISHED
        raise ValueError(f"Unsupported goal state for task {info.name}: {goal}")


class DefaultPhaseFactory:
    def __init__(self, step_factory):
        self.step_factory = step_factory

    def get_phase(self, pod_spec: PodSpec, strategy=None) -> DefaultPhase:
        steps = []
        for i in range(pod_spec.count):
            pi = PodInstance(pod_spec, i)
            steps.append(self.step_factory.get_step(pi, [t.name for t in pod_spec.tasks]))
        return DefaultPhase(pod_spec.type, steps, strategy if strategy is not None else SerialStrategy(), [])


class DeployPlanFactory:
    def __init__(self, phase_factory: DefaultPhaseFactory, strategy_generator=serial_generator):
        self.phase_factory = phase_factory
        self.strategy_generator = strategy_generator

    def get_plan(self, service_spec: ServiceSpec) -> DefaultPlan:
        phases = [self.phase_factory.get_phase(p) for p in service_spec.pods]
        return DefaultPlan(constants.DEPLOY_PLAN_NAME, phases, self.strategy_generator(phases))


class PlanGenerator:
    """Builds plans from the YAML ``plans:`` section."""

    def __init__(self, step_factory):
        self.step_factory = step_factory

    def generate(self, raw_plan: Dict, plan_name: str, pod_specs) -> DefaultPlan:
        phases = [self._phase(raw_phase or {}, phase_name, pod_specs)
                  for phase_name, raw_phase in (raw_plan.get("phases") or {}).items()]
        return DefaultPlan(plan_name, phases, plan_strategy_generator(raw_plan.get("strategy"))(phases))

    def _phase(self, raw_phase: Dict, phase_name: str, pod_specs) -> DefaultPhase:
        pod = next((p for p in pod_specs if p.type == raw_phase.get("pod")), None)
        if pod is None:
            raise ValueError(f"Unable to find pod '{raw_phase.get('pod')}' referenced by phase '{phase_name}'")
        strategy = raw_phase.get("strategy")
        raw_steps = raw_phase.get("steps")
        if not raw_steps:
            steps = [self._step(PodInstance(pod, i), [t.name for t in pod.tasks]) for i in range(pod.count)]
            return DefaultPhase(phase_name, steps, phase_strategy_generator(strategy)(steps), [])
        index_to_tasks: Dict[str, List[List[str]]] = {}
        for entry in raw_steps:
            if not isinstance(entry, dict) or len(entry) != 1:
                raise ValueError(f"Malformed step in phase '{phase_name}': Map should contain a single entry, "
                                 f"but has {len(entry) if isinstance(entry, dict) else 'none'}: {entry}")
            (k, v), = entry.items()
            index_to_tasks[str(k)] = v
        if strategy in PARALLEL_STRATEGY_TYPES:
            helper = DependencyStrategyHelper([])
            all_steps = []
            for i in range(pod.count):
                task_lists = self._task_lists(index_to_tasks, i, phase_name)
                pod_steps = []
                for names in task_lists:
                    step = self._step(PodInstance(pod, i), list(names))
                    if not pod_steps:
                        helper.add_element(step)
                    else:
                        for prev in pod_steps:
                            helper.add_dependency(step, prev)
                    pod_steps.append(step)
                all_steps.extend(pod_steps)
            strat = DependencyStrategy(helper)
            if strategy.endswith("-canary"):
                strat = CanaryStrategy(strat, all_steps)
            return DefaultPhase(phase_name, all_steps, strat, [])
        steps = []
        for i in range(pod.count):
            for names in self._task_lists(index_to_tasks, i, phase_name):
                steps.append(self._step(PodInstance(pod, i), list(names)))
        return DefaultPhase(phase_name, steps, phase_strategy_generator(strategy)(steps), [])

    @staticmethod
    def _task_lists(index_to_tasks, i: int, phase_name: str):
        lists = index_to_tasks.get(str(i))
        if lists is None:
            lists = index_to_tasks.get(DEFAULT_POD_INDEX_LABEL)
            if lists is None:
                raise ValueError(f"Malformed steps in phase '{phase_name}': Missing '{i}' step entry, and no "
                                 "'default' defined")
        return lists

    def _step(self, pod_instance: PodInstance, tasks: List[str]):
        names = {t.name for t in pod_instance.pod.tasks}
        if not set(tasks) <= names:
            raise ValueError("Malformed step: step refers to a task that does not exist")
        return self.step_factory.get_step(pod_instance, tasks)
