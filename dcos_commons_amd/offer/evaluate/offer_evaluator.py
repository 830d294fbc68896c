"""The core offer matcher.

Reference: sdk/.../offer/evaluate/OfferEvaluator.java:65-857. For one ``PodInstanceRequirement``
it builds the stage pipeline once -- *new* (first launch / permanent replace: placement, fresh
reservations) or *existing* (relaunch in place on the pod's reservations, reusing a live executor)
-- then runs it against each offer with a fresh ``MesosResourcePool`` and ``PodInfoBuilder``, and
returns the recommendations of the first offer that passes every stage.

MI355X-first notes: the evaluator is the CPU hot loop of the scheduler (the reference has no
numeric kernels). ``evaluate`` reads the StateStore once per call (not per offer), and callers may
pass a pre-fetched task map (``all_tasks``) so a whole offer cycle touches storage once.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

from dcos_commons_amd import trace
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import task_utils
from dcos_commons_amd.offer.history import OfferOutcome, OfferOutcomeTracker, OfferOutcomeTrackerV2
from dcos_commons_amd.offer.resource_pool import MesosResourcePool
from dcos_commons_amd.offer.resources import get_resource_id, new_reservation, new_root_volume
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement, RecoveryType
from dcos_commons_amd.specification.specs import GoalState, NamedVIPSpec, PortSpec, ResourceSpec, VolumeType
from dcos_commons_amd.utils.logging_utils import get_logger

from .outcome import EvaluationOutcome
from .pod_info_builder import PodInfoBuilder
from .resource_mappers import ExecutorResourceMapper, TaskResourceMapper
from .stages import (
    DestroyEvaluationStage,
    ExecutorEvaluationStage,
    LaunchEvaluationStage,
    NamedVIPEvaluationStage,
    PlacementRuleEvaluationStage,
    PortEvaluationStage,
    ResourceEvaluationStage,
    UnreserveEvaluationStage,
    VolumeEvaluationStage,
    get_role,
)


def _ordered_resource_specs(resource_set) -> List[ResourceSpec]:
    static_ports, dynamic_ports, simple = [], [], []
    for r in resource_set.resources:
        if isinstance(r, PortSpec):
            (dynamic_ports if r.port == 0 else static_ports).append(r)
        else:
            simple.append(r)
    return static_ports + dynamic_ports + simple


def _executor_resource_specs(scheduler_config, role: str, principal: str, pre_reserved_role: str):
    return [ResourceSpec(name=name, value=value, role=role, principal=principal, pre_reserved_role=pre_reserved_role)
            for name, value in sorted(scheduler_config.executor_resources().items())]


def _outcome_lines(outcome, indent: str = "") -> List[str]:
    lines = [f"  {indent}{outcome}"]
    for c in outcome.children:
        lines.extend(_outcome_lines(c, indent + "  "))
    return lines


def _outcome_reasons(out: List[str], outcome) -> None:
    out.append(f"{'PASS' if outcome.passing else 'FAIL'}({outcome.source}):{outcome.reason}")
    for c in outcome.children:
        _outcome_reasons(out, c)


def _required_reservations(stages) -> set:
    """Reservation IDs the pipeline's task resource and volume stages consume by ID (executor
    resources are left out: a running executor's are not taken from the offer)."""
    return {s.resource_id for s in stages
            if isinstance(s, (ResourceEvaluationStage, VolumeEvaluationStage)) and s.task_names and s.resource_id}


class _LazyText:
    """Renders on first ``str()`` (log formatting) or ``render()`` (debug trackers), once."""

    __slots__ = ("_fn", "_text")

    def __init__(self, fn):
        self._fn, self._text = fn, None

    def render(self) -> str:
        if self._text is None:
            self._text = self._fn()
        return self._text

    __str__ = render


class OfferEvaluator:
    def __init__(self, framework_store, state_store, service_name: str, target_config_id, template_url_factory,
                 scheduler_config, resource_namespace: Optional[str] = None,
                 offer_outcome_tracker: Optional[OfferOutcomeTracker] = None,
                 offer_outcome_tracker_v2: Optional[OfferOutcomeTrackerV2] = None, tls_stage_factory=None):
        self.framework_store = framework_store
        self.state_store = state_store
        self.service_name = service_name
        self.target_config_id = target_config_id
        self.template_url_factory = template_url_factory
        self.scheduler_config = scheduler_config
        self.resource_namespace = resource_namespace
        self.offer_outcome_tracker = offer_outcome_tracker
        self.offer_outcome_tracker_v2 = offer_outcome_tracker_v2
        self.tls_stage_factory = tls_stage_factory
        self._framework_id: Optional[str] = None
        self._executor_specs: Dict[tuple, List[ResourceSpec]] = {}
        # untouched PodInfoBuilder templates, reused across offer cycles (see _template)
        self._templates: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.logger = get_logger(__name__, resource_namespace)

    _TEMPLATE_CACHE_SIZE = 512

    def _template(self, requirement: PodInstanceRequirement, target_config, override_map,
                  fid_proto: P.FrameworkID) -> PodInfoBuilder:
        """The offer-independent PodInfoBuilder of a requirement: every task's command,
        environment, checks, labels and container info, and the executor. Building it renders the
        pod's whole task environment (a reference hdfs or cassandra task carries hundreds of
        variables), so it is built once per (pod instance, target config, requirement env, goal
        overrides) and every evaluation -- each offer cycle, each offer -- works on a copy. The
        first instance's template is also kept per pod type: the other instances are moved from it
        (``PodInfoBuilder.for_instance``), so an N-pod parallel deploy renders the tasks once."""
        pi = requirement.pod_instance
        shared = (pi.pod.type, str(target_config), tuple(sorted(requirement.environment.items())),
                  tuple(sorted((k, str(v)) for k, v in override_map.items())), fid_proto.value)
        key = (pi.index,) + shared
        hit = self._templates.get(key)
        if hit is not None and hit[0] is pi.pod:
            self._templates.move_to_end(key)
            return hit[1]
        tpl = None
        # another instance of the pod with the same inputs: move its template to this index
        # (PodInfoBuilder.for_instance) instead of rendering every task again
        sibling = self._templates.get(shared)
        if sibling is not None and sibling[0] is pi.pod:
            tpl = sibling[1].for_instance(pi)
        if tpl is None:
            tpl = PodInfoBuilder(requirement, self.service_name, target_config, self.template_url_factory,
                                 self.scheduler_config, (), fid_proto, override_map)
            self._templates[shared] = (pi.pod, tpl)
        self._templates[key] = (pi.pod, tpl)
        while len(self._templates) > self._TEMPLATE_CACHE_SIZE:
            self._templates.popitem(last=False)
        return tpl

    def _executor_specs_for(self, role: str, principal: str, pre_reserved_role: str) -> List[ResourceSpec]:
        """The executor's resource specs (immutable) for one role/principal, built once."""
        key = (role, principal, pre_reserved_role)
        specs = self._executor_specs.get(key)
        if specs is None:
            specs = self._executor_specs[key] = _executor_resource_specs(self.scheduler_config, role, principal,
                                                                         pre_reserved_role)
        return specs

    def _fid(self) -> P.FrameworkID:
        fid = self.framework_store.fetch_framework_id()
        if fid is None:
            raise RuntimeError("FrameworkID is not yet stored; cannot evaluate offers before registration")
        return fid

    def evaluate(self, requirement: PodInstanceRequirement, offers: Sequence[P.Offer],
                 all_tasks: Optional[Dict[str, P.TaskInfo]] = None) -> list:
        if not trace.enabled():
            return self._evaluate(requirement, offers, all_tasks)
        with trace.span("evaluate", "offers", step=requirement.name, offers=len(offers)) as sp:
            recs = self._evaluate(requirement, offers, all_tasks)
            sp.set(recs=len(recs))
            return recs

    def _evaluate(self, requirement: PodInstanceRequirement, offers: Sequence[P.Offer],
                  all_tasks: Optional[Dict[str, P.TaskInfo]]) -> list:
        fid_proto = self._fid()
        if self._framework_id is None:
            self._framework_id = fid_proto.value
        if not offers:
            return []  # nothing to match: the pipeline would be built for no offer
        if all_tasks is None:
            all_tasks = {t.name: t for t in self.state_store.fetch_tasks_shared()}
        pi = requirement.pod_instance
        this_pod = {}
        for name in task_utils.get_task_names(pi):
            t = all_tasks.get(name)
            if t is not None:
                this_pod[name] = t
        stages = self.get_evaluation_pipeline(requirement, list(all_tasks.values()), this_pod)
        role = get_role(pi.pod)
        override_map = {ts.name: self.state_store.fetch_goal_override_status(f"{pi.name}-{ts.name}").target
                        for ts in pi.pod.tasks}
        target_config = self.get_target_config(requirement, this_pod)
        required = _required_reservations(stages)
        template = None
        prior_ports = None
        for i, offer in enumerate(offers):
            if required:
                missing = required.difference(get_resource_id(r) for r in offer.resources)
                if missing:
                    # an in-place relaunch consumes these reservations by ID: an offer without
                    # one of them fails its resource/volume stage whatever else it holds (e.g. an
                    # offer from another agent, or from the pod's agent while a killed task still
                    # holds them), so the pipeline is not run on it
                    o = EvaluationOutcome.fail(
                        "ReservationPrecheck", "Offer lacks %d of the %d reservation(s) this relaunch reuses: %s",
                        len(missing), len(required), sorted(missing))
                    self.logger.info("Offer %d, %s: %s for %s", i + 1, offer.id.value, o.reason, requirement.name)
                    self._track(requirement, False, offer, lambda o=o: "\n".join(_outcome_lines(o)), [o])
                    continue
            pool = MesosResourcePool(offer, role)
            # each offer's stages work on a copy of the cached offer-independent template, with
            # this pod's prior ports
            if template is None:
                template = self._template(requirement, target_config, override_map, fid_proto)
                prior_ports = PodInfoBuilder.prior_ports(this_pod.values())
            builder = template.clone()
            builder.ports_by_task = prior_ports
            outcomes = []
            failed = 0
            for stage in stages:
                o = stage.evaluate(pool, builder)
                outcomes.append(o)
                if not o.passing:
                    failed += 1
            details = _LazyText(lambda outcomes=outcomes: "\n".join(
                line for o in outcomes for line in _outcome_lines(o)))
            if failed:
                self.logger.info("Offer %d, %s: failed %d of %d evaluation stages for %s:\n%s", i + 1,
                                 offer.id.value, failed, len(stages), requirement.name, details)
                self._track(requirement, False, offer, details.render, outcomes)
                continue
            recs = [r for o in outcomes for r in o.get_offer_recommendations()]
            self.logger.info("Offer %d: passed all %d evaluation stages, returning %d recommendations for %s",
                             i + 1, len(stages), len(recs), requirement.name)
            self._track(requirement, True, offer, details.render, outcomes)
            return recs
        return []

    def prewarm(self, requirement: PodInstanceRequirement, stop=lambda: False) -> bool:
        """Builds what the first evaluation of a new footprint for ``requirement`` would build
        before it could match an offer: the pod's PodInfoBuilder template (the other instances
        are moved from it) and the wire templates of its new reservations and ROOT volumes. The
        scheduler runs it for its candidate steps between registering and its first offers,
        which is a master round trip of idle time (``OfferProcessor._loop``); without it the
        first pod of every deploy pays ~2x the evaluation of the next ones. ``stop()`` is asked
        between the pieces; False when it ended the prewarm early."""
        fid_proto = self._fid()
        if self._framework_id is None:
            self._framework_id = fid_proto.value
        pi = requirement.pod_instance
        this_pod = {}
        for name in task_utils.get_task_names(pi):
            t = self.state_store.fetch_task_shared(name)
            if t is not None:
                this_pod[name] = t
        if not self._uses_new_pipeline(requirement, this_pod):
            return True     # a relaunch on existing reservations: nothing new is built
        override_map = {ts.name: self.state_store.fetch_goal_override_status(f"{pi.name}-{ts.name}").target
                        for ts in pi.pod.tasks}
        self._template(requirement, self.get_target_config(requirement, this_pod), override_map, fid_proto)
        ns, fid = self.resource_namespace, self._framework_id
        tasks = sorted(pi.pod.tasks, key=lambda t: t.name)
        if not tasks:
            return True
        first = _ordered_resource_specs(tasks[0].resource_set)
        specs = list(self._executor_specs_for(first[0].role, first[0].principal, first[0].pre_reserved_role)) \
            if first else []
        volumes = list(pi.pod.volumes)
        for ts in tasks:
            specs.extend(r for r in ts.resource_set.resources if not isinstance(r, (PortSpec, NamedVIPSpec)))
            volumes.extend(ts.resource_set.volumes)
        for spec in specs:
            if stop():
                return False
            new_reservation(spec, ns, fid)
        for v in volumes:
            if v.type == VolumeType.ROOT:
                if stop():
                    return False
                new_reservation(v, ns, fid)
                new_root_volume(v, "00000000-0000-4000-8000-000000000000", ns, fid)
        return True

    def _track(self, requirement, passed, offer, details, outcomes) -> None:
        if self.offer_outcome_tracker is not None:
            self.offer_outcome_tracker.track(OfferOutcome(requirement.name, passed, offer, details))
        if self.offer_outcome_tracker_v2 is not None:
            def reasons(outcomes=outcomes) -> List[str]:
                out: List[str] = []
                for o in outcomes:
                    _outcome_reasons(out, o)
                return out

            s = self.offer_outcome_tracker_v2.summary
            s.add_offer(OfferOutcome(requirement.name, passed, offer, reasons))
            if not passed:
                s.add_failure_agent(offer.agent_id.value)
                for o in outcomes:
                    if not o.passing:
                        s.add_failure_reason(o.source)

    # -- pipelines ---------------------------------------------------------------------
    @staticmethod
    def _uses_new_pipeline(requirement: PodInstanceRequirement, this_pod: Dict[str, P.TaskInfo]) -> bool:
        """New footprint (OfferEvaluator.java:250-262): a permanent replace, a pod whose tasks are
        all permanently failed, or one that never reserved anything; otherwise an in-place relaunch
        on the pod's existing reservations."""
        ids = [get_resource_id(r) for t in this_pod.values() for r in t.resources]
        no_launched = all((i or "") == "" for i in ids if i is not None)
        all_perm_failed = bool(this_pod) and all(TaskLabelReader(t).is_permanently_failed()
                                                 for t in this_pod.values())
        return requirement.recovery_type == RecoveryType.PERMANENT or all_perm_failed or no_launched

    def get_evaluation_pipeline(self, requirement: PodInstanceRequirement, all_tasks, this_pod: Dict[str, P.TaskInfo]):
        new = self._uses_new_pipeline(requirement, this_pod)
        pod = requirement.pod_instance.pod
        tls = self.tls_stage_factory if any(t.transport_encryption for t in pod.tasks) else None
        if new:
            return self._new_pipeline(requirement, all_tasks, tls)
        executor_info = self._executor_info(requirement, this_pod)
        eid = executor_info.executor_id if executor_info.executor_id.value else None
        return [ExecutorEvaluationStage(self.service_name, eid)] + \
            self._existing_pipeline(requirement, this_pod, all_tasks, executor_info, tls)

    def _executor_info(self, requirement, this_pod: Dict[str, P.TaskInfo]) -> P.ExecutorInfo:
        names = task_utils.get_task_names(requirement.pod_instance, requirement.tasks_to_launch)
        for t in this_pod.values():
            if t.name in names:
                continue
            if self._has_reusable_executor(t):
                return t.executor
        first = next(iter(this_pod.values()))
        e = P.ExecutorInfo()
        e.CopyFrom(first.executor)
        e.executor_id.value = ""
        return e

    def _has_reusable_executor(self, t: P.TaskInfo) -> bool:
        status = self.state_store.fetch_status(t.name)
        if status is None or TaskLabelReader(t).is_permanently_failed():
            return False
        return status.state in (P.TASK_STAGING, P.TASK_STARTING, P.TASK_RUNNING)

    def _new_pipeline(self, requirement, all_tasks, tls):
        pi = requirement.pod_instance
        pod = pi.pod
        ns, fid = self.resource_namespace, self._framework_id
        stages = [ExecutorEvaluationStage(self.service_name, None)]
        if pod.placement_rule is not None:
            stages.append(PlacementRuleEvaluationStage(all_tasks, pod.placement_rule))
        for v in pod.volumes:
            stages.append(VolumeEvaluationStage.get_new(v, [], ns, fid))
        if tls is not None:
            for ts in pod.tasks:
                if ts.transport_encryption:
                    stages.append(tls(ts.name))
        rs_by_task = {ts.name: ts.resource_set for ts in sorted(pod.tasks, key=lambda t: t.name)}
        added_executor = False
        added_sets = set()
        for task_name, rs in rs_by_task.items():
            specs = _ordered_resource_specs(rs)
            if not added_executor:
                added_executor = True
                for spec in self._executor_specs_for(specs[0].role, specs[0].principal, specs[0].pre_reserved_role):
                    stages.append(ResourceEvaluationStage(spec, [], None, ns, fid))
            if rs.id not in added_sets:
                names = sorted(n for n, r in rs_by_task.items() if r.id == rs.id)
                added_sets.add(rs.id)
                for spec in specs:
                    if isinstance(spec, NamedVIPSpec):
                        stages.append(NamedVIPEvaluationStage(spec, names, None, ns, fid))
                    elif isinstance(spec, PortSpec):
                        stages.append(PortEvaluationStage(spec, names, None, ns, fid))
                    else:
                        stages.append(ResourceEvaluationStage(spec, names, None, ns, fid))
                for v in rs.volumes:
                    stages.append(VolumeEvaluationStage.get_new(v, names, ns, fid))
            stages.append(LaunchEvaluationStage(self.service_name, task_name,
                                                task_name in requirement.tasks_to_launch))
        return stages

    def _existing_pipeline(self, requirement, this_pod, all_tasks, executor_info, tls):
        pi = requirement.pod_instance
        pod = pi.pod
        ns, fid = self.resource_namespace, self._framework_id
        stages = []
        if tls is not None:
            for ts in pod.tasks:
                if ts.transport_encryption:
                    stages.append(tls(ts.name))
        if pod.placement_rule is not None and requirement.recovery_type == RecoveryType.PERMANENT:
            stages.append(PlacementRuleEvaluationStage(all_tasks, pod.placement_rule))
        first_spec = next(r for ts in pod.tasks for r in ts.resource_set.resources)
        mapper = ExecutorResourceMapper(
            pod, self._executor_specs_for(first_spec.role, first_spec.principal, first_spec.pre_reserved_role),
            executor_info.resources, ns, fid)
        for r in mapper.orphaned_resources:
            stages.append(DestroyEvaluationStage(r))
        for r in mapper.orphaned_resources:
            stages.append(UnreserveEvaluationStage(r))
        stages.extend(mapper.evaluation_stages)
        rs_by_task = {ts.name: ts.resource_set for ts in sorted(pod.tasks, key=lambda t: t.name)}
        updated = set()
        for task_name in requirement.tasks_to_launch:
            rs = rs_by_task.get(task_name)
            if rs is None:
                raise ValueError(f"Unable to find task to launch {task_name} among defined tasks "
                                 f"{list(rs_by_task)} in pod {requirement.name}. Malformed ServiceSpec?")
            if rs.id in updated:
                continue
            updated.add(rs.id)
            names_in_set = sorted(n for n, r in rs_by_task.items() if r.id == rs.id)
            infos = [this_pod.get(f"{pi.name}-{n}") for n in names_in_set]
            info = next((x for x in infos if x is not None), None)
            if info is not None:
                tm = TaskResourceMapper(names_in_set, rs, info, ns, fid)
                for r in tm.orphaned_resources:
                    stages.append(UnreserveEvaluationStage(r))
                stages.extend(tm.evaluation_stages)
            for n in names_in_set:
                stages.append(LaunchEvaluationStage(self.service_name, n, n in requirement.tasks_to_launch))
        return stages

    def get_target_config(self, requirement: PodInstanceRequirement, this_pod: Dict[str, P.TaskInfo]):
        if requirement.recovery_type == RecoveryType.NONE:
            return self.target_config_id
        running, other = {}, {}
        pi = requirement.pod_instance
        for ts in pi.pod.tasks:
            if ts.name not in requirement.tasks_to_launch:
                continue
            name = f"{pi.name}-{ts.name}"
            info = this_pod.get(name)
            if info is None:
                continue
            try:
                target = TaskLabelReader(info).get_target_configuration()
            except (TaskException, ValueError):
                continue
            (running if ts.goal == GoalState.RUNNING else other)[name] = target
        for m in (running, other):
            if m:
                return next(iter(m.values()))
        return self.target_config_id
