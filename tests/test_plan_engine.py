"""Plan engine: aggregate status rules, strategies (serial / parallel / canary / dependency), plan
managers and the coordinator's dirty-asset exclusion. Reference: scheduler/plan/PlanUtilsTest,
strategy/{SerialStrategyTest,ParallelStrategyTest,CanaryStrategyTest,DependencyStrategyTest},
DefaultPlanCoordinatorTest, DefaultPhaseTest."""
import pytest

from dcos_commons_amd.scheduler.plan.elements import AbstractStep, DefaultPhase, DefaultPlan, get_aggregate_status
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanCoordinator, DefaultPlanManager
from dcos_commons_amd.scheduler.plan.status import Status as S
from dcos_commons_amd.scheduler.plan.strategy import (
    CanaryStrategy,
    DependencyStrategy,
    DependencyStrategyHelper,
    ParallelStrategy,
    RandomStrategy,
    SerialStrategy,
    phase_strategy_generator,
)


class TStep(AbstractStep):
    def __init__(self, name, req=None):
        super().__init__(name)
        self.req = req

    def get_pod_instance_requirement(self):
        return self.req

    def start(self):
        self.set_status(S.STARTING)


def names(steps):
    return [s.get_name() for s in steps]


# -- aggregate status (PlanUtils.getAggregateStatus, rule order matters) -----------------------

@pytest.mark.parametrize("children,candidates,errors,interrupted,expected", [
    ([], [], ["err"], False, S.ERROR),
    ([S.ERROR], [], [], False, S.ERROR),
    ([], [], [], False, S.COMPLETE),
    ([S.COMPLETE, S.COMPLETE], [], [], False, S.COMPLETE),
    ([S.DELAYED], [], [], True, S.WAITING),
    ([S.DELAYED, S.DELAYED], [], [], False, S.DELAYED),
    ([S.COMPLETE, S.PENDING], [], [], True, S.WAITING),
    ([S.COMPLETE, S.WAITING], [], [], False, S.WAITING),
    ([S.COMPLETE, S.WAITING], [S.WAITING], [], False, S.WAITING),
    ([S.PREPARED, S.WAITING], [], [], False, S.IN_PROGRESS),
    ([S.COMPLETE, S.IN_PROGRESS], [S.IN_PROGRESS], [], False, S.IN_PROGRESS),
    ([S.COMPLETE, S.PENDING], [S.PENDING], [], False, S.IN_PROGRESS),
    ([S.COMPLETE, S.STARTING], [S.STARTING], [], False, S.IN_PROGRESS),
    ([S.COMPLETE, S.STARTED], [S.STARTED], [], False, S.IN_PROGRESS),
    ([S.PENDING, S.PENDING], [S.PENDING], [], False, S.PENDING),
    ([S.STARTING, S.PENDING], [S.STARTING], [], False, S.STARTING),
    ([S.STARTED, S.PENDING], [S.STARTED], [], False, S.STARTED),
])
def test_aggregate_status(children, candidates, errors, interrupted, expected):
    assert get_aggregate_status("foo", children, candidates, errors, interrupted) == expected


# -- strategies -------------------------------------------------------------------------------

def test_serial_strategy_one_at_a_time():
    steps = [TStep(f"s{i}") for i in range(3)]
    st = SerialStrategy()
    assert names(st.get_candidates(steps, [])) == ["s0"]
    steps[0].set_status(S.COMPLETE)
    assert names(st.get_candidates(steps, [])) == ["s1"]
    st.interrupt()
    assert st.get_candidates(steps, []) == []
    st.proceed()
    steps[1].set_status(S.COMPLETE)
    steps[2].set_status(S.COMPLETE)
    assert st.get_candidates(steps, []) == []


def test_serial_strategy_blocks_on_in_progress_step():
    steps = [TStep(f"s{i}") for i in range(2)]
    st = SerialStrategy()
    steps[0].set_status(S.STARTING)
    assert names(st.get_candidates(steps, [])) == ["s0"]  # still the head: not completed


def test_parallel_strategy_all_eligible():
    steps = [TStep(f"s{i}") for i in range(3)]
    st = ParallelStrategy()
    assert names(st.get_candidates(steps, [])) == ["s0", "s1", "s2"]
    steps[1].set_status(S.COMPLETE)
    assert names(st.get_candidates(steps, [])) == ["s0", "s2"]
    st.interrupt()
    assert st.get_candidates(steps, []) == []


def test_canary_strategy_requires_two_proceeds():
    steps = [TStep(f"s{i}") for i in range(4)]
    st = CanaryStrategy(SerialStrategy(), steps)
    assert st.get_name() == "serial-canary"
    assert st.is_interrupted()
    assert st.get_candidates(steps, []) == []  # waits for the operator
    st.proceed()  # first canary
    assert names(st.get_candidates(steps, [])) == ["s0"]
    steps[0].set_status(S.COMPLETE)
    assert st.get_candidates(steps, []) == []  # waiting for the second proceed
    st.proceed()
    assert names(st.get_candidates(steps, [])) == ["s1"]
    steps[1].set_status(S.COMPLETE)
    # after both canaries the post-canary strategy runs the rest
    assert names(st.get_candidates(steps, [])) == ["s2"]


def test_parallel_canary_generator():
    steps = [TStep(f"s{i}") for i in range(4)]
    st = phase_strategy_generator("parallel-canary")(steps)
    assert st.get_name() == "parallel-canary"
    st.proceed()
    steps[0].set_status(S.COMPLETE)
    st.proceed()
    steps[1].set_status(S.COMPLETE)
    assert names(st.get_candidates(steps, [])) == ["s2", "s3"]
    with pytest.raises(ValueError):
        phase_strategy_generator("bogus")


def test_dependency_strategy_dag():
    a, b, c = TStep("a"), TStep("b"), TStep("c")
    h = DependencyStrategyHelper([a, b, c])
    h.add_dependency(c, a)  # c after a
    h.add_dependency(c, b)  # c after b
    st = DependencyStrategy(h)
    assert sorted(names(st.get_candidates([a, b, c], []))) == ["a", "b"]
    a.set_status(S.COMPLETE)
    assert names(st.get_candidates([a, b, c], [])) == ["b"]
    b.set_status(S.COMPLETE)
    assert names(st.get_candidates([a, b, c], [])) == ["c"]


# -- phases, plans, managers ----------------------------------------------------------------

def test_phase_and_plan_status_roll_up():
    steps = [TStep("s0"), TStep("s1")]
    phase = DefaultPhase("p", steps, SerialStrategy())
    plan = DefaultPlan("deploy", [phase], SerialStrategy())
    assert plan.get_status() == S.PENDING
    steps[0].set_status(S.COMPLETE)
    assert phase.get_status() == S.IN_PROGRESS and plan.get_status() == S.IN_PROGRESS
    steps[1].set_status(S.COMPLETE)
    assert plan.is_complete()
    plan.restart()
    assert all(s.get_status() == S.PENDING for s in steps)
    plan.force_complete()
    assert plan.is_complete()


def test_plan_errors_make_status_error():
    plan = DefaultPlan("deploy", [DefaultPhase("p", [TStep("s")], SerialStrategy())], SerialStrategy(), ["bad"])
    assert plan.get_status() == S.ERROR and plan.has_errors()


def test_interrupted_plan_is_waiting_and_has_no_candidates():
    steps = [TStep("s0")]
    plan = DefaultPlan("deploy", [DefaultPhase("p", steps, SerialStrategy())], SerialStrategy())
    pm = DefaultPlanManager.create_interrupted(plan)
    assert plan.get_status() == S.WAITING
    assert pm.get_candidates([]) == []
    plan.proceed()
    assert names(pm.get_candidates([])) == ["s0"]


class _Req:
    """Minimal PodInstanceRequirement stand-in for dirty-asset checks."""

    def __init__(self, pod):
        self.pod = pod
        self.tasks_to_launch = ["t"]

        class _PI:
            name = pod
        self.pod_instance = _PI()

    def conflicts_with(self, other):
        return self.pod == other.pod

    def __hash__(self):
        return hash(self.pod)

    def __eq__(self, o):
        return isinstance(o, _Req) and o.pod == self.pod


def test_coordinator_excludes_dirty_assets():
    """Two plans touching the same pod: only the first plan's step is a candidate; a step that
    is already in progress in one plan makes the pod dirty for the others."""
    a1, b1 = TStep("a-deploy", _Req("pod-0")), TStep("a-other", _Req("pod-0"))
    p1 = DefaultPlan("deploy", [DefaultPhase("p", [a1], SerialStrategy())], SerialStrategy())
    p2 = DefaultPlan("other", [DefaultPhase("p", [b1], SerialStrategy())], SerialStrategy())
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(p1), DefaultPlanManager.create_proceeding(p2)])
    assert names(coord.get_candidates()) == ["a-deploy"]
    a1.set_status(S.PREPARED)  # in flight: its asset is dirty for other plans
    assert names(coord.get_candidates()) == ["a-deploy"]
    a1.set_status(S.COMPLETE)
    assert names(coord.get_candidates()) == ["a-other"]


# -- cached aggregate statuses (elements._status_gen) --------------------------------------------

def _plan(strategy=SerialStrategy, n=3):
    steps = [TStep(f"s{i}") for i in range(n)]
    phase = DefaultPhase("p", steps, strategy())
    return DefaultPlan("deploy", [phase], SerialStrategy()), phase, steps


def test_cached_plan_status_follows_every_kind_of_change():
    from dcos_commons_amd.scheduler.plan import elements

    plan, phase, steps = _plan()
    assert plan.get_status() == S.PENDING
    gen = elements.status_generation()
    assert plan.get_status() == S.PENDING and plan._status_cache == (gen, S.PENDING)   # served from cache
    steps[0].set_status(S.COMPLETE)
    assert phase.get_status() == S.IN_PROGRESS and plan.get_status() == S.IN_PROGRESS
    phase.interrupt()                                        # strategy flag
    assert plan.get_status() == S.WAITING
    phase.proceed()
    steps[1].interrupt()                                     # step flag: an interrupted PENDING step is WAITING
    assert steps[1].get_status() == S.WAITING and phase.get_status() == S.WAITING
    steps[1].proceed()
    for s in steps:
        s.force_complete()
    assert plan.get_status() == S.COMPLETE
    steps[2].restart()
    assert plan.get_status() == S.IN_PROGRESS


def test_uncacheable_aggregates_are_recomputed():
    class Flip:                                             # not an AbstractStep: changes unannounced
        def __init__(self):
            self.status = S.PENDING

        def get_status(self):
            return self.status

        def get_errors(self):
            return []

        def is_interrupted(self):
            return False

        def get_pod_instance_requirement(self):
            return None

    f = Flip()
    phase = DefaultPhase("p", [f], ParallelStrategy())
    assert phase.get_status() == S.PENDING and phase._status_cache is None
    f.status = S.COMPLETE
    assert phase.get_status() == S.COMPLETE
    plan, phase2, steps = _plan(RandomStrategy)              # random candidates: never cached
    plan.get_status()
    assert phase2._status_cache is None and plan._status_cache is None


def test_delayed_step_is_not_cached_past_its_backoff():
    from dcos_commons_amd.scheduler.plan import elements

    plan, phase, steps = _plan(ParallelStrategy, n=1)
    steps[0].set_status(S.DELAYED)
    assert phase.get_status() == S.DELAYED
    assert phase._status_cache is None and not phase._last_cacheable and plan._status_cache is None
    steps[0]._status = S.PENDING                             # what the backoff expiry does, with no bump
    assert phase.get_status() == S.PENDING and elements.status_generation() >= 0
