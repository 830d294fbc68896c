"""DeploymentStep state machine and launch backoff.

Pinned against the reference's DeploymentStepTest (minimum-state table, display-status table,
error retention, PREPARED handling, step/task status coherence) and
backoff/ExponentialBackoffTest (delay growth, cap, clear) under
sdk/scheduler/src/test/java/com/mesosphere/sdk/scheduler/plan/. Real specs, real StateStore.
"""
import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import common_id_utils
from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.scheduler.plan import backoff as B
from dcos_commons_amd.scheduler.plan.deployment_step import DeploymentStep, compute_status
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import PodInstance
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister

S = Status


# ---------------------------------------------------------------------------------------
# DeploymentStep.getStatus(Set<Status>, hasErrors, isPrepared)


@pytest.mark.parametrize("statuses,errors,prepared,expected", [
    (set(), False, False, S.PENDING),
    (set(), False, True, S.PREPARED),
    ({S.DELAYED}, False, True, S.DELAYED),
    (set(), True, False, S.ERROR),
    (set(), True, True, S.ERROR),
    ({S.PREPARED, S.ERROR, S.COMPLETE}, False, False, S.ERROR),
    ({S.DELAYED, S.PREPARED, S.COMPLETE}, False, True, S.DELAYED),
    ({S.PREPARED, S.PENDING}, False, False, S.PENDING),
    ({S.PREPARED, S.STARTING}, False, False, S.PREPARED),
    ({S.STARTING, S.STARTED, S.COMPLETE}, False, False, S.STARTING),
    ({S.STARTED, S.COMPLETE}, False, False, S.STARTED),
    ({S.COMPLETE}, False, False, S.COMPLETE),
])
def test_minimum_status(statuses, errors, prepared, expected):
    assert compute_status(statuses, errors, prepared) == expected


# ---------------------------------------------------------------------------------------
# the step against real specs


SPEC = """\
name: svc
pods:
  pod:
    count: 1
    tasks:
      server:
        goal: RUNNING
        cmd: ./server
        cpus: 0.1
        memory: 32
        {readiness}
      init:
        goal: ONCE
        cmd: ./init
        cpus: 0.1
        memory: 32
"""


def _spec(readiness=False):
    rc = "readiness-check:\n          cmd: ./ready\n          interval: 5\n          delay: 0\n          timeout: 10" \
        if readiness else ""
    raw = RawServiceSpec.from_string(SPEC.format(readiness=rc))
    return mappers.ServiceSpecGenerator(raw, SchedulerConfig.for_testing(), "/tmp", {}).build()


@pytest.fixture
def store():
    return StateStore(MemPersister())


@pytest.fixture(autouse=True)
def disabled_backoff():
    B.set_instance(B.DisabledBackoff())
    yield
    B.set_instance(None)


def _step(store, tasks=("server",), readiness=False):
    pi = PodInstance(_spec(readiness).pods[0], 0)
    return DeploymentStep("pod-0:[" + ", ".join(tasks) + "]", PodInstanceRequirement(pi, list(tasks)), store)


def _launch(step, task="server", readiness=False):
    """Simulate a matched offer: the step gets the LaunchOfferRecommendation of its task."""
    ti = P.TaskInfo(name=f"pod-0-{task}")
    ti.task_id.CopyFrom(common_id_utils.to_task_id("svc", f"pod-0-{task}"))
    ti.agent_id.value = "agent"
    w = TaskLabelWriter(ti)
    w.set_type("pod")
    w.set_index(0)
    if readiness:
        hc = P.HealthCheck()
        hc.command.value = "./ready"
        w.set_readiness_check(hc)
    ti.labels.CopyFrom(w.to_proto())
    step.update_offer_status([LaunchOfferRecommendation(P.Offer(), ti, P.ExecutorInfo())])
    return ti.task_id


def _status(tid, state, **kw):
    st = P.TaskStatus(state=state, **kw)
    st.task_id.CopyFrom(tid)
    return st


def test_launch_then_running_completes(store):
    step = _step(store)
    assert step.get_status() == S.PENDING
    tid = _launch(step)
    assert step.get_status() == S.STARTING
    step.update(_status(tid, P.TASK_STARTING))
    assert step.get_status() == S.STARTING
    step.update(_status(tid, P.TASK_RUNNING))
    assert step.get_status() == S.COMPLETE


def test_readiness_gates_completion(store):
    step = _step(store, readiness=True)
    tid = _launch(step, readiness=True)
    pending_check = _status(tid, P.TASK_RUNNING)
    pending_check.check_status.type = P.CheckInfo.COMMAND
    pending_check.check_status.command.SetInParent()
    step.update(pending_check)
    assert step.get_status() == S.STARTED
    ready = _status(tid, P.TASK_RUNNING)
    ready.check_status.type = P.CheckInfo.COMMAND
    ready.check_status.command.exit_code = 0
    step.update(ready)
    assert step.get_status() == S.COMPLETE


@pytest.mark.parametrize("state,expected", [
    (P.TASK_KILLED, S.PENDING), (P.TASK_LOST, S.PENDING), (P.TASK_DROPPED, S.PENDING),
    (P.TASK_GONE, S.PENDING), (P.TASK_UNREACHABLE, S.PENDING), (P.TASK_GONE_BY_OPERATOR, S.PENDING),
    (P.TASK_KILLING, S.PENDING),
    # FAILED/ERROR delay the step; with backoff disabled it is immediately eligible again
    (P.TASK_FAILED, S.PENDING), (P.TASK_ERROR, S.PENDING),
    # a RUNNING-goal task that FINISHes must run again
    (P.TASK_FINISHED, S.PENDING),
])
def test_terminal_states(store, state, expected):
    step = _step(store)
    tid = _launch(step)
    step.update(_status(tid, state))
    assert step.get_status() == expected


def test_unknown_is_discarded_and_foreign_ids_ignored(store):
    step = _step(store)
    tid = _launch(step)
    step.update(_status(tid, P.TASK_UNKNOWN))
    assert step.get_status() == S.STARTING
    other = P.TaskID(value="svc__pod-0-server__00000000-0000-0000-0000-000000000000")
    step.update(_status(other, P.TASK_FAILED))
    assert step.get_status() == S.STARTING


def test_once_task_finishing_completes(store):
    step = _step(store, tasks=("init",))
    tid = _launch(step, task="init")
    step.update(_status(tid, P.TASK_RUNNING))
    assert step.get_status() == S.STARTED        # ONCE goal: RUNNING is not the goal
    step.update(_status(tid, P.TASK_FINISHED))
    assert step.get_status() == S.COMPLETE


def test_complete_is_terminal(store):
    step = _step(store)
    tid = _launch(step)
    step.update(_status(tid, P.TASK_RUNNING))
    step.update(_status(tid, P.TASK_FAILED))     # a completed deploy step ignores later failures
    assert step.get_status() == S.COMPLETE


def test_error_is_retained_across_updates(store):
    step = _step(store)
    step.add_error("bad things")
    tid = _launch(step)
    for st in (P.TASK_STARTING, P.TASK_RUNNING, P.TASK_FAILED):
        step.update(_status(tid, st))
        assert step.get_status() == S.ERROR
    assert step.get_errors() == ["bad things"]


def test_failure_with_backoff_delays_then_recovers():
    clock = [1000.0]
    B.set_instance(B.ExponentialBackoff(2.0, 10, 40, clock=lambda: clock[0]))
    store = StateStore(MemPersister())
    step = _step(store)
    tid = _launch(step)
    step.update(_status(tid, P.TASK_FAILED))
    assert step.get_status() == S.DELAYED
    clock[0] += 9.9
    assert step.get_status() == S.DELAYED
    clock[0] += 0.2
    assert step.get_status() == S.PENDING       # delay elapsed: eligible again


def test_restart_clears_backoff():
    clock = [0.0]
    B.set_instance(B.ExponentialBackoff(2.0, 10, 40, clock=lambda: clock[0]))
    store = StateStore(MemPersister())
    step = _step(store)
    tid = _launch(step)
    step.update(_status(tid, P.TASK_FAILED))
    assert step.get_status() == S.DELAYED
    step.restart()
    assert step.get_status() == S.PENDING
    assert B.get_instance().get_delay("pod-0-server") is None


def test_interrupted_pending_step_is_waiting(store):
    step = _step(store)
    step.interrupt()
    assert step.get_status() == S.WAITING
    step.proceed()
    assert step.get_status() == S.PENDING
    step.force_complete()
    assert step.get_status() == S.COMPLETE and step.is_complete()


def test_override_progress_follows_the_step(store):
    """A PAUSED override goes PENDING -> IN_PROGRESS -> COMPLETE as the relaunch proceeds."""
    step = _step(store)
    store.store_goal_override_status("pod-0-server", GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING))
    tid = _launch(step)
    assert store.fetch_goal_override_status("pod-0-server").progress == OverrideProgress.IN_PROGRESS
    step.update(_status(tid, P.TASK_RUNNING))
    st = store.fetch_goal_override_status("pod-0-server")
    assert st.target == GoalStateOverride.PAUSED and st.progress == OverrideProgress.COMPLETE
    # the display status only says PAUSED when every task of the pod is paused ("init" is not)
    assert step.get_display_status() == "COMPLETE"
    store.store_goal_override_status("pod-0-init", GoalStateOverride.PAUSED.new_status(OverrideProgress.COMPLETE))
    assert step.get_display_status() == "PAUSED"


def test_display_status_table(store):
    from dcos_commons_amd.scheduler.plan.deployment_step import display_status
    store.store_goal_override_status("paused-0", GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING))
    store.store_goal_override_status("paused-1", GoalStateOverride.PAUSED.new_status(OverrideProgress.COMPLETE))
    cases = [
        (S.IN_PROGRESS, [], "IN_PROGRESS"), (S.COMPLETE, [], "COMPLETE"), (S.DELAYED, [], "DELAYED"),
        (S.IN_PROGRESS, ["paused-0"], "PAUSING"), (S.IN_PROGRESS, ["paused-1"], "PAUSING"),
        (S.IN_PROGRESS, ["paused-0", "paused-1"], "PAUSING"),
        (S.IN_PROGRESS, ["no-override-0", "no-override-1"], "IN_PROGRESS"),
        (S.IN_PROGRESS, ["no-override-0", "paused-0"], "IN_PROGRESS"),
        (S.IN_PROGRESS, ["no-override-0", "paused-0", "paused-1"], "IN_PROGRESS"),
        (S.COMPLETE, ["paused-0"], "PAUSED"), (S.COMPLETE, ["paused-1"], "PAUSED"),
        (S.COMPLETE, ["paused-0", "paused-1"], "PAUSED"),
        (S.COMPLETE, ["no-override-0", "no-override-1"], "COMPLETE"),
        (S.COMPLETE, ["no-override-0", "paused-1"], "COMPLETE"),
    ]
    for status, names, expected in cases:
        assert display_status(store, status, names) == expected, (status, names)


def test_parameters_reach_the_requirement(store):
    step = _step(store)
    step.update_parameters({"VERSION": "2"})
    assert step.get_pod_instance_requirement().environment == {"VERSION": "2"}


# ---------------------------------------------------------------------------------------
# ExponentialBackoff


def test_exponential_backoff_growth_cap_and_clear():
    now = [0.0]
    b = B.ExponentialBackoff(1.5, 10, 20, clock=lambda: now[0])
    tid = common_id_utils.to_task_id("svc", "pod-0-server")
    assert b.get_delay("pod-0-server") is None
    b.add_delay(tid)
    assert b.get_delay("pod-0-server") == pytest.approx(10)
    b.add_delay(tid)
    assert b.get_delay("pod-0-server") == pytest.approx(15)
    b.add_delay(tid)
    assert b.get_delay("pod-0-server") == pytest.approx(20)     # capped
    now[0] += 5
    assert b.get_delay("pod-0-server") == pytest.approx(15)
    now[0] += 16
    assert b.get_delay("pod-0-server") is None
    assert b.clear_delay(tid) is True and b.clear_delay(tid) is False
    b.add_delay(tid)
    assert b.get_delay("pod-0-server") == pytest.approx(10)     # cleared: starts over


def test_disabled_backoff_never_delays():
    b = B.DisabledBackoff()
    b.add_delay("pod-0-server")
    assert b.get_delay("pod-0-server") is None and b.clear_delay("pod-0-server") is False
