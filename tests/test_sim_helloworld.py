"""Tick-by-tick simulation of the helloworld service (reference:
frameworks/helloworld/src/test/java/com/mesosphere/sdk/helloworld/scheduler/ServiceTest.java)."""
import os

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.state import state_store_utils
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.testing import Expect, Send, ServiceTestRunner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SVC = os.path.join(ROOT, "frameworks", "helloworld", "specs", "svc.yml")

# every test runs under the scheduler defaults and with every deviation from the reference off
pytestmark = pytest.mark.usefixtures("sched_profile")

ENV = dict(FRAMEWORK_NAME="hello-world", FRAMEWORK_PRINCIPAL="hello-world-principal", FRAMEWORK_USER="nobody",
           HELLO_COUNT="1", HELLO_PLACEMENT='[["hostname", "UNIQUE"]]', HELLO_CPUS="0.1", HELLO_MEM="252",
           HELLO_DISK="25", SLEEP_DURATION="1000", WORLD_COUNT="2", WORLD_PLACEMENT='[["hostname", "UNIQUE"]]',
           WORLD_CPUS="0.2", WORLD_MEM="512", WORLD_DISK="25", WORLD_READINESS_CHECK_INTERVAL="5",
           WORLD_READINESS_CHECK_DELAY="0", WORLD_READINESS_CHECK_TIMEOUT="10")


def runner(**env):
    e = dict(ENV)
    e.update(env)
    # reference cadence: every work-set change revives immediately (no burst spacing in the sim)
    return ServiceTestRunner(SVC).set_env(e).set_scheduler_env(SDK_REVIVE_INTERVAL_S="0", SDK_FAST_UNSUPPRESS="false",
                                                               SDK_REVIVE_ONLY_UNMATCHED="false")


def default_deployment_ticks():
    return [
        Send.register(),
        Expect.reconciled_implicitly(),
        # one hello pod, then two world pods
        Send.offer_builder("hello").build(),
        Expect.launched_tasks("hello-0-server"),
        Expect.revived_offers(1),
        # an offer before hello-0 is running is declined
        Send.offer_builder("world").build(),
        Expect.declined_last_offer(),
        # hello has no readiness check: RUNNING completes the step
        Send.task_status("hello-0-server", P.TASK_RUNNING).build(),
        Send.offer_builder("world").build(),
        Expect.launched_tasks("world-0-server"),
        Expect.revived_offers(2),
        # world-0 has a readiness check: RUNNING with a pending check is not enough
        Send.task_status("world-0-server", P.TASK_RUNNING).set_check_pending().build(),
        Send.offer_builder("world").build(),
        Expect.declined_last_offer(),
        Expect.deploy_step_status("world", "world-0:[server]", Status.STARTED),
        # readiness passes; world-1 still cannot share world-0's host (hostname:UNIQUE)
        Send.task_status("world-0-server", P.TASK_RUNNING).set_readiness_check_exit_code(0).build(),
        Send.offer_builder("world").build(),
        Expect.declined_last_offer(),
        # the work set changed (world-0 => world-1) at that offer cycle
        Expect.revived_offers(3),
        # a different host works
        Send.offer_builder("world").set_hostname("host-foo").build(),
        Expect.launched_tasks("world-1-server"),
        Send.task_status("world-1-server", P.TASK_RUNNING).set_readiness_check_exit_code(0).build(),
        # nothing left to launch
        Send.offer_builder("world").set_hostname("host-bar").build(),
        Expect.declined_last_offer(),
        Expect.all_plans_complete(),
        Expect.known_tasks("hello-0-server", "world-0-server", "world-1-server"),
    ]


def test_default_deployment():
    result = runner().run(default_deployment_ticks())
    assert state_store_utils.get_deployment_was_completed(StateStore(result.persister))
    # after deployment the scheduler goes idle and suppresses offers
    res2 = runner().set_state(result.persister).run([Send.register(), Send.empty_offers(),
                                                     Expect.suppressed_offers(1)])
    assert res2 is not None


def test_deploy_plan_http_view_during_deployment():
    ticks = [Send.register(), Send.offer_builder("hello").build(), Expect.launched_tasks("hello-0-server"),
             Expect.http("GET", "/v1/plans/deploy", 202),
             Expect.http("GET", "/v1/pod", 200, lambda r: r.json() == ["hello-0"]),
             Send.task_status("hello-0-server", P.TASK_RUNNING).build(),
             Expect.http("GET", "/v1/pod/hello-0/status", 200,
                         lambda r: r.json()["tasks"][0]["status"] == "RUNNING")]
    runner().run(ticks)


def test_transient_restart_reuses_reservations():
    ticks = default_deployment_ticks() + [
        Send.task_status("world-0-server", P.TASK_FAILED).build(),
        Send.empty_offers(),
        Expect.recovery_step_status("world-0:[server]", "world-0:[server]", Status.PREPARED),
        Send.offer_builder("world").set_pod_index_to_reoffer(0).build(),
        Expect.launched_tasks("world-0-server"),
        Expect.recovery_step_status("world-0:[server]", "world-0:[server]", Status.STARTING),
        Send.task_status("world-0-server", P.TASK_RUNNING).set_readiness_check_exit_code(0).build(),
        Expect.recovery_step_status("world-0:[server]", "world-0:[server]", Status.COMPLETE),
        Expect.all_plans_complete(),
    ]
    result = runner().run(ticks)
    # a transient relaunch does not reserve anything new: the last accept only relaunched
    last = result.cluster_state.driver.accepts[-1]
    assert [o.type for o in last.operations] == [P.Offer.Operation.LAUNCH_GROUP]


def _replace_prefix():
    return default_deployment_ticks() + [
        Send.replace_pod("world-0"),
        Expect.task_name_killed("world-0-server", 1),
        Send.task_status("world-0-server", P.TASK_KILLED).build(),
        Send.empty_offers(),
        Expect.recovery_step_status("world-0:[server]", "world-0:[server]", Status.PREPARED),
    ]


def test_replace_pod_recycles_reservations_in_one_accept():
    """MI355X build: the stale reservations are UNRESERVEd at the head of the same ACCEPT that
    re-reserves and launches the replacement."""
    ticks = _replace_prefix() + [
        Send.offer_builder("world").set_pod_index_to_reoffer(0).build(),
        Expect.unreserved_tasks("world-0-server"),
        Expect.launched_tasks("world-0-server"),
        Send.task_status("world-0-server", P.TASK_RUNNING).set_readiness_check_exit_code(0).build(),
        Expect.all_plans_complete(),
    ]
    # the MI355X behaviour is SDK_RESERVATION_GC_ALL_OFFERS (off under the reference flags)
    result = runner().set_scheduler_env(SDK_RESERVATION_GC_ALL_OFFERS="true").run(ticks)
    ops = [o.type for o in result.cluster_state.driver.accepts[-1].operations]
    Op = P.Offer.Operation
    assert ops.index(Op.UNRESERVE) < ops.index(Op.RESERVE) < ops.index(Op.LAUNCH_GROUP)


def test_replace_pod_reference_cleanup_then_fresh_offer():
    """Reference behaviour (SDK_RESERVATION_GC_ALL_OFFERS=false): the stale reservations are
    released from an unused offer, the replacement lands on a fresh offer."""
    ticks = _replace_prefix() + [
        Send.offer_builder("world").set_pod_index_to_reoffer(0).set_hostname("host-foo").build(),
        Expect.unreserved_tasks("world-0-server"),
        Send.offer_builder("world").set_hostname("host-new").build(),
        Expect.launched_tasks("world-0-server"),
        Send.task_status("world-0-server", P.TASK_RUNNING).set_readiness_check_exit_code(0).build(),
        Expect.all_plans_complete(),
    ]
    runner().set_scheduler_env(SDK_RESERVATION_GC_ALL_OFFERS="false").run(ticks)


def test_pause_and_resume_pod():
    ticks = default_deployment_ticks() + [
        Send.http("POST", "/v1/pod/hello-0/pause", b"", expect_status=200),
        Expect.task_name_killed("hello-0-server", 1),
        Expect.http("GET", "/v1/pod/hello-0/status", 200,
                    lambda r: r.json()["tasks"][0]["status"] == "PAUSING"),
    ]
    runner().run(ticks)


def test_zombie_task_is_killed():
    ticks = default_deployment_ticks() + [
        Send.task_status("hello-0-server", P.TASK_RUNNING).set_task_id("hello-world__hello-0-server__zombie").build(),
        Expect.that(lambda sim: None),
    ]
    result = runner().run(ticks)
    assert "hello-world__hello-0-server__zombie" in result.cluster_state.driver.kills


def test_config_update_relaunches_changed_pods():
    first = runner().run(default_deployment_ticks())
    ticks = [
        Send.register(),
        Expect.reconciled_explicitly("hello-0-server", "world-0-server", "world-1-server"),
        Send.task_status("hello-0-server", P.TASK_RUNNING).build(),
        Send.task_status("world-0-server", P.TASK_RUNNING).set_readiness_check_exit_code(0).build(),
        Send.task_status("world-1-server", P.TASK_RUNNING).set_readiness_check_exit_code(0).build(),
        Send.empty_offers(),
        # only hello changed (cpus): world steps are already complete
        Expect.deploy_step_status("hello", "hello-0:[server]", Status.PREPARED),
        Expect.deploy_step_status("world", "world-0:[server]", Status.COMPLETE),
        Expect.task_name_killed("hello-0-server", 1),
    ]
    runner(HELLO_CPUS="0.2").set_state(first.persister).run(ticks)


@pytest.mark.parametrize("count", [1, 3])
def test_parallel_gpu_spec_launches_all_pods_at_once(count):
    spec = os.path.join(ROOT, "frameworks", "helloworld", "specs", "gpu.yml")
    env = dict(ENV, HELLO_COUNT=str(count), HELLO_GPUS="1", GPU_PROBE_CMD="true")
    gpu = P.Resource(name="gpus", type=P.Value.SCALAR, role="*")
    gpu.scalar.value = 1
    ticks = [Send.register()]
    for i in range(count):
        ticks.append(Send.offer_builder("hello").set_hostname(f"gpu-host-{i}").add_resources(gpu).build())
    ticks.append(Expect.that(lambda sim: None))
    result = ServiceTestRunner(spec).set_env(env).set_scheduler_env(SDK_REVIVE_INTERVAL_S="0").run(ticks)
    launched = sorted(t.name for a in result.cluster_state.driver.accepts for t in a.launched_tasks())
    assert launched == [f"hello-{i}-server" for i in range(count)]
