"""Deterministic simulation harness for service schedulers.

Reference: sdk/testing/src/main/java/com/mesosphere/sdk/testing/{ServiceTestRunner,Send,Expect,
SendOffer,SendTaskStatus,ClusterState,AcceptEntry}.java. A test is a list of *ticks*: ``Send``
ticks push an event into the scheduler (registration, offers, task statuses, pod commands) and
``Expect`` ticks assert on what the scheduler did (accepts, declines, kills, revives, plan
status, persisted state). The scheduler runs single-threaded: every offer is processed
synchronously inside the tick that delivered it, so each tick observes a settled state.

    result = ServiceTestRunner("svc.yml").set_env(...).run([
        Send.register(),
        Expect.reconciled_implicitly(),
        Send.offer_builder("hello").build(),
        Expect.launched_tasks("hello-0-server"),
        Send.task_status("hello-0-server", P.TASK_RUNNING).build(),
        Expect.deploy_step_status("hello", "hello-0:[server]", Status.COMPLETE),
    ])
"""
from .harness import (  # noqa: F401
    AcceptEntry,
    ClusterState,
    Expect,
    RecordingDriver,
    Send,
    ServiceTestResult,
    ServiceTestRunner,
)
