"""helloworld scale and soak load on the local cluster.

Reference: frameworks/helloworld/tests/scale/test_scale.py (+ threading_utils.py). Many
hello-world services are installed in parallel batches, one thread per service, each with its
own service account when the cluster runs strict; the load ends with a parallel cleanup. The
reference only checks that the instances were created; this suite also checks that every
``normal`` service completed its deploy and every ``crashloop`` one kept failing without
blocking the others, and that the cleanup left no reservations behind.
"""
import pytest

from dcos_commons_amd.testing.sdk import sdk_install, sdk_plan, sdk_tasks
from dcos_commons_amd.testing.sdk.threading_utils import spawn_threads, wait_and_get_failures
from tests.integration import hw_config as config
from tests.integration.conftest import make_cluster

JOB_RUN_TIMEOUT = 10 * 60
SERVICE_COUNT, BATCH_SIZE = 6, 3


@pytest.fixture(scope="module")
def local_cluster():
    c = make_cluster(agents=6)
    yield c
    c.shutdown()


pytestmark = pytest.mark.usefixtures("local_cluster")

SCENARIOS = {
    "normal": {"service": {"yaml": "simple"}},
    "crashloop": {"service": {"yaml": "crash-loop", "sleep": 1,
                              "task_failure_backoff": {"enabled": True, "initial_backoff": 1, "max_launch_delay": 2}}},
}


def _launch_load(service_name, scenario):
    options = {"service": dict(SCENARIOS[scenario]["service"], name=service_name)}
    if scenario == "normal":
        sdk_install.install(config.PACKAGE_NAME, service_name, 1, additional_options=options)
        sdk_plan.wait_for_completed_deployment(service_name)
    else:
        sdk_install.install(config.PACKAGE_NAME, service_name, 0, additional_options=options,
                            wait_for_deployment=False, wait_for_all_conditions=False)
        sdk_plan.wait_for_kicked_off_deployment(service_name)
    return service_name


def _uninstall(service_name):
    sdk_install.uninstall(config.PACKAGE_NAME, service_name)


@pytest.mark.parametrize("scenario", ["normal", "crashloop"])
def test_scaling_load_and_cleanup(scenario):
    names = [f"hello-world-{scenario}-{i}" for i in range(SERVICE_COUNT)]
    durations = []
    for start in range(0, len(names), BATCH_SIZE):
        threads = spawn_threads(names[start:start + BATCH_SIZE], _launch_load, scenario=scenario)
        failures = wait_and_get_failures(threads, timeout=JOB_RUN_TIMEOUT)
        assert not failures, [(t.name, t.error) for t in failures]
        durations.extend(t.duration_s for t in threads)
    # every instance was created and registered with the master
    registered = {f["name"] for f in sdk_install._cluster().frameworks()}
    assert set(names) <= registered
    for name in names:
        if scenario == "normal":
            assert sdk_plan.get_deployment_plan(name)["status"] == "COMPLETE"
            sdk_tasks.check_running(name, 1)
        else:
            # somewhere in its crash loop: waiting out the backoff, relaunching, or running until it exits
            assert sdk_plan.get_deployment_plan(name)["status"] in (
                "PENDING", "PREPARED", "STARTING", "STARTED", "DELAYED", "IN_PROGRESS")
    assert max(durations) < JOB_RUN_TIMEOUT

    cleanup = spawn_threads(names, _uninstall)
    failures = wait_and_get_failures(cleanup, timeout=JOB_RUN_TIMEOUT)
    assert not failures, [(t.name, t.error) for t in failures]
    assert not sdk_install._cluster().reserved_resources()
