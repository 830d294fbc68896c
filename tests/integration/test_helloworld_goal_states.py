"""Task goal states on the local cluster (``finish_state.yml``): a ONCE task runs a single time
ever, a FINISH task reruns whenever its pod's configuration changes, and both must exit 0 before
their pod's server launches.

Reference: frameworks/helloworld/tests/test_goal_states.py.
"""
import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_plan, sdk_tasks
from tests.integration import hw_config as config

PKG = config.PACKAGE_NAME
SVC = "/test/integration/hello-goals"


@pytest.fixture(scope="module", autouse=True)
def finish_state_service(local_cluster):
    sdk_install.install(PKG, SVC, 3, additional_options={"service": {"yaml": "finish_state"}})
    yield
    sdk_install.uninstall(PKG, SVC)


def _completed(task_name):
    # newest first, as Mesos lists them
    return [t.id for t in sdk_tasks.get_summary(with_completed=True, task_name=task_name) if t.is_completed]


def test_install():
    config.check_running(SVC)
    sdk_plan.wait_for_completed_deployment(SVC)
    assert len(_completed("hello-0-once")) == 1 and len(_completed("world-0-init")) == 1
    # both ran before their pod's server: the server found what they wrote
    assert sdk_cmd.service_task_exec(SVC, "world-0-server", "true")[0] == 0


def test_once_task_does_not_restart_on_config_update():
    sdk_plan.wait_for_completed_deployment(SVC)
    once = _completed("hello-0-once")
    assert once
    server = sdk_tasks.get_task_ids(SVC, "hello-0-server")
    config.bump_hello_cpus(SVC)
    sdk_tasks.check_tasks_updated(SVC, "hello-0-server", server)
    sdk_tasks.check_task_not_relaunched(SVC, "hello-0-once", once[0], with_completed=True)
    config.check_running(SVC)


def test_finish_task_restarts_on_config_update():
    init = _completed("world-0-init")
    assert init
    config.bump_world_cpus(SVC)
    sdk_tasks.check_task_relaunched("world-0-init", init[0], ensure_new_task_not_completed=False)
    sdk_plan.wait_for_completed_deployment(SVC)
    assert len(_completed("world-0-init")) == len(init) + 1
    config.check_running(SVC)
