"""System-integration tier on the local DC/OS stand-in (``dcos_commons_amd.testing.cluster``).

Reference: the per-framework ``frameworks/*/tests`` suites run against a live DC/OS cluster through
``testing/sdk_*.py``. Here every module gets a fresh local cluster: ZooKeeper, a Mesos
master with 5 agents behind the v1 HTTP API, schedulers as supervised processes, and task commands
running for real in agent sandboxes.
"""
import os

import pytest

from dcos_commons_amd.testing.cluster import LocalCluster, use

CLI = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                   "native", "build", "sdk-cli")


def pytest_collection_modifyitems(config, items):
    for item in items:
        if "/integration/" in str(item.fspath):
            item.add_marker(pytest.mark.integration)


def make_cluster(**kw) -> LocalCluster:
    kw.setdefault("agents", 5)
    # lock waits short: a test that starts a second scheduler must not wait 3 x 10 s
    kw.setdefault("scheduler_env", {"SDK_LOCK_WAIT_S": "1"})
    c = LocalCluster(**kw).start()
    use(c)
    return c


@pytest.fixture(scope="module")
def local_cluster():
    c = make_cluster()
    yield c
    c.shutdown()


needs_cli = pytest.mark.skipif(not os.path.exists(CLI), reason="native sdk-cli not built")


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_makereport(item, call):
    outcome = yield
    report = outcome.get_result()
    if "/integration/" in str(item.fspath) and report.failed:
        from dcos_commons_amd.testing.sdk import sdk_diag

        sdk_diag.handle_test_report(item, report, out_dir=os.environ.get("SDK_DIAG_DIR",
                                                                         os.path.join("/tmp", "sdk-diag", item.name)))
