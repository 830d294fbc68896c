import os
import sys

import pytest

# every offer cycle in the suite checks that no caller modified a shared (read-only) TaskInfo
# (StateStore.fetch_tasks_shared); set before the package is imported
os.environ.setdefault("SDK_DEBUG_SHARED_TASKS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "integration: runs services on the local DC/OS stand-in")


@pytest.fixture(autouse=True)
def _test_mode():
    """ProcessExit raises instead of exiting; deadlock detection raises instead of exiting."""
    from dcos_commons_amd.framework.process_exit import ProcessExit

    ProcessExit.set_test_mode(True)
    yield


@pytest.fixture(params=["mi355x", "reference"])
def sched_profile(request):
    """Runs a test under both scheduler flag profiles (``testing.profiles``): the defaults, and
    every deviation from the reference switched off. Suites opt in with
    ``pytestmark = pytest.mark.usefixtures("sched_profile")``."""
    from dcos_commons_amd.testing import profiles

    prev = profiles.use(request.param)
    yield request.param
    profiles.ACTIVE = prev


def reference_path(*parts):
    p = os.path.join(REFERENCE, *parts)
    return p if os.path.exists(p) else None
