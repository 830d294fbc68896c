"""Test-SDK pieces that need a cluster service: Metronome jobs and universe repositories.

Reference: testing/sdk_jobs.py (the cassandra/hdfs data read/write jobs, e.g.
frameworks/cassandra/tests/test_tls.py ``InstallJobContext`` + ``run_job``) and
testing/sdk_repository.py (stub universes added for a test session). Jobs here talk to a deployed
service through its scheduler API; the stub universe is a package repository published by
``tools.universe`` and installed from.
"""
import os

import pytest

from dcos_commons_amd.testing.sdk import sdk_install, sdk_jobs, sdk_plan, sdk_repository
from tests.integration import hw_config as config
from tests.test_tools import needs_native

pytestmark = pytest.mark.usefixtures("local_cluster")


def _job(name, cmd, env=None):
    return {"id": name, "description": f"{name} job", "run": {"cmd": cmd, "cpus": 0.1, "mem": 64, "disk": 0,
                                                             "env": dict(env or {})}}


def test_jobs_against_a_deployed_service():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1, additional_options={"service": {"yaml": "simple"}})
    try:
        url = sdk_install._cluster().marathon.scheduler_url(config.SERVICE_NAME)
        write = _job("write-data", 'echo "$PAYLOAD" > data && curl -sf -X PUT -F "file=@data" '
                                    '"$API/v1/state/files/job-data"', {"PAYLOAD": "hello-from-job", "API": url})
        verify = _job("verify-data", 'curl -sf "$API/v1/state/files/job-data" | grep -q hello-from-job', {"API": url})
        fail = _job("fail", "exit 3")
        with sdk_jobs.InstallJobContext([write, verify, fail]):
            sdk_jobs.run_job(write)
            sdk_jobs.run_job(verify)
            with pytest.raises(Exception, match="has failed"):
                sdk_jobs.run_job(fail, timeout_seconds=30)
            run_id = sdk_jobs.run_job(fail, timeout_seconds=30, raise_on_failure=False)
            hist = sdk_install._cluster().metronome.job("fail", embed_history=True)["history"]
            assert run_id in [r["id"] for r in hist["failedFinishedRuns"]]
        # the context removed the jobs
        with pytest.raises(KeyError):
            sdk_install._cluster().metronome.job("write-data")
        with sdk_jobs.RunJobContext(before_jobs=[verify]):
            pass
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


@needs_native
def test_stub_universe_session(tmp_path, monkeypatch):
    from dcos_commons_amd.tools import build_package
    from dcos_commons_amd.tools.publish_http import HTTPPublisher

    assert sdk_repository.parse_stub_universe_url_string("a,b c,,a") == ["a", "b", "c"]
    hello = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                         "frameworks", "helloworld")
    artifacts = build_package.build_artifacts(config.PACKAGE_NAME, hello, str(tmp_path / "artifacts"))
    pub = HTTPPublisher(config.PACKAGE_NAME, "9.9.9-stub", os.path.join(hello, "universe"), artifacts,
                        http_dir=str(tmp_path / "http"))
    monkeypatch.setenv("STUB_UNIVERSE_URL", pub.start())
    try:
        with sdk_repository.universe_session():
            assert [r["name"] for r in sdk_repository.get_repos()] == ["testpkg-0"]
            assert "9.9.9-stub" in sdk_repository.get_package_versions(config.PACKAGE_NAME)
            sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                                additional_options={"service": {"yaml": "simple"}}, package_version="9.9.9-stub")
            try:
                sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
            finally:
                sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
        assert sdk_repository.get_repos() == []
    finally:
        pub.stop()
