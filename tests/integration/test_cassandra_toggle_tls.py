"""Turning transport encryption on and off on a running Cassandra service.

Reference: frameworks/cassandra/tests/test_toggle_tls.py, in the same order on one service: the
default installation, TLS with plaintext still accepted, plaintext disabled, TLS disabled, and on
and off again. Without Cassandra binaries (synthetic payloads) the checks are what every node is
handed: its rendered ``cassandra.yaml`` (internode / client encryption, ``optional``), the
keystore and truststore mounted from the secret store only while TLS is on, and its data volume,
which every rollout keeps (the reference checks the data through a client job instead).
"""
import pytest

from dcos_commons_amd.testing.sdk import sdk_install, sdk_plan, sdk_security, sdk_tasks, sdk_upgrade
from tests.integration.test_cassandra import PACKAGE
from tests.integration.test_cassandra_features import (ACCOUNT_OPTIONS, SVC, _keystore_volumes, _rendered,
                                                       _server_info, local_cluster)  # noqa: F401


@pytest.fixture(scope="module", autouse=True)
def cassandra_service(local_cluster):  # noqa: F811
    sdk_install.install(PACKAGE, SVC, 3, additional_options=ACCOUNT_OPTIONS)
    yield
    sdk_install.uninstall(PACKAGE, SVC)
    assert not [n for n in sdk_security.list_secrets(SVC) if "keystore" in n or "truststore" in n]


def _data_volumes():
    """Persistence IDs of every node's volumes."""
    out = {}
    for i in range(3):
        info = _server_info(i)
        out[i] = sorted(r["disk"]["persistence"]["id"] for r in info.get("resources", []) + info["executor"].get(
            "resources", []) if "persistence" in r.get("disk", {}))
    return out


def _update(enabled, allow_plaintext):
    ids = sdk_tasks.get_task_ids(SVC, "node")
    sdk_upgrade.update_or_upgrade_or_downgrade(
        PACKAGE, SVC, to_version=None, expected_running_tasks=3,
        to_options={"service": {"security": {"transport_encryption": {"enabled": enabled,
                                                                        "allow_plaintext": allow_plaintext}}}})
    sdk_tasks.check_tasks_updated(SVC, "node", ids)
    sdk_plan.wait_for_completed_deployment(SVC)


def _assert_plaintext():
    for i in range(3):
        assert _keystore_volumes(i) == []
        assert "internode_encryption: none" in _rendered(i, "cassandra")


def _assert_tls(optional):
    for i in range(3):
        vols = _keystore_volumes(i)
        assert any(v.endswith("node.keystore") for v in vols) and any(v.endswith("node.truststore") for v in vols)
        cfg = _rendered(i, "cassandra")
        assert "internode_encryption: all" in cfg and f"optional: {str(optional).lower()}" in cfg


def test_default_installation():
    _assert_plaintext()


def test_enable_tls_and_plaintext():
    _update(True, True)
    _assert_tls(optional=True)
    names = sdk_security.list_secrets(SVC)
    assert any("keystore" in n for n in names) and any("truststore" in n for n in names)


def test_disable_plaintext():
    _update(True, False)
    _assert_tls(optional=False)


def test_disable_tls():
    _update(False, False)
    _assert_plaintext()


def test_enabling_then_disabling_tls():
    before = _data_volumes()
    _update(True, True)
    _update(True, False)
    _update(False, False)
    _assert_plaintext()
    assert _data_volumes() == before        # every rollout relaunched in place: the data stayed
