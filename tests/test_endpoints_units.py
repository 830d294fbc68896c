"""Endpoint queries on the reference's own task fixture: ports across tasks, hidden and unnamed
ports, VIPs, a custom endpoint shadowing a port of the same name, foldered service names, and the
address fallback from the offer hostname to the task's IP (current status first, then the
``<task>:task-status`` property).

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/http/queries/EndpointsQueriesTest.java.
"""
import pytest

import testutils as U
from dcos_commons_amd.http import resources as R
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from test_http_queries import Router

CFG = SchedulerConfig.for_testing()
CUSTOM = "custom"
CUSTOM_VALUE = "hi\nhey\nhello"
OVERLAY_HOSTNAME = "overlay-hostname"


def _base(name=U.TASK_NAME):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(U.TASK_ID)
    t.agent_id.CopyFrom(U.AGENT_ID)
    return t


def _with_metadata(name):
    t = _base(name)
    TaskLabelWriter(t).set_hostname(P.Offer(hostname=U.HOSTNAME)).set_type("some-task-type").apply()
    return t


def _with_ports(name, ports):
    """ports: (name or None, number, visible, vip label (key, value) or None)."""
    t = _with_metadata(name)
    t.discovery.visibility = P.DiscoveryInfo.CLUSTER
    for pname, number, visible, label in ports:
        p = t.discovery.ports.ports.add(number=number, protocol="tcp")
        if pname is not None:
            p.name = pname
        if visible:
            p.visibility = P.DiscoveryInfo.EXTERNAL
        if label is not None:
            p.labels.labels.add(key=label[0], value=label[1])
    return t


TASKS = [
    _base(),
    _with_metadata(U.TASK_NAME),
    _with_ports("ports-1", [("porta", 1234, True, None), ("portb", 1235, True, None)]),
    _with_ports("ports-2", [("porta", 1243, True, None), (None, 1244, True, None)]),      # unnamed: ignored
    _with_ports("hidden-ports", [("porta-hidden", 1, False, None), ("portb-hidden", 2, False, None)]),
    _with_ports("vips-1", [("porta", 2345, True, ("VIP_abc", "vip1:5432")),
                           (CUSTOM, 2347, True, ("VIP_ghi", "custom:6432")),            # shadowed by 'custom'
                           ("novip", 2348, True, ("ignored_not_vip", "ignored:6432"))]),
    _with_ports("vips-2", [("porta", 3456, True, ("VIP_abc", "vip1:5432")),
                           ("portb", 3457, True, ("VIP_def", "vip2:6432")),
                           (CUSTOM, 3458, True, ("VIP_ghi", "custom:6432")),
                           ("novip", 3459, True, ("ignored_not_vip", "ignored:6432"))]),
]


class FakeStore:
    def __init__(self, statuses=None, properties=None):
        self.statuses = statuses or {}
        self.properties = properties or {}

    def fetch_tasks(self):
        return list(TASKS)

    def fetch_status(self, name):
        return self.statuses.get(name)

    def fetch_property(self, key):
        if key not in self.properties:
            from dcos_commons_amd.state.state_store import StateStoreException
            from dcos_commons_amd.storage.persister import Reason

            raise StateStoreException(Reason.NOT_FOUND, key)
        return self.properties[key]


def _router(service, store=None):
    return Router([R.EndpointsResource(store or FakeStore(), service, CFG, {CUSTOM: lambda: CUSTOM_VALUE})])


def _dns(task, net, port):
    return f"{task}.{net}.{CFG.autoip_tld()}:{port}"


@pytest.mark.parametrize("service,net", [("svc-name", "svc-name"), ("/path/to/svc-name", "pathtosvc-name")])
def test_all_endpoints(service, net):
    r = _router(service)
    listing = r.get("/v1/endpoints")
    assert listing.status == 200 and listing.json() == [CUSTOM, "novip", "porta", "portb"]
    custom = r.get(f"/v1/endpoints/{CUSTOM}")
    assert custom.status == 200 and custom.body == CUSTOM_VALUE

    novip = r.get("/v1/endpoints/novip").json()
    assert set(novip) == {"dns", "address"}  # a non-VIP label is no VIP
    assert novip["dns"] == [_dns("vips-1", net, 2348), _dns("vips-2", net, 3459)]
    assert novip["address"] == [f"{U.HOSTNAME}:2348", f"{U.HOSTNAME}:3459"]

    porta = r.get("/v1/endpoints/porta").json()
    assert len(porta) == 3 and porta["vip"] == f"vip1.{net}.{CFG.vip_tld()}:5432"
    assert porta["dns"] == [_dns("ports-1", net, 1234), _dns("ports-2", net, 1243), _dns("vips-1", net, 2345),
                            _dns("vips-2", net, 3456)]
    assert porta["address"] == [f"{U.HOSTNAME}:{p}" for p in (1234, 1243, 2345, 3456)]

    portb = r.get("/v1/endpoints/portb").json()
    assert len(portb) == 3 and portb["vip"] == f"vip2.{net}.{CFG.vip_tld()}:6432"
    assert portb["dns"] == [_dns("ports-1", net, 1235), _dns("vips-2", net, 3457)]
    assert portb["address"] == [f"{U.HOSTNAME}:1235", f"{U.HOSTNAME}:3457"]


def _status(ip):
    s = P.TaskStatus(state=P.TASK_RUNNING)
    s.task_id.CopyFrom(U.TASK_ID)
    s.container_status.network_infos.add().ip_addresses.add(ip_address=ip)
    return s


def _porta_addresses(store):
    e = _router("svc-name", store).get("/v1/endpoints/porta").json()
    assert e["dns"] == [_dns(t, "svc-name", p) for t, p in
                        (("ports-1", 1234), ("ports-2", 1243), ("vips-1", 2345), ("vips-2", 3456))]
    return {a.rsplit(":", 1)[0] for a in e["address"]}


def test_overlay_address_fallbacks():
    names = [t.name for t in TASKS]
    assert _porta_addresses(FakeStore()) == {U.HOSTNAME}  # no status: the offer hostname
    overlay = {n: _status(OVERLAY_HOSTNAME) for n in names}
    assert _porta_addresses(FakeStore(overlay)) == {OVERLAY_HOSTNAME}
    other = {f"{n}:task-status": _status("otherHost").SerializeToString() for n in names}
    assert _porta_addresses(FakeStore(overlay, other)) == {OVERLAY_HOSTNAME}  # the live status wins
    assert _porta_addresses(FakeStore({}, other)) == {"otherHost"}  # then the last IP-bearing status


def test_unknown_endpoint():
    assert _router("svc-name").get("/v1/endpoints/porta-hidden").status == 404
