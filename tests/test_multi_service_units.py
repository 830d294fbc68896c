"""Unit tests of the multi-service layer with fake services.

Mirrors the reference's scheduler/multi suites (sdk/scheduler/src/test/java/com/mesosphere/sdk/
scheduler/multi/{MultiServiceEventClientTest,ParallelFootprintDisciplineTest,
DisciplineSelectionStoreTest,MultiServiceManagerTest,ServiceStoreTest}.java and
http/endpoints/MultiHealthResourceTest.java): status aggregation across services, offers handed
to each WORKING service in turn with the offers earlier services consumed pruned, uninstall and
removal of finished services, task-status routing, footprint slots, the persisted selection and
service list, and the multi-service health endpoint.
"""
from types import SimpleNamespace

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.common_id_utils import to_task_id
from dcos_commons_amd.offer.recommendations import ReserveOfferRecommendation
from dcos_commons_amd.scheduler.mesos_event_client import (
    ClientStatusResponse,
    OfferResponse,
    OfferResult,
    TaskStatusResponse,
    TaskStatusResult,
)
from dcos_commons_amd.scheduler.multi import (
    DisciplineSelectionStore,
    MultiHealthResource,
    MultiServiceEventClient,
    MultiServiceManager,
    OfferDiscipline,
    ParallelFootprintDiscipline,
    ServiceStore,
)
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanManager
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.storage import persister_utils
from dcos_commons_amd.storage.mem_persister import MemPersister

SERVICE_NAME = "test-service"


def offer(i: int) -> P.Offer:
    o = P.Offer()
    o.id.value = str(i)
    o.framework_id.value = "test-framework-id"
    o.agent_id.value = "test-agent-id"
    o.hostname = "test-hostname"
    return o


def cpus(v: float) -> P.Resource:
    r = P.Resource(name="cpus", type=P.Value.SCALAR)
    r.scalar.value = v
    return r


def consume_first(offers):
    return OfferResponse.processed([ReserveOfferRecommendation(offers[0], cpus(3))] if offers else [])


def consume_last(offers):
    return OfferResponse.processed([ReserveOfferRecommendation(offers[-1], cpus(5))] if offers else [])


def no_changes(offers):
    return OfferResponse.processed([])


def not_ready(offers):
    return OfferResponse.not_ready([])


class FakeStateStore:
    def __init__(self):
        self.deleted = 0

    def delete_all_data_if_namespaced(self):
        self.deleted += 1


class FakeService:
    """An AbstractScheduler stand-in: canned client status, offer behaviour and status result."""

    def __init__(self, name, status=None, on_offers=no_changes, status_result=None):
        self.service_spec = SimpleNamespace(name=name)
        self.status = status or ClientStatusResponse.idle()
        self.on_offers = on_offers
        self.status_result = status_result or TaskStatusResponse.processed()
        self.state_store = FakeStateStore()
        self.offer_calls = []
        self.status_calls = []
        self.registered_calls = []
        self.uninstall_scheduler = None

    def get_client_status(self):
        return self.status

    def offers(self, offers):
        self.offer_calls.append([o.id.value for o in offers])
        return self.on_offers(list(offers))

    def task_status(self, status):
        self.status_calls.append(status)
        return self.status_result

    def registered(self, re_registered):
        self.registered_calls.append(re_registered)

    def to_uninstall_scheduler(self):
        return self.uninstall_scheduler


class FakeManager:
    """Records the calls MultiServiceEventClient makes on its MultiServiceManager."""

    def __init__(self, services=()):
        self.services = list(services)
        self.uninstalled = []
        self.removed = []
        self.matching = {}

    def all_services(self):
        return list(self.services)

    def get_service(self, name):
        return next((s for s in self.services if s.service_spec.name == name), None)

    def get_service_sanitized(self, name):
        return self.matching.get(("sanitized", name))

    def get_matching_service(self, status):
        return self.matching.get(status.task_id.value)

    def uninstall_services(self, names):
        self.uninstalled.append(list(names))

    def remove_services(self, names):
        self.removed.append(list(names))

    def registered(self, re_registered):
        pass


class RecordingDiscipline(OfferDiscipline):
    def __init__(self):
        self.updates = []
        self.statuses = []

    def update_services(self, names):
        self.updates.append(set(names))

    def update_service_status(self, name, status):
        self.statuses.append((name, status))
        return True


def client(manager, uninstalling=False, discipline=None, removed=None):
    removed_names = removed if removed is not None else []
    step = SimpleNamespace(set_complete=lambda: None) if uninstalling else None
    return MultiServiceEventClient(SERVICE_NAME, SchedulerConfig.for_testing(), manager,
                                   discipline=discipline or RecordingDiscipline(),
                                   uninstall_callback=removed_names.append, deregister_step=step)


# ---------------------------------------------------------------------------------------
# MultiServiceEventClient


def test_no_services_uninstalling_is_ready_to_remove():
    assert client(FakeManager(), uninstalling=True).get_client_status() == ClientStatusResponse.ready_to_remove()


def test_no_services_is_idle_and_offers_are_declined():
    c = client(FakeManager())
    assert c.get_client_status() == ClientStatusResponse.idle()
    r = c.offers([])
    assert r.result == OfferResult.PROCESSED and not r.recommendations
    assert c.get_client_status() == ClientStatusResponse.idle()
    r = c.offers([offer(1), offer(2), offer(3)])
    assert r.result == OfferResult.PROCESSED and not r.recommendations


@pytest.mark.parametrize("uninstalling", [False, True])
def test_finished_service_is_uninstalled_then_removed(uninstalling):
    s1 = FakeService("1", ClientStatusResponse.ready_to_uninstall())
    m = FakeManager([s1])
    d = RecordingDiscipline()
    removed = []
    c = client(m, uninstalling=uninstalling, discipline=d, removed=removed)

    assert c.get_client_status() == ClientStatusResponse.idle()
    assert d.updates == [{"1"}] and d.statuses == [("1", ClientStatusResponse.ready_to_uninstall())]
    assert m.uninstalled == [["1"]]
    assert c.offers([]).result == OfferResult.PROCESSED
    assert s1.state_store.deleted == 0 and removed == []

    s1.status = ClientStatusResponse.ready_to_remove()
    assert c.get_client_status() == ClientStatusResponse.idle()
    assert d.updates == [{"1"}, {"1"}]
    assert d.statuses[-1] == ("1", ClientStatusResponse.ready_to_remove())
    assert s1.state_store.deleted == 1
    assert m.removed == [["1"]] and removed == ["1"]
    assert c.offers([]).result == OfferResult.PROCESSED

    # once the manager no longer lists it: IDLE normally, READY_TO_REMOVE while uninstalling the framework
    m.services = []
    assert c.offers([]).result == OfferResult.PROCESSED
    expected = ClientStatusResponse.ready_to_remove() if uninstalling else ClientStatusResponse.idle()
    assert c.get_client_status() == expected


def test_finished_and_uninstalled_services_in_one_pass():
    s = {n: FakeService(n) for n in "1234"}
    s["1"].status = s["3"].status = ClientStatusResponse.ready_to_remove()
    s["2"].status = s["4"].status = ClientStatusResponse.ready_to_uninstall()
    m = FakeManager(s.values())
    d = RecordingDiscipline()
    removed = []
    c = client(m, discipline=d, removed=removed)
    assert c.get_client_status() == ClientStatusResponse.idle()
    assert d.updates == [{"1", "2", "3", "4"}]
    assert [n for n, _ in d.statuses] == ["1", "2", "3", "4"]
    assert s["1"].state_store.deleted == 1 and s["3"].state_store.deleted == 1
    assert m.removed == [["1", "3"]] and removed == ["1", "3"]
    assert m.uninstalled == [["2", "4"]]


def test_empty_offers_still_reach_every_working_service():
    s = {"1": FakeService("1", ClientStatusResponse.launching(True), consume_first),
         "2": FakeService("2", ClientStatusResponse.footprint(False), consume_last),
         "3": FakeService("3", ClientStatusResponse.idle()),
         "4": FakeService("4", ClientStatusResponse.ready_to_uninstall()),
         "5": FakeService("5", ClientStatusResponse.ready_to_remove())}
    m = FakeManager(s.values())
    c = client(m)
    assert c.get_client_status() == ClientStatusResponse.footprint(True)
    r = c.offers([])
    assert r.result == OfferResult.PROCESSED and not r.recommendations
    assert s["1"].offer_calls == [[]] and s["2"].offer_calls == [[]]
    assert s["3"].offer_calls == [] and s["4"].offer_calls == [] and s["5"].offer_calls == []
    assert m.uninstalled == [["4"]] and m.removed == [["5"]]
    assert s["5"].state_store.deleted == 1


def test_offers_consumed_by_earlier_services_are_pruned_for_later_ones():
    behaviours = [consume_first, consume_last, no_changes] * 3
    states = [ClientStatusResponse.launching(False), ClientStatusResponse.footprint(False),
              ClientStatusResponse.launching(False), ClientStatusResponse.footprint(False),
              ClientStatusResponse.launching(True), ClientStatusResponse.footprint(False),
              ClientStatusResponse.launching(False), ClientStatusResponse.footprint(False),
              ClientStatusResponse.launching(False)]
    services = [FakeService(str(i + 1), st, b) for i, (st, b) in enumerate(zip(states, behaviours))]
    c = client(FakeManager(services))
    assert c.get_client_status() == ClientStatusResponse.footprint(True)
    r = c.offers([offer(i) for i in range(1, 8)])
    assert r.result == OfferResult.PROCESSED
    assert sorted(int(rec.offer_id.value) for rec in r.recommendations) == [1, 2, 3, 5, 6, 7]
    seen = [s.offer_calls[0] for s in services]
    assert seen == [
        ["1", "2", "3", "4", "5", "6", "7"],
        ["2", "3", "4", "5", "6", "7"],  # 1 ate the first
        ["2", "3", "4", "5", "6"],       # 2 ate the last
        ["2", "3", "4", "5", "6"],       # 3 changed nothing
        ["3", "4", "5", "6"],
        ["3", "4", "5"],
        ["3", "4", "5"],
        ["4", "5"],
        ["4"],                           # only the middle offer is left
    ]


def test_a_service_that_is_not_ready_makes_the_round_not_ready():
    s1 = FakeService("1", ClientStatusResponse.launching(False), no_changes)
    s2 = FakeService("2", ClientStatusResponse.launching(False), not_ready)
    s3 = FakeService("3", ClientStatusResponse.idle())
    c = client(FakeManager([s1, s2, s3]))
    assert c.get_client_status() == ClientStatusResponse.launching(False)
    r = c.offers([])
    assert r.result == OfferResult.NOT_READY and not r.recommendations
    r = c.offers([offer(1), offer(2), offer(3)])
    assert r.result == OfferResult.NOT_READY and not r.recommendations
    assert s1.offer_calls == [[], ["1", "2", "3"]] and s2.offer_calls == [[], ["1", "2", "3"]]
    assert s3.offer_calls == []


@pytest.mark.parametrize("statuses,expected", [
    ([ClientStatusResponse.launching(False), ClientStatusResponse.launching(True), ClientStatusResponse.idle()],
     ClientStatusResponse.launching(True)),
    ([ClientStatusResponse.launching(False)] * 3, ClientStatusResponse.launching(False)),
    ([ClientStatusResponse.idle()] * 3, ClientStatusResponse.idle()),
    ([ClientStatusResponse.launching(True), ClientStatusResponse.footprint(False),
      ClientStatusResponse.launching(False)], ClientStatusResponse.footprint(True)),
])
def test_client_status_aggregation(statuses, expected):
    services = [FakeService(str(i), st) for i, st in enumerate(statuses)]
    c = client(FakeManager(services))
    assert c.offers([]).result == OfferResult.PROCESSED
    assert c.get_client_status() == expected


def test_status_for_no_known_service_is_unknown():
    m = FakeManager()
    st = P.TaskStatus(state=P.TASK_FINISHED)
    st.task_id.CopyFrom(to_task_id("2", "foo"))
    assert client(m).task_status(st).result == TaskStatusResult.UNKNOWN_TASK


def test_status_falls_back_to_the_service_named_like_the_framework():
    s3 = FakeService("3")
    m = FakeManager([s3])
    m.matching[("sanitized", SERVICE_NAME)] = s3
    st = P.TaskStatus(state=P.TASK_FINISHED)
    st.task_id.CopyFrom(to_task_id("3", "foo"))
    assert client(m).task_status(st).result == TaskStatusResult.PROCESSED
    assert s3.status_calls == [st]


@pytest.mark.parametrize("result", [TaskStatusResponse.unknown_task(), TaskStatusResponse.processed()])
def test_status_is_routed_to_the_matching_service(result):
    s2 = FakeService("2", status_result=result)
    m = FakeManager([s2])
    st = P.TaskStatus(state=P.TASK_FINISHED)
    st.task_id.CopyFrom(to_task_id("2", "foo"))
    m.matching[st.task_id.value] = s2
    assert client(m).task_status(st).result == result.result
    assert s2.status_calls == [st]


# ---------------------------------------------------------------------------------------
# ParallelFootprintDiscipline / DisciplineSelectionStore


@pytest.fixture
def store():
    return DisciplineSelectionStore(MemPersister())


@pytest.mark.parametrize("limit", [0, -1])
def test_discipline_rejects_non_positive_limits(store, limit):
    with pytest.raises(ValueError):
        ParallelFootprintDiscipline(limit, store)


def test_discipline_needs_update_services_first(store):
    with pytest.raises(RuntimeError):
        ParallelFootprintDiscipline(1, store).update_service_status("1", ClientStatusResponse.launching(False))


FP = ClientStatusResponse.footprint(False)
LAUNCH = ClientStatusResponse.launching(False)


def test_slot_is_released_by_every_non_reserving_state(store):
    d = ParallelFootprintDiscipline(1, store)
    d.update_services(["1", "2", "3"])
    assert d.update_service_status("1", FP) and not d.update_service_status("2", FP)
    assert d.update_service_status("1", ClientStatusResponse.ready_to_uninstall())
    assert d.update_service_status("2", FP) and not d.update_service_status("1", FP)
    assert d.update_service_status("2", LAUNCH)
    assert d.update_service_status("1", FP) and not d.update_service_status("2", FP)
    assert d.update_service_status("1", ClientStatusResponse.ready_to_remove())
    assert d.update_service_status("2", FP) and not d.update_service_status("1", FP)


def test_single_slot(store):
    d = ParallelFootprintDiscipline(1, store)
    d.update_services(["1", "2", "3"])
    assert store.fetch_selected_services() == set()
    assert d.update_service_status("1", LAUNCH)
    assert d.update_service_status("2", FP)
    assert not d.update_service_status("3", FP)
    assert d.update_service_status("3", LAUNCH)  # may still launch
    assert d.update_service_status("2", FP)
    d.update_services(["1", "3"])  # 2 removed: its slot frees up
    assert d.update_service_status("3", FP)
    assert not d.update_service_status("1", FP)
    assert d.update_service_status("3", FP)


def test_single_slot_starts_occupied(store):
    store.store_selected_services({"2"})
    d = ParallelFootprintDiscipline(1, DisciplineSelectionStore(store.persister))
    d.update_services(["1", "2", "3"])
    assert store.fetch_selected_services() == {"2"}
    assert not d.update_service_status("1", FP)
    assert d.update_service_status("2", FP)
    assert not d.update_service_status("3", FP)
    assert not d.update_service_status("1", FP)
    assert d.update_service_status("2", LAUNCH)
    assert d.update_service_status("1", FP)


def test_single_slot_prunes_unknown_stored_services(store):
    store.store_selected_services({"2", "3"})
    reader = DisciplineSelectionStore(store.persister)
    d = ParallelFootprintDiscipline(1, reader)
    d.update_services(["1", "2"])
    assert DisciplineSelectionStore(store.persister).fetch_selected_services() == {"2"}
    assert not d.update_service_status("1", FP)
    assert d.update_service_status("2", FP)
    assert d.update_service_status("2", LAUNCH)
    assert d.update_service_status("1", FP)
    assert not d.update_service_status("2", FP)


def test_multi_slot(store):
    d = ParallelFootprintDiscipline(2, store)
    d.update_services(["1", "2", "3"])
    assert store.fetch_selected_services() == set()
    assert d.update_service_status("1", FP) and d.update_service_status("2", FP)
    assert d.update_service_status("1", FP) and d.update_service_status("2", FP)
    assert not d.update_service_status("3", FP)
    assert d.update_service_status("1", LAUNCH)
    assert d.update_service_status("3", FP)
    assert not d.update_service_status("1", FP)
    d.update_services(["1", "3"])
    assert DisciplineSelectionStore(store.persister).fetch_selected_services() == {"3"}
    assert d.update_service_status("1", FP) and d.update_service_status("3", FP)


def test_multi_slot_starts_occupied(store):
    store.store_selected_services({"2"})
    d = ParallelFootprintDiscipline(2, DisciplineSelectionStore(store.persister))
    d.update_services(["1", "2", "3"])
    assert d.update_service_status("1", FP)
    assert not d.update_service_status("3", FP)
    assert d.update_service_status("2", FP)
    assert not d.update_service_status("3", FP)
    assert d.update_service_status("2", LAUNCH)
    assert d.update_service_status("3", FP)


def test_multi_slot_prunes_unknown_stored_services(store):
    store.store_selected_services({"2", "3"})
    d = ParallelFootprintDiscipline(2, DisciplineSelectionStore(store.persister))
    d.update_services(["1", "2"])
    assert DisciplineSelectionStore(store.persister).fetch_selected_services() == {"2"}
    assert d.update_service_status("1", FP) and d.update_service_status("2", FP)


def test_slot_count_change_keeps_the_services_already_selected(store):
    p = store.persister
    d = ParallelFootprintDiscipline(1, DisciplineSelectionStore(p))
    d.update_services(["1", "2", "3"])
    assert d.update_service_status("2", FP)
    assert not d.update_service_status("1", FP) and not d.update_service_status("3", FP)
    d.update_services(["1", "2", "3"])
    assert DisciplineSelectionStore(p).fetch_selected_services() == {"2"}

    d = ParallelFootprintDiscipline(2, DisciplineSelectionStore(p))  # more slots after a restart
    d.update_services(["1", "2", "3"])
    assert d.update_service_status("1", FP) and d.update_service_status("2", FP)
    assert not d.update_service_status("3", FP)
    d.update_services(["1", "2", "3"])
    assert DisciplineSelectionStore(p).fetch_selected_services() == {"1", "2"}

    d = ParallelFootprintDiscipline(1, DisciplineSelectionStore(p))  # fewer slots: both keep theirs
    d.update_services(["1", "2", "3"])
    assert d.update_service_status("1", FP) and d.update_service_status("2", FP)
    assert not d.update_service_status("3", FP)
    d.update_services(["1", "2", "3"])
    assert DisciplineSelectionStore(p).fetch_selected_services() == {"1", "2"}
    assert d.update_service_status("2", LAUNCH)
    assert not d.update_service_status("3", FP)  # the freed slot is over the new limit
    assert d.update_service_status("1", LAUNCH)
    assert d.update_service_status("3", FP)


SELECTED_A = {"foo", "/path/to/bar"}
SELECTED_B = {"baz"}


def test_selection_store_round_trip_and_change_detection(store):
    assert store.store_selected_services(SELECTED_A)
    assert store.fetch_selected_services() == SELECTED_A
    assert not store.store_selected_services(SELECTED_A)
    assert store.store_selected_services(SELECTED_B)
    assert not store.store_selected_services(SELECTED_B)
    assert store.store_selected_services(set())
    assert not store.store_selected_services(set())
    assert store.fetch_selected_services() == set()


def test_selection_store_layout_and_fresh_reader(store):
    assert store.fetch_selected_services() == set()
    store.store_selected_services(SELECTED_A)
    raw = store.persister.get("SelectedServices").decode()
    assert set(raw.split("__")) == SELECTED_A  # reference layout: names joined by "__"
    assert DisciplineSelectionStore(store.persister).fetch_selected_services() == SELECTED_A
    assert persister_utils.get_all_keys(store.persister) == ["/SelectedServices"]
    persister_utils.clear_all_data(store.persister)
    assert persister_utils.get_all_keys(store.persister) == []


# ---------------------------------------------------------------------------------------
# MultiServiceManager


def svc(name):
    s = FakeService(name)
    return s


def test_manager_registration_callbacks_may_call_back_into_the_manager():
    m = MultiServiceManager()
    loopback = []
    s1, s2 = svc("1"), svc("2")
    u1, u2 = svc("1"), svc("2")
    s1.uninstall_scheduler, s2.uninstall_scheduler = u1, u2

    def cb1(re):
        m.get_service("1")
        loopback.append("1")

    def cb2(re):
        m.get_service_names()
        loopback.append("2")
    for s, cb in ((s1, cb1), (u1, cb1), (s2, cb2), (u2, cb2)):
        s.registered = cb
    m.registered(False)
    m.put_service(s1)
    assert loopback == ["1"]
    m.put_service(s2)
    assert loopback == ["1", "2"]
    m.registered(True)
    assert loopback == ["1", "2", "1", "2"]
    m.uninstall_services(["1", "2"])
    assert loopback == ["1", "2", "1", "2", "1", "2"]
    assert m.get_service("1") is u1 and m.get_service("2") is u2


def test_manager_put_replace_remove():
    m = MultiServiceManager()
    s1, s2 = svc("1"), svc("2")
    m.put_service(s1)
    assert m.get_service_names() == ["1"]
    m.put_service(s2)
    assert m.get_service_names() == ["1", "2"]
    m.put_service(s2)  # reconfiguration
    assert m.get_service_names() == ["1", "2"]
    m.remove_services(["2"])
    assert m.get_service_names() == ["1"]
    m.put_service(s2)
    assert m.get_service_names() == ["1", "2"]


def test_manager_sanitized_name_conflict_message():
    m = MultiServiceManager()
    m.put_service(svc("/path/to/1"))
    with pytest.raises(ValueError) as e:
        m.put_service(svc("/path.to/1"))
    assert str(e.value) == ("Service named '/path.to/1' conflicts with existing service '/path/to/1': "
                            "matching sanitized name 'path.to.1'")
    m.remove_services(["/path/to/1"])
    m.put_service(svc("/path.to/1"))


def _status(service_name):
    st = P.TaskStatus(state=P.TASK_FINISHED)
    st.task_id.CopyFrom(to_task_id(service_name, "foo"))
    return st


def test_manager_routes_statuses_by_sanitized_service_name():
    m = MultiServiceManager()
    s1, s2 = svc("/path/to/1"), svc("2")
    m.put_service(s1)
    m.put_service(s2)
    assert m.get_matching_service(_status("/path/to/1")) is s1
    assert m.get_matching_service(_status("path.to.1")) is s1
    assert m.get_matching_service(_status("/path/to/2")) is None
    assert m.get_matching_service(_status("path.to.2")) is None
    assert m.get_matching_service(_status("2")) is s2
    m.remove_services(["/path/to/1", "2"])
    assert m.get_matching_service(_status("/path/to/1")) is None
    assert m.get_matching_service(_status("2")) is None
    bad = P.TaskStatus(state=P.TASK_RUNNING)
    bad.task_id.value = "not-an-sdk-task-id"
    assert m.get_matching_service(bad) is None


def test_manager_registers_services_added_after_registration():
    m = MultiServiceManager()
    s1, s2 = svc("1"), svc("2")
    m.put_service(s1)
    m.registered(False)
    assert s1.registered_calls == [False]
    m.put_service(s2)
    assert s2.registered_calls == [False]
    m.put_service(s2)  # reconfiguration re-registers
    assert s2.registered_calls == [False, False]


def test_manager_uninstall_requested_service_once():
    m = MultiServiceManager()
    class UninstallingService:  # an uninstall scheduler has no uninstall scheduler of its own
        service_spec = SimpleNamespace(name="1")

        def registered(self, re_registered):
            pass
    s1 = svc("1")
    u1 = UninstallingService()
    s1.uninstall_scheduler = u1
    m.put_service(s1)
    m.uninstall_services(["1", "1", "2"])  # the second "1" and the unknown "2" are ignored
    assert m.get_service_names() == ["1"] and m.get_service("1") is u1
    m.remove_services(["1"])
    assert m.get_service_names() == []


# ---------------------------------------------------------------------------------------
# ServiceStore


FOO, BAR = b"foo-data", b"bar-data"


class Factory:
    def __init__(self, names):
        self.names = dict(names)
        self.calls = []
        self.fail = set()

    def __call__(self, context):
        self.calls.append(context)
        if context in self.fail:
            raise RuntimeError("BANG")
        return svc(self.names[context])


def test_service_store_put_get_and_uninstall_callback():
    f = Factory({FOO: "foo", BAR: "bar"})
    st = ServiceStore(MemPersister(), f)
    assert st.get("foo") is None
    assert st.put(FOO).service_spec.name == "foo"
    assert st.get("foo") == FOO and len(st.recover()) == 1
    assert st.get("bar") is None
    st.put(BAR)
    assert st.get("foo") == FOO and st.get("bar") == BAR and len(st.recover()) == 2
    st.uninstall_callback()("foo")
    assert st.get("foo") is None and len(st.recover()) == 1
    st.uninstall_callback()("bar")
    assert st.get("bar") is None and st.recover() == []


def test_service_store_does_not_persist_a_context_the_factory_rejects():
    f = Factory({FOO: "foo", BAR: "bar"})
    f.fail.add(BAR)
    st = ServiceStore(MemPersister(), f)
    with pytest.raises(RuntimeError, match="BANG"):
        st.put(BAR)
    assert st.get("bar") is None


def test_service_store_slashed_names_are_escaped():
    f = Factory({FOO: "/path/to/foo"})
    p = MemPersister()
    st = ServiceStore(p, f)
    assert st.get("/path/to/foo") is None
    st.put(FOO)
    assert st.get("/path/to/foo") == FOO
    assert p.get("/ServiceList/path__to__foo/Context") == FOO
    st.uninstall_callback()("/path/to/foo")
    assert st.get("/path/to/foo") is None


def test_service_store_recovers_from_the_persister_alone():
    f = Factory({FOO: "foo", BAR: "bar"})
    p = MemPersister()
    ServiceStore(p, f).put(FOO)
    ServiceStore(p, f).put(BAR)
    st = ServiceStore(p, f)
    assert st.get("foo") == FOO and st.get("bar") == BAR
    assert sorted(s.service_spec.name for s in st.recover()) == ["bar", "foo"]
    assert f.calls.count(FOO) == 2 and f.calls.count(BAR) == 2


def test_service_store_recovery_skips_services_that_fail_to_build():
    f = Factory({FOO: "foo", BAR: "bar"})
    p = MemPersister()
    ServiceStore(p, f).put(FOO)
    ServiceStore(p, f).put(BAR)
    f.fail.add(FOO)
    assert [s.service_spec.name for s in ServiceStore(p, f).recover()] == ["bar"]


def test_service_store_context_limit():
    f = Factory({b"x" * (100 * 1024 + 1): "big"})
    st = ServiceStore(MemPersister(), f)
    with pytest.raises(ValueError, match="limit is 102400 bytes"):
        st.put(b"x" * (100 * 1024 + 1))
    assert st.get("big") is None


# ---------------------------------------------------------------------------------------
# MultiHealthResource


class FakePlan:
    def __init__(self, errors=(), complete=True):
        self.errors = list(errors)
        self.complete = complete

    def get_errors(self):
        return self.errors

    def is_complete(self):
        return self.complete

    def interrupt(self):
        pass

    def proceed(self):
        pass


class EmptyManager:
    def all_services(self):
        return []


@pytest.mark.parametrize("p1,p2,code", [
    (FakePlan(["err"], True), FakePlan([], False), 417),
    (FakePlan(["err"], True), FakePlan([], True), 417),
    (FakePlan([], False), FakePlan([], True), 202),
    (FakePlan([], True), FakePlan([], True), 200),
])
def test_multi_health_codes(p1, p2, code):
    cfg = SchedulerConfig.for_testing(PACKAGE_NAME="pkg", PACKAGE_VERSION="9.9")
    res = MultiHealthResource(EmptyManager(), cfg,
                              [DefaultPlanManager.create_proceeding(p1), DefaultPlanManager.create_proceeding(p2)])
    r = res.health()
    assert r.status == code
    body = r.json()
    assert body["PACKAGE_NAME"] == "pkg" and body["PACKAGE_VERSION"] == "9.9"
    assert set(body) == {"PACKAGE_NAME", "PACKAGE_VERSION", "PACKAGE_BUILT_AT", "SDK_NAME", "SDK_VERSION",
                         "SDK_GIT_SHA", "SDK_BUILT_AT"}


def test_multi_health_without_plans_is_ok():
    assert MultiHealthResource(EmptyManager(), SchedulerConfig.for_testing()).health().status == 200
