"""ZooKeeper client / persister / locker over the jute protocol (reference:
curator/CuratorPersisterTest.java, CuratorLockerTest.java, CuratorUtilsTest.java)."""
import threading
import time

import pytest

from dcos_commons_amd.framework.process_exit import ProcessExit, ProcessExitError
from dcos_commons_amd.storage import zookeeper as Z
from dcos_commons_amd.storage.persister import PersisterException, Reason
from dcos_commons_amd.storage.zk_persister import ZkLocker, ZooKeeperPersister, get_service_root_path, \
    init_service_name
from dcos_commons_amd.testing.zk_server import ZkServer


@pytest.fixture
def zk():
    srv = ZkServer().start()
    yield srv
    srv.stop()


@pytest.fixture
def client(zk):
    c = Z.ZkClient(zk.connect_string, session_timeout_ms=2000).start()
    yield c
    c.close()


def test_connect_string_parsing():
    assert Z.parse_connect_string("a:1,b:2/x/y") == ([("a", 1), ("b", 2)], "/x/y")
    assert Z.parse_connect_string("a") == ([("a", 2181)], "")
    assert get_service_root_path("/path/to/svc") == "/dcos-service-path__to__svc"


def test_basic_crud_versions_and_errors(client):
    assert client.create("/a", b"1") == "/a"
    with pytest.raises(Z.NodeExistsError):
        client.create("/a")
    with pytest.raises(Z.NoNodeError):
        client.create("/x/y")
    data, st = client.get("/a")
    assert data == b"1" and st.version == 0 and st.data_length == 1
    st = client.set("/a", b"22", version=0)
    assert st.version == 1
    with pytest.raises(Z.BadVersionError):
        client.set("/a", b"3", version=0)
    client.create("/a/child", None)
    assert client.get("/a/child")[0] is None  # null data is preserved (not b"")
    assert client.exists("/a").num_children == 1
    with pytest.raises(Z.NotEmptyError):
        client.delete("/a")
    client.delete("/a", recursive=True)
    assert client.exists("/a") is None
    client.create("/p/q/r", b"v", make_parents=True)
    assert client.get_children("/p") == ["q"]


def test_sequential_and_ephemeral_nodes(zk, client):
    client.create("/seq")
    a = client.create("/seq/n-", sequence=True)
    b = client.create("/seq/n-", sequence=True)
    assert a == "/seq/n-0000000000" and b == "/seq/n-0000000001"
    other = Z.ZkClient(zk.connect_string, session_timeout_ms=500).start()
    other.create("/eph", b"x", ephemeral=True)
    with pytest.raises(Z.NoChildrenForEphemeralsError):
        other.create("/eph/child")
    assert client.exists("/eph") is not None
    other.close()  # closing the session removes its ephemerals immediately
    assert client.exists("/eph") is None
    third = Z.ZkClient(zk.connect_string, session_timeout_ms=300).start()
    third.create("/eph2", ephemeral=True)
    zk.drop_connections()  # connection lost; the session reattaches before it expires
    time.sleep(0.2)
    assert third.exists("/eph2") is not None
    third._closed.set()  # stop the client without closing its session, then let it expire
    third._drop_connection()
    deadline = time.time() + 5
    while client.exists("/eph2") is not None and time.time() < deadline:
        time.sleep(0.05)
    assert client.exists("/eph2") is None


def test_watches_fire_once(client, zk):
    other = Z.ZkClient(zk.connect_string).start()
    events = []
    client.create("/w", b"0")
    client.get("/w", watch=events.append)
    client.get_children("/w", watch=events.append)
    client.exists("/w/new", watch=events.append)
    other.set("/w", b"1")
    other.create("/w/new")
    other.set("/w", b"2")  # data watch was one-shot
    deadline = time.time() + 5
    while len(events) < 3 and time.time() < deadline:
        time.sleep(0.01)
    time.sleep(0.05)
    kinds = sorted((e.type, e.path) for e in events)
    assert kinds == [(Z.EVENT_CREATED, "/w/new"), (Z.EVENT_DATA_CHANGED, "/w"), (Z.EVENT_CHILD_CHANGED, "/w")]
    other.close()


def test_multi_is_atomic(client):
    client.create("/m", b"0")
    res = client.multi([Z.Check("/m", 0), Z.Create("/m/a", b"1"), Z.SetData("/m", b"x"), Z.Delete("/m/a")])
    assert res[1] == "/m/a" and res[2].version == 1 and res[3] is None
    with pytest.raises(Z.TransactionError) as e:
        client.multi([Z.Create("/m/b", b"1"), Z.Create("/m/b", b"2"), Z.SetData("/m", b"y")])
    assert e.value.results == [0, Z.NodeExistsError.code, -2]
    assert isinstance(e.value.failed, Z.NodeExistsError)
    assert client.exists("/m/b") is None and client.get("/m")[0] == b"x"  # rolled back


def test_chroot_and_digest_acls(zk):
    admin = Z.ZkClient(zk.connect_string + "/jail", auth=[("digest", b"u:p")],
                       default_acl=list(Z.CREATOR_ALL_ACL) + list(Z.READ_ACL_UNSAFE))
    root = Z.ZkClient(zk.connect_string).start()
    root.create("/jail")
    admin.start()
    time.sleep(0.05)  # auth packet is processed before later requests on the same connection
    admin.create("/secret", b"s")
    assert root.get("/jail/secret")[0] == b"s"  # world-readable
    with pytest.raises(Z.NoAuthError):
        root.set("/jail/secret", b"hacked")
    admin.set("/secret", b"ok")
    assert admin.get_children("/") == ["secret"]
    admin.close()
    root.close()


def test_persister_root_semantics(zk):
    p = ZooKeeperPersister(zk.connect_string, "/team/db")
    assert p.root == "/dcos-service-team__db"
    assert p.get("/") is None and list(p.get_children("")) == []
    p.set("lock/x", b"held")  # lock node must survive root deletion
    p.set_many({"Tasks/a/Info": b"1", "FrameworkID": b"fw"})
    p.recursive_delete("/")
    assert list(p.get_children("/")) == ["lock"]
    with pytest.raises(ValueError):
        p.recursive_copy("lock", "lock2")
    init_service_name(p, "/team/db")
    init_service_name(p, "/team/db")
    q = ZooKeeperPersister(zk.connect_string, "team.db")  # different name, different root: fine
    init_service_name(q, "team.db")
    clash = ZooKeeperPersister(zk.connect_string, "/dcos-service-team__db")  # same root as p
    with pytest.raises(ValueError):
        init_service_name(clash, "team.db")
    p.close()
    q.close()
    clash.close()


def test_persister_storage_error_when_server_gone():
    srv = ZkServer().start()
    p = ZooKeeperPersister(srv.connect_string, "svc", session_timeout_ms=500)
    p.client.connect_timeout_s = 0.3
    p.set("a", b"1")
    srv.stop()
    with pytest.raises(PersisterException) as e:
        p.get("a")
    assert e.value.reason == Reason.STORAGE_ERROR
    p.client._closed.set()


def test_locker_excludes_second_scheduler(zk):
    ProcessExit.set_test_mode(True)
    first = ZkLocker("svc", zk.connect_string, wait_s=0.2)
    assert first.lock_internal()
    second = ZkLocker("svc", zk.connect_string, wait_s=0.1)
    t0 = time.time()
    assert not second.lock_internal()  # 3 attempts x 0.1 s
    assert time.time() - t0 >= 0.25
    # waiting contender gets the lock as soon as the holder releases
    third = ZkLocker("svc", zk.connect_string, wait_s=5)
    got = []
    th = threading.Thread(target=lambda: got.append(third.lock_internal()))
    th.start()
    time.sleep(0.2)
    first.unlock_internal()
    th.join(5)
    assert got == [True]
    with pytest.raises(RuntimeError):
        first.unlock_internal()
    third.unlock_internal()
    # process-level API: a failed lock exits with LOCK_UNAVAILABLE
    holder = ZkLocker("svc2", zk.connect_string)
    assert holder.lock_internal()
    with pytest.raises(ProcessExitError) as e:
        ZkLocker.lock("svc2", zk.connect_string, wait_s=0.05)
    assert e.value.code == ProcessExit.LOCK_UNAVAILABLE
    holder.unlock_internal()
    inst = ZkLocker.lock("svc2", zk.connect_string, wait_s=1)
    with pytest.raises(RuntimeError):
        ZkLocker.lock("svc3", zk.connect_string)
    ZkLocker.unlock()
    assert ZkLocker._instance is None and inst.client is None


def test_crashed_holder_lease_expires(zk):
    holder = ZkLocker("svc", zk.connect_string, session_timeout_ms=300)
    assert holder.lock_internal()
    holder.client._closed.set()  # the process dies without releasing
    holder.client._drop_connection()
    waiter = ZkLocker("svc", zk.connect_string, wait_s=3)
    assert waiter.lock_internal()
    waiter.unlock_internal()


def test_factory_zk_and_file_backends_take_the_lock(zk, tmp_path):
    from types import SimpleNamespace

    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
    from dcos_commons_amd.storage.factory import FileLocker, persister_for_service
    from dcos_commons_amd.storage.persister_cache import PersisterCache

    ProcessExit.set_test_mode(True)
    spec = SimpleNamespace(name="/folder/svc", zookeeper_connection=zk.connect_string)
    p = persister_for_service(spec, SchedulerConfig.for_testing(SDK_PERSISTER="zk"))
    try:
        assert isinstance(p, PersisterCache)
        assert ZkLocker._instance is not None
        p.set("FrameworkID", b"x")
        raw = Z.ZkClient(zk.connect_string).start()
        assert raw.get("/dcos-service-folder__svc/FrameworkID")[0] == b"x"
        assert raw.get("/dcos-service-folder__svc/servicename")[0] == b"/folder/svc"
        assert raw.get_children("/dcos-service-folder__svc/lock/leases")  # lease held
        raw.close()
    finally:
        ZkLocker.unlock()
    cfg = SchedulerConfig.for_testing(SDK_PERSISTER="file", SDK_STATE_DIR=str(tmp_path))
    fp = persister_for_service(spec, cfg)
    fp.set("a", b"1")
    other = FileLocker(str(tmp_path / "dcos-service-folder__svc"), wait_s=0.05)
    assert not other.lock()  # a second scheduler for the same service is refused
    FileLocker._held[other.path].unlock()
    assert other.lock()
    other.unlock()


def test_lock_failure_exits_outside_the_instance_lock_and_hooks_register_once(zk, monkeypatch):
    """``ZkLocker.lock`` called ``ProcessExit.exit`` while holding ``_instance_lock``;
    the exit runs ``unlock`` as a shutdown hook, which needs that lock. The hook was also appended
    on every ``lock()``."""
    from dcos_commons_amd.framework import process_exit as PE

    monkeypatch.setattr(PE, "_hooks", [])
    monkeypatch.setattr(ZkLocker, "_hooks_registered", False)
    free_at_exit = []

    def fake_exit(code, cause=None):
        got = []

        def probe():
            ok = ZkLocker._instance_lock.acquire(timeout=1)
            if ok:
                ZkLocker._instance_lock.release()
            got.append(ok)

        th = threading.Thread(target=probe)
        th.start()
        th.join(2)
        free_at_exit.append(bool(got and got[0]))
        raise ProcessExitError(code, cause)

    monkeypatch.setattr(ProcessExit, "exit", staticmethod(fake_exit))
    holder = ZkLocker("svc4", zk.connect_string)
    assert holder.lock_internal()
    with pytest.raises(ProcessExitError):
        ZkLocker.lock("svc4", zk.connect_string, wait_s=0.05)
    assert free_at_exit == [True]
    holder.unlock_internal()
    for _ in range(3):
        ZkLocker.lock("svc4", zk.connect_string, wait_s=1)
        ZkLocker.unlock()
    assert PE._hooks.count(ZkLocker.unlock) == 1


def test_shutdown_hooks_run_from_a_handler_that_interrupts_hook_registration(monkeypatch):
    """SIGTERM landing while the main thread is inside ``add_shutdown_hook`` ran the
    hooks under a non-reentrant lock already held by that thread (deadlock)."""
    from dcos_commons_amd.framework import process_exit as PE

    monkeypatch.setattr(PE, "_hooks", [])
    monkeypatch.setattr(PE, "_hooks_ran", False)
    ran = []
    PE.add_shutdown_hook(lambda: ran.append(1))
    done = threading.Event()

    def body():
        with PE._hooks_lock:  # the interrupted add_shutdown_hook
            PE.run_shutdown_hooks()  # what the signal handler runs on the same thread
        done.set()

    th = threading.Thread(target=body, daemon=True)
    th.start()
    assert done.wait(2), "run_shutdown_hooks deadlocked on the hooks lock"
    assert ran == [1]
    PE.run_shutdown_hooks()  # at most once
    assert ran == [1]
