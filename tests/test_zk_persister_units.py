"""ZooKeeper persister units against the in-repo ZooKeeper server: service root naming, multi-op
writes and deletes from every starting state, digest ACLs, root deletion that keeps the lock,
the ``servicename`` node, copies that carry null-data nodes, and illegal copy endpoints.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/curator/{CuratorPersisterTest,
CuratorUtilsTest}.java. The reference's mock-Curator cases become real round trips here.
"""
import itertools

import pytest

from dcos_commons_amd.storage import persister_utils as PU
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import PersisterException, Reason
from dcos_commons_amd.storage.zk_persister import ZooKeeperPersister, get_service_root_path, init_service_name
from dcos_commons_amd.testing.zk_server import ZkServer

PATH_1, PATH_2 = "/path/1", "/path/2"
PATH_SUB_1, PATH_SUB_2 = "/path/sub/1", "/path/sub/2"
DATA = {PATH_1: b"one", PATH_2: b"two", PATH_SUB_1: b"sub_one", PATH_SUB_2: b"sub_two"}
_names = itertools.count()


@pytest.fixture(scope="module")
def zk():
    srv = ZkServer().start()
    yield srv
    srv.stop()


@pytest.fixture
def persister(zk):
    p = ZooKeeperPersister(zk.connect_string, f"svc-{next(_names)}")
    yield p
    p.close()


@pytest.mark.parametrize("name,root", [
    ("/test", "/dcos-service-test"), ("test", "/dcos-service-test"),
    ("/path/to/myteam/test", "/dcos-service-path__to__myteam__test"),
    ("path/to/myteam/test", "/dcos-service-path__to__myteam__test"),
    ("//test", "/dcos-service-__test"),
    ("/path/to/myteam//test", "/dcos-service-path__to__myteam____test"),
])
def test_service_root_path(name, root):
    assert get_service_root_path(name) == root


@pytest.mark.parametrize("name", ["/folder/path/to/myservice", "unfoldered"])
def test_data_lives_under_the_service_root(zk, name):
    p = ZooKeeperPersister(zk.connect_string, name)
    p.set(PATH_1, b"one")
    assert p.client.get(get_service_root_path(name) + PATH_1)[0] == b"one"
    p.recursive_delete("/")
    p.close()


def _setup(p, state):
    """The reference's starting states for multi-op writes/deletes."""
    if state == "empty":
        return
    p.set_many({k: b"x" for k in DATA})
    if state == "ones_missing":
        p.recursive_delete(PATH_1)
        p.recursive_delete(PATH_SUB_1)
    elif state == "roots_missing":
        p.recursive_delete(PATH_1)
        p.recursive_delete(PATH_2)
    elif state == "subs_missing":
        p.recursive_delete("/path/sub")


STATES = ["empty", "ones_missing", "roots_missing", "subs_missing", "full"]


@pytest.mark.parametrize("state", STATES)
def test_set_many_from_every_state(persister, state):
    _setup(persister, state)
    persister.set_many(DATA)
    assert {k: persister.get(k) for k in DATA} == DATA


@pytest.mark.parametrize("state", STATES[1:])
def test_delete_many_root_from_every_state(persister, state):
    _setup(persister, state)
    persister.recursive_delete_many(["/"])
    assert PU.get_all_keys(persister) == []


def test_delete_many_without_a_service_root_fails(persister):
    with pytest.raises(PersisterException) as e:
        persister.recursive_delete_many(["/"])
    assert e.value.reason == Reason.STORAGE_ERROR


def test_deleting_an_already_deleted_path_fails(persister):
    _setup(persister, "full")
    persister.recursive_delete("/path")
    with pytest.raises(PersisterException) as e:
        persister.recursive_delete(PATH_1)
    assert e.value.reason == Reason.NOT_FOUND


def test_acls(zk):
    root = f"acl-{next(_names)}"
    open_p = ZooKeeperPersister(zk.connect_string, root)
    acl_p = ZooKeeperPersister(zk.connect_string, root, "testuser", "testpw")
    wrong_p = ZooKeeperPersister(zk.connect_string, root, "testuser", "otherpw")
    try:
        acl_p.set(PATH_1, b"one")
        assert acl_p.get(PATH_1) == b"one"
        assert open_p.get(PATH_1) == b"one"  # world-readable
        for other in (open_p, wrong_p):
            with pytest.raises(PersisterException) as e:
                other.set(PATH_1, b"two")
            assert e.value.reason == Reason.STORAGE_ERROR and "NoAuth" in type(e.value.__cause__).__name__
        acl_p.recursive_delete("/path")
    finally:
        for p in (open_p, acl_p, wrong_p):
            p.close()
    with pytest.raises(ValueError):
        ZooKeeperPersister(zk.connect_string, root, "user-without-password", "")


def test_delete_root_keeps_the_lock(persister):
    for path, v in [("lock", b"1"), ("a", b"2"), ("a/1", b"1"), ("a/lock", b"2"), ("a/2/a", b"1"), ("a/3", b"2"),
                    ("a/3/a/1", b"1"), ("b", b"2"), ("c", b"1"), ("d/1/a/1", b"2")]:
        persister.set(path, v)
    persister.recursive_delete("")
    assert list(persister.get_children("")) == ["lock"]
    assert persister.get("lock") == b"1"
    assert PU.get_all_keys(persister) == ["/lock"]


def test_service_name_node(zk):
    name = f"/path/to/myservice{next(_names)}"
    p = ZooKeeperPersister(zk.connect_string, name)
    init_service_name(p, name)
    assert list(p.get_children("")) == ["servicename"]
    assert p.get("servicename") == name.encode()
    init_service_name(p, name)  # idempotent
    p.close()


def test_double_underscore_service_name_is_rejected(zk):
    with pytest.raises(ValueError, match="double underscore"):
        ZooKeeperPersister(zk.connect_string, "/path/to__myservice")


def test_service_name_collision():
    p = MemPersister()
    init_service_name(p, "/path/to/myservice")
    with pytest.raises(ValueError, match="Collision"):
        init_service_name(p, "/path/to.myservice")


def test_recursive_copy_keeps_null_data(persister):
    for path, v in [("lock", b"1"), ("x", b"2"), ("x/1", b"1"), ("x/lock", b"2"), ("x/2/a", b"1"), ("x/3", b"2"),
                    ("x/3/a/1", b"1"), ("x/5/1", None), ("y", b"2"), ("z", b"1"), ("w/1/a/1", b"2"),
                    ("w/1/a/2", None)]:
        persister.set(path, v)
    persister.recursive_copy("/x", "/p")
    assert list(persister.get_children("/p")) == ["1", "2", "3", "5", "lock"]
    assert list(persister.get_children("/p/5")) == ["1"]
    assert [persister.get(k) for k in ("p", "p/1", "p/lock", "p/2/a", "p/3", "p/3/a/1", "p/5/1")] == \
        [b"2", b"1", b"2", b"1", b"2", b"1", None]


@pytest.mark.parametrize("src,dst", [("lock", "/does-not-matter"), ("/does-not-matter", "ROOT")])
def test_recursive_copy_refuses_the_lock_and_the_root(persister, src, dst):
    with pytest.raises(ValueError):
        persister.recursive_copy(src, persister.root if dst == "ROOT" else dst)


@pytest.mark.parametrize("setup,src,dst", [({"x": b"2", "y": b"1"}, "/x", "/y"), ({"y": b"1"}, "/x", "/y"),
                                           ({}, "/x", "/x")])
def test_recursive_copy_failures(persister, setup, src, dst):
    for k, v in setup.items():
        persister.set(k, v)
    with pytest.raises(PersisterException):
        persister.recursive_copy(src, dst)
