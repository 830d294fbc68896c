"""Persister semantics (reference: storage/MemPersisterTest, PersisterCacheTest, PersisterUtilsTest,
curator/CuratorPersisterTest). Every backend must behave identically, so the contract tests run
against the memory, file and cached backends."""
import os

import pytest

from dcos_commons_amd.storage import persister_utils as PU
from dcos_commons_amd.storage.file_persister import FilePersister
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import PersisterException, Reason
from dcos_commons_amd.storage.persister_cache import PersisterCache


@pytest.fixture(scope="module")
def zk_server():
    from dcos_commons_amd.testing.zk_server import ZkServer

    srv = ZkServer().start()
    yield srv
    srv.stop()


@pytest.fixture(params=["mem", "file", "cache-mem", "cache-file", "zk", "cache-zk"])
def persister(request, tmp_path):
    kind = request.param
    if kind in ("zk", "cache-zk"):
        from dcos_commons_amd.storage.zk_persister import ZooKeeperPersister

        zk = request.getfixturevalue("zk_server")
        p = ZooKeeperPersister(zk.connect_string, "/test/" + request.node.name.replace("[", "-").rstrip("]"))
        request.addfinalizer(p.close)
        return PersisterCache(p) if kind == "cache-zk" else p
    if kind == "mem":
        return MemPersister()
    if kind == "file":
        return FilePersister(str(tmp_path / "state"), fsync=False)
    if kind == "cache-mem":
        return PersisterCache(MemPersister())
    return PersisterCache(FilePersister(str(tmp_path / "state"), fsync=False))


def test_get_missing_is_not_found(persister):
    with pytest.raises(PersisterException) as e:
        persister.get("/nope")
    assert e.value.reason == Reason.NOT_FOUND
    with pytest.raises(PersisterException):
        persister.get_children("/nope")


def test_set_creates_parents_without_data(persister):
    persister.set("/a/b/c", b"v")
    assert persister.get("/a/b/c") == b"v"
    assert persister.get("/a/b") is None
    assert persister.get("/a") is None
    assert list(persister.get_children("/a")) == ["b"]
    assert list(persister.get_children("/")) == ["a"]


def test_overwrite_and_empty_value(persister):
    persister.set("/x", b"1")
    persister.set("/x", b"")
    assert persister.get("/x") == b""


def test_children_sorted_and_names_with_special_chars(persister):
    for n in ["z", "a", "m-1", "hello world", "pct%2F"]:
        persister.set("/p/" + n, n.encode())
    assert sorted(persister.get_children("/p")) == sorted(["z", "a", "m-1", "hello world", "pct%2F"])
    assert persister.get("/p/hello world") == b"hello world"
    assert persister.get("/p/pct%2F") == b"pct%2F"


def test_set_many_get_many(persister):
    persister.set_many({"/t/a": b"1", "/t/b/c": b"2", "/u": b"3"})
    got = persister.get_many(["/t/a", "/t/b/c", "/u", "/missing", "/t/b"])
    assert got == {"/t/a": b"1", "/t/b/c": b"2", "/u": b"3", "/missing": None, "/t/b": None}


def test_recursive_delete(persister):
    persister.set_many({"/d/a/1": b"1", "/d/a/2": b"2", "/d/b": b"3"})
    persister.recursive_delete("/d/a")
    assert list(persister.get_children("/d")) == ["b"]
    with pytest.raises(PersisterException) as e:
        persister.recursive_delete("/d/a")
    assert e.value.reason == Reason.NOT_FOUND
    persister.recursive_delete_many(["/d/b", "/never"])  # missing paths are ignored
    assert list(persister.get_children("/d")) == []


def test_recursive_copy(persister):
    persister.set_many({"/src/a": b"1", "/src/b/c": b"2"})
    persister.recursive_copy("/src", "/dst")
    assert persister.get("/dst/a") == b"1" and persister.get("/dst/b/c") == b"2"
    with pytest.raises(PersisterException) as e:
        persister.recursive_copy("/src", "/dst")
    assert e.value.reason == Reason.LOGIC_ERROR
    with pytest.raises(PersisterException):
        persister.recursive_copy("/nosrc", "/dst2")


def test_get_all_data_and_clear(persister):
    persister.set_many({"/a/b": b"1", "/c": b"2"})
    data = PU.get_all_data(persister)
    assert data["/a/b"] == b"1" and data["/c"] == b"2"
    assert "/a/b" in PU.get_all_keys(persister)
    PU.clear_all_data(persister)
    assert list(persister.get_children("/")) == []


def test_file_persister_survives_restart(tmp_path):
    root = str(tmp_path / "s")
    p = FilePersister(root, fsync=False)
    p.set_many({"/Tasks/t1/TaskInfo": b"\x00\x01binary", "/Properties/k": b"v"})
    p.recursive_delete("/Properties")
    p.close()
    q = FilePersister(root, fsync=False)
    assert q.get("/Tasks/t1/TaskInfo") == b"\x00\x01binary"
    with pytest.raises(PersisterException):
        q.get("/Properties/k")


def test_file_persister_replays_interrupted_batch(tmp_path):
    """A batch whose journal was written but not applied (crash) is completed on open."""
    import json

    root = str(tmp_path / "s")
    p = FilePersister(root, fsync=False)
    p.set("/keep", b"1")
    journal = os.path.join(root, ".journal")
    ops = [{"op": "set", "path": "/a/b", "data": "aGVsbG8="}, {"op": "del", "path": "/keep"}]
    with open(journal, "w") as f:
        json.dump(ops, f)
    q = FilePersister(root, fsync=False)
    assert q.get("/a/b") == b"hello"
    with pytest.raises(PersisterException):
        q.get("/keep")
    assert not os.path.exists(journal)


def test_persister_cache_refresh_sees_backend_changes():
    backend = MemPersister()
    cache = PersisterCache(backend)
    cache.set("/a", b"1")
    backend.set("/a", b"2")  # out-of-band change
    assert cache.get("/a") == b"1"
    cache.refresh()
    assert cache.get("/a") == b"2"


def test_paths():
    assert PU.join_paths("a", "b") == "a/b"
    assert PU.join_paths("/a/", "/b") == "/a/b"
    assert PU.get_parent_paths("/a/b/c") == ["/a", "/a/b"]
    assert PU.get_service_namespaced_root("path/to/svc") == "Services/path__to__svc"
    assert PU.with_escaped_slashes("/a/b") == "a__b"
    assert PU.get_parent_paths("a/b/c") == ["a", "a/b"]
    with pytest.raises(ValueError):
        PU.with_escaped_slashes("bad__name")


def test_schema_migration_single_to_multi():
    from dcos_commons_amd.state.schema_version_store import SchemaVersion, SchemaVersionStore

    p = MemPersister()
    SchemaVersionStore(p).store(SchemaVersion.SINGLE_SERVICE)
    p.set_many({"/FrameworkID": b"fw", "/Tasks/t/TaskInfo": b"ti", "/ConfigTarget": b"cfg",
                "/Configurations/x": b"c", "/Properties/k": b"v"})
    PU.check_and_migrate("svc", p)
    assert p.get("/FrameworkID") == b"fw"
    assert p.get("/Services/svc/Tasks/t/TaskInfo") == b"ti"
    assert p.get("/Services/svc/ConfigTarget") == b"cfg"
    assert SchemaVersionStore(p).get_or_set_version(SchemaVersion.SINGLE_SERVICE) == SchemaVersion.MULTI_SERVICE
    backups = [c for c in p.get_children("/") if c.startswith("backup-")]
    assert len(backups) == 1 and p.get(f"/{backups[0]}/Tasks/t/TaskInfo") == b"ti"
    with pytest.raises(PersisterException):
        p.get("/Tasks")
