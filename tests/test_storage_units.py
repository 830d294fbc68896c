"""Storage and config-store units: the reference's tree scenarios run against every persister
backend (memory, file, ZooKeeper, and each behind the write-through cache), path helpers, the
cache's behavior when the backing store fails, concurrent writers, and the versioned config store.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/storage/{MemPersisterTest,PersisterCacheTest,
PersisterUtilsTest}.java and state/ConfigStoreTest.java. ``test_storage`` holds the basic
per-backend contract; this suite adds the reference's exact trees and failure cases.
"""
import threading
import uuid

import pytest

from dcos_commons_amd.config.serialization import StringConfiguration
from dcos_commons_amd.state.config_store import ConfigStore, ConfigStoreException
from dcos_commons_amd.storage import persister_utils as PU
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import Persister, PersisterException, Reason
from dcos_commons_amd.storage.persister_cache import PersisterCache
from test_storage import persister, zk_server  # noqa: F401  (shared backend fixtures)

VAL = b"someval"
VAL2 = b"someval2"
TREE = ["/a", "/a/1", "/a/2/a", "/a/3", "/a/3/a/1", "/b", "/c", "/d/1/a/1"]


def _children(p, path):
    """Children of ``path`` under each of its four spellings must agree (MemPersisterTest.checkChildren)."""
    spellings = {path, "/" + path, path + "/", "/" + path + "/"}
    results = {s: sorted(c for c in p.get_children(s) if c != "servicename") for s in spellings}
    assert len({tuple(v) for v in results.values()}) == 1, results
    return results[path]


def _not_found(p, path):
    for s in (path, "/" + path, path + "/", "/" + path + "/"):
        with pytest.raises(PersisterException) as e:
            p.get_children(s)
        assert e.value.reason == Reason.NOT_FOUND


def _fill(p):
    for path in TREE:
        p.set(path, VAL)


def test_missing_root(persister):  # noqa: F811
    assert persister.get("") is None
    assert _children(persister, "") == []


def test_delete_missing(persister):  # noqa: F811
    with pytest.raises(PersisterException):
        persister.recursive_delete("key")


def test_get_children_tree(persister):  # noqa: F811
    _fill(persister)
    _not_found(persister, "notfound")
    assert _children(persister, "") == ["a", "b", "c", "d"]
    assert _children(persister, "a") == ["1", "2", "3"]
    for missing in ("a/notfound", "a/3/notfound", "a/3/a/notfound", "a/3/a/1/notfound"):
        _not_found(persister, missing)
    expected = {"a/1": [], "a/2": ["a"], "a/2/a": [], "a/3": ["a"], "a/3/a": ["1"], "a/3/a/1": [], "b": [],
                "c": [], "d": ["1"], "d/1": ["a"], "d/1/a": ["1"], "d/1/a/1": []}
    for path, kids in expected.items():
        assert _children(persister, path) == kids, path


def test_delete_children(persister):  # noqa: F811
    _fill(persister)
    steps = [("/a/1", "a", ["2", "3"]), ("/a/3/a", "a", ["2", "3"]), ("/b", "", ["a", "c", "d"]),
             ("/c", "", ["a", "d"]), ("/d/1", "", ["a", "d"]), ("/a", "", ["d"]), ("/d", "", [])]
    for delete, parent, kids in steps:
        persister.recursive_delete(delete)
        assert _children(persister, parent) == kids, delete


@pytest.mark.parametrize("root", ["", "/"])
def test_delete_root(persister, root):  # noqa: F811
    _fill(persister)
    persister.recursive_delete(root)
    assert persister.get("") is None
    assert _children(persister, "") == []


def test_recursive_copy(persister):  # noqa: F811
    for path, v in [("x", VAL2), ("x/1", VAL), ("x/lock", VAL2), ("x/2/a", VAL), ("x/3", VAL2),
                    ("x/3/a/1", VAL), ("y", VAL2), ("z", VAL), ("w/1/a/1", VAL2)]:
        persister.set(path, v)
    persister.recursive_copy("/x", "/p")
    assert sorted(persister.get_children("/p")) == ["1", "2", "3", "lock"]
    assert list(persister.get_children("/p/1")) == [] and list(persister.get_children("/p/lock")) == []
    assert list(persister.get_children("/p/2")) == ["a"] and list(persister.get_children("/p/3")) == ["a"]
    assert list(persister.get_children("/p/3/a")) == ["1"]
    assert [persister.get(k) for k in ("p", "p/1", "p/lock", "p/2/a", "p/3", "p/3/a/1")] == \
        [VAL2, VAL, VAL2, VAL, VAL2, VAL]
    assert persister.get("x/3/a/1") == VAL  # the source is untouched


@pytest.mark.parametrize("setup,src,dst", [
    ({"x": VAL2, "y": VAL}, "/x", "/y"),   # target exists
    ({"y": VAL}, "/x", "/y"),              # source missing
    ({}, "/x", "/x"),                      # source == destination
])
def test_recursive_copy_failures(persister, setup, src, dst):  # noqa: F811
    for k, v in setup.items():
        persister.set(k, v)
    with pytest.raises((PersisterException, ValueError)):
        persister.recursive_copy(src, dst)


def test_set_get_delete_keys(persister):  # noqa: F811
    persister.set("key", VAL)
    assert persister.get("key") == VAL and PU.get_all_keys(persister) == ["/key"]
    persister.set("key2", VAL2)
    assert PU.get_all_keys(persister) == ["/key", "/key2"]
    persister.recursive_delete("key")
    with pytest.raises(PersisterException):
        persister.get("key")
    assert PU.get_all_keys(persister) == ["/key2"]
    persister.recursive_delete("key2")
    assert PU.get_all_keys(persister) == []


def test_set_many_get_many_delete_many(persister):  # noqa: F811
    assert persister.get_many(["key", "key2"]) == {"key": None, "key2": None}
    persister.set_many({"key": VAL})
    assert persister.get_many(["key", "key2"]) == {"key": VAL, "key2": None}
    persister.set_many({"key": VAL2, "key2": VAL2})
    assert persister.get_many(["key", "key2"]) == {"key": VAL2, "key2": VAL2}
    persister.recursive_delete_many(["key", "key2"])
    assert persister.get_many(["key", "key2"]) == {"key": None, "key2": None}
    assert PU.get_all_keys(persister) == []


def test_concurrent_set_get_delete(persister):  # noqa: F811
    errors = []

    def worker(i):
        key = f"key-{i}"
        try:
            for _ in range(20):
                persister.set(key, VAL)
                assert persister.get(key) == VAL
                persister.set(key, VAL2)
                assert persister.get(key) == VAL2
                persister.set_many({key: VAL})
                assert persister.get_many([key])[key] == VAL
                persister.recursive_delete(key)
                with pytest.raises(PersisterException):
                    persister.get(key)
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert errors == []


# ---------------------------------------------------------------------------------------
# PersisterUtils


@pytest.mark.parametrize("a,b,joined", [
    ("test", "path", "test/path"), ("test", "/path", "test/path"), ("test/", "path", "test/path"),
    ("test/", "/path", "test/path"), ("test//", "/path", "test//path"), ("test/", "//path", "test//path"),
    ("/test", "path", "/test/path"), ("/test", "/path", "/test/path"), ("/test/", "path", "/test/path"),
    ("/test/", "/path", "/test/path"), ("/test//", "/path", "/test//path"), ("/test/", "//path", "/test//path"),
])
def test_join_paths(a, b, joined):
    assert PU.join_paths(a, b) == joined


@pytest.mark.parametrize("path,parents", [
    ("", []), ("test", []), ("test/", []), ("test/path", ["test"]),
    ("test/path/foo", ["test", "test/path"]),
    ("test/path/foo/bar/baz", ["test", "test/path", "test/path/foo", "test/path/foo/bar"]),
    ("/", []), ("//", []), ("/test", []), ("/test/", []), ("/test/path", ["/test"]),
    ("/test/path/foo/bar/baz", ["/test", "/test/path", "/test/path/foo", "/test/path/foo/bar"]),
])
def test_parent_paths(path, parents):
    assert PU.get_parent_paths(path) == parents


def test_all_keys_and_data():
    p = MemPersister()
    p.set_many({k: b"" for k in TREE})
    assert PU.get_all_keys(p) == sorted(["/a", "/a/1", "/a/2", "/a/2/a", "/a/3", "/a/3/a", "/a/3/a/1", "/b", "/c",
                                         "/d", "/d/1", "/d/1/a", "/d/1/a/1"])
    assert PU.get_all_data(p) == {k: b"" for k in TREE}


# ---------------------------------------------------------------------------------------
# PersisterCache over a failing backend


def test_cache_loads_existing_data():
    backing = MemPersister()
    data = {"ConfigTarget": VAL, "Configurations/abad-coffee": VAL2, "FrameworkID": VAL,
            "Properties/suppressed": VAL2, "SchemaVersion": VAL}
    for n in range(3):
        data[f"Tasks/node-{n}/TaskInfo"] = VAL2
        data[f"Tasks/node-{n}/TaskStatus"] = VAL
    backing.set_many(data)
    cache = PersisterCache(backing)
    assert PU.get_all_data(cache) == {"/" + k: v for k, v in data.items()}
    assert "/Tasks/node-1" in PU.get_all_keys(cache) and "/Properties" in PU.get_all_keys(cache)


class FailingPersister(Persister):
    """A backend that holds nothing (so deletes of missing keys succeed silently, like the
    reference's mock) and fails the configured operations."""

    def __init__(self, fail_set=(), fail_set_many=False, fail_delete=()):
        self.fail_set, self.fail_set_many, self.fail_delete = set(fail_set), fail_set_many, set(fail_delete)

    def _fail(self):
        raise PersisterException(Reason.STORAGE_ERROR, "hi")

    def get(self, path):
        self._fail()

    def get_children(self, path):
        return []

    def get_many(self, paths):
        return {p: None for p in paths}

    def set(self, path, data):
        if path in self.fail_set:
            self._fail()

    def set_many(self, path_bytes):
        if self.fail_set_many:
            self._fail()

    def recursive_copy(self, src, dst):
        pass

    def recursive_delete(self, path):
        if path in self.fail_delete:
            self._fail()

    def recursive_delete_many(self, paths):
        for p in paths:
            self.recursive_delete(p)

    def close(self):
        pass


def test_cache_unchanged_when_set_fails():
    cache = PersisterCache(FailingPersister(fail_set={"key2"}))
    cache.set("key", VAL)
    with pytest.raises(PersisterException):
        cache.set("key2", VAL2)
    assert PU.get_all_keys(cache) == ["/key"] and cache.get("key") == VAL
    with pytest.raises(PersisterException):
        cache.get("key2")


def test_cache_unchanged_when_set_many_fails():
    cache = PersisterCache(FailingPersister(fail_set_many=True))
    with pytest.raises(PersisterException):
        cache.set_many({"key": VAL, "key2": VAL2})
    assert PU.get_all_keys(cache) == []


def test_cache_unchanged_when_delete_fails():
    cache = PersisterCache(FailingPersister(fail_delete={"key2"}))
    cache.set("key", VAL)
    cache.set("key2", VAL2)
    cache.recursive_delete("key")
    with pytest.raises(PersisterException):
        cache.recursive_delete("key2")
    assert PU.get_all_keys(cache) == ["/key2"] and cache.get("key2") == VAL2


def test_cache_tolerates_a_backend_that_deletes_missing_keys():
    cache = PersisterCache(FailingPersister())
    cache.set("key", VAL)
    cache.recursive_delete("key")
    cache.recursive_delete("key")  # logged, not raised


def test_cache_close_empties_it():
    backing = MemPersister()
    cache = PersisterCache(backing)
    cache.set("key", VAL)
    cache.close()
    assert PU.get_all_keys(backing) == []
    with pytest.raises(PersisterException):
        cache.get("key")


def test_cache_refresh_picks_up_out_of_band_writes():
    backing = MemPersister()
    cache = PersisterCache(backing)
    cache.set("key", VAL)
    backing.set("key", VAL2)
    assert cache.get("key") == VAL  # served from the mirror
    cache.refresh()
    assert cache.get("key") == VAL2


# ---------------------------------------------------------------------------------------
# ConfigStore


NAMESPACE = "test-namespace"
CONFIG = StringConfiguration("test-config")


@pytest.fixture
def config_store():
    p = MemPersister()
    return ConfigStore(StringConfiguration.Factory(), p), p


def _absent(p, path):
    with pytest.raises(PersisterException) as e:
        p.get(path)
    assert e.value.reason == Reason.NOT_FOUND


@pytest.mark.parametrize("namespace", [None, NAMESPACE])
def test_config_store_path_mapping(namespace):
    p = MemPersister()
    store = ConfigStore(StringConfiguration.Factory(), p, namespace)
    cid = store.store(CONFIG)
    store.set_target_config(cid)
    here, there = ("", f"Services/{NAMESPACE}/") if namespace is None else (f"Services/{NAMESPACE}/", "")
    assert p.get(here + "ConfigTarget") == str(cid).encode()
    assert len(p.get(f"{here}Configurations/{cid}")) > 0
    _absent(p, there + "ConfigTarget")
    _absent(p, f"{there}Configurations/{cid}")
    assert store.get_target_config() == cid
    # a fresh store (no in-process cache) reads the same config back
    assert ConfigStore(StringConfiguration.Factory(), p, namespace).fetch(cid) == CONFIG


def test_config_store_fetch_repeat_clear(config_store):
    store, _ = config_store
    cid = store.store(CONFIG)
    assert store.fetch(cid) == CONFIG
    store.store(CONFIG)
    store.clear(cid)
    with pytest.raises(ConfigStoreException) as e:
        store.fetch(cid)
    assert e.value.reason == Reason.NOT_FOUND
    store.clear(uuid.uuid4())  # clearing an unknown id is a no-op


def test_config_store_list_and_keys(config_store):
    store, _ = config_store
    ids = [store.store(CONFIG) for _ in range(3)]
    assert sorted(store.list()) == sorted(ids)
    assert store.has_key(ids[0]) and not store.has_key(uuid.uuid4())


def test_config_store_target(config_store):
    store, _ = config_store
    with pytest.raises(ConfigStoreException) as e:
        store.get_target_config()
    assert e.value.reason == Reason.NOT_FOUND
    cid = store.store(CONFIG)
    store.set_target_config(cid)
    store.set_target_config(cid)
    assert store.get_target_config() == cid


def test_config_store_rejects_foreign_children(config_store):
    store, p = config_store
    p.set("Configurations/not-a-uuid", b"x")
    with pytest.raises(ConfigStoreException) as e:
        store.list()
    assert e.value.reason == Reason.SERIALIZATION_ERROR
