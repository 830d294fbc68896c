"""The application knobs of the shipped cassandra and hdfs packages (``tools.package_knobs``).

Covered: the generated regions of the package files are in sync with the tables; with the package
defaults every knob reaches its config file with the application's default (and a knob whose
default is empty stays out of it); a knob set as a package option reaches the rendered file of
every pod; the option schemas are valid (type matches default)."""
import re
import xml.etree.ElementTree as ET

import pytest
import yaml

from dcos_commons_amd.tools import package_knobs as K

import test_cassandra
import test_hdfs


def test_generated_regions_are_up_to_date():
    for framework in K.PACKAGES:
        for path, content in K.render_files(framework).items():
            with open(path, encoding="utf-8") as f:
                assert f.read() == content, f"{path} is out of date: python -m dcos_commons_amd.tools.package_knobs"


def test_knob_tables_are_consistent():
    py = {"integer": int, "number": (int, float), "boolean": bool, "string": str}
    for knobs in (K.CASSANDRA, K.HDFS_SITE, K.CORE_SITE):
        keys = [k.key for k in knobs]
        assert len(keys) == len(set(keys))
        for k in knobs:
            assert isinstance(k.default, py[k.type]) and not (k.type == "integer" and isinstance(k.default, bool)), k
    settings = [k.setting for k in K.HDFS_SITE + K.CORE_SITE]
    assert len(settings) == len(set(settings))
    assert len(K.CASSANDRA) >= 90 and len(K.HDFS_SITE) + len(K.CORE_SITE) >= 160


def _yaml_value(k):
    return k.default if k.type != "string" else str(k.default)


def test_cassandra_yaml_carries_every_knob_default_and_an_override():
    cfg = yaml.safe_load(test_cassandra.runner().run().get_task_config("node", "server", "cassandra"))
    for k in K.CASSANDRA:
        if K._value(k) == "":
            assert k.setting not in cfg, k.setting            # left to Cassandra's auto-sizing
        else:
            assert cfg[k.setting] == _yaml_value(k), k.setting
    r = test_cassandra.runner().set_options("cassandra.tombstone_warn_threshold", "5",
                                            "cassandra.key_cache_size_in_mb", "64",
                                            "cassandra.commitlog_sync", "batch").run()
    for i in range(3):
        cfg = yaml.safe_load(r.get_task_config("node", "server", "cassandra"))
        assert cfg["tombstone_warn_threshold"] == 5 and cfg["key_cache_size_in_mb"] == 64
        assert cfg["commitlog_sync"] == "batch"


def _props(xml: str) -> dict:
    root = ET.fromstring(xml)
    return {p.findtext("name"): p.findtext("value") for p in root.iter("property")}


@pytest.mark.parametrize("name,knobs", [("hdfs-site", K.HDFS_SITE), ("core-site", K.CORE_SITE)])
def test_hadoop_site_files_carry_every_knob_default(name, knobs):
    r = test_hdfs.runner().run()
    for pod, task in (("journal", "node"), ("name", "node"), ("data", "node")):
        props = _props(r.get_task_config(pod, task, name))
        for k in knobs:
            if K._value(k) == "":
                assert k.setting not in props, k.setting
            else:
                assert props[k.setting] == K._value(k), (pod, k.setting)


def test_hdfs_option_reaches_every_pod():
    r = test_hdfs.runner().set_options("hdfs.blocksize", "268435456",
                                       "hdfs.client_read_shortcircuit_streams_cache_expiry_ms", "1000",
                                       "hdfs.domain_socket_path", "/var/lib/hadoop-hdfs/dn_socket",
                                       "hdfs.fs_trash_interval", "1440").run()
    for pod in ("journal", "name", "data"):
        site = _props(r.get_task_config(pod, "node", "hdfs-site"))
        assert site["dfs.blocksize"] == "268435456"
        assert site["dfs.client.read.shortcircuit.streams.cache.expiry.ms"] == "1000"
        assert site["dfs.domain.socket.path"] == "/var/lib/hadoop-hdfs/dn_socket"
        assert _props(r.get_task_config(pod, "node", "core-site"))["fs.trash.interval"] == "1440"
    # the reference's test_modify_app_config field is a scheduler env var of this package too
    assert r.scheduler_environment["TASKCFG_ALL_CLIENT_READ_SHORTCIRCUIT_STREAMS_CACHE_EXPIRY_MS"] == "1000"


def test_marathon_env_names_are_unique():
    for framework in K.PACKAGES:
        text = K.render_files(framework)[next(p for p in K.render_files(framework) if p.endswith(".mustache"))]
        # an inverted section is the else-branch of the section before it: one of the two renders
        text = re.sub(r"\{\{\^([^}]+)\}\}.*?\{\{/\1\}\}", "", text, flags=re.S)
        names = re.findall(r'^\s*"([A-Z0-9_]+)":', text, re.M)
        dupes = {n for n in names if names.count(n) > 1}
        assert not dupes, (framework, dupes)
