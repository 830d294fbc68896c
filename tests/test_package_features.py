"""Every shipped cassandra and hdfs config template, rendered with the optional features on:
TLS (transport encryption), Kerberos, metrics reporting, the G1 collector, secure JMX.

The harness renders every config file of every task of pod 0 strictly (a value the task
environment lacks fails the run), so each case below also proves the templates it turns on
render; the assertions check what the application will read."""
import os
import subprocess
import xml.etree.ElementTree as ET

import pytest

from dcos_commons_amd.testing import ServiceTestRunner
from dcos_commons_amd.testing.cosmos import render_marathon_app

import test_cassandra
import test_hdfs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CRED = '{"uid": "svc", "private_key": "k"}'


def _props(xml: str) -> dict:
    return {p.findtext("name"): p.findtext("value") for p in ET.fromstring(xml).iter("property")}


# -- cassandra -----------------------------------------------------------------------------------
def test_cassandra_defaults_render_cms_metrics_and_cqlsh():
    r = test_cassandra.runner().run()
    jvm = r.get_task_config("node", "server", "jvm")
    assert "-XX:+UseConcMarkSweepGC" in jvm and "-Xmx" in jvm and "-Xmn" in jvm and "PrintGCDetails" not in jvm
    metrics = r.get_task_config("node", "server", "metrics-reporter")
    assert "statsd:" in metrics and "port: 99999" in metrics        # the task's STATSD_UDP_PORT
    cqlshrc = r.get_task_config("node", "server", "cqlshrc")
    assert "port = 9042" in cqlshrc and "[ssl]" not in cqlshrc
    server = r.service_spec.pod("node").task("server")
    assert "metricsReporterConfigFile" in server.command.value and "jmx-ssl-setup" not in server.command.value
    assert not r.service_spec.pod("node").secrets


def test_cassandra_g1_with_gc_logging():
    r = test_cassandra.runner().set_options("nodes.heap.gc", "G1", "nodes.heap.gc_logging", "true",
                                            "nodes.heap.g1_max_pause_ms", "300").run()
    jvm = r.get_task_config("node", "server", "jvm")
    assert "-XX:+UseG1GC" in jvm and "-XX:MaxGCPauseMillis=300" in jvm and "ConcMarkSweep" not in jvm
    assert "-Xmn" not in jvm and "-Xloggc:" in jvm
    jvm_spec = next(c for c in r.service_spec.pod("node").task("server").config_files if c.name == "jvm")
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "frameworks", "cassandra",
                           "specs", "jvm_G1.options"), encoding="utf-8") as f:
        assert jvm_spec.template_content == f.read()


def test_cassandra_tls_cqlsh_and_metrics_off():
    r = (test_cassandra.runner().set_options("service.security.transport_encryption.enabled", "true",
                                             "cassandra.metrics_enabled", "false")
         .set_scheduler_env(DCOS_SERVICE_ACCOUNT_CREDENTIAL=CRED).run())
    cqlshrc = r.get_task_config("node", "server", "cqlshrc")
    assert "[ssl]" in cqlshrc and "node.ca" in cqlshrc and "ssl_transport_factory" in cqlshrc
    assert "metricsReporterConfigFile" not in r.service_spec.pod("node").task("server").command.value


def test_cassandra_access_control_defaults():
    """Without service.security.authentication/authorization the nodes run AllowAll*; the cache and
    back-pressure settings carry the package defaults (reference cassandra config.json)."""
    import yaml
    cfg = yaml.safe_load(test_cassandra.runner().run().get_task_config("node", "server", "cassandra"))
    assert cfg["authenticator"] == "AllowAllAuthenticator" and cfg["authorizer"] == "AllowAllAuthorizer"
    assert cfg["role_manager"] == "CassandraRoleManager" and cfg["permissions_cache_max_entries"] == 1000
    for name in ("roles", "credentials", "permissions"):
        assert cfg[f"{name}_validity_in_ms"] == 2000 and cfg[f"{name}_update_interval_in_ms"] == 2000
    assert cfg["seed_provider"][0]["class_name"] == "org.apache.cassandra.locator.SimpleSeedProvider"
    (bp,) = cfg["back_pressure_strategy"]
    assert bp["class_name"].endswith("RateBasedBackPressure")
    assert bp["parameters"] == [{"high_ratio": 0.9, "factor": 5, "flow": "FAST"}]
    assert cfg["start_native_transport"] is True and "commitlog_sync_batch_window_in_ms" not in cfg


def test_cassandra_authentication_and_authorization(tmp_path):
    """PasswordAuthenticator + CassandraAuthorizer with a superuser password secret: the secret is
    mounted in the node pod (merged with the secure JMX secrets when both are on), and the init
    step replaces the default login by the configured superuser before altering system_auth."""
    import base64
    import yaml
    custom = base64.b64encode(b"auth_read_consistency_level: LOCAL_QUORUM").decode()
    r = (test_cassandra.runner().set_options(
        "service.security.authentication.enabled", "true",
        "service.security.authentication.superuser.name", "admin",
        "service.security.authentication.superuser.password_secret_path", "cassandra/su-pw",
        "service.security.authentication.authentication_custom_cassandra_yml", custom,
        "service.security.authorization.enabled", "true",
        "service.security.authorization.permissions_validity_in_ms", "0",
        "service.jmx.enabled", "true", "service.jmx.password_file", "c/jmx-pw", "service.jmx.access_file", "c/acc",
        "service.jmx.key_store", "c/ks", "service.jmx.key_store_password_file", "c/ks-pw",
        "service.rlimits.rlimit_nofile.soft", "200000", "service.rlimits.rlimit_nofile.hard", "300000",
        "cassandra.back_pressure_flow", "SLOW").run())
    cfg = yaml.safe_load(r.get_task_config("node", "server", "cassandra"))
    assert cfg["authenticator"] == "PasswordAuthenticator" and cfg["authorizer"] == "CassandraAuthorizer"
    assert cfg["permissions_validity_in_ms"] == 0
    assert cfg["back_pressure_strategy"][0]["parameters"][0]["flow"] == "SLOW"
    pod = r.service_spec.pod("node")
    files = sorted(s.file_path for s in pod.secrets)
    assert files == ["jmx/access_file", "jmx/key_store", "jmx/key_store_password_file", "jmx/password_file",
                     "superuser/password"]
    assert next(s for s in pod.secrets if s.file_path == "superuser/password").secret_path == "cassandra/su-pw"
    (rl,) = pod.rlimits
    assert (rl.soft, rl.hard) == (200000, 300000)
    # the init step's script, with a stub cqlsh that logs its arguments
    init = pod.task("init_system_keyspaces").command.value
    sandbox = tmp_path / "sb"
    (sandbox / "apache-cassandra-3.11.6" / "bin").mkdir(parents=True)
    (sandbox / "superuser").mkdir()
    (sandbox / "superuser" / "password").write_text("s3cret")
    log = sandbox / "cqlsh.log"
    stub = sandbox / "apache-cassandra-3.11.6" / "bin" / "cqlsh"
    stub.write_text(f'#!/bin/bash\necho "$*" >> {log}\ncase "$*" in *"CREATE ROLE"*) touch {sandbox}/created;; esac\n'
                    f'[ "$2" != admin ] || [ -f {sandbox}/created ]\n')     # admin logs in once created
    stub.chmod(0o755)
    script = init.replace("{{CASSANDRA_VERSION}}", "3.11.6")
    env = dict(os.environ, CASSANDRA_AUTHENTICATOR="PasswordAuthenticator", SUPERUSER_NAME="admin",
               FRAMEWORK_HOST="cassandra.autoip", CASSANDRA_NATIVE_TRANSPORT_PORT="9042",
               CASSANDRA_LOCATION_DATA_CENTER="dc1")
    for _ in range(2):     # a rerun finds the superuser and does not recreate it
        subprocess.run(["bash", "-c", script], cwd=sandbox, env=env, check=True)
    lines = log.read_text().splitlines()
    creates = [l for l in lines if "CREATE ROLE" in l]
    assert len(creates) == 1 and creates[0].startswith("-u cassandra -p cassandra") and "'s3cret'" in creates[0]
    assert any("ALTER ROLE cassandra" in l and "SUPERUSER = false" in l for l in lines)
    alters = [l for l in lines if "ALTER KEYSPACE system_auth" in l]
    assert len(alters) == 2 and all(l.startswith("-u admin -p s3cret") for l in alters)
    # the schema backup logs in the same way
    (sandbox / "container-path" / "snapshot").mkdir(parents=True)
    backup = pod.task("backup-schema").command.value.replace("{{CASSANDRA_VERSION}}", "3.11.6")
    subprocess.run(["bash", "-c", backup], cwd=sandbox, env=dict(env, POD_INSTANCE_INDEX="0"), check=True)
    assert log.read_text().splitlines()[-1].startswith("-u admin -p s3cret -e DESC SCHEMA")


def test_cassandra_marathon_health_check_rlimits_and_profile():
    app = render_marathon_app(os.path.join(ROOT, "frameworks", "cassandra", "universe"), {})
    (hc,) = app["healthChecks"]
    assert (hc["intervalSeconds"], hc["timeoutSeconds"], hc["delaySeconds"]) == (30, 20, 15)
    env = app["env"]
    assert env["RLIMIT_NOFILE_SOFT"] == env["RLIMIT_NOFILE_HARD"] == "128000"
    assert "CASSANDRA_VOLUME_PROFILE" not in env and "NODE_POD_SECRETS" not in env
    assert env["TASKCFG_ALL_CASSANDRA_AUTHENTICATOR"] == "AllowAllAuthenticator"
    app = render_marathon_app(os.path.join(ROOT, "frameworks", "cassandra", "universe"),
                              {"nodes.volume_profile": "xfs", "service.security.authentication.enabled": "true",
                               "service.security.authentication.superuser.password_secret_path": "c/pw",
                               "service.security.authentication.authentication_custom_cassandra_yml": "YTogYg=="})
    env = app["env"]
    assert env["CASSANDRA_VOLUME_PROFILE"] == "xfs" and env["NODE_POD_SECRETS"] == "yes"
    assert env["TASKCFG_ALL_CASSANDRA_AUTHENTICATOR"] == "PasswordAuthenticator"
    assert env["SUPERUSER_PASSWORD_SECRET"] == "c/pw"
    # decoded by the scheduler into every node's cassandra.yaml (models/cassandra.py)
    assert env["TASKCFG_ALL_AUTHENTICATION_CUSTOM_YAML_BLOCK_BASE64"] == "YTogYg=="


def test_cassandra_secure_jmx(tmp_path):
    r = (test_cassandra.runner()
         .set_options("service.jmx.enabled", "true", "service.jmx.password_file", "cassandra/jmx-pw",
                      "service.jmx.access_file", "cassandra/jmx-access", "service.jmx.key_store", "cassandra/ks",
                      "service.jmx.key_store_password_file", "cassandra/ks-pw",
                      "service.jmx.add_trust_store", "true", "service.jmx.trust_store", "cassandra/ts",
                      "service.jmx.trust_store_password_file", "cassandra/ts-pw").run())
    pod = r.service_spec.pod("node")
    files = sorted(s.file_path for s in pod.secrets)
    assert files == ["jmx/access_file", "jmx/key_store", "jmx/key_store_password_file", "jmx/password_file",
                     "jmx/trust_store", "jmx/trust_store_password_file"]
    server = pod.task("server")
    assert "bash ./jmx-ssl-setup.sh" in server.command.value and "LOCAL_JMX=no" in server.command.value
    ports = {p.port_name: p for p in server.resource_set.resources if getattr(p, "port_name", "")}
    assert "jmx-rmi" in ports and "7198" in str(ports["jmx-rmi"].value)
    # the rendered setup script, run in a sandbox holding the secrets, writes the JVM flags
    script = r.get_task_config("node", "server", "jmx-ssl-setup")
    sandbox = tmp_path / "sandbox"
    (sandbox / "jmx").mkdir(parents=True)
    for name, text in (("password_file", "admin secret\n"), ("access_file", "admin readwrite\n"),
                       ("key_store", "KS"), ("key_store_password_file", "kspass\n"), ("trust_store", "TS"),
                       ("trust_store_password_file", "tspass\n")):
        (sandbox / "jmx" / name).write_text(text)
    (sandbox / "jmx-ssl-setup.sh").write_text(script)
    p = subprocess.run(["bash", "jmx-ssl-setup.sh"], cwd=sandbox, env=dict(os.environ, MESOS_SANDBOX=str(sandbox)),
                       capture_output=True, text=True, timeout=30)
    assert p.returncode == 0, p.stderr
    opts = (sandbox / "jmx.options").read_text()
    assert "-Dcom.sun.management.jmxremote.port=7199" in opts and "rmi.port=7198" in opts
    assert "keyStorePassword=kspass" in opts and "trustStorePassword=tspass" in opts
    assert oct((sandbox / "jmx" / "password_file").stat().st_mode & 0o777) == "0o400"
    # a missing secret stops the task before Cassandra starts
    (sandbox / "jmx" / "access_file").unlink()
    assert subprocess.run(["bash", "jmx-ssl-setup.sh"], cwd=sandbox, env=dict(os.environ, MESOS_SANDBOX=str(sandbox)),
                          capture_output=True, text=True, timeout=30).returncode == 1


# -- hdfs ----------------------------------------------------------------------------------------
def _hdfs(**options):
    r = test_hdfs.runner()
    flat = [x for kv in options.items() for x in kv]
    return r.set_options(*flat).set_scheduler_env(DCOS_SERVICE_ACCOUNT_CREDENTIAL=CRED).run()


def test_hdfs_metrics2_per_role():
    r = test_hdfs.runner().run()
    for pod, prefix in (("journal", "journalnode"), ("name", "namenode"), ("data", "datanode")):
        m = r.get_task_config(pod, "node", "hadoop-metrics2")
        assert f"{prefix}.sink.statsd.class=org.apache.hadoop.metrics2.sink.StatsDSink" in m
        assert f"{prefix}.sink.statsd.server.port=99999" in m and f"service.name={pod}-0" in m
    off = test_hdfs.runner().set_options("hdfs.metrics_enabled", "false").run()
    assert "sink.statsd" not in off.get_task_config("data", "node", "hadoop-metrics2")


def test_hdfs_https_with_tls():
    r = _hdfs(**{"service.security.transport_encryption.enabled": "true",
                 "service.security.transport_encryption.excluded_ciphers": "TLS_RSA_WITH_RC4_128_MD5"})
    for pod in ("journal", "name", "data"):
        site = _props(r.get_task_config(pod, "node", "hdfs-site"))
        assert site["dfs.http.policy"] == "HTTPS_ONLY"
        assert site["dfs.https.server.keystore.resource"] == "ssl-server.xml"
        server = _props(r.get_task_config(pod, "node", "ssl-server"))
        assert server["ssl.server.keystore.location"].endswith("/node.keystore")
        assert server["ssl.server.exclude.cipher.list"] == "TLS_RSA_WITH_RC4_128_MD5"
        client = _props(r.get_task_config(pod, "node", "ssl-client"))
        assert client["ssl.client.truststore.location"].endswith("/node.truststore")
    names = {c.name for c in r.service_spec.pod("name").task("zkfc").config_files}
    assert "ssl-client" in names and "ssl-server" not in names


def test_hdfs_node_type_options():
    """Per node type: rlimits, volume profile, placement, readiness checks (reference hdfs
    config.json journal_node / name_node / data_node sections)."""
    r = _hdfs(**{"journal_node.rlimits.rlimit_nofile.soft": "200000", "journal_node.rlimits.rlimit_nofile.hard": "200000",
                 "name_node.rlimits.rlimit_nofile.hard": "300000",
                 "data_node.volume_profile": "xfs", "data_node.disk_type": "MOUNT",
                 "name_node.placement": '[["hostname", "UNIQUE"]]',
                 "journal_node.readiness_check.interval": "7", "journal_node.lagging_tx_count": "5",
                 "name_node.readiness_check.timeout": "99"})
    spec = r.service_spec
    assert spec.pod("journal").rlimits[0].soft == 200000 and spec.pod("name").rlimits[0].hard == 300000
    assert spec.pod("data").rlimits[0].soft == 128000
    assert "xfs" in repr(spec.pod("data").task("node").resource_set)
    assert "MaxPerHostname" in repr(spec.pod("name").placement_rule)     # hostname:UNIQUE
    jrc = spec.pod("journal").task("node").readiness_check
    assert jrc.interval == 7 and "CurrentLagTxns" in jrc.command and "-le 5" in jrc.command
    assert spec.pod("name").task("node").readiness_check.timeout == 99
    r = _hdfs(**{"journal_node.enable_readiness_check": "false"})
    assert r.service_spec.pod("journal").task("node").readiness_check is None


def test_hdfs_journal_readiness_check_script(tmp_path):
    """The JournalNode readiness check passes on a first deployment (no journal yet) and then only
    while the journal's CurrentLagTxns metric is within journal_node.lagging_tx_count."""
    cmd = _hdfs(**{"journal_node.lagging_tx_count": "5"}).service_spec.pod("journal").task("node").readiness_check.command
    (tmp_path / "bin").mkdir()
    curl = tmp_path / "bin" / "curl"
    env = dict(os.environ, PATH=f"{tmp_path / 'bin'}:{os.environ['PATH']}", MESOS_CONTAINER_IP="127.0.0.1")

    def check(lag):
        curl.write_text('#!/bin/bash\necho \'{"beans" : [ {"name" : "Hadoop:service=JournalNode,name=Journal-hdfs",'
                        f'\n "CurrentLagTxns" : {lag}, "LastWrittenTxId" : 42 }} ] }}\'\n')
        curl.chmod(0o755)
        return subprocess.run(["bash", "-c", cmd], cwd=tmp_path, env=env).returncode == 0

    assert check(100)                              # no journal-data/hdfs: first deployment
    (tmp_path / "journal-data" / "hdfs").mkdir(parents=True)
    assert check(3) and check(5) and not check(6)


def test_hdfs_security_and_plaintext_options():
    r = _hdfs(**{"service.security.transport_encryption.enabled": "true",
                 "service.security.transport_encryption.allow_plaintext": "true",
                 "hdfs.block_access_token_enable": "true", "hdfs.security_authorization": "false",
                 "name_node.handler_count": "40", "hdfs.ha_fencing_methods": "shell(/bin/false)"})
    site = _props(r.get_task_config("name", "node", "hdfs-site"))
    assert site["dfs.http.policy"] == "HTTP_AND_HTTPS" and site["dfs.block.access.token.enable"] == "true"
    assert site["dfs.namenode.handler.count"] == "40" and site["dfs.ha.fencing.methods"] == "shell(/bin/false)"
    assert _props(r.get_task_config("name", "node", "core-site"))["hadoop.security.authorization"] == "false"
    # defaults: plaintext HTTP off, authorization on, tokens off
    r = _hdfs()
    site = _props(r.get_task_config("data", "node", "hdfs-site"))
    assert site["dfs.block.access.token.enable"] == "false" and site["dfs.namenode.handler.count"] == "10"
    assert _props(r.get_task_config("data", "node", "core-site"))["hadoop.security.authorization"] == "true"


def test_hdfs_site_files_have_no_duplicate_properties():
    for opts in ({}, {"service.security.transport_encryption.enabled": "true"}):
        r = _hdfs(**opts)
        for pod in ("journal", "name", "data"):
            for name in ("hdfs-site", "core-site"):
                names = [p.findtext("name") for p in ET.fromstring(r.get_task_config(pod, "node", name)).iter("property")]
                assert len(names) == len(set(names)), (pod, name, {n for n in names if names.count(n) > 1})


def test_hdfs_marathon_env_and_health_check():
    app = render_marathon_app(os.path.join(ROOT, "frameworks", "hdfs", "universe"),
                              {"name_node.hadoop_namenode_opts": "-XX:+UseG1GC", "hdfs.hadoop_heapsize": "2048",
                               "service.security.custom_domain": "example.tld"})
    (hc,) = app["healthChecks"]
    assert (hc["intervalSeconds"], hc["timeoutSeconds"], hc["delaySeconds"]) == (30, 20, 15)
    env = app["env"]
    assert env["TASKCFG_ALL_HADOOP_NAMENODE_OPTS"] == "-XX:+UseG1GC" and env["TASKCFG_ALL_HADOOP_HEAPSIZE"] == "2048"
    assert env["TASKCFG_ALL_HADOOP_ROOT_LOGGER"] == "INFO,console" and env["SERVICE_TLD"] == "example.tld"
    assert env["JOURNAL_READINESS_CHECK_ENABLED"] == "true" and env["NAME_NODE_READINESS_CHECK_TIMEOUT"] == "180"
    # reference option paths of renamed knobs, with the reference package's defaults
    assert env["TASKCFG_ALL_NAME_NODE_HEARTBEAT_RECHECK_INTERVAL"] == "60000"
    assert env["TASKCFG_ALL_CLIENT_READ_SHORTCIRCUIT_STREAMS_CACHE_EXPIRY_MS"]


@pytest.mark.skipif(not os.path.isdir("/root/reference/frameworks"), reason="no reference tree")
@pytest.mark.parametrize("framework", ["helloworld", "cassandra", "hdfs"])
def test_every_reference_option_path_exists(framework):
    """An options file written for the reference package installs unchanged: every leaf option of
    its universe/config.json is a leaf of ours (the debug.* JVM-debugger options of the reference
    helloworld scheduler have no counterpart: the scheduler is not a JVM)."""
    import json

    def leaves(d, p=""):
        out = {}
        for k, v in d.get("properties", {}).items():
            out.update(leaves(v, p + k + ".") if v.get("type") == "object" and "properties" in v else {p + k: v})
        return out

    with open(f"/root/reference/frameworks/{framework}/universe/config.json", encoding="utf-8") as f:
        ref = leaves(json.load(f))
    with open(os.path.join(ROOT, "frameworks", framework, "universe", "config.json"), encoding="utf-8") as f:
        ours = leaves(json.load(f))
    missing = sorted(k for k in ref if k not in ours and not k.startswith("debug."))
    assert not missing, missing


def test_hdfs_kerberos_krb5_conf_and_jvm_flag():
    r = _hdfs(**{"service.security.kerberos.enabled": "true", "service.security.kerberos.realm": "EXAMPLE.COM",
                 "service.security.kerberos.kdc.hostname": "kdc.example.com",
                 "service.security.kerberos.kdc.port": "88"})
    krb5 = r.get_task_config("name", "node", "krb5")
    assert "default_realm = EXAMPLE.COM" in krb5 and "kdc = kdc.example.com:88" in krb5
    assert "udp_preference_limit = 1" in krb5
    for pod in ("journal", "name", "data"):
        cmd = r.service_spec.pod(pod).task("node").command.value
        assert "-Djava.security.krb5.conf=" in cmd and "./keytab-fix" in cmd
        assert "hadoop.security.authentication" in r.get_task_config(pod, "node", "core-site")
    assert {c.name for c in r.service_spec.pod("name").task("format").config_files} >= {"krb5"}


def test_hdfs_everything_on():
    """TLS, Kerberos and metrics together: every template of every pod renders."""
    r = _hdfs(**{"service.security.transport_encryption.enabled": "true",
                 "service.security.kerberos.enabled": "true", "hdfs.metrics_enabled": "true"})
    for pod in ("journal", "name", "data"):
        names = {c.name for c in r.service_spec.pod(pod).task("node").config_files}
        assert names == {"core-site", "hdfs-site", "hadoop-metrics2", "ssl-server", "ssl-client", "krb5"}
        for name in names:
            assert r.get_task_config(pod, "node", name)


def test_cassandra_everything_on():
    """TLS, password authentication with authorization, secure JMX, G1 and metrics together: every
    template of the node pod renders and the pod's secrets are merged under one ``secrets`` key."""
    import yaml
    r = (test_cassandra.runner().set_options(
        "service.security.transport_encryption.enabled", "true",
        "service.security.authentication.enabled", "true",
        "service.security.authentication.superuser.password_secret_path", "c/su",
        "service.security.authorization.enabled", "true",
        "service.jmx.enabled", "true", "service.jmx.password_file", "c/pw", "service.jmx.access_file", "c/acc",
        "service.jmx.key_store", "c/ks", "service.jmx.key_store_password_file", "c/ksp",
        "nodes.heap.gc", "G1", "cassandra.metrics_enabled", "true")
        .set_scheduler_env(DCOS_SERVICE_ACCOUNT_CREDENTIAL=CRED).run())
    task = r.service_spec.pod("node").task("server")
    names = {c.name for c in task.config_files}
    assert names == {"cassandra", "rackdc", "jvm", "metrics-reporter", "cqlshrc", "jmx-ssl-setup"}
    for name in names:
        assert r.get_task_config("node", "server", name)
    cfg = yaml.safe_load(r.get_task_config("node", "server", "cassandra"))
    assert cfg["client_encryption_options"]["enabled"] is True and cfg["authorizer"] == "CassandraAuthorizer"
    assert len(r.service_spec.pod("node").secrets) == 5 and [t.name for t in task.transport_encryption] == ["node"]


# -- helloworld ----------------------------------------------------------------------------------
def _hello(spec="svc.yml"):
    return ServiceTestRunner.for_framework("helloworld", spec).set_scheduler_env(SDK_REVIVE_INTERVAL_S="0")


def test_helloworld_rlimits_and_labels():
    """hello.rlimits / world.rlimits (default 128000 open files, like the reference package) and
    hello.labels reach the pods and the hello task."""
    r = _hello().run()
    for pod in ("hello", "world"):
        (rl,) = r.service_spec.pod(pod).rlimits
        assert (rl.name, rl.soft, rl.hard) == ("RLIMIT_NOFILE", 128000, 128000)
    assert not r.service_spec.pod("hello").task("server").labels
    r = _hello().set_options("hello.labels", "team:infra,tier:gold",
                             "world.rlimits.rlimit_nofile.soft", "4096").run()
    assert r.service_spec.pod("hello").task("server").labels == {"team": "infra", "tier": "gold"}
    assert r.service_spec.pod("world").rlimits[0].soft == 4096


def test_helloworld_scenario_options():
    """port_one (multiport), seccomp-* (seccomp), volume_profile (profile-mount-volume)."""
    r = _hello("multiport.yml").set_options("hello.port_one", "4321").run()
    ports = {p.port_name: p for p in r.service_spec.pod("multiport").task("server").resource_set.resources
             if getattr(p, "port_name", "")}
    assert "4321" in str(ports["static"].value)
    pod = _hello("seccomp.yml").run().service_spec.pod("hello")
    assert not pod.seccomp_unconfined and pod.seccomp_profile_name is None
    pod = _hello("seccomp.yml").set_options("hello.seccomp-unconfined", "true").run().service_spec.pod("hello")
    assert pod.seccomp_unconfined
    pod = _hello("seccomp.yml").set_options("hello.seccomp-profile-name", "default.json").run().service_spec.pod("hello")
    assert not pod.seccomp_unconfined and pod.seccomp_profile_name == "default.json"
    for profile, expect in (("", "fast-nvme"), ("xfs", "xfs")):
        r = _hello("profile-mount-volume.yml").set_options("hello.volume_profile", profile).run()
        text = repr(r.service_spec.pod("hello").to_dict() if hasattr(r.service_spec.pod("hello"), "to_dict")
                    else r.service_spec.pod("hello"))
        assert expect in text


def test_helloworld_marathon_health_check_and_env():
    app = render_marathon_app(os.path.join(ROOT, "frameworks", "helloworld", "universe"),
                              {"service.check.intervalSeconds": "30", "service.verbose_mesos_logging": "0"})
    (hc,) = app["healthChecks"]
    assert hc["path"] == "/v1/health" and hc["intervalSeconds"] == 30 and hc["timeoutSeconds"] == 20
    assert hc["delaySeconds"] == 15
    env = app["env"]
    assert env["GLOG_v"] == "0" and env["HELLO_PORT_ONE"] == "1729" and env["HELLO_SECCOMP_UNCONFINED"] == "false"
    assert "HELLO_SECCOMP_PROFILE_NAME" not in env and "HELLO_VOLUME_PROFILE" not in env
    assert env["KEYSTORE_APP_VERSION"] and env["NGINX_CONTAINER_VERSION"]
