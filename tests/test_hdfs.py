"""HDFS service (reference: frameworks/hdfs/src/test/java/.../scheduler/{ServiceTest,
HDFSUserAuthMapperBuilderTest}.java and HdfsRecoveryPlanOverrider behaviour). Renders the package,
checks TLS ports/configs, client config endpoints, validators and auth_to_local mapping, and
simulates the HA bring-up order plus journal/name replacement via the ``replace`` plan."""
import base64
import os

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.models import hdfs as H
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.testing import Expect, Send, ServiceTestRunner
from dcos_commons_amd.testing.cosmos import render_scheduler_environment

# every test runs under the scheduler defaults and with every deviation from the reference off
pytestmark = pytest.mark.usefixtures("sched_profile")

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "frameworks", "hdfs")


def runner():
    r = ServiceTestRunner.for_framework("hdfs")
    for pod in ("journal", "name", "data"):
        r.set_pod_env(pod, SERVICE_ZK_ROOT="/dcos-service-hdfs", DECODED_AUTH_TO_LOCAL="")
    return (r.set_recovery_manager_factory(H.HdfsRecoveryPlanOverriderFactory())
            .set_custom_validators([H.HDFSZoneValidator()])
            .set_builder_customizer(lambda b: setattr(b, "original_service_spec",
                                                      H.with_placement_rules(b.original_service_spec)))
            .set_scheduler_env(SDK_REVIVE_INTERVAL_S="0"))


def test_spec_renders_every_config():
    r = runner().run()
    spec = r.service_spec
    assert [p.type for p in spec.pods] == ["journal", "name", "data"]
    assert [p.count for p in spec.pods] == [3, 2, 3]
    hdfs_site = r.get_task_config("name", "node", "hdfs-site")
    assert "qjournal://journal-0-node.hdfs.autoip.dcos.thisdcos.directory:8485;" in hdfs_site
    assert "name-1-node.hdfs.autoip.dcos.thisdcos.directory:9001" in hdfs_site
    assert "https-address" not in hdfs_site
    core = r.get_task_config("data", "node", "core-site")
    assert "/dcos-service-hdfs/hadoop-ha" in core and "<value>kerberos</value>" not in core
    assert sorted(r.raw_service_spec.plans) == ["deploy", "replace", "update"]


def test_tls_adds_https_ports_and_addresses():
    r = (runner().set_options("service.security.transport_encryption.enabled", "true",
                              "hdfs.name_node_https_port", "2000", "hdfs.journal_node_https_port", "2001",
                              "hdfs.data_node_https_port", "2002")
         .set_scheduler_env(DCOS_SERVICE_ACCOUNT_CREDENTIAL='{"uid": "hdfs", "private_key": "k"}').run())
    spec = r.service_spec

    def port(pod, task, name):
        res = spec.pod(pod).task(task).resource_set.resources
        return next(x for x in res if getattr(x, "port_name", None) == name)

    assert port("name", "node", "name-https").port == 2000
    cfg = r.get_task_config("name", "node", "hdfs-site")
    assert "dfs.namenode.https-address.hdfs.name-0-node" in cfg and "dfs.namenode.https-address.hdfs.name-1-node" in cfg
    assert port("journal", "node", "journal-https").port == 2001
    cfg = r.get_task_config("journal", "node", "hdfs-site")
    assert "0.0.0.0:2001" in cfg and "dfs.journalnode.https-address" in cfg
    assert port("data", "node", "data-https").port == 2002
    cfg = r.get_task_config("data", "node", "hdfs-site")
    assert "0.0.0.0:2002" in cfg and "dfs.datanode.https.address" in cfg
    assert [t.name for t in spec.pod("data").task("node").transport_encryption] == ["node"]


@pytest.mark.parametrize("name", [H.HDFS_SITE_XML, H.CORE_SITE_XML])
def test_render_client_configs(name):
    env = render_scheduler_environment(os.path.join(ROOT, "universe"))
    cfg = SchedulerConfig.for_testing(**env)
    text = H.render_client_config(os.path.join(ROOT, "specs", name), "hdfs", cfg, "", env)
    assert text.startswith("<?xml") and "{{" not in text
    if name == H.HDFS_SITE_XML:
        assert "sandboxpath/name-data" in text


def _zone_spec(placement):
    r = ServiceTestRunner.for_framework("hdfs")
    for pod in ("journal", "name", "data"):
        r.set_pod_env(pod, SERVICE_ZK_ROOT="", DECODED_AUTH_TO_LOCAL="")
    return r.set_options("data_node.placement", placement).run().service_spec


def test_zone_validator():
    v = H.HDFSZoneValidator()
    plain = _zone_spec('[["hostname", "UNIQUE"]]')
    zoned = _zone_spec('[["@zone", "GROUP_BY", "3"]]')
    zoned2 = _zone_spec('[["@zone", "MAX_PER", "2"]]')
    assert v.validate(plain, zoned) and v.validate(zoned, plain)
    assert v.validate(zoned, zoned2) == []


def test_region_awareness():
    assert runner().set_options("service.region", "Europe").run().scheduler_environment["SERVICE_REGION"] == "Europe"


# -- auth_to_local (HDFSUserAuthMapperBuilderTest) ------------------------------------------
AUTH_ENV = {H.PRIMARY_ENV_KEY: "hdfs", H.REALM_ENV_KEY: "LOCAL", H.FRAMEWORK_USER_ENV_KEY: "nobody"}


def test_auth_mapper_requires_keys():
    with pytest.raises(RuntimeError) as e:
        H.HDFSUserAuthMapperBuilder({H.PRIMARY_ENV_KEY: "hdfs"}, "host")
    assert H.REALM_ENV_KEY in str(e.value) and H.FRAMEWORK_USER_ENV_KEY in str(e.value)


def test_auth_mapper_rules():
    assert H.HDFSUserAuthMapperBuilder(AUTH_ENV, "h").add_user_auth_mapping_from_env().build() == ""
    env = dict(AUTH_ENV, **{H.TASKCFG_ALL_AUTH_TO_LOCAL: base64.b64encode(b"RULE:custom\n\nRULE:two").decode()})
    b = H.HDFSUserAuthMapperBuilder(env, "hdfs.autoip.dcos.thisdcos.directory").add_user_auth_mapping_from_env()
    b.add_default_user_auth_mapping("name", "node", 2)
    assert b.build().split("\n") == [
        "RULE:custom", "", "RULE:two",
        "RULE:[2:$1/$2@$0](hdfs/name-0-node.hdfs.autoip.dcos.thisdcos.directory@LOCAL)s/.*/nobody/",
        "RULE:[2:$1/$2@$0](hdfs/name-1-node.hdfs.autoip.dcos.thisdcos.directory@LOCAL)s/.*/nobody/"]
    # empty env mapping lines are dropped, the env rules are kept first
    b2 = H.HDFSUserAuthMapperBuilder(AUTH_ENV, "x").add_user_auth_mapping_from_env()
    b2.add_default_user_auth_mapping("data", "node", 1).add_default_user_auth_mapping("journal", "node", 1)
    assert len(b2.build().split("\n")) == 2


def test_kerberos_mapping_reaches_core_site():
    env = render_scheduler_environment(os.path.join(ROOT, "universe"), {"service.security.kerberos.enabled": "true"})
    cfg = SchedulerConfig.for_testing(**env)
    b = H.create_scheduler_builder(os.path.join(ROOT, "specs", "svc.yml"), cfg, env)
    mapping = b.original_service_spec.pod("data").task("node").command.env[H.DECODED_AUTH_TO_LOCAL]
    assert mapping.count("RULE:") == 3 + 2 + 2 + 3
    assert "hadoop.security.auth_to_local" in b.endpoint_producers[H.CORE_SITE_XML]
    assert "(hdfs/journal-2-node.hdfs.autoip.dcos.thisdcos.directory@LOCAL)" in b.endpoint_producers[H.CORE_SITE_XML]


def test_main_builder_placement_and_endpoints():
    env = render_scheduler_environment(os.path.join(ROOT, "universe"))
    cfg = SchedulerConfig.for_testing(**env)
    b = H.create_scheduler_builder(os.path.join(ROOT, "specs", "svc.yml"), cfg, env)
    spec = b.original_service_spec
    journal_rule = str(spec.pod("journal").placement_rule)
    assert "TaskTypeRule" in journal_rule and "journal" in journal_rule and "name" in journal_rule
    assert spec.pod("name").task("node").command.env[H.SERVICE_ZK_ROOT_TASKENV] == "/dcos-service-hdfs"
    assert "dfs.nameservices" in b.endpoint_producers[H.HDFS_SITE_XML]
    assert b.region_awareness_enabled
    with pytest.raises(RuntimeError):
        H.HdfsRecoveryPlanOverriderFactory().create(None, [])


# -- simulated deployment --------------------------------------------------------------------
def _running(task, ready=True):
    s = Send.task_status(task, P.TASK_RUNNING)
    return (s.set_readiness_check_exit_code(0) if ready else s).build()


def deploy_ticks():
    t = [Send.register()]
    for i in range(3):
        t += [Send.offer_builder("journal").set_hostname(f"j{i}").build(), Expect.launched_tasks(f"journal-{i}-node"),
              _running(f"journal-{i}-node", ready=False)]
    t += [
        # name-0: format, then node
        Send.offer_builder("name").set_hostname("n0").build(), Expect.launched_tasks("name-0-format"),
        Send.task_status("name-0-format", P.TASK_FINISHED).build(),
        Send.offer_builder("name").set_pod_index_to_reoffer(0).build(), Expect.launched_tasks("name-0-node"),
        _running("name-0-node"),
        # name-1: bootstrapStandby, then node
        Send.offer_builder("name").set_hostname("n1").build(), Expect.launched_tasks("name-1-bootstrap"),
        Send.task_status("name-1-bootstrap", P.TASK_FINISHED).build(),
        Send.offer_builder("name").set_pod_index_to_reoffer(1).build(), Expect.launched_tasks("name-1-node"),
        _running("name-1-node"),
        # zkfc: format ZK on name-0, then a zkfc next to each namenode
        Send.offer_builder("name").set_pod_index_to_reoffer(0).build(), Expect.launched_tasks("name-0-zkfc-format"),
        Send.task_status("name-0-zkfc-format", P.TASK_FINISHED).build(),
        Send.offer_builder("name").set_pod_index_to_reoffer(0).build(), Expect.launched_tasks("name-0-zkfc"),
        _running("name-0-zkfc"),
        Send.offer_builder("name").set_pod_index_to_reoffer(1).build(), Expect.launched_tasks("name-1-zkfc"),
        _running("name-1-zkfc"),
    ]
    for i in range(3):
        t += [Send.offer_builder("data").set_hostname(f"d{i}").build(), Expect.launched_tasks(f"data-{i}-node"),
              _running(f"data-{i}-node")]
    t += [Expect.plan_status("deploy", Status.COMPLETE)]
    return t


def _offer_on_agent_of(pod_type, task_name):
    def send(sim):
        agent = sim.state.last_launched(task_name).agent_id.value
        Send.offer_builder(pod_type).set_hostname("n0").set_agent_id(agent).build().send(sim)
    return send


def test_ha_deploy_order():
    def journal_avoids_name(sim):
        hosts = {}
        for a in sim.driver.accepts:
            for task in a.launched_tasks():
                hosts.setdefault(task.name.split("-")[0], set()).add(
                    next(lb.value for lb in task.labels.labels if lb.key == "offer_hostname"))
        assert not hosts["journal"] & hosts["name"]

    ticks = deploy_ticks() + [
        # a journal offer on a namenode host is refused by the injected TaskTypeRule
        Send.replace_pod("journal-1"),
        Send.task_status("journal-1-node", P.TASK_KILLED).build(),
        Send(_offer_on_agent_of("journal", "name-0-node"), "journal offer on name-0's agent"),
        Expect.declined_last_offer(),
        Expect.that(journal_avoids_name, "journal and name never share a host"),
    ]
    runner().run(ticks)


def test_replace_namenode_uses_bootstrap_then_node():
    def check(sim):
        plan = sim.scheduler.get_plan("recovery")
        phases = [ph.get_name() for ph in plan.get_children()]
        assert phases == ["permanent-name-failure-recovery"], phases
        steps = [s.get_name() for s in plan.get_children()[0].get_children()]
        assert steps == ["name-0:[bootstrap]", "name-0:[node, zkfc]"], steps

    ticks = deploy_ticks() + [
        Send.replace_pod("name-0"),
        Send.task_status("name-0-node", P.TASK_KILLED).build(),
        Send.task_status("name-0-zkfc", P.TASK_KILLED).build(),
        Send.offer_builder("name").set_hostname("n-new").build(),
        Expect.launched_tasks("name-0-bootstrap"),
        Expect.that(check, "namenode replacement phase"),
        Send.task_status("name-0-bootstrap", P.TASK_FINISHED).build(),
        Send.offer_builder("name").set_pod_index_to_reoffer(0).build(),
        Expect.launched_tasks("name-0-node", "name-0-zkfc"),
        _running("name-0-node"), _running("name-0-zkfc"),
        Expect.plan_status("recovery", Status.COMPLETE),
    ]
    runner().run(ticks)


def test_replace_journal_and_data():
    def check(sim):
        names = [ph.get_name() for ph in sim.scheduler.get_plan("recovery").get_children()]
        assert "permanent-journal-failure-recovery" in names and "data-2:[node]" in names, names

    ticks = deploy_ticks() + [
        Send.replace_pod("journal-2"),
        Send.task_status("journal-2-node", P.TASK_KILLED).build(),
        Send.replace_pod("data-2"),
        Send.task_status("data-2-node", P.TASK_KILLED).build(),
        Send.offer_builder("journal").set_hostname("j-new").build(),
        Expect.launched_tasks("journal-2-bootstrap"),
        Expect.that(check, "journal replaced via override, data via default recovery"),
    ]
    runner().run(ticks)


@pytest.mark.parametrize("framework,pods", [("hdfs", ("journal", "name", "data")), ("cassandra", ("node",))])
@pytest.mark.parametrize("labels,expected", [("", ()), ("k_0:v_0,k_1:v_1", (("k_0", "v_0"), ("k_1", "v_1")))])
def test_virtual_network_plugin_labels_reach_every_pod(framework, pods, labels, expected):
    """the reference passes ``virtual_network_plugin_labels`` (config.json:45) as CNI
    labels on every overlay-network pod (hdfs svc.yml:23-27,170-174,476-480; cassandra svc.yml:9-13)."""
    r = ServiceTestRunner.for_framework(framework)
    for pod in pods:
        if framework == "hdfs":
            r.set_pod_env(pod, SERVICE_ZK_ROOT="/dcos-service-hdfs", DECODED_AUTH_TO_LOCAL="")
        else:
            r.set_pod_env(pod, {"LOCAL_SEEDS": "a,b"})
    r = r.set_options("service.virtual_network_enabled", "true", "service.virtual_network_name", "dcos",
                      "service.virtual_network_plugin_labels", labels).run()
    for pod in pods:
        nets = r.service_spec.pod(pod).networks
        assert [n.name for n in nets] == ["dcos"]
        assert tuple(sorted(nets[0].labels)) == expected
