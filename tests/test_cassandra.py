"""Cassandra service (reference: frameworks/cassandra/src/test/java/.../scheduler/ServiceTest.java,
CassandraRecoveryPlanOverriderTest.java). Runs the package through its Universe options, renders
the node config templates, checks the zone/env validators and simulates a full deployment plus
seed and non-seed node replacement with ``replace_address``."""
import os

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.models import cassandra as C
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.testing import Expect, Send, ServiceTestRunner

NODE_ENV = {"LOCAL_SEEDS": "foo,bar"}  # what Main injects into every pod

# every test runs under the scheduler defaults and with every deviation from the reference off
pytestmark = pytest.mark.usefixtures("sched_profile")


def runner():
    return (ServiceTestRunner.for_framework("cassandra").set_pod_env("node", NODE_ENV)
            .set_custom_validators(C.custom_validators())
            .set_recovery_manager_factory(C.CassandraRecoveryPlanOverriderFactory(2))
            .set_builder_customizer(lambda b: b.set_custom_resources([C.SeedsResource(["foo", "bar"])]))
            .set_scheduler_env(SDK_REVIVE_INTERVAL_S="0"))


def test_spec_renders_with_package_defaults():
    r = runner().run()
    spec = r.service_spec
    assert spec.name == "cassandra" and spec.user == "nobody"
    node = spec.pod("node")
    assert node.count == 3 and len(node.tasks) == 13
    assert sorted(r.raw_service_spec.plans) == ["backup-azure", "backup-s3", "cleanup", "deploy", "repair", "replace",
                                                "restore-azure", "restore-s3"]
    cfg = r.get_task_config("node", "server", "cassandra")
    assert '- seeds: "foo,bar"' in cfg and "internode_encryption: none" in cfg
    assert "native_transport_port: 9042" in cfg and "authenticator: AllowAllAuthenticator" in cfg
    assert r.get_task_config("node", "server", "rackdc") == "dc=datacenter1\nrack=rack1\n"
    assert r.scheduler_environment["NODES"] == "3" and "PORT_API" in r.scheduler_environment


def test_spec_custom_user_and_seeds():
    env = dict(NODE_ENV, REMOTE_SEEDS="baz")
    r = runner().set_options("service.user", "foo").set_pod_env("node", env).run()
    assert r.service_spec.user == "foo"
    assert r.service_spec.pods[0].user == "foo"
    assert '- seeds: "foo,bar,baz"' in r.get_task_config("node", "server", "cassandra")


def test_spec_ssl():
    r = (runner().set_options("service.security.transport_encryption.enabled", "true")
         .set_scheduler_env(DCOS_SERVICE_ACCOUNT_CREDENTIAL='{"uid": "cassandra", "private_key": "k"}').run())
    cfg = r.get_task_config("node", "server", "cassandra")
    assert "internode_encryption: all" in cfg
    assert "client_encryption_options:\n    enabled: true\n    optional: false" in cfg
    server = r.service_spec.pod("node").task("server")
    assert [t.name for t in server.transport_encryption] == ["node"]


def test_region_awareness():
    r = runner().set_options("service.region", "Europe").run()
    assert r.scheduler_environment["SERVICE_REGION"] == "Europe"


def _spec_with(placement, **options):
    rr = ServiceTestRunner.for_framework("cassandra").set_pod_env("node", NODE_ENV)
    rr.set_options("nodes.placement_constraint", placement, **options)
    return rr.run().service_spec


def test_zone_validator_rejects_toggling_zones_but_allows_changes():
    v = C.CassandraZoneValidator()
    no_zone = _spec_with('[["hostname", "MAX_PER", "1"]]')
    zone = _spec_with('[["@zone", "GROUP_BY", "3"]]')
    zone2 = _spec_with('[["@zone", "MAX_PER", "2"]]')
    assert v.validate(no_zone, zone)  # enabling racks
    assert v.validate(zone, no_zone)  # disabling racks
    assert v.validate(zone, zone2) == []
    assert v.validate(None, zone) == []


def test_data_center_env_may_only_be_set_once():
    rack = C.custom_validators()[2]
    a = ServiceTestRunner.for_framework("cassandra").set_pod_env("node", NODE_ENV).run().service_spec
    b = (ServiceTestRunner.for_framework("cassandra").set_pod_env("node", NODE_ENV)
         .set_options("service.rack", "rack2").run().service_spec)
    errs = rack.validate(a, b)
    assert errs and "CASSANDRA_LOCATION_RACK" in str(errs[0])


def _check_seeds(resp):
    assert resp.json() == {"seeds": ["foo", "bar"]}, resp.json()


def _deploy_ticks():
    ticks = [Send.register()]
    for i in range(3):
        ticks += [
            Send.offer_builder("node").set_hostname(f"host-{i}").build(),
            Expect.launched_tasks(f"node-{i}-server"),
            Send.task_status(f"node-{i}-server", P.TASK_RUNNING).set_readiness_check_exit_code(0)
            .set_ip(f"10.0.0.{i + 1}").build(),
        ]
    ticks += [
        # keyspace-deploy: node 0 runs init_system_keyspaces once; the other steps are empty
        Send.offer_builder("node").set_pod_index_to_reoffer(0).add_unreserved_resources().build(),
        Expect.launched_tasks("node-0-init_system_keyspaces"),
        Send.task_status("node-0-init_system_keyspaces", P.TASK_FINISHED).build(),
        Expect.plan_status("deploy", Status.COMPLETE),
        Expect.http("GET", "/v1/seeds", 200, _check_seeds),
    ]
    return ticks


def _launched_server_cmd(sim, task_name):
    for a in reversed(sim.driver.accepts):
        for t in a.launched_tasks():
            if t.name == task_name:
                return t.command.value
    raise AssertionError(f"{task_name} never launched")


def test_deploy_then_replace_seed_node_restarts_others():
    replaced = {}

    def check_phase(sim):
        plan = sim.scheduler.get_plan("recovery")
        phases = [p.get_name() for p in plan.get_children()]
        assert phases == [C.RECOVERY_PHASE_NAME], phases
        steps = [s.get_name() for s in plan.get_children()[0].get_children()]
        assert steps == ["node-0:[server]", "node-1:[server]", "node-2:[server]"], steps
        replaced["cmd"] = _launched_server_cmd(sim, "node-0-server")

    ticks = _deploy_ticks() + [
        Send.replace_pod("node-0"),
        Expect.task_name_killed("node-0-server"),
        Send.task_status("node-0-server", P.TASK_KILLED).build(),
        Send.offer_builder("node").set_hostname("host-new").build(),
        Expect.launched_tasks("node-0-server"),
        Expect.that(check_phase, "seed replacement phase restarts the other nodes"),
    ]
    runner().run(ticks)
    assert "-Dcassandra.replace_address=10.0.0.1 -Dcassandra.consistent.rangemovement=false" in replaced["cmd"]


def test_replace_non_seed_node_is_single_step():
    def check(sim):
        plan = sim.scheduler.get_plan("recovery")
        steps = [s.get_name() for ph in plan.get_children() for s in ph.get_children()]
        assert steps == ["node-2:[server]"], steps
        assert "-Dcassandra.replace_address=10.0.0.3" in _launched_server_cmd(sim, "node-2-server")

    ticks = _deploy_ticks() + [
        Send.replace_pod("node-2"),
        Send.task_status("node-2-server", P.TASK_KILLED).build(),
        Send.offer_builder("node").set_hostname("host-new").build(),
        Expect.launched_tasks("node-2-server"),
        Expect.that(check, "non-seed replacement"),
    ]
    runner().run(ticks)


def test_transient_failure_is_not_overridden():
    def check(sim):
        plan = sim.scheduler.get_plan("recovery")
        assert [ph.get_name() for ph in plan.get_children()] == ["node-1:[server]"]
        assert "replace_address" not in _launched_server_cmd(sim, "node-1-server")

    ticks = _deploy_ticks() + [
        Send.task_status("node-1-server", P.TASK_FAILED).build(),
        Send.offer_builder("node").set_pod_index_to_reoffer(1).build(),
        Expect.launched_tasks("node-1-server"),
        Expect.that(check, "transient recovery uses the default phase"),
    ]
    runner().run(ticks)


def test_main_builder_injects_seeds_and_resources(tmp_path):
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
    from dcos_commons_amd.testing.cosmos import render_scheduler_environment

    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "frameworks", "cassandra")
    env = render_scheduler_environment(os.path.join(root, "universe"), {"service.remote_seeds": "dc2-a,dc2-b"})
    import base64

    env[C.AUTH_YAML_BASE64_ENV] = base64.b64encode(b"roles_validity_in_ms: 5").decode()
    cfg = SchedulerConfig.for_testing(**env)
    b = C.create_scheduler_builder(os.path.join(root, "specs", "svc.yml"), cfg, env)
    spec = b.original_service_spec
    server = spec.pod("node").task("server")
    seeds = server.command.env["LOCAL_SEEDS"]
    assert seeds == "node-0-server.cassandra.autoip.dcos.thisdcos.directory," \
                    "node-1-server.cassandra.autoip.dcos.thisdcos.directory"
    assert server.command.env["AUTHENTICATION_CUSTOM_YAML_BLOCK"] == "roles_validity_in_ms: 5"
    res = b.custom_resources[0]
    route = res.routes()[0]
    assert route.handler(None).json()["seeds"][-2:] == ["dc2-a", "dc2-b"]
    assert b.region_awareness_enabled
    with pytest.raises(RuntimeError):
        C.CassandraRecoveryPlanOverriderFactory().create(None, [])
