"""Every hello-world scenario spec renders, builds a scheduler and deploys to COMPLETE in the
simulator (reference: frameworks/helloworld/src/main/dist/*.yml exercised by helloworld's
ServiceTest / CustomStepsTest), plus scenario-specific checks of the launched TaskInfos."""
import os

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.testing import Expect, Send, ServiceTestRunner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS = os.path.join(ROOT, "frameworks", "helloworld", "specs")

ENV = dict(FRAMEWORK_NAME="hello-world", FRAMEWORK_PRINCIPAL="hello-world-principal", FRAMEWORK_USER="nobody",
           HELLO_COUNT="2", HELLO_PLACEMENT='[["hostname", "UNIQUE"]]', HELLO_CPUS="0.1", HELLO_MEM="252",
           HELLO_DISK="25", HELLO_GPUS="1", SLEEP_DURATION="1000", WORLD_COUNT="2",
           WORLD_PLACEMENT='[["hostname", "UNIQUE"]]', WORLD_CPUS="0.2", WORLD_MEM="512", WORLD_DISK="25",
           WORLD_READINESS_CHECK_INTERVAL="5", WORLD_READINESS_CHECK_DELAY="0", WORLD_READINESS_CHECK_TIMEOUT="10",
           HELLO_VERSION="1", HELLO_SECRET1="hello-world/secret1", HELLO_SECRET2="hello-world/secret2", WORLD_SECRET1="hello-world/secret1",
           WORLD_SECRET2="hello-world/secret2", WORLD_SECRET3="hello-world/secret3",
           DISCOVERY_TASK_PREFIX="custom", GPU_PROBE_CMD="true", PRE_RESERVED_ROLE="slave_public",
           TASKCFG_ALL_GREETING="hi", TASKCFG_HELLO_TARGET="everyone", HELLO_VOLUME_PROFILE="xfs")

# scenarios that need a DC/OS CA (tests/test_tls.py and test_reference_conformance.py deploy it);
# pre-reserved and profiled-disk scenarios get offers carrying those resources (harness SendOffer)
RENDER_ONLY = {"tls.yml"}
ALL = sorted(f for f in os.listdir(SPECS) if f.endswith(".yml"))


def _launched(sim):
    return {t.name: t for a in sim.driver.accepts for t in a.launched_tasks()}


def _executor(sim, task_name):
    """The pod's ExecutorInfo (LAUNCH_GROUP carries it next to the task group)."""
    for a in reversed(sim.driver.accepts):
        if any(t.name == task_name for t in a.launched_tasks()):
            return a.executors()[-1]
    raise AssertionError(f"{task_name} not launched")


@pytest.mark.parametrize("spec", ALL)
def test_scenario_deploys(spec):
    r = ServiceTestRunner(os.path.join(SPECS, spec)).set_env(ENV).set_scheduler_env(SDK_REVIVE_INTERVAL_S="0")
    if spec == "tls.yml":
        r.set_scheduler_env(DCOS_SERVICE_ACCOUNT_CREDENTIAL='{"uid": "u", "private_key": "k"}')
    if spec in RENDER_ONLY:
        r.run([Send.register(), Expect.plan_status("deploy", Status.PENDING)])
        return
    r.run([Send.register(), Send.drive_plan("deploy"), Expect.plan_status("deploy", Status.COMPLETE)])


def _run(spec, checks, env=None, sched=None):
    r = ServiceTestRunner(os.path.join(SPECS, spec)).set_env(dict(ENV, **(env or {})))
    r.set_scheduler_env(SDK_REVIVE_INTERVAL_S="0", **(sched or {}))
    return r.run([Send.register(), Send.drive_plan("deploy"), Expect.that(checks, f"{spec} checks")])


def test_taskcfg_routing():
    def check(sim):
        t = _launched(sim)
        hello = {v.name: v.value for v in t["hello-0-server"].command.environment.variables}
        world = {v.name: v.value for v in t["world-0-server"].command.environment.variables}
        assert hello["GREETING"] == "hi" and hello["TARGET"] == "everyone"  # TASKCFG_HELLO_*: hello only
        assert world["GREETING"] == "hi" and "TARGET" not in world
        assert hello["OUTPUT_FILENAME"] == "out" and world["SLEEP_DURATION"] == "5"
    _run("taskcfg.yml", check, env={"TASKCFG_ALL_OUTPUT_FILENAME": "out", "TASKCFG_ALL_SLEEP_DURATION": "5"})


def test_discovery_prefix_and_kill_grace_and_uris():
    def check(sim):
        t = _launched(sim)
        assert t["hello-1-server"].discovery.name == "hello-svc-1"
        assert t["hello-1-server"].discovery.visibility == P.DiscoveryInfo.CLUSTER
        assert t["setup-0-once"].discovery.name == "setup-job-0"
    _run("discovery.yml", check)

    def grace(sim):
        t = _launched(sim)["hello-0-server"]
        assert t.kill_policy.grace_period.nanoseconds == 30 * 10 ** 9
    _run("graceful-shutdown.yml", grace)

    def uris(sim):
        t = _launched(sim)
        assert [u.value for u in t["world-0-server"].command.uris][-2:] == [
            "https://downloads.example.com/world-artifact.zip", "https://downloads.example.com/config.json"]
    _run("uri.yml", uris)


def test_container_features():
    def shm(sim):
        linux = _executor(sim, "hello-0-server").container.linux_info  # pod-level: executor container
        assert linux.ipc_mode == P.LinuxInfo.PRIVATE and linux.shm_size == 128
    _run("shm.yml", shm)

    def seccomp(sim):  # seccomp applies to the task container (PodInfoBuilder.java:592-605)
        assert _launched(sim)["hello-0-server"].container.linux_info.seccomp.unconfined
    _run("seccomp.yml", seccomp, env={"HELLO_SECCOMP_UNCONFINED": "true"})

    def profile(sim):
        seccomp = _launched(sim)["hello-0-server"].container.linux_info.seccomp
        assert not seccomp.unconfined and seccomp.profile_name == "default.json"
    _run("seccomp.yml", profile, env={"HELLO_SECCOMP_PROFILE_NAME": "default.json"})

    def host_vol(sim):
        vols = {v.container_path: v for v in _launched(sim)["hello-0-server"].container.volumes}
        assert vols["host-etc"].host_path == "/etc" and vols["host-etc"].mode == P.Volume.RO
        assert vols["host-tmp"].mode == P.Volume.RW
    _run("host-volume.yml", host_vol)

    def secrets(sim):
        t = _launched(sim)["hello-0-server"]
        env_secrets = {v.name: v.secret.reference.name for v in t.command.environment.variables
                       if v.type == P.Environment.Variable.SECRET}
        assert env_secrets == {"HELLO_SECRET1_ENV": "hello-world/secret1", "HELLO_SECRET1_AGAIN": "hello-world/secret1"}
        files = {v.container_path: v.source.secret.reference.name for v in t.container.volumes
                 if v.source.type == P.Volume.Source.SECRET}
        assert files == {"secrets/secret2": "hello-world/secret2", "secrets/secret1": "hello-world/secret1"}
    _run("secrets.yml", secrets)


def test_enable_disable_plan_steps():
    def without(sim):
        assert not any(n.endswith("-server-a") for n in _launched(sim))
        assert {"hello-0-server-b", "hello-1-server-b"} <= set(_launched(sim))
    _run("enable-disable.yml", without, env={"TEST_BOOLEAN": "false"})

    def with_a(sim):
        assert {"hello-0-server-a", "hello-1-server-a", "hello-0-server-b"} <= set(_launched(sim))
    _run("enable-disable.yml", with_a, env={"TEST_BOOLEAN": "true"})


def test_multiport_and_overlay_ports():
    def ports(sim):
        t = _launched(sim)["multiport-0-server"]
        env = {v.name: v.value for v in t.command.environment.variables}
        ports = {p.name: p.number for p in t.discovery.ports.ports}
        assert ports["static"] == 4444 and ports["dynamic"] not in (0, 4444)
        assert env["CUSTOM_ENV"] == str(ports["keyed"])  # only explicit env-keys become variables
        assert 7000 <= ports["ranged"] <= 7100
        vips = [lb.key for p in t.discovery.ports.ports for lb in p.labels.labels if lb.key.startswith("VIP_")]
        assert vips
    _run("multiport.yml", ports)

    def overlay(sim):
        t = _launched(sim)
        # with the default executor, NetworkInfos live on the executor (PodInfoBuilder.java:642)
        assert [n.name for n in _executor(sim, "overlay-0-server").container.network_infos] == ["dcos"]
        assert not [r for r in t["overlay-0-server"].resources if r.name == "ports"]  # overlay: no host ports
        bridge = _executor(sim, "bridge-0-server").container.network_infos[0]
        assert bridge.name == "mesos-bridge" and bridge.port_mappings[0].host_port == 4045
        assert [r for r in t["host-0-server"].resources if r.name == "ports"]
    _run("overlay.yml", overlay)


def test_gpu_and_mount_volumes():
    def gpus(sim):
        t = _launched(sim)["hello-0-server"]
        assert [r.scalar.value for r in t.resources if r.name == "gpus"] == [1.0]
    _run("gpu_resource.yml", gpus)

    def mount(sim):
        disks = [r for r in _executor(sim, "hello-0-node").resources if r.name == "disk"]
        assert disks and disks[0].disk.source.type == P.Resource.DiskInfo.Source.MOUNT
        own = {t: [r.disk.source.type for r in _launched(sim)[f"hello-0-{t}"].resources if r.name == "disk"]
               for t in ("node", "agent")}
        assert own["node"] == [P.Resource.DiskInfo.Source.MOUNT] and own["agent"] == [0]   # 0: no source, ROOT
    _run("pod-mount-volume.yml", mount)


def test_operator_started_plans():
    def sidecar(sim):
        assert sim.scheduler.get_plan("sidecar").get_status() in (Status.WAITING, Status.PENDING)
    r = ServiceTestRunner(os.path.join(SPECS, "sidecar.yml")).set_env(ENV).set_scheduler_env(SDK_REVIVE_INTERVAL_S="0")
    r.run([Send.register(), Send.drive_plan("deploy"), Expect.that(sidecar, "sidecar plan waits for start"),
           Send.http("POST", "/v1/plans/sidecar/start", b"{}", 200),
           Send.drive_plan("sidecar"), Expect.plan_status("sidecar", Status.COMPLETE),
           # the never-started "toxic" sidecar is known too: it shares the sidecar resource set,
           # whose reservation is recorded on every task of the set
           Expect.known_tasks("hello-0-server", "hello-1-server", "hello-0-backup", "hello-1-backup",
                              "hello-0-verify", "hello-1-verify", "hello-0-toxic", "hello-1-toxic")])


def test_update_plan_rolls_out_config_change():
    first = (ServiceTestRunner(os.path.join(SPECS, "update_plan.yml")).set_env(ENV)
             .set_scheduler_env(SDK_REVIVE_INTERVAL_S="0")
             .run([Send.register(), Send.drive_plan("deploy"), Send.empty_offers()]))

    def check(sim):
        assert sim.scheduler.get_plan("deploy").get_children()[0].get_name() == "hello-update"
    (ServiceTestRunner(os.path.join(SPECS, "update_plan.yml")).set_env(dict(ENV, HELLO_VERSION="2"))
     .set_scheduler_env(SDK_REVIVE_INTERVAL_S="0").set_state(first)
     .run([Send.register(), Expect.that(check, "update plan serves as deploy"), Send.drive_plan("deploy"),
           Expect.that(lambda sim: _assert_version(sim, "2"), "new version launched")]))


def _assert_version(sim, v):
    t = {x.name: x for a in sim.driver.accepts for x in a.launched_tasks()}["hello-1-server"]
    assert {e.name: e.value for e in t.command.environment.variables}["VERSION"] == v
