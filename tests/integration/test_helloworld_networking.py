"""helloworld networking scenarios on the local cluster.

Reference: frameworks/helloworld/tests/{test_overlay.py, test_discovery.py, test_multiple_ports.py,
test_web_url.py, test_custom_service_tld.py}. Overlay tasks report the ``dcos`` network and an
address from the overlay subnet (9.x) with no host port reservation, host tasks report their
agent's 10.x address and no network name; the endpoints API serves both kinds with autoip DNS
names and VIPs, CNI labels reach the executor's NetworkInfo, and Mesos-DNS carries one SRV record
per advertised port. Custom discovery prefixes name the DNS entries, multi-port tasks get every
port they ask for, the spec's web-url reaches the FrameworkInfo, and a custom service TLD
replaces the autoip domain of endpoint DNS names.
"""
import pytest

from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_hosts, sdk_install, sdk_networks, sdk_plan, sdk_tasks,
                                          sdk_utils)
from tests.integration import hw_config as config

pytestmark = pytest.mark.usefixtures("local_cluster")
OVERLAY = "hello-overlay"   # its own service: runs next to the single-scenario installs below


@pytest.fixture(scope="module")
def overlay_service(local_cluster):
    sdk_install.install(config.PACKAGE_NAME, OVERLAY, 5,
                        additional_options={"service": {"yaml": "overlay"}})
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, OVERLAY)


def test_overlay_network(overlay_service):
    sdk_plan.wait_for_completed_deployment(OVERLAY)
    tasks = sdk_tasks.get_service_tasks(OVERLAY)
    assert {t.name for t in tasks} == {"overlay-vip-0-server", "overlay-0-server", "bridge-0-server",
                                       "host-vip-0-server", "host-0-server"}
    for t in tasks:
        if t.name.startswith("host-"):
            assert "ports" in t.resources, f"Task {t.name} should have port resources"
            sdk_networks.check_task_network(t.name, expected_network_name=None)
            assert sdk_networks.get_task_ip(OVERLAY, t.name) == t.host
        elif t.name.startswith("overlay-"):
            assert "ports" not in t.resources, f"Task {t.name} should NOT have port resources"
            sdk_networks.check_task_network(t.name)
            assert sdk_networks.get_task_ip(OVERLAY, t.name).startswith("9.")
        else:
            # bridge: container port 8080 is reached through the reserved host port 4045
            assert "ports" in t.resources
            sdk_networks.check_task_network(t.name, expected_network_name="mesos-bridge")

    names = sdk_networks.get_endpoint_names(config.PACKAGE_NAME, OVERLAY)
    assert {"overlay-vip", "host-vip"} <= set(names), names
    overlay = sdk_networks.get_endpoint(config.PACKAGE_NAME, OVERLAY, "overlay-vip")
    assert len(overlay["address"]) == 1
    assert overlay["address"][0].startswith("9") and overlay["address"][0].split(":")[-1] == "4044"
    assert overlay["dns"] == [sdk_hosts.autoip_host(OVERLAY, "overlay-vip-0-server", 4044)]
    assert overlay["vip"] == sdk_hosts.vip_host(OVERLAY, "overlay-vip", 80)
    sdk_networks.check_endpoint_on_overlay(config.PACKAGE_NAME, OVERLAY, "overlay-vip", 1)

    host = sdk_networks.get_endpoint(config.PACKAGE_NAME, OVERLAY, "host-vip")
    assert len(host["address"]) == 1
    assert host["address"][0].startswith("10") and host["address"][0].split(":")[-1] == "4044"
    assert host["dns"] == [sdk_hosts.autoip_host(OVERLAY, "host-vip-0-server", 4044)]


def test_cni_labels(overlay_service):
    r = sdk_cmd.service_request("GET", OVERLAY, "/v1/pod/overlay-vip-0/info").json()
    assert len(r) == 1, "Got multiple responses from v1/pod/overlay-vip-0/info"
    labels = r[0]["info"]["executor"]["container"]["networkInfos"][0]["labels"]["labels"]
    assert {(l["key"], l["value"]) for l in labels} == {("key0", "val0"), ("key1", "val1")}
    # and the running container's status carries them
    status = [s for s in sdk_tasks.get_all_status_history("overlay-vip-0-server") if s["state"] == "TASK_RUNNING"][-1]
    ni = status["container_status"]["network_infos"][0]
    assert ni["name"] == "dcos" and {l["key"] for l in ni["labels"]["labels"]} == {"key0", "key1"}


def test_srv_records(overlay_service):
    expected = {"overlay-vip-0-server": ["overlay-vip"], "overlay-0-server": ["overlay-http"],
                "host-vip-0-server": ["host-vip"], "host-0-server": ["host-http"],
                "bridge-0-server": ["bridge-http"]}

    @sdk_utils.retry(timeout_s=30, interval_s=0.5)
    def check():
        records = sdk_networks.get_srv_records(OVERLAY)
        assert expected.keys() == records.keys(), "Mismatch between expected and actual tasks"
        for task_name, ports in expected.items():
            for port in ports:
                assert f"_{port}._{task_name}._tcp.{OVERLAY}.mesos." in records[task_name], \
                    (task_name, records[task_name])
    check()


def test_task_dns_prefix_points_to_all_tasks():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 3,
                        additional_options={"service": {"yaml": "discovery"}, "hello": {"count": 3}})
    try:
        for i in range(3):
            pod_info = sdk_cmd.service_request("GET", config.SERVICE_NAME, f"/v1/pod/hello-{i}/info").json()
            assert all(p["info"]["discovery"]["name"] == f"hello-svc-{i}" for p in pod_info)
        setup = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/pod/setup-0/info").json()
        assert setup[0]["info"]["discovery"]["name"] == "setup-job-0"
        # Mesos-DNS names every hello task by its prefix and serves its advertised port
        records = sdk_networks.get_srv_records(config.SERVICE_NAME)
        for i in range(3):
            assert f"hello-svc-{i}.{config.SERVICE_NAME}.mesos." in records[f"hello-{i}-server"]
            assert f"_http._hello-svc-{i}._tcp.{config.SERVICE_NAME}.mesos." in records[f"hello-{i}-server"]
        ep = sdk_networks.get_endpoint(config.PACKAGE_NAME, config.SERVICE_NAME, "http")
        assert len(ep["address"]) == 3 and len(ep["dns"]) == 3
        assert all(d.startswith("hello-svc-") for d in ep["dns"]), ep["dns"]
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_launch_task_with_multiple_ports():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"yaml": "multiport"}})
    try:
        assert sdk_tasks.get_summary(with_completed=True, task_name="multiport-0-server"), \
            "Unable to find matching task"
        info = sdk_cmd.service_request("GET", config.SERVICE_NAME, "/v1/pod/multiport-0/info").json()[0]["info"]
        ports = {p["name"]: p["number"] for p in info["discovery"]["ports"]["ports"]}
        assert ports["static"] == 1729 and 7000 <= ports["ranged"] <= 7100     # the package's hello.port_one
        assert len(set(ports.values())) == 5, ports
        # every port is reserved for the task: the agent's port ranges cover them
        ranges = [(int(r["begin"]), int(r["end"])) for res in info["resources"] if res["name"] == "ports"
                  for r in res["ranges"]["range"]]
        assert all(any(b <= p <= e for b, e in ranges) for p in ports.values()), (ports, ranges)
        # the task saw its keyed port in the environment
        rc, out, _ = sdk_cmd.run_cli("task log multiport-0-server")
        assert rc == 0 and str(ports["keyed"]) in out, out
        assert sdk_networks.get_endpoint(config.PACKAGE_NAME, config.SERVICE_NAME, "advertised")["vip"] == \
            sdk_hosts.vip_host(config.SERVICE_NAME, "multiport-vip", 80)
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_web_url():
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"yaml": "web-url"}})
    try:
        plan = sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
        assert len(plan["phases"]) == 1 and plan["phases"][0]["name"] == "hello"
        assert len(plan["phases"][0]["steps"]) == 1
        fws = [f for f in sdk_cmd.cluster_request("GET", "/mesos/frameworks").json()["frameworks"]
               if f["name"] == config.SERVICE_NAME and f["active"]]
        assert fws and fws[0]["webui_url"] == f"http://{config.SERVICE_NAME}.example.com/ui"
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)


def test_custom_service_tld():
    custom_tld = "custom.example.tld"
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 1,
                        additional_options={"service": {"custom_service_tld": custom_tld, "yaml": "custom_tld"}})
    try:
        assert sdk_networks.get_endpoint_names(config.PACKAGE_NAME, config.SERVICE_NAME) == ["http"]
        ep = sdk_networks.get_endpoint(config.PACKAGE_NAME, config.SERVICE_NAME, "http")
        assert set(ep) == {"address", "dns"}
        assert len(ep["address"]) == 1 and all(len(a.split(":")) == 2 for a in ep["address"])
        assert len(ep["dns"]) == 1 and all(custom_tld in d for d in ep["dns"]), ep["dns"]
        assert ep["dns"][0].startswith(f"hello-0-server.{config.SERVICE_NAME}.")
    finally:
        sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
