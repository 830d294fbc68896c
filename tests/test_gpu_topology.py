"""MI355X node discovery (``ops.gpu``) and topology-aware GPU placement.

The reference only knows a ``gpus`` scalar (``offer/Constants.java:62``) and the ``GPU_RESOURCES``
capability (``framework/FrameworkRunner.java:191-194``). Here agents derive ``gpus``, ``gpu_model``,
``gpu_arch`` and ``xgmi_hive`` from the node (KFD topology, ``amd-smi static --json``,
``rocminfo``), placement rules use those attributes unchanged (``[["xgmi_hive","GROUP_BY"]]``,
``CLUSTER``, ``MAX_PER``), and an agent hands a ``gpus: N`` task N devices of one xGMI hive.

Parsers run on recorded-format fixtures: the KFD sysfs tree (``synthetic_kfd_tree`` writes the
kernel's ``properties`` layout), an ``amd-smi static --json`` document in the layout of
``amdsmi_commands.py`` (ROCm 7.2), and ``rocminfo`` agent blocks. ``tests/fixtures/gpu/mi355x_box``
is the discovery dump of the MI355X box this repository's GPU runs use
(``scripts/dev/dump_gpu_discovery.sh``), when present.
"""
import json
import os
import time

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver, gpu_agent_specs
from dcos_commons_amd.ops import gpu as G
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.storage.mem_persister import MemPersister

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS = os.path.join(ROOT, "frameworks", "helloworld", "specs")
BOX_FIXTURE = os.path.join(ROOT, "tests", "fixtures", "gpu", "mi355x_box")

AMD_SMI_STATIC = json.dumps([
    {"gpu": i, "asic": {"market_name": "AMD Instinct MI355X", "vendor_id": "0x1002", "vendor_name": "Advanced Micro Devices Inc. [AMD/ATI]",
                        "subvendor_id": "0x1002", "device_id": "0x75a3", "subsystem_id": "0x75a3", "rev_id": "0x00",
                        "asic_serial": f"0x{0xABCDEF00 + i:X}", "oam_id": i, "num_compute_units": 256,
                        "target_graphics_version": "gfx950"},
     "bus": {"bdf": f"0000:{0x05 + 0x10 * i:02x}:00.0", "max_pcie_width": 16, "max_pcie_speed": {"value": 32, "unit": "GT/s"},
             "pcie_interface_version": "Gen 5", "slot_type": "OAM"},
     "vram": {"type": "HBM", "vendor": "N/A", "size": {"value": 294896, "unit": "MB"}, "bit_width": 8192,
              "max_bandwidth": {"value": 8000, "unit": "GB/s"}}} for i in range(8)])

ROCMINFO = """ROCk module version 6.12.12 is loaded
=====================
HSA System Attributes
=====================
Runtime Version:         1.18

==========
HSA Agents
==========
*******
Agent 1
*******
  Name:                    AMD EPYC 9575F 64-Core Processor
  Marketing Name:          AMD EPYC 9575F 64-Core Processor
  Vendor Name:             CPU
  Node:                    0
  Device Type:             CPU
*******
Agent 2
*******
  Name:                    gfx950
  Uuid:                    GPU-4b6f2a0c1d2e3f40
  Marketing Name:          AMD Instinct MI355X
  Vendor Name:             AMD
  Node:                    2
  Device Type:             GPU
  Chip ID:                 30115(0x75a3)
  Compute Unit:            256
  ISA Info:
    ISA 1
      Name:                    amdgcn-amd-amdhsa--gfx950:sramecc+:xnack-
*******
Agent 3
*******
  Name:                    gfx950
  Marketing Name:          AMD Instinct MI355X
  Vendor Name:             AMD
  Node:                    3
  Device Type:             GPU
  Chip ID:                 30115(0x75a3)
  Compute Unit:            256
*** Done ***
"""


def _node(tmp_path, hives, **kw):
    root = tmp_path / "node"
    G.synthetic_kfd_tree(str(root / "kfd"), hives, **kw)
    return str(root)


# -- parsers -----------------------------------------------------------------------------------
def test_kfd_topology_devices_hives_and_xgmi_links(tmp_path):
    inv = G.discover(env={}, fixture_dir=_node(tmp_path, [0xA1] * 4 + [0xB2] * 4))
    assert inv.count == 8 and inv.source == "kfd"
    d0 = inv.devices[0]
    assert (d0.arch, d0.model, d0.compute_units, d0.kfd_node) == ("gfx950", "MI355X", 256, 2)
    assert d0.vram_mib == 288 * 1024 and d0.bdf == "0000:05:00.0"
    assert inv.hives() == {"a1": [0, 1, 2, 3], "b2": [4, 5, 6, 7]}
    assert d0.xgmi_peers == (1, 2, 3) and inv.devices[5].xgmi_peers == (4, 6, 7)
    assert inv.attributes() == {"gpu_vendor": "amd", "gpu_model": "MI355X", "gpu_arch": "gfx950",
                                "xgmi_hive": "a1+b2"}
    assert inv.subset([4, 5]).attributes()["xgmi_hive"] == "b2"
    assert G.GpuInventory.from_dict(json.loads(json.dumps(inv.to_dict()))).devices == inv.devices


def test_gfx_target_version_and_models():
    assert G.arch_from_gfx_target_version(90500) == "gfx950"
    assert G.arch_from_gfx_target_version(90402) == "gfx942"
    assert G.arch_from_gfx_target_version(90010) == "gfx90a"
    assert G.model_from_market_name("AMD Instinct MI355X") == "MI355X"
    assert G.model_from_market_name("AMD Instinct MI300X VF") == "MI300X"


def test_gpu_without_hive_and_unknown_device(tmp_path):
    inv = G.discover(env={}, fixture_dir=_node(tmp_path, [0, 0], device_id=0x1234))
    assert [d.hive for d in inv.devices] == [G.NO_HIVE, G.NO_HIVE]
    assert inv.devices[0].xgmi_peers == () and inv.devices[0].model == "MI350"   # gfx950 family
    assert inv.attributes()["xgmi_hive"] == G.NO_HIVE


def test_amd_smi_static_json():
    inv = G.parse_amd_smi_static(AMD_SMI_STATIC)
    assert inv.count == 8 and inv.source == "amd-smi"
    d = inv.devices[3]
    assert (d.index, d.model, d.arch, d.compute_units, d.device_id) == (3, "MI355X", "gfx950", 256, 0x75A3)
    assert d.bdf == "0000:35:00.0" and d.vram_mib == 294896
    assert G.parse_amd_smi_static(json.dumps({"gpu_data": json.loads(AMD_SMI_STATIC)[:2]})).count == 2


def test_rocminfo_gpu_agents():
    inv = G.parse_rocminfo(ROCMINFO)
    # (rocminfo's "Node" numbers the runtime's agents, not KFD topology nodes: not kept)
    assert [(d.index, d.arch, d.model, d.kfd_node, d.compute_units) for d in inv.devices] == [
        (0, "gfx950", "MI355X", None, 256), (1, "gfx950", "MI355X", None, 256)]
    assert inv.devices[0].device_id == 0x75A3


def test_kfd_wiring_refined_by_amd_smi_name(tmp_path):
    node = _node(tmp_path, [0xA1] * 8, device_id=0x1234)   # KFD alone cannot name the model
    with open(os.path.join(node, "amd_smi_static.json"), "w") as f:
        f.write(AMD_SMI_STATIC)
    inv = G.discover(env={}, fixture_dir=node)
    assert inv.source == "kfd+amd-smi"
    assert {d.model for d in inv.devices} == {"MI355X"} and inv.devices[7].xgmi_peers == (0, 1, 2, 3, 4, 5, 6)


def test_tools_only_when_there_is_no_kfd_tree(tmp_path):
    node = tmp_path / "tools-only"
    node.mkdir()
    (node / "rocminfo.txt").write_text(ROCMINFO)
    inv = G.discover(env={}, fixture_dir=str(node))
    assert inv.count == 2 and inv.source == "rocminfo"


def test_visible_devices_restrict_and_renumber(tmp_path):
    node = _node(tmp_path, [0xA1] * 4 + [0xB2] * 4)
    inv = G.discover(env={"ROCR_VISIBLE_DEVICES": "1,2,5,6", "HIP_VISIBLE_DEVICES": "1,2"}, fixture_dir=node)
    # ROCR picks physical 1,2,5,6 -> 0..3; HIP then picks 1,2 of those = physical 2 and 5
    assert [d.kfd_node for d in inv.devices] == [4, 7]
    assert [d.index for d in inv.devices] == [0, 1] and [d.hive for d in inv.devices] == ["a1", "b2"]
    assert inv.devices[0].xgmi_peers == ()   # its hive peers are not visible
    assert G.discover(env={"HIP_VISIBLE_DEVICES": ""}, fixture_dir=node).count == 8   # empty = unset


def test_visible_devices_by_uuid(tmp_path, caplog):
    """ROCm also takes ``GPU-<unique id>`` entries: they select the device with that KFD
    unique id; an entry no device matches leaves the inventory unfiltered, with a warning, instead
    of advertising zero GPUs."""
    node = _node(tmp_path, [0xA1] * 4 + [0xB2] * 4)
    full = G.discover(env={}, fixture_dir=node)
    u3, u6 = full.devices[3].unique_id, full.devices[6].unique_id
    assert u3 and u6
    inv = G.discover(env={"HIP_VISIBLE_DEVICES": f"GPU-{u6},GPU-{u3.upper()}"}, fixture_dir=node)
    assert [d.kfd_node for d in inv.devices] == [full.devices[6].kfd_node, full.devices[3].kfd_node]
    assert [d.index for d in inv.devices] == [0, 1]
    mixed = G.discover(env={"ROCR_VISIBLE_DEVICES": f"1,GPU-{u6}"}, fixture_dir=node)
    assert [d.kfd_node for d in mixed.devices] == [full.devices[1].kfd_node, full.devices[6].kfd_node]
    with caplog.at_level("WARNING"):
        unknown = G.discover(env={"HIP_VISIBLE_DEVICES": "GPU-deadbeefdeadbeef"}, fixture_dir=node)
    assert unknown.count == 8 and "cannot identify" in caplog.text


@pytest.mark.skipif(not os.path.isdir(BOX_FIXTURE), reason="no recorded MI355X box dump")
def test_recorded_mi355x_box_dump():
    """The dump of the MI355X box (one GPU granted of its node's eight): only the granted GPU's KFD
    properties are readable, its io_links show the node's seven xGMI links, amd-smi names the part
    ``AMD Instinct MI355 OAM`` (device 0x75a3)."""
    inv = G.discover(env={}, fixture_dir=BOX_FIXTURE)
    assert inv.count == 1 and inv.source.startswith("kfd")
    d = inv.devices[0]
    assert (d.arch, d.model, d.compute_units, d.vram_mib) == ("gfx950", "MI355X", 256, 294896)
    assert d.xgmi_links == 7 and d.xgmi_peers == () and d.hive not in ("", G.NO_HIVE)
    assert d.bdf == "0000:f4:00.0" and d.kfd_node == 6
    assert inv.attributes() == {"gpu_vendor": "amd", "gpu_model": "MI355X", "gpu_arch": "gfx950",
                                "xgmi_hive": d.hive}
    # the box's ROCR/HIP_VISIBLE_DEVICES=0 is already what the container was granted
    assert G.discover(env={"ROCR_VISIBLE_DEVICES": "0", "HIP_VISIBLE_DEVICES": "0"}, fixture_dir=BOX_FIXTURE).count == 1
    assert G.discover(env={"ROCR_VISIBLE_DEVICES": "5"}, fixture_dir=BOX_FIXTURE).count == 1
    # rocminfo alone: the same part, no wiring
    r = G.parse_rocminfo(open(os.path.join(BOX_FIXTURE, "rocminfo.txt")).read())
    assert [(x.arch, x.model, x.compute_units) for x in r.devices] == [("gfx950", "MI355X", 256)]


def test_restricted_kfd_tree_uses_amd_smi_list_and_link_graph(tmp_path):
    """No readable GPU properties at all: amd-smi enumerates the granted GPUs, ``amd-smi list``
    maps them to KFD nodes, and the still-readable xGMI links give hive and peers (the hive label
    is host + lowest node of the link component: hives never span hosts)."""
    node = _node(tmp_path, [0xA1] * 4 + [0xB2] * 4)
    for n in range(2, 10):
        open(os.path.join(node, "kfd", "nodes", str(n), "properties"), "w").close()
    granted = json.loads(AMD_SMI_STATIC)[:2]
    with open(os.path.join(node, "amd_smi_static.json"), "w") as f:
        json.dump({"gpu_data": granted}, f)
    with open(os.path.join(node, "amd_smi_list.json"), "w") as f:
        json.dump([{"gpu": 0, "node_id": 3}, {"gpu": 1, "node_id": 7}], f)
    inv = G.discover(env={"SDK_GPU_HOST_LABEL": "host-a"}, fixture_dir=node)
    assert inv.count == 2 and "kfd-links" in inv.source
    assert [(d.kfd_node, d.hive, d.xgmi_links) for d in inv.devices] == [(3, "host-a:2", 3), (7, "host-a:6", 3)]
    assert all(d.xgmi_peers == () for d in inv.devices)     # granted GPUs sit in different hives


# -- device selection --------------------------------------------------------------------------
HIVES = {i: ("a1" if i < 4 else "b2") for i in range(8)}


def test_select_devices_stays_inside_one_hive_best_fit():
    assert G.select_devices(range(8), 2, HIVES) == [0, 1]
    assert G.select_devices([0, 1, 2, 4, 5, 6, 7], 4, HIVES) == [4, 5, 6, 7]      # only b2 fits
    assert G.select_devices([0, 1, 2, 4, 5, 6, 7], 2, HIVES) == [0, 1]            # a1: fewest free that fit
    assert G.select_devices([3, 4, 5, 6, 7], 1, HIVES) == [3]                     # keep b2 whole
    assert G.select_devices([0, 4], 2, HIVES) == [0, 4]                            # no hive fits: spans
    assert G.select_devices([0, 1, 4], 3, HIVES) == [0, 1, 4]
    assert G.select_devices([2, 0, 1], 2) == [0, 1]                               # no topology
    with pytest.raises(ValueError):
        G.select_devices([0], 2, HIVES)


def test_select_devices_prefers_direct_xgmi_peers():
    # a partial mesh: 0-1 and 2-3 linked, 1-2 not
    peers = {0: (1,), 1: (0,), 2: (3,), 3: (2,)}
    hives = {i: "h" for i in range(4)}
    assert G.select_devices([1, 2, 3], 2, hives, peers) == [2, 3]


# -- placement on a live scheduler -------------------------------------------------------------
def _env(count, gpus=1, placement='[["hostname", "UNIQUE"]]'):
    from dcos_commons_amd.benchmarks.deploy_bench import helloworld_env

    env = helloworld_env(count, gpus, "true")
    env["HELLO_PLACEMENT"] = placement
    return env


def _deploy(agent_specs, env, timeout=30.0):
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_WAIT_S="0.5")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    master = LocalMaster(allocation_interval_s=0.05)
    for s in agent_specs:
        master.add_agent(s)
    runner = SchedulerRunner(SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw),
                             driver_factory=lambda s, i: LocalSchedulerDriver(master, s, i))
    runner.run(block=False)
    try:
        api = runner.framework_runner.api_server.router
        t0 = time.time()
        while api.get("/v1/plans/deploy").status != 200:
            if time.time() - t0 > timeout:
                raise AssertionError(api.get("/v1/plans/deploy").json())
            time.sleep(0.01)
        return master.placement()
    finally:
        runner.stop()
        master.shutdown()


@pytest.fixture
def two_hive_node(tmp_path):
    return G.discover(env={}, fixture_dir=_node(tmp_path, [0xA1] * 4 + [0xB2] * 4))


def test_agents_from_discovery_carry_model_and_hive(two_hive_node):
    specs = gpu_agent_specs(8, "auto", lambda i: f"gpu-agent-{i}", inventory=two_hive_node)
    assert [s.gpu_devices for s in specs] == [[i] for i in range(8)]
    assert [s.attributes["xgmi_hive"] for s in specs] == ["a1"] * 4 + ["b2"] * 4
    assert all(s.attributes["gpu_model"] == "MI355X" and s.gpus == 1 for s in specs)
    whole = AgentSpec.from_gpu_inventory("node", two_hive_node)
    assert whole.gpus == 8 and whole.attributes["xgmi_hive"] == "a1+b2"


def test_max_per_one_pins_eight_pods_one_to_one(two_hive_node):
    specs = gpu_agent_specs(8, "auto", lambda i: f"gpu-agent-{i}", inventory=two_hive_node, cpus=4, mem=8192,
                            disk=20000)
    placed = _deploy(specs, _env(8, placement='[["hostname", "MAX_PER", "1"]]'))
    hello = [p for p in placed if p["task"].startswith("hello-")]
    assert len(hello) == 8 and len({p["hostname"] for p in hello}) == 8
    dev_of = {s.hostname: s.gpu_devices for s in specs}
    assert all(p["gpu_devices"] == dev_of[p["hostname"]] for p in hello)


def test_group_by_hive_spreads_pods_evenly(two_hive_node):
    """``GROUP_BY`` with the number of hives (Marathon semantics, AbstractRoundRobinRule.java:56):
    without the count the rule cannot know a second hive exists before a pod lands there."""
    specs = gpu_agent_specs(8, "auto", lambda i: f"gpu-agent-{i}", inventory=two_hive_node, cpus=4, mem=8192,
                            disk=20000)
    placed = _deploy(specs, _env(4, placement='[["xgmi_hive", "GROUP_BY", "2"], ["hostname", "UNIQUE"]]'))
    hives = [p["attributes"]["xgmi_hive"] for p in placed if p["task"].startswith("hello-")]
    assert sorted(hives) == ["a1", "a1", "b2", "b2"]


def test_cluster_on_one_hive(two_hive_node):
    specs = gpu_agent_specs(8, "auto", lambda i: f"gpu-agent-{i}", inventory=two_hive_node, cpus=4, mem=8192,
                            disk=20000)
    placed = _deploy(specs, _env(3, placement='[["xgmi_hive", "CLUSTER", "b2"], ["hostname", "UNIQUE"]]'))
    hello = [p for p in placed if p["task"].startswith("hello-")]
    assert len(hello) == 3 and {p["attributes"]["xgmi_hive"] for p in hello} == {"b2"}
    assert all(p["gpu_devices"][0] >= 4 for p in hello)


def test_multi_gpu_pods_land_inside_one_hive(two_hive_node):
    """One 8-GPU node (two hives of 4) as one agent: four ``gpus: 2`` pods use all eight devices,
    and no pod's pair crosses a hive; two ``gpus: 4`` pods get one whole hive each."""
    node = AgentSpec.from_gpu_inventory("mi355x-node", two_hive_node, cpus=16, mem=65536, disk=100000)
    placed = _deploy([node], _env(4, gpus=2, placement='[["hostname", "MAX_PER", "4"]]'))
    pairs = [p["gpu_devices"] for p in placed if p["task"].startswith("hello-")]
    assert sorted(d for pair in pairs for d in pair) == list(range(8))
    assert all(len({HIVES[d] for d in pair}) == 1 for pair in pairs), pairs
    placed = _deploy([node], _env(2, gpus=4, placement='[["hostname", "MAX_PER", "2"]]'))
    quads = sorted(p["gpu_devices"] for p in placed if p["task"].startswith("hello-"))
    assert quads == [[0, 1, 2, 3], [4, 5, 6, 7]]
