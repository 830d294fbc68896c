"""MI355X node discovery on a real box (``ops.gpu.discover``): what the KFD topology, amd-smi and
rocminfo report must agree with what the HIP runtime (torch) sees, and it must be what the
agents advertise. The CPU suite covers the parsers with the recorded box output
(``tests/fixtures/gpu/mi355x_box``); this runs them against the live driver.
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def inventory():
    from dcos_commons_amd.ops import gpu as G

    G._LIVE_CACHE.clear()
    return G.discover()


def test_discovered_devices_match_the_hip_runtime(inventory):
    import torch

    assert torch.cuda.is_available()
    n = torch.cuda.device_count()
    assert inventory.count == n, inventory.to_dict()
    for i, dev in enumerate(inventory.devices):
        props = torch.cuda.get_device_properties(i)
        assert dev.index == i
        assert dev.arch == "gfx950", dev
        assert props.gcnArchName.startswith("gfx950")
        assert dev.vendor == "amd"
        assert dev.model == "MI355X", dev
        # compute units and HBM as the KFD topology reports them, against the runtime's view
        if dev.compute_units:
            assert dev.compute_units == props.multi_processor_count
        if dev.vram_mib:
            assert abs(dev.vram_mib * 2 ** 20 - props.total_memory) < 4 * 2 ** 30
            assert dev.vram_mib > 250 * 1024        # 288 GB HBM3E


def test_agents_advertise_what_was_discovered(inventory):
    from dcos_commons_amd.mesos.local_master import AgentSpec

    spec = AgentSpec.from_gpu_inventory("node-0", inventory)
    assert spec.gpus == inventory.count
    attrs = dict(spec.attributes)
    assert attrs["gpu_model"] == "MI355X" and attrs["gpu_arch"] == "gfx950" and attrs["gpu_vendor"] == "amd"
    assert attrs.get("xgmi_hive") == inventory.attributes().get("xgmi_hive")


def test_readiness_probe_runs_on_every_discovered_device(inventory):
    from dcos_commons_amd.benchmarks.runner import gpu_check_runner

    check = gpu_check_runner()
    for dev in inventory.devices:
        assert check(None, [dev.index]) is True
