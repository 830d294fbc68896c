"""GPU pods on the local cluster: MI355X agents, whole-GPU pods, readiness on the assigned device.

Reference: frameworks/helloworld/src/main/dist/gpu_resource.yml + the GPU_RESOURCES capability
(the only GPU surface of the reference is the ``gpus`` scalar). The MI355X build pins
each pod to devices of its agent and the agent exports them to the task as
``HIP_VISIBLE_DEVICES``/``ROCR_VISIBLE_DEVICES``. On CPU the readiness command checks that export;
on the GPU box (``-m gpu``) it is the real HIP probe (MFMA GEMM numerics + HBM pattern) running in
the task process on the device the agent assigned.
"""
import os

import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_plan, sdk_tasks
from tests.integration.conftest import make_cluster

PACKAGE = "hello-world"


def _gpu_options(count, probe_command=None):
    opts = {"service": {"yaml": "gpu", "mi355x_probe": {"quick": True}},
            "hello": {"count": count, "gpus": 1, "placement": '[["hostname", "MAX_PER", "2"]]'}}
    if probe_command is not None:
        opts["service"]["mi355x_probe"]["command"] = probe_command
    return opts


def test_gpu_pods_get_distinct_devices_exported():
    c = make_cluster(agents=2, gpus_per_agent=2)
    try:
        svc = "hello-gpu"
        sdk_install.install(PACKAGE, svc, 4, additional_options=_gpu_options(
            4, probe_command='test -n "$HIP_VISIBLE_DEVICES" -a "$HIP_VISIBLE_DEVICES" = "$ROCR_VISIBLE_DEVICES"'))
        tasks = sdk_tasks.get_service_tasks(svc)
        assert len(tasks) == 4
        seen = set()
        for t in tasks:
            rc, out, _ = sdk_cmd.service_task_exec(svc, t.name, 'echo "$HIP_VISIBLE_DEVICES"')
            assert rc == 0
            seen.add((t.host, out.strip()))
            assert t.resources["gpus"] == 1.0
        # 2 agents x 2 devices: every pod has its own device
        assert seen == {(h, d) for h in {t.host for t in tasks} for d in ("0", "1")}
        fw = [f for f in c.frameworks() if f["name"] == svc]
        assert fw
        sdk_install.uninstall(PACKAGE, svc)
    finally:
        c.shutdown()


@pytest.mark.gpu
def test_gpu_pod_readiness_runs_the_hip_probe_on_its_device():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dcos_commons_amd import ops

    ops.lib()   # the probe extension must be built in-tree: a missing one is a failure
    n = torch.cuda.device_count()
    c = make_cluster(agents=1, gpus_per_agent=n)
    try:
        svc = "hello-mi355x"
        sdk_install.install(PACKAGE, svc, 1, additional_options=_gpu_options(1), timeout_seconds=240)
        plan = sdk_plan.get_deployment_plan(svc)
        assert plan["status"] == "COMPLETE"
        task = sdk_tasks.get_service_tasks(svc)[0]
        rc, out, _ = sdk_cmd.service_task_exec(svc, task.name, 'echo "$HIP_VISIBLE_DEVICES"')
        assert rc == 0 and out.strip() in {str(i) for i in range(n)}
        # the readiness command itself, re-run in the task: healthy JSON report for device 0 of the task
        rc, out, err = sdk_cmd.service_task_exec(
            svc, task.name, "python3 -m dcos_commons_amd.ops.gpu_health --device 0 --readiness --json")
        assert rc == 0, err
        assert '"healthy": true' in out
        sdk_install.uninstall(PACKAGE, svc)
    finally:
        c.shutdown()
