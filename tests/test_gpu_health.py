"""GPU readiness-check logic that runs without a device (the kernels are covered by test_gpu_ops)."""


def test_readiness_probe_is_one_native_call_on_the_requested_device(monkeypatch):
    """The readiness probe hands the whole check of ``device`` to ``ops.readiness`` (one native
    call that makes the device current for its launches and restores the caller's device,
    csrc/probe_api.hip ``DeviceGuard``) and judges the two numbers it returns. The device
    bookkeeping itself runs on the GPU box (test_gpu_ops); this pins the Python contract."""
    from dcos_commons_amd import ops
    from dcos_commons_amd.ops import gpu_health

    calls = []
    answers = iter([(2e-7, 0), (5e-3, 0), (2e-7, 3)])

    def fake_readiness(device, seed=0, inject=0):
        calls.append((device, seed, inject))
        return next(answers)

    monkeypatch.setattr(ops, "readiness", fake_readiness)
    healthy = gpu_health.readiness_probe(device=5)
    assert healthy["healthy"] and healthy["device"] == 5 and healthy["mem_bad_words"] == 0
    assert not gpu_health.readiness_probe(device=5)["healthy"]     # GEMM error above 1e-3
    assert not gpu_health.readiness_probe(device=5)["healthy"]     # bad memory words
    assert calls == [(5, 4326, 0)] * 3
