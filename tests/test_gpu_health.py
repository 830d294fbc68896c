"""GPU readiness-check logic that runs without a device (the kernels are covered by test_gpu_ops)."""


def test_freivalds_check_matches_dense_reference():
    import torch

    from dcos_commons_amd.ops.gpu_health import MAX_GEMM_REL_ERR, freivalds_rel_err

    g = torch.Generator().manual_seed(7)
    a = torch.randn((256, 512), generator=g).to(torch.bfloat16)
    bt = torch.randn((256, 512), generator=g).to(torch.bfloat16)
    c = a.float() @ bt.float().t()
    assert freivalds_rel_err(a, bt, c, g) < 1e-5
    bad = c.clone()
    bad[32:48, 64:80] = 0  # one 16x16 MFMA tile lost
    dense = float(torch.linalg.norm(bad - c) / torch.linalg.norm(c))
    projected = freivalds_rel_err(a, bt, bad, g)
    assert dense > MAX_GEMM_REL_ERR and projected > MAX_GEMM_REL_ERR
    assert 0.3 < projected / dense < 3


def test_readiness_probe_runs_its_kernels_on_the_requested_device(monkeypatch):
    """the readiness probe makes its device current for the HIP launches and restores
    the caller's device afterwards (gpu_health.py ``torch.cuda.device(dev)``). The one-GPU box
    cannot show this (``test_readiness_probe_on_a_non_default_device`` skips there), so the device
    bookkeeping is checked here with the CUDA runtime replaced by a recorder. The multi-GPU
    hardware path itself stays unverified until a multi-GPU run exists."""
    import contextlib

    import torch

    from dcos_commons_amd import ops
    from dcos_commons_amd.ops import gpu_health

    current = {"dev": 0}
    seen = []

    @contextlib.contextmanager
    def fake_device(dev):
        idx = dev.index if isinstance(dev, torch.device) else int(dev)
        prev, current["dev"] = current["dev"], idx
        try:
            yield
        finally:
            current["dev"] = prev

    real_gen, real_randn, real_empty = torch.Generator, torch.randn, torch.empty

    def on_cpu(fn):
        def wrapped(*a, **kw):
            kw.pop("device", None)
            return fn(*a, **kw)
        return wrapped

    def gemm(a, bt):
        seen.append(("gemm", current["dev"]))
        return a.float() @ bt.float().t()

    def pattern_write(buf, seed):
        seen.append(("write", current["dev"]))

    def pattern_check(buf, seed):
        seen.append(("check", current["dev"]))
        return 0

    monkeypatch.setattr(torch.cuda, "device", fake_device)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: current["dev"])
    monkeypatch.setattr(torch, "Generator", on_cpu(real_gen))
    monkeypatch.setattr(torch, "randn", on_cpu(real_randn))
    monkeypatch.setattr(torch, "empty", lambda *a, **kw: real_empty(8, dtype=kw.get("dtype")))
    monkeypatch.setattr(ops, "gemm_bf16_nt", gemm)
    monkeypatch.setattr(ops, "pattern_write", pattern_write)
    monkeypatch.setattr(ops, "pattern_check", pattern_check)

    current["dev"] = 2  # the caller's device
    rep = gpu_health.readiness_probe(device=5)
    assert rep["healthy"] and rep["device"] == 5
    assert seen == [("gemm", 5), ("write", 5), ("check", 5)]
    assert torch.cuda.current_device() == 2  # restored
