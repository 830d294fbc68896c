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
