"""Numerics of the HIP probe kernels vs plain PyTorch fp32 references (MI355X only)."""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dcos_commons_amd import ops

    ops.lib()  # must load: a GPU box without the extension is a failure, not a skip
    return torch.device("cuda", 0)


@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (256, 384, 512), (1024, 512, 2048), (384, 1152, 192)])
def test_gemm_bf16_matches_fp32_reference(dev, m, n, k):
    from dcos_commons_amd import ops

    g = torch.Generator(device=dev)
    g.manual_seed(m * 31 + n * 7 + k)
    a = torch.randn((m, k), generator=g, device=dev).to(torch.bfloat16)
    bt = torch.randn((n, k), generator=g, device=dev).to(torch.bfloat16)
    c = ops.gemm_bf16_nt(a, bt)
    ref = a.float() @ bt.float().t()
    torch.cuda.synchronize()
    rel = (torch.linalg.norm(c - ref) / torch.linalg.norm(ref)).item()
    assert rel < 1e-5, rel
    assert torch.allclose(c, ref, rtol=1e-3, atol=1e-2)


def test_gemm_exact_integer_asymmetric(dev):
    """A = I-like selector with an asymmetric B catches row/col swaps in the epilogue."""
    from dcos_commons_amd import ops

    m, n, k = 128, 256, 128
    a = torch.zeros((m, k), device=dev)
    a[torch.arange(m), torch.arange(m) % k] = 1.0
    bt = (torch.arange(n, device=dev).view(n, 1) * 3 + torch.arange(k, device=dev).view(1, k) % 5).float()
    c = ops.gemm_bf16_nt(a.to(torch.bfloat16), bt.to(torch.bfloat16))
    ref = a @ bt.to(torch.bfloat16).float().t()
    assert torch.equal(c, ref)


def test_gemm_rejects_bad_shapes(dev):
    from dcos_commons_amd import ops

    a = torch.zeros((100, 64), device=dev, dtype=torch.bfloat16)
    with pytest.raises(ops.ProbeError):
        ops.gemm_bf16_nt(a, a)


def test_hbm_copy_and_pattern(dev):
    from dcos_commons_amd import ops

    src = torch.randint(-2**31, 2**31 - 1, (8 * 2**20 + 4,), device=dev, dtype=torch.int32)
    dst = torch.empty_like(src)
    ops.hbm_copy(src, dst)
    assert torch.equal(src, dst)
    ops.pattern_write(dst, seed=5)
    assert ops.pattern_check(dst, seed=5) == 0
    dst[12345] ^= 1
    assert ops.pattern_check(dst, seed=5) == 1
    assert ops.pattern_check(dst, seed=6) > 0


def test_mfma_peak_is_fast(dev):
    from dcos_commons_amd import ops

    secs, flops = ops.mfma_peak(0, blocks=1024, iters=256)
    assert flops / secs / 1e12 > 100.0


def test_gpu_health_reports_healthy(dev):
    from dcos_commons_amd.ops import gpu_health

    rep = gpu_health.run_probe(0, quick=True)
    assert rep["healthy"], rep
    r2 = gpu_health.readiness_probe(0)
    assert r2["healthy"], r2
