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


@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (512, 768, 384), (768, 512, 256), (1024, 1024, 2048),
                                   (2048, 256, 1152)])
def test_gemm_glds256_matches_fp32_reference(dev, m, n, k):
    """256x256 LDS-DMA pipeline: one-iteration (K=128), odd iteration counts, rectangular grids."""
    from dcos_commons_amd import ops

    g = torch.Generator(device=dev)
    g.manual_seed(m + 3 * n + 11 * k)
    a = (torch.rand((m, k), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand((n, k), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    c = ops.gemm_bf16_nt(a, bt, variant="glds256")
    ref = a.float() @ bt.float().t()
    torch.cuda.synchronize()
    rel = (torch.linalg.norm(c - ref) / torch.linalg.norm(ref)).item()
    assert rel < 1e-5, rel
    c128 = ops.gemm_bf16_nt(a, bt, variant="tile128")
    assert torch.allclose(c, c128, rtol=1e-4, atol=1e-3)


def test_gemm_glds256_exact_integer_layout(dev):
    """Exact small-integer products pin every row/column of the interleaved wave decomposition."""
    from dcos_commons_amd import ops

    m, n, k = 512, 768, 256
    a = ((torch.arange(m, device=dev).view(m, 1) * 7 + torch.arange(k, device=dev).view(1, k)) % 5 - 2).float()
    bt = ((torch.arange(n, device=dev).view(n, 1) * 3 + torch.arange(k, device=dev).view(1, k) * 11) % 7 - 3).float()
    c = ops.gemm_bf16_nt(a.to(torch.bfloat16), bt.to(torch.bfloat16), variant="glds256")
    assert torch.equal(c, a @ bt.t())


def test_gemm_rejects_bad_shapes(dev):
    from dcos_commons_amd import ops

    a = torch.zeros((100, 64), device=dev, dtype=torch.bfloat16)
    with pytest.raises(ops.ProbeError):
        ops.gemm_bf16_nt(a, a)
    b = torch.zeros((256, 64), device=dev, dtype=torch.bfloat16)  # K % 128 != 0
    with pytest.raises(ops.ProbeError):
        ops.gemm_bf16_nt(b, b, variant="glds256")
    assert ops.gemm_bf16_nt(b, b).shape == (256, 256)  # auto falls back to the 128 kernel


@pytest.mark.parametrize("n,blocks", [(4, 4096), (4 * 1023 + 4, 7), (4 * 1024 * 5, 1), (4 * 300001, 4096)])
def test_hbm_copy_spans_and_tails(dev, n, blocks):
    from dcos_commons_amd import ops

    src = torch.randint(-2**31, 2**31 - 1, (n,), device=dev, dtype=torch.int32)
    dst = torch.zeros(n + 64, device=dev, dtype=torch.int32)
    ops.hbm_copy(src, dst[:n], blocks=blocks)
    assert torch.equal(src, dst[:n]) and not dst[n:].any()  # nothing written past the end


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


def test_readiness_probe_on_a_non_default_device(dev):
    """the readiness probe must make its device current before launching (the HIP
    kernels run on the current device's stream)."""
    from dcos_commons_amd.ops.gpu_health import readiness_probe

    if torch.cuda.device_count() < 2:
        pytest.skip("needs a second visible GPU")
    torch.cuda.set_device(0)
    rep = readiness_probe(1)
    assert rep["healthy"], rep
    assert torch.cuda.current_device() == 0       # the caller's current device is restored


# ---------------------------------------------------------------------------------------
# fused readiness path (csrc/probe_kernels.hip readiness_prep_kernel / gemm_check_kernel,
# csrc/probe_api.hip amdprobe_readiness)


@pytest.mark.parametrize("m,n,k", [(256, 256, 512), (16, 48, 8), (128, 384, 64), (512, 128, 1024)])
def test_gemm_check_kernel_matches_fp32_reference(dev, m, n, k):
    from dcos_commons_amd import ops

    g = torch.Generator(device=dev)
    g.manual_seed(m + 3 * n + 7 * k)
    a = torch.randn((m, k), generator=g, device=dev).to(torch.bfloat16)
    bt = torch.randn((n, k), generator=g, device=dev).to(torch.bfloat16)
    ref = a.float() @ bt.float().t()
    d2, w2 = ops.gemm_check(a, bt, ref)
    ref_w2 = float((ref * ref).sum())
    assert abs(w2 - ref_w2) / ref_w2 < 1e-4
    assert (d2 / w2) ** 0.5 < 1e-5                     # an exact product passes
    bad = ref.clone()
    bad[:16, :16] = 0                                  # one lost MFMA tile
    ref_d2 = float((ref[:16, :16] ** 2).sum())
    d2b, _ = ops.gemm_check(a, bt, bad)
    assert abs(d2b - ref_d2) / ref_d2 < 1e-3
    d2i, _ = ops.gemm_check(a, bt, ref, inject=1)      # the planted fault: the same tile read as zeros
    assert abs(d2i - ref_d2) / ref_d2 < 1e-3
    with pytest.raises(ops.ProbeError):
        ops.gemm_check(a[:, :k - 1].contiguous() if k > 8 else a, bt[:, :k - 1].contiguous() if k > 8 else bt[:8],
                       ref)


def _mix32(v):
    import numpy as np

    v = v ^ (v >> np.uint64(33))
    v = v * np.uint64(0xFF51AFD7ED558CCD)
    v = v ^ (v >> np.uint64(33))
    v = v * np.uint64(0xC4CEB9FE1A85EC53)
    v = v ^ (v >> np.uint64(33))
    return (v & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def test_readiness_fill_matches_the_host_hash(dev):
    import numpy as np

    from dcos_commons_amd import ops

    seed = 4321
    ab = torch.empty(4096, dtype=torch.int32, device=dev)      # 1024 chunks of 16 B
    ops.readiness_fill(ab, seed)
    torch.cuda.synchronize()
    with np.errstate(over="ignore"):
        i = np.arange(1024, dtype=np.uint64)
        base = (i << np.uint64(2)) ^ (np.uint64(seed) << np.uint64(40))
        words = np.stack([_mix32(base + np.uint64(j)) for j in range(4)], axis=1).reshape(-1)
        words = (words & np.uint32(0x807F807F)) | np.uint32(0x3F003F00)
    assert np.array_equal(ab.cpu().numpy().view(np.uint32), words)
    vals = ab.view(torch.bfloat16).float().abs()
    assert bool(((vals >= 0.5) & (vals < 1.0)).all())


def test_fused_readiness_passes_and_catches_planted_faults(dev):
    import time

    from dcos_commons_amd import ops
    from dcos_commons_amd.ops.gpu_health import MAX_GEMM_REL_ERR

    rel, bad = ops.readiness(0, seed=4321)
    assert rel < 1e-4 and bad == 0
    again = ops.readiness(0, seed=4321)               # fresh operands and pattern (call counter in the seed)
    assert again[1] == 0 and again[0] < 1e-4
    rel1, bad1 = ops.readiness(0, seed=4321, inject=1)
    assert rel1 > MAX_GEMM_REL_ERR and bad1 == 0
    rel2, bad2 = ops.readiness(0, seed=4321, inject=2)
    assert rel2 < 1e-4 and bad2 >= 1
    # a GEMM or pattern write that silently drops its stores must not pass on the previous call's data
    rel3, bad3 = ops.readiness(0, seed=4321, inject=3)
    assert rel3 > MAX_GEMM_REL_ERR and bad3 == 0
    rel4, bad4 = ops.readiness(0, seed=4321, inject=4)
    assert rel4 < 1e-4 and bad4 > 1000
    rel5, bad5 = ops.readiness(0, seed=4321)                    # healthy again
    assert rel5 < 1e-4 and bad5 == 0
    assert ops.readiness(0, seed=7)[1] == 0
    with pytest.raises(ops.ProbeError):
        ops.readiness(torch.cuda.device_count(), seed=1)
    assert torch.cuda.current_device() == 0                     # the caller's device is kept
    t0 = time.perf_counter()
    for _ in range(20):
        ops.readiness(0, seed=4321)
    per_call_ms = (time.perf_counter() - t0) / 20 * 1e3
    print(f"fused readiness: {per_call_ms:.3f} ms per call")
    assert per_call_ms < 5.0


def test_fused_readiness_from_many_threads(dev):
    from concurrent.futures import ThreadPoolExecutor

    from dcos_commons_amd import ops

    with ThreadPoolExecutor(8) as pool:
        results = list(pool.map(lambda s: ops.readiness(0, seed=s), range(32)))
    assert all(rel < 1e-4 and bad == 0 for rel, bad in results)
