"""MI355X device ops: HIP probe kernels behind a torch-tensor API.

The kernels live in ``csrc/probe_kernels.hip`` (MFMA bf16 GEMM, MFMA issue-rate loop, HBM
streaming copy, HBM pattern test) and are compiled for gfx950 into the in-tree
``_amdprobe.so`` (``python -m dcos_commons_amd.ops.build``). They back the GPU readiness/health
check that gates pods which request ``gpus`` (``dcos_commons_amd.ops.gpu_health``).

There is deliberately no PyTorch fallback: on a machine with a GPU, a missing or stale
extension raises ``ProbeUnavailable`` instead of silently running something else.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_amdprobe.so")
_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()

GEMM_TILE_M = 128
GEMM_TILE_N = 128
GEMM_TILE_K = 64


class ProbeUnavailable(RuntimeError):
    pass


class ProbeError(RuntimeError):
    pass


def _bind(lib: ctypes.CDLL) -> None:
    vp, i, sz, f, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_float, ctypes.c_double
    lib.amdprobe_version.restype = i
    lib.amdprobe_gemm_bf16_nt.argtypes = [vp, vp, vp, i, i, i, vp]
    lib.amdprobe_gemm_bf16_nt.restype = i
    lib.amdprobe_gemm_bf16_nt_variant.argtypes = [vp, vp, vp, i, i, i, i, vp]
    lib.amdprobe_gemm_bf16_nt_variant.restype = i
    lib.amdprobe_mfma_peak.argtypes = [vp, i, i, f, vp]
    lib.amdprobe_mfma_peak.restype = i
    lib.amdprobe_mfma_peak_flops.argtypes = [i, i]
    lib.amdprobe_mfma_peak_flops.restype = d
    lib.amdprobe_hbm_copy.argtypes = [vp, vp, sz, i, vp]
    lib.amdprobe_hbm_copy.restype = i
    lib.amdprobe_pattern_write.argtypes = [vp, sz, ctypes.c_uint, i, vp]
    lib.amdprobe_pattern_write.restype = i
    lib.amdprobe_pattern_check.argtypes = [vp, sz, ctypes.c_uint, vp, i, vp]
    lib.amdprobe_pattern_check.restype = i
    lib.amdprobe_gemm_check.argtypes = [vp, vp, vp, i, i, i, i, vp, vp]
    lib.amdprobe_gemm_check.restype = i
    lib.amdprobe_readiness_fill.argtypes = [vp, sz, ctypes.c_uint, vp, vp]
    lib.amdprobe_readiness_fill.restype = i
    lib.amdprobe_readiness.argtypes = [i, ctypes.c_uint, i, ctypes.POINTER(d), ctypes.POINTER(ctypes.c_ulonglong)]
    lib.amdprobe_readiness.restype = i


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ProbeUnavailable(f"{LIB_PATH} is not built; run `python -m dcos_commons_amd.ops.build`")
                l = ctypes.CDLL(LIB_PATH)
                _bind(l)
                _lib = l
    return _lib


def _stream(device=None):
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _check(rc: int, what: str) -> None:
    if rc == -1:
        raise ProbeError(f"{what}: shape rejected by the kernel's launch contract")
    if rc == -2:
        raise ProbeError(f"{what}: operands must be 16-byte aligned")
    if rc != 0:
        raise ProbeError(f"{what}: HIP error {rc}")


GEMM_VARIANTS = {"auto": 0, "tile128": 1, "glds256": 2}


def gemm_bf16_nt(a, bt, out=None, variant: str = "auto"):
    """``a[M,K] @ bt[N,K]^T`` in fp32 on an MFMA kernel (M, N % 128 == 0, K % 64 == 0).

    ``auto`` runs the 256x256 LDS-DMA pipelined kernel when M, N % 256 == 0 and K % 128 == 0 and
    the 128x128 register-staged kernel otherwise; ``tile128`` / ``glds256`` force one."""
    import torch

    if a.dtype != torch.bfloat16 or bt.dtype != torch.bfloat16:
        raise ProbeError("gemm_bf16_nt expects bf16 operands")
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ProbeError(f"gemm_bf16_nt shape mismatch: {tuple(a.shape)} x {tuple(bt.shape)}^T")
    m, k = a.shape
    n = bt.shape[0]
    if m % GEMM_TILE_M or n % GEMM_TILE_N or k % GEMM_TILE_K:
        raise ProbeError(f"gemm_bf16_nt needs M,N % 128 == 0 and K % 64 == 0, got {m}x{n}x{k}")
    a, bt = a.contiguous(), bt.contiguous()
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    if variant not in GEMM_VARIANTS:
        raise ProbeError(f"unknown GEMM variant {variant!r}: {sorted(GEMM_VARIANTS)}")
    _check(lib().amdprobe_gemm_bf16_nt_variant(a.data_ptr(), bt.data_ptr(), out.data_ptr(), m, n, k,
                                               GEMM_VARIANTS[variant], _stream(a.device)), "gemm_bf16_nt")
    return out


def mfma_peak(device=0, blocks: int = 2048, iters: int = 2048):
    """Runs the MFMA issue-rate loop; returns (elapsed_s, flops)."""
    import torch

    out = torch.empty(blocks * 256, dtype=torch.float32, device=device)
    s = _stream(out.device)
    # warm-up launch
    _check(lib().amdprobe_mfma_peak(out.data_ptr(), blocks, 8, 1.0, s), "mfma_peak")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _check(lib().amdprobe_mfma_peak(out.data_ptr(), blocks, iters, 1.0, s), "mfma_peak")
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3, lib().amdprobe_mfma_peak_flops(blocks, iters)


def hbm_copy(src, dst, blocks: int = 4096):
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nbytes:
        raise ProbeError("hbm_copy destination too small")
    _check(lib().amdprobe_hbm_copy(src.data_ptr(), dst.data_ptr(), nbytes, blocks, _stream(src.device)), "hbm_copy")


def pattern_write(buf, seed: int, blocks: int = 2048):
    nbytes = buf.numel() * buf.element_size()
    _check(lib().amdprobe_pattern_write(buf.data_ptr(), nbytes, seed & 0xFFFFFFFF, blocks, _stream(buf.device)),
           "pattern_write")


def pattern_check(buf, seed: int, blocks: int = 2048) -> int:
    import torch

    nbytes = buf.numel() * buf.element_size()
    errs = torch.zeros(1, dtype=torch.int64, device=buf.device)
    _check(lib().amdprobe_pattern_check(buf.data_ptr(), nbytes, seed & 0xFFFFFFFF, errs.data_ptr(), blocks,
                                        _stream(buf.device)), "pattern_check")
    return int(errs.item())


def gemm_check(a, bt, c, inject: int = 0):
    """Dense check of ``c == a @ bt.T`` on the GPU (an fp32 VALU reference per element): returns
    ``(sum((c - a bt^T)^2), sum((a bt^T)^2))``. M, N % 16 == 0, K % 8 == 0, K <= 1024."""
    import torch

    m, k = a.shape
    n = bt.shape[0]
    if a.dtype != torch.bfloat16 or bt.dtype != torch.bfloat16 or c.dtype != torch.float32 or \
            tuple(c.shape) != (m, n) or bt.shape[1] != k:
        raise ProbeError(f"gemm_check: bad operands {tuple(a.shape)} {tuple(bt.shape)} {tuple(c.shape)}")
    a, bt, c = a.contiguous(), bt.contiguous(), c.contiguous()
    out = torch.zeros(4, dtype=torch.float32, device=a.device)
    _check(lib().amdprobe_gemm_check(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, inject, out.data_ptr(),
                                     _stream(a.device)), "gemm_check")
    o = out.cpu()
    return float(o[0]), float(o[1])


def readiness_fill(ab, seed: int):
    """The readiness operand fill into ``ab`` (any dtype, byte size % 16)."""
    import torch

    res = torch.empty(8, dtype=torch.int32, device=ab.device)
    _check(lib().amdprobe_readiness_fill(ab.data_ptr(), ab.numel() * ab.element_size(), seed & 0xFFFFFFFF,
                                         res.data_ptr(), _stream(ab.device)), "readiness_fill")


READINESS_SHAPE = (256, 256, 512)   # M, N, K of the readiness GEMM (csrc/probe_api.hip)
READINESS_PATTERN_BYTES = 64 << 20


def readiness(device: int = 0, seed: int = 0, inject: int = 0):
    """The whole readiness check of one device in one native call (no framework ops): hashed bf16
    operands, the MFMA GEMM, a dense fp32 check of every product element and the 64 MiB HBM
    pattern test on a private stream, then one 32-byte read-back. Returns ``(gemm_rel_err, bad_words)``. ``inject`` = 1 or
    2 plants a product / memory fault, 3 / 4 skips the GEMM / pattern write (tests). Each call mixes
    a call counter into ``seed``, so stale buffers from an earlier call never verify. The GIL is released for the duration (ctypes)."""
    rel = ctypes.c_double(0.0)
    bad = ctypes.c_ulonglong(0)
    _check(lib().amdprobe_readiness(int(device), seed & 0xFFFFFFFF, int(inject), ctypes.byref(rel),
                                    ctypes.byref(bad)), "readiness")
    return rel.value, int(bad.value)


def require_native_on_gpu() -> None:
    """Raise if a GPU is present but the HIP extension is not loadable (no silent fallback)."""
    import torch

    if torch.cuda.is_available():
        lib()
