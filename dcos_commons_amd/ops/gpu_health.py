"""GPU readiness/health check for pods that are given MI355X GPUs.

Runs the HIP probe kernels on one device and decides healthy / unhealthy:

* **MFMA GEMM numerics** -- bf16 ``C = A @ Bt^T`` on the probe GEMM (256x256 LDS-DMA pipeline
  where the shape tiles, else 128x128) checked against the same bf16 values in fp32: the full
  probe compares with a dense fp32 matmul, the readiness probe with an fp32 VALU reference of
  every element computed on the device (``ops.readiness``, one native call). Relative error
  must stay < 1e-3;
* **MFMA rate** -- register-resident ``v_mfma_f32_32x32x16_bf16`` loop (TFLOP/s);
* **HBM** -- 16-B/lane streaming copy of a buffer larger than the 256 MiB Infinity Cache
  (read+write GB/s) and an address-hashed write/verify pattern (bad words must be 0).

``python -m dcos_commons_amd.ops.gpu_health --device 0 --json`` prints the report and exits 0
only when healthy; it is the readiness-check command used for GPU pods.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

MIN_TFLOPS = 200.0       # far below the ~2.5 PF dense peak: catches a broken/throttled matrix pipe
MIN_HBM_GBPS = 1000.0    # far below the ~5.5 TB/s measured copy rate: catches a degraded stack
MAX_GEMM_REL_ERR = 1e-3


def readiness_probe(device: int = 0) -> dict:
    """The fast form used as a pod readiness check: numerics + memory integrity only, as ONE
    native call (``ops.readiness``): hashed bf16 operands, the MFMA GEMM, a dense fp32 check of
    every product element and the 64 MiB pattern test on a private stream with a single read-back. It sits on the deploy and
    recovery critical path of every GPU pod, and the GIL is released while it runs."""
    from dcos_commons_amd import ops

    t0 = time.perf_counter()
    rel, bad = ops.readiness(device, seed=4321 + device)
    return {"device": device, "gemm_rel_err": rel, "mem_bad_words": bad,
            "healthy": bool(rel < MAX_GEMM_REL_ERR and bad == 0), "probe_seconds": round(time.perf_counter() - t0, 4)}


def run_probe(device: int = 0, quick: bool = True) -> dict:
    import torch

    from dcos_commons_amd import ops

    t_start = time.perf_counter()
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    props = torch.cuda.get_device_properties(dev)
    report = {"device": device, "name": props.name, "arch": getattr(props, "gcnArchName", ""),
              "total_mem_gib": round(props.total_memory / 2**30, 1), "cus": props.multi_processor_count}
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + device)

    # 1. MFMA GEMM numerics
    m = n = 512 if quick else 2048
    k = 1024 if quick else 4096
    a = torch.randn((m, k), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
    bt = torch.randn((n, k), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
    c = ops.gemm_bf16_nt(a, bt)
    ref = a.float() @ bt.float().t()
    rel = float(torch.linalg.norm(c - ref) / torch.linalg.norm(ref))
    report["gemm_rel_err"] = rel

    # GEMM throughput on a square shape
    s = 2048 if quick else 8192
    a2 = torch.randn((s, s), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
    b2 = torch.randn((s, s), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
    out = torch.empty((s, s), dtype=torch.float32, device=dev)
    ops.gemm_bf16_nt(a2, b2, out)
    reps = 5 if quick else 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.gemm_bf16_nt(a2, b2, out)
    e1.record()
    e1.synchronize()
    report["gemm_tflops"] = round(2.0 * s * s * s * reps / (e0.elapsed_time(e1) / 1e3) / 1e12, 1)
    del a2, b2, out

    # 2. MFMA issue rate
    secs, flops = ops.mfma_peak(device, blocks=2048, iters=512 if quick else 4096)
    report["mfma_tflops"] = round(flops / secs / 1e12, 1)

    # 3. HBM bandwidth (buffers larger than the Infinity Cache)
    nbytes = (512 if quick else 2048) * 2**20
    src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    dst = torch.empty_like(src)
    ops.pattern_write(src, seed=7)
    ops.hbm_copy(src, dst)
    reps = 5
    e0.record()
    for _ in range(reps):
        ops.hbm_copy(src, dst)
    e1.record()
    e1.synchronize()
    report["hbm_copy_gbps"] = round(2.0 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9, 1)

    # 4. HBM integrity: the copy must preserve the pattern, and a fresh pattern must verify
    bad = ops.pattern_check(dst, seed=7)
    ops.pattern_write(src, seed=99)
    bad += ops.pattern_check(src, seed=99)
    report["mem_bad_words"] = bad
    del src, dst
    torch.cuda.synchronize(dev)

    report["healthy"] = bool(rel < MAX_GEMM_REL_ERR and bad == 0 and report["mfma_tflops"] > MIN_TFLOPS and
                             report["hbm_copy_gbps"] > MIN_HBM_GBPS)
    report["probe_seconds"] = round(time.perf_counter() - t_start, 3)
    return report


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--full", action="store_true", help="larger shapes (slower, more precise)")
    ap.add_argument("--readiness", action="store_true", help="fast numerics + memory check only")
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args(argv)
    rep = readiness_probe(args.device) if args.readiness else run_probe(args.device, quick=not args.full)
    print(json.dumps(rep) if args.json else "\n".join(f"{k}: {v}" for k, v in rep.items()))
    return 0 if rep["healthy"] else 1


if __name__ == "__main__":
    sys.exit(main())
