"""Interleaved A/B timing of the probe GEMM variants on uniform random [-1, 1) bf16 operands.

Rounds alternate the variants in one process (cdna_hip_programming.md §5.4 rule 24); prints one
JSON line per shape with the median and best TFLOP/s per variant and torch.matmul (hipBLASLt) as
the library reference on the same data.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dcos_commons_amd import ops


def time_ms(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for size in (int(x) for x in args.sizes.split(",")):
        m = n = k = size
        g = torch.Generator(device=dev)
        g.manual_seed(size)
        a = (torch.rand((m, k), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand((n, k), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty((m, n), device=dev, dtype=torch.float32)
        flop = 2.0 * m * n * k
        arms = {
            "glds256": lambda: ops.gemm_bf16_nt(a, bt, out, variant="glds256"),
            "tile128": lambda: ops.gemm_bf16_nt(a, bt, out, variant="tile128"),
            "torch_matmul_bf16out": lambda: torch.matmul(a, bt.t()),
        }
        res = {name: [] for name in arms}
        for _ in range(args.rounds):
            for name, fn in arms.items():
                res[name].append(flop / (time_ms(fn, args.reps) * 1e-3) / 1e12)
        ref = a.float() @ bt.float().t()
        ops.gemm_bf16_nt(a, bt, out, variant="glds256")
        torch.cuda.synchronize()
        rel = (torch.linalg.norm(out - ref) / torch.linalg.norm(ref)).item()
        print(json.dumps({"shape": [m, n, k], "rel_err_glds256": rel,
                          **{f"{name}_tflops_median": round(statistics.median(v), 1) for name, v in res.items()},
                          **{f"{name}_tflops_best": round(max(v), 1) for name, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
