"""Runs the fused readiness probe N times on device 0 (a rocprofv3 --pmc target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dcos_commons_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for _ in range(n):
    rel, bad = ops.readiness(0, seed=4321)
print(f"readiness x{n}: rel_err={rel:.3e} bad_words={bad}")
