"""Interleaved A/B of scheduler flag profiles on DeployBench (synthetic readiness): medians of
deploy / restart / replace wall-clock per agent count. Used to decide whether a scheduler change
pays off on a quiet machine (the GPU box), since the build container's CPU timing is noisy.

    python scripts/ab_profiles.py --agents 1 8 --reps 15 --profile base= --profile nostream=SDK_STREAM_LAUNCHES=false
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dcos_commons_amd.benchmarks import deploy_bench as DB  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--profile", action="append", default=[],
                    help="NAME=K1=V1,K2=V2 (scheduler env overrides on top of the mi355x profile)")
    args = ap.parse_args()
    profiles = {}
    for spec in args.profile or ["base="]:
        name, _, kvs = spec.partition("=")
        env = dict(DB.PROFILES["mi355x"])
        for kv in filter(None, kvs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        DB.PROFILES["ab-" + name] = env
        profiles[name] = "ab-" + name
    for n in args.agents:
        benches = {name: DB.DeployBench(n, profile=p, allocation_interval_s=1.0) for name, p in profiles.items()}
        for b in benches.values():
            b.run_cycle()
        res = {name: [] for name in profiles}
        for _ in range(args.reps):
            for name, b in benches.items():
                res[name].append(b.run_cycle())
        for name, rs in res.items():
            print(json.dumps({"profile": name, "agents": n, "reps": args.reps,
                              "deploy_ms": round(statistics.median(r.deploy_s for r in rs) * 1000, 3),
                              "restart_ms": round(statistics.median(r.mttr_restart_s for r in rs) * 1000, 3),
                              "replace_ms": round(statistics.median(r.mttr_replace_s for r in rs) * 1000, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
