"""python scripts/dev/ab_deploy.py <repo> <n> <cycles> [--gpu]: helloworld DeployBench of the tree at
<repo>, pinned to CPUs 4-7. Readiness is a 0.2 ms GIL-free sleep, or with --gpu the tree's own HIP
probe on device 0 (every pod on the one card, as in the one-GPU rehearsal). Prints mean/median
deploy, MTTRs and process CPU per cycle."""
import json
import logging
import os
import sys
import time

repo = os.path.abspath(sys.argv[1])
sys.path.insert(0, repo)
os.chdir(repo)
logging.disable(logging.WARNING)
os.sched_setaffinity(0, [4, 5, 6, 7])
from dcos_commons_amd.benchmarks.deploy_bench import DeployBench  # noqa: E402

n = int(sys.argv[2])
gpu = "--gpu" in sys.argv
if gpu:
    from dcos_commons_amd.benchmarks.runner import gpu_check_runner  # noqa: E402

    runner = gpu_check_runner()
elif "--inline-fake" in sys.argv:
    def runner(task, devices):   # the fused probe's shape: one short GIL-releasing call, run inline
        time.sleep(0.00007)
        return True
    runner.inline = True
else:
    def runner(task, devices):
        time.sleep(0.0002)
        return True
b = DeployBench(n, check_runner=runner, gpu_devices=[0] * n)
for _ in range(3):
    b.run_cycle()
cs, ds, rs, ps = [], [], [], []
for _ in range(int(sys.argv[3])):
    c0 = time.process_time()
    r = b.run_cycle()
    cs.append(time.process_time() - c0)
    ds.append(r.deploy_s)
    rs.append(r.mttr_restart_s)
    ps.append(r.mttr_replace_s)


def m(x):
    return round(sum(x) / len(x) * 1000, 2)


def md(x):
    return round(sorted(x)[len(x) // 2] * 1000, 2)


print(json.dumps({"repo": repo, "n": n, "gpu": gpu, "cpu_ms": m(cs), "deploy_ms": m(ds), "deploy_med": md(ds),
                  "restart_ms": m(rs), "replace_ms": m(ps)}))
