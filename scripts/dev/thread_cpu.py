"""CPU time per thread over N-pod helloworld deploy cycles (in-process DeployBench, inline fake probe):
python scripts/dev/thread_cpu.py N [cycles]. Shows which thread (offer loop, master dispatcher, agent
check threads, API server, bench driver) spends the interpreter's time."""
import collections
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import logging  # noqa: E402

logging.disable(logging.WARNING)
from dcos_commons_amd.benchmarks.deploy_bench import DeployBench  # noqa: E402

cpu = collections.defaultdict(float)
lock = threading.Lock()
orig_run = threading.Thread.run


def run(self, *a, **k):
    t0 = time.thread_time()
    try:
        return orig_run(self, *a, **k)
    finally:
        name = self.name.split("-")[0] if self.name.startswith(("check", "agent", "wait", "Thread")) else self.name
        with lock:
            cpu[name] += time.thread_time() - t0


threading.Thread.run = run
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 20


def runner(task, devices):
    time.sleep(0.00007)
    return True


runner.inline = True
b = DeployBench(n, check_runner=runner, gpu_devices=[0] * n)
for _ in range(3):
    b.run_cycle()
cpu.clear()
t0 = time.thread_time()
deploy = 0.0
for _ in range(cycles):
    deploy += b.run_cycle().deploy_s
cpu["main(bench)"] += time.thread_time() - t0
time.sleep(0.5)
total = sum(cpu.values())
print(f"{n} pods: deploy {deploy / cycles * 1e3:.2f} ms; CPU per cycle (deploy+restart+replace) {total / cycles * 1e3:.2f} ms")
for k, v in sorted(cpu.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v / cycles * 1e3:7.2f} ms")
