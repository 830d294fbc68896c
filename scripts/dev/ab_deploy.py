"""python scripts/dev/ab_deploy.py <repo> <n> <cycles>: helloworld DeployBench of the tree at <repo>, synthetic readiness (0.2 ms GIL-free sleep), pinned to CPUs 4-7; prints mean/median deploy, MTTRs and process CPU per cycle."""
import sys, os, time, json, logging
repo=os.path.abspath(sys.argv[1]); sys.path.insert(0, repo); os.chdir(repo)
logging.disable(logging.WARNING)
os.sched_setaffinity(0,[4,5,6,7])
from dcos_commons_amd.benchmarks.deploy_bench import DeployBench
n=int(sys.argv[2])
b=DeployBench(n, check_runner=lambda t, d: (time.sleep(0.0002), True)[1], gpu_devices=[0]*n)
for _ in range(3): b.run_cycle()
cs=[];ds=[];rs=[];ps=[]
for _ in range(int(sys.argv[3])):
    c0=time.process_time()
    r=b.run_cycle()
    cs.append(time.process_time()-c0); ds.append(r.deploy_s); rs.append(r.mttr_restart_s); ps.append(r.mttr_replace_s)
m=lambda x: round(sum(x)/len(x)*1000,2)
md=lambda x: round(sorted(x)[len(x)//2]*1000,2)
print(json.dumps({"repo":repo,"n":n,"cpu_ms":m(cs),"deploy_ms":m(ds),"deploy_med":md(ds),"restart_ms":m(rs),"replace_ms":m(ps)}))
