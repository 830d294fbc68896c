# In-process deploy anatomy on one MI355X box: traced 1- and 8-pod deploy timelines with the HIP
# readiness probe (span wall and thread CPU), and CPU time per thread over 8-pod cycles.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/inproc
SDK_TRACE=1 timeout -k 10 120 python -u scripts/dev/deploy_timeline.py 8 --gpu > gpurun_out/inproc/timeline_n8.txt 2>&1 && \
SDK_TRACE=1 timeout -k 10 120 python -u scripts/dev/deploy_timeline.py 1 --gpu > gpurun_out/inproc/timeline_n1.txt 2>&1 && \
timeout -k 10 120 python -u scripts/dev/thread_cpu.py 8 30 > gpurun_out/inproc/thread_cpu_n8.txt 2>&1 && \
timeout -k 10 120 python -u scripts/dev/thread_cpu.py 1 30 > gpurun_out/inproc/thread_cpu_n1.txt 2>&1
