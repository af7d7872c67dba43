#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
(cat /sys/fs/cgroup/cpu.max; nproc; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; python -c "from ray_amd._private.raylet import detect_cpus; print('detect', detect_cpus())") > gpurun_out/cpuinfo.log 2>&1
timeout -k 10 400 python -u bench.py --workload ppo --steps 3 --warmup 1 > gpurun_out/bench_ppo.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload microbench > gpurun_out/bench_micro.log 2>&1 || exit $?
