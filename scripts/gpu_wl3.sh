#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload ppo --steps 3 --warmup 1 > gpurun_out/bench_ppo_gpurunner.log 2>&1 || exit $?
RAY_AMD_RUNNER_GPUS=0 timeout -k 10 400 python -u bench.py --workload ppo --steps 3 --warmup 1 > gpurun_out/bench_ppo_cpurunner.log 2>&1 || exit $?
