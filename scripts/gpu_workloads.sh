#!/bin/bash
# GPU box: the non-default bench workloads (BASELINE.json configs 1, 3, 4, 5), each under
# its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload data --steps 40 --warmup 5 > gpurun_out/bench_data.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload ppo --steps 3 --warmup 1 > gpurun_out/bench_ppo.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload impala --steps 3 --warmup 1 > gpurun_out/bench_impala.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload microbench > gpurun_out/bench_micro.log 2>&1 || exit $?
echo done
