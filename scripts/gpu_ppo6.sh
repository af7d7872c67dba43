#!/bin/bash
# end-to-end PPO with env-runner inference on fractional GPU shares (8 x 0.125)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
RAY_AMD_RUNNER_GPUS=0.125 timeout -k 10 400 python -u bench.py --workload ppo --steps 5 --warmup 2 > gpurun_out/bench_ppo6_gpurunners.log 2>&1 || exit $?
RAY_AMD_RUNNER_GPUS=0.125 RAY_AMD_PPO_ASYNC=1 timeout -k 10 400 python -u bench.py --workload ppo --steps 5 --warmup 2 > gpurun_out/bench_ppo6_gpurunners_async.log 2>&1 || exit $?
echo done
