#!/bin/bash
# PPO: conv numerics, learner bench, end-to-end PPO (async + sync) through bench.py
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_rllib_gpu.py -k "conv or nature or bias_relu or ppo or rllib or learner or heads or linear_relu" > gpurun_out/ppo5_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ppo_learner_bench.py > gpurun_out/ppo_learner5.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload ppo --steps 5 --warmup 2 > gpurun_out/bench_ppo5_async.log 2>&1 || exit $?
RAY_AMD_PPO_ASYNC=0 timeout -k 10 400 python -u bench.py --workload ppo --steps 5 --warmup 2 > gpurun_out/bench_ppo5_sync.log 2>&1 || exit $?
echo done
