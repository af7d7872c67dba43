#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_rllib_gpu.py -k "conv or nature or bias_relu or ppo or rllib or learner or heads or linear_relu" > gpurun_out/ppo7_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/conv_bench.py --fwd-caps 0 --wg-rows 512 > gpurun_out/conv_bench7.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ppo_learner_bench.py > gpurun_out/ppo_learner7.log 2>&1 || exit $?
echo done
