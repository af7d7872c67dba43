#!/bin/bash
# conv kernels: numerics, per-layer microbench (knob sweeps), learner bench + trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
rm -rf gpurun_out/ppoprof4
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "conv or nature or bias_relu" > gpurun_out/conv_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/conv_bench.py --fwd-caps 0 --wg-rows 256,512 > gpurun_out/conv_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ppo_learner_bench.py > gpurun_out/ppo_learner4.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ppoprof4" -o run -- python3 "$R/scripts/ppo_learner_bench.py" --iters 2 --warmup 1 > "$R/gpurun_out/ppoprof4.log" 2>&1 || exit $?
echo done
