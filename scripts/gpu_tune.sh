#!/bin/bash
# kernel tests, then TunableOp-tune the GPT-2 bench GEMMs and measure tuned vs heuristic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/tunableop
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/kt.log 2>&1
echo "pytest rc=$?" >> gpurun_out/kt.log
MB=${MB:-16}
timeout -k 10 900 python bench.py --steps 10 --warmup 3 --micro-batch $MB --tunableop tune > gpurun_out/bench_tune_mb$MB.log 2>&1 || exit $?
cp profiles/tunableop/*.csv gpurun_out/tunableop/ 
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch $MB --tunableop off > gpurun_out/bench_off_mb$MB.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch $MB --tunableop auto > gpurun_out/bench_auto_mb$MB.log 2>&1 || exit $?
