#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
RAY_AMD_WGRAD_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_ws.log 2>&1 || exit $?
RAY_AMD_WGRAD_STREAM=1 timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_ws.log 2>&1 || exit $?
RAY_AMD_WGRAD_STREAM=0 timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_nows.log 2>&1 || exit $?
RAY_AMD_WGRAD_STREAM=1 timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_ws2.log 2>&1 || exit $?
echo done
