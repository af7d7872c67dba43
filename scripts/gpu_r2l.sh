#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k flash --timeout 120 --timeout-method thread > gpurun_out/t_s2.log 2>&1 || exit $?
RAY_AMD_ATTN_BWD=split2 timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_s2.log 2>&1 || exit $?
RAY_AMD_ATTN_BWD=split timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_s1.log 2>&1 || exit $?
RAY_AMD_ATTN_BWD=split2 timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_s2b.log 2>&1 || exit $?
echo done
