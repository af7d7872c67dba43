#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu -k "flash_attention" --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_attn.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_fused.log 2>&1 || exit $?
RAY_AMD_ATTN_BWD=split timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_split.log 2>&1 || exit $?
echo done
