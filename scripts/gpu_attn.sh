#!/bin/bash
# flash-attention numerics + kernel timing vs SDPA, then the full GPT-2 profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "flash or gpt2" > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/attn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
PYTHONPATH=$PWD timeout -k 10 180 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || exit $?
cat gpurun_out/attn_bench.log
bash scripts/gpu_profile.sh
