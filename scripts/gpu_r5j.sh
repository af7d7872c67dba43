#!/bin/bash
# round 5, call J: gemm.hip with inline-asm LDS DMA — numerics, then the GPT-2 MLP passes
# fused into GEMM epilogues vs hipBLASLt + separate elementwise kernels
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/mlp_fused_bench.py --rounds 3 --variants 0,3 > $O/mlp.log 2>&1 || { echo "mlp rc=$?"; tail -20 $O/mlp.log; exit 1; }
tail -1 $O/mlp.log
exit 0
