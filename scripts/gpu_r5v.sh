#!/bin/bash
# round 5, call V: embedding backward kernel (coalesced atomics) — numerics + timing vs torch
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "embedding or flat_fp32" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/embed_bench.py > $O/embed.log 2>&1 || { echo "embed rc=$?"; tail -5 $O/embed.log; exit 1; }
tail -1 $O/embed.log
exit 0
