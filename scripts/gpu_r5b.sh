#!/bin/bash
# round 5, call B: hand-written wgrad kernel — numerics vs fp32, then speed vs hipBLASLt
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v -k "wgrad" --timeout 120 --timeout-method thread > $O/wgrad_tests.log 2>&1; rc=$?
echo "wgrad tests rc=$rc"; tail -12 $O/wgrad_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/wgrad_bench.py --rounds 3 > $O/wgrad_bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/wgrad_bench.log; exit 1; }
cat $O/wgrad_bench.log
exit 0
