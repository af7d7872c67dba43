#!/bin/bash
# GPU box: norm/colsum knob A/B, correctness of the touched kernels, bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/r2_perf_bench.py --part norm > gpurun_out/r2_norm.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py tests/test_kernels_gpu.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_d.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_d.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_d.log 2>&1 || exit $?
echo done
