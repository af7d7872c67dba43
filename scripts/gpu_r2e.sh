#!/bin/bash
# GPU box: HBM object store tests + throughput bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hbm_store_gpu.py tests/test_gpu_object_store.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_hbm.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_hbm.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/hbm_store_bench.py > gpurun_out/hbm_bench.log 2>&1 || exit $?
echo done
