#!/bin/bash
# GPU box: data GPU tests, image_normalize variants, PPO (sync/async) + IMPALA benches.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_data_gpu.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r2g.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_r2g.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/r2_perf_bench.py --part imgnorm > gpurun_out/imgnorm2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload ppo --steps 5 --warmup 2 > gpurun_out/ppo_sync.log 2>&1 || exit $?
RAY_AMD_PPO_ASYNC=1 timeout -k 10 400 python -u bench.py --workload ppo --steps 5 --warmup 2 > gpurun_out/ppo_async.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload impala --steps 5 --warmup 2 > gpurun_out/impala.log 2>&1 || exit $?
echo done
