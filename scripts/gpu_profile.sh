#!/bin/bash
# GPU box: kernel tests + bench + rocprofv3 kernel stats of the bench step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/kt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/kt.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch 16 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 3 --micro-batch 16 ${BENCH_ARGS} > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log" 2>&1
echo "prof rc=$?" >> "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log"
