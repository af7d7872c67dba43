#!/bin/bash
# GPU box: attention/kernel numerics tests, GPT-2 bench at the default config, then a
# rocprofv3 kernel-stats pass of a short bench run. MB (default 64) = per-GPU batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
MB=${MB:-64}
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/kt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/kt.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --micro-batch $MB ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 3 --warmup 2 --micro-batch $MB ${BENCH_ARGS} > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log" 2>&1
echo "prof rc=$?" >> "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log"
