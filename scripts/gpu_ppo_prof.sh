#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ppoprof
timeout -k 10 300 python -u scripts/ppo_learner_bench.py > gpurun_out/ppo_learner.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/ppoprof" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/scripts/ppo_learner_bench.py" --iters 2 --warmup 1 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/ppoprof.log" 2>&1
echo "prof rc=$?" >> "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/ppoprof.log"
